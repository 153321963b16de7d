"""Restated MVCC validation of one block (TEST INFRASTRUCTURE ONLY -- the oracle).

Follows (citations under /root/reference/core/ledger/kvledger/txmgmt):
  validation/batch_preparer.go:192-286  preprocessProtoBlock: skip txs already invalid in the
        committer's TRANSACTIONS_FILTER; GetActionFromEnvelope error -> NIL_TXACTION(16);
        rwset parse error -> INVALID_OTHER_REASON(255); (LevelDB: validateWriteset is a no-op)
  validation/validator.go:81-118        validateAndPrepareBatch: transactions in block order;
        a VALID tx's write set enters `updates` at Height{blockNum, txIdx}
  validation/validator.go:134-200       validateTx / validateKVRead: MVCC_READ_CONFLICT(11) if
        the key was written by an earlier VALID tx of this block (updates.Exists) or the
        committed version differs from the read version (version.AreSame; nil <=> absent)
  validation/tx_ops.go + types.go:81-112 applyWriteSet: puts and deletes enter `updates`;
        a write is a delete when rwsetutil.IsKVWriteDelete / IsKVWriteHashDelete say so
        (rwsetutil/rwset_proto_util.go:366-375: is_delete, empty value, or value hash ==
        SHA-256 of the empty string)
  validation/validator.go:246-293       validateNsHashedReadSets / validateKVReadHash: hashed
        reads are point reads of the key hash in the hashed-data namespace; the state DB keeps
        them under ns + "$$h" + coll (privacyenabledstate/db.go:31-33,355-357), which is the
        (namespace, key) the oracle and the engine use for them
  validation/validator.go:134-162       per namespace in order: public reads (11), then range
        queries (PHANTOM_READ_CONFLICT 12, oracle/rangequery.py), then the collections' hashed
        reads (11)
  validation/tx_ops.go:17-53,97-230     prepareTxOps: per key a delete wins, an upsert puts, and a
        metadata-only write puts the key's latest value again (a new version) if the key exists
        in the preceding updates or the committed state, else it is a no-op
  validation/tx_ops.go:17-53,97-148 + statemetadata/metadata.go  the keys' metadata at commit:
        a delete drops it, an upsert keeps it (retrieveLatestMetadata), a metadata write beside
        an upsert replaces it, a metadata-only write replaces it when the key exists (entries
        nil: deleted); the state's VALIDATION_PARAMETER (last entry of that name) is what the
        key-level endorsement check reads (StateDB.kvmeta, oracle/v20.py ChannelModel.kvmeta)
A key written twice (or given two metadata writes) by one transaction is outside the modelled
state (txOps adds the operation flags) and raises Unsupported; so does what the reference errors
out or panics on: a range query with maxDegree < 2 or a versionless raw read, a metadata write to
a key an earlier transaction of the block deleted (PutValAndMetadata(nil value)).
"""
import bisect
import hashlib

from .protowire import DecodeError, decode
from .rangequery import RangeQueryError, combined_iterator, validate_range_query
from .v20 import Unsupported, get_action_from_envelope, parse_rwset

MVCC_READ_CONFLICT, PHANTOM_READ_CONFLICT, NIL_TXACTION, INVALID_OTHER_REASON = 11, 12, 16, 255
_EMPTY_HASH = hashlib.sha256(b"").digest()


def hashed_ns(ns, coll):
    """privacyenabledstate.deriveHashedDataNs (privacyenabledstate/db.go:355-357)"""
    return ns + "$$h" + coll


def _kb(key):
    """state DB keys are bytes (public keys are UTF-8 strings, hashed keys raw hash bytes)"""
    return key.encode() if isinstance(key, str) else bytes(key)


class StateDB:
    """committed versions: {(ns, key bytes): (block_num, tx_num)}; kvmeta: the keys'
    VALIDATION_PARAMETER metadata {(ns, coll, key bytes): bytes} (coll "" = public)"""

    def __init__(self, versions=None, kvmeta=None):
        self.v = {(ns, _kb(k)): h for (ns, k), h in dict(versions or {}).items()}
        self.kvmeta = dict(kvmeta or {})

    def get_version(self, ns, key):
        return self.v.get((ns, _kb(key)))

    def range(self, ns, start, end):
        """GetStateRangeScanIterator: keys of ns in [start, end), end b"" = no bound; sorted"""
        out = sorted((k, h) for (n, k), h in self.v.items()
                     if n == ns and k >= start and (end == b"" or k < end))
        return out


def _ver(v):
    return None if v is None else (v.get("block_num", 0), v.get("tx_num", 0))


def _tx_rwsets(env_bytes):
    """-> list, per NsReadWriteSet in order, of dict(ns, reads [(key, ver|None)], rqs [dict],
    colls [(hashed ns, hashed reads [(key hash, ver|None)])], writes [(hashed, ns, key,
    is_delete)]) -- or an int code."""
    try:
        cca, _ = get_action_from_envelope(env_bytes)
    except (DecodeError, ValueError, KeyError, IndexError):
        return NIL_TXACTION
    try:
        rw = parse_rwset(cca.get("results"))
    except DecodeError:
        return INVALID_OTHER_REASON
    out = []
    for ns in rw:
        kv = ns["kv"]
        name = ns["namespace"]
        e = dict(ns=name, reads=[], rqs=[], colls=[], writes=[], meta=[], mdw=[], dels=[])
        for m in kv.get("metadata_writes", []):
            e["meta"].append((False, name, m.get("key", "")))
            e["mdw"].append((False, "", name, _kb(m.get("key", "")), _vp(m)))
        for r in kv.get("reads", []):
            e["reads"].append((r.get("key", ""), _ver(r.get("version"))))
        for q in kv.get("range_queries_info", []):
            rq = dict(start=_kb(q.get("start_key", "")), end=_kb(q.get("end_key", "")),
                      exhausted=bool(q.get("itr_exhausted", False)), raw=None, merkle=None)
            if q.get("raw_reads") is not None:
                rq["raw"] = [(_kb(r.get("key", "")), _ver(r.get("version")))
                             for r in q["raw_reads"].get("kv_reads", [])]
            if q.get("reads_merkle_hashes") is not None:
                m = q["reads_merkle_hashes"]
                rq["merkle"] = (m.get("max_degree", 0), m.get("max_level", 0),
                                [bytes(h) for h in m.get("max_level_hashes", [])])
            e["rqs"].append(rq)
        for w in kv.get("writes", []):
            e["writes"].append((False, name, w.get("key", ""), bool(w.get("is_delete", False)) or not w.get("value")))
            if e["writes"][-1][3]:
                e["dels"].append(("", _kb(w.get("key", ""))))
        for c in ns["coll"]:
            hns, h = hashed_ns(name, c["name"]), c["hashed"]
            e["colls"].append((hns, [(bytes(r.get("key_hash") or b""), _ver(r.get("version")))
                                     for r in h.get("hashed_reads", [])]))
            for w in h.get("hashed_writes", []):
                vh = bytes(w.get("value_hash") or b"")
                e["writes"].append((True, hns, bytes(w.get("key_hash") or b""),
                                    bool(w.get("is_delete", False)) or not vh or vh == _EMPTY_HASH))
                if e["writes"][-1][3]:
                    e["dels"].append((c["name"], bytes(w.get("key_hash") or b"")))
            for m in h.get("metadata_writes", []):
                e["meta"].append((True, hns, bytes(m.get("key_hash") or b"")))
                e["mdw"].append((True, c["name"], hns, bytes(m.get("key_hash") or b""), _vp(m)))
        out.append(e)
    # a key written twice by one transaction: txOps adds the operation flags
    # (validation/tx_ops.go:183-191), a state the engine does not model
    seen, mseen = set(), set()
    for e in out:
        for hashed, nsname, key, _ in e["writes"]:
            if (hashed, nsname, _kb(key)) in seen:
                raise Unsupported("key written twice by one transaction")
            seen.add((hashed, nsname, _kb(key)))
    for e in out:
        for hashed, nsname, key in e["meta"]:
            if (hashed, nsname, _kb(key)) in mseen:
                raise Unsupported("two metadata writes of one key in one transaction")
            mseen.add((hashed, nsname, _kb(key)))
    for e in out:  # a metadata write beside a KVWrite of the key follows the write
        e["meta"] = [m for m in e["meta"] if (m[0], m[1], _kb(m[2])) not in seen]
    return out


def _vp(mw):
    """statemetadata.Deserialize(...)[VALIDATION_PARAMETER]: the last entry of that name"""
    vp = b""
    for en in mw.get("entries", []):
        if en.get("name", "") == "VALIDATION_PARAMETER":
            vp = bytes(en.get("value") or b"")
    return vp


def _range_ok(state, updates, ns, rq):
    """validateRangeQuery (validator.go:218-244) over committed state + public updates"""
    start, end = rq["start"], rq["end"]
    db_items = [(k, h, False) for k, h in state.range(ns, start, end)]
    keys = sorted(k for (hashed, n, k) in updates if not hashed and n == ns)
    lo = bisect.bisect_left(keys, start) if start else 0
    hi = bisect.bisect_left(keys, end) if end else len(keys)
    upd_items = [(k, updates[(False, ns, k)][0], updates[(False, ns, k)][1]) for k in keys[lo:hi]]

    def end_lookup():  # serveEndKeyIfNeeded: updates.Get, else db.GetState
        u = updates.get((False, ns, end))
        if u is not None:
            return u
        h = state.get_version(ns, end)
        return None if h is None else (h, False)

    itr = combined_iterator(db_items, upd_items, end, not rq["exhausted"], end_lookup)
    try:
        return validate_range_query(rq, itr)
    except RangeQueryError as e:
        raise Unsupported("range query the reference errors out on: %s" % e)


def validate_block(state, block_bytes, flags, block_num, commit=False, updates_out=None):
    """flags: committer TxValidationFlags (list of ints) -> new flags list.  updates_out (dict):
    receives the block's update batch {(hashed, ns, key bytes): (height, is_delete)}."""
    blk = decode("Block", block_bytes)
    data = (blk.get("data") or {}).get("data", [])
    flags = list(flags)
    updates = {}  # (ns, key) -> (height, is_delete)
    kvops = []    # key-level parameter changes in block order: ((ns, coll, key), vp | b"")
    for i, d in enumerate(data):
        if flags[i] != 0:
            continue
        try:
            env = decode("Envelope", d)
            payl = decode("Payload", env.get("payload"))
            if payl.get("header") is None:
                raise Unsupported("nil payload header (the reference dereferences nil)")
            chdr = decode("ChannelHeader", payl["header"].get("channel_header"))
        except DecodeError:
            raise Unsupported("unparsable committer-valid envelope (the reference halts)")
        if chdr.get("type", 0) != 3:
            raise Unsupported("non-endorser transaction in MVCC")
        sets = _tx_rwsets(d)
        if isinstance(sets, int):
            flags[i] = sets
            continue
        code = 0
        for e in sets:  # validateTx (validator.go:134-162)
            ns = e["ns"]
            if any((False, ns, _kb(k)) in updates or state.get_version(ns, k) != v for k, v in e["reads"]):
                code = MVCC_READ_CONFLICT
            elif not all(_range_ok(state, updates, ns, rq) for rq in e["rqs"]):
                code = PHANTOM_READ_CONFLICT
            elif any((True, hns, _kb(k)) in updates or state.get_version(hns, k) != v
                     for hns, hreads in e["colls"] for k, v in hreads):
                code = MVCC_READ_CONFLICT
            if code:
                break
        if code:
            flags[i] = code
            continue
        for e in sets:
            for hashed, ns, key, is_del in e["writes"]:
                updates[(hashed, ns, _kb(key))] = ((block_num, i), is_del)
        for e in sets:  # metadata-only writes (prepareTxOps: retrieveLatestState)
            for hashed, ns, key in e["meta"]:
                u = updates.get((hashed, ns, _kb(key)))
                if u is not None and u[1]:
                    raise Unsupported("metadata write to a key deleted earlier in the block (the reference panics)")
                if u is not None or state.get_version(ns, key) is not None:
                    updates[(hashed, ns, _kb(key))] = ((block_num, i), False)
        for e in sets:  # the keys' metadata (tx_ops.go:17-53, 97-148)
            wr = {(h, n, _kb(k)): d for h, n, k, d in e["writes"]}
            for coll, key in e["dels"]:
                kvops.append(((e["ns"], coll, key), b""))
            for hashed, coll, fns, key, vp in e["mdw"]:
                d = wr.get((hashed, fns, key))
                if d is None:  # metadata only: replaced iff the key exists (its update is this tx's)
                    u = updates.get((hashed, fns, key))
                    if u is None or u[0] != (block_num, i):
                        continue
                elif d:
                    continue
                kvops.append(((e["ns"], coll, key), vp))
    if updates_out is not None:
        updates_out.update(updates)
    if commit:
        for (_, ns, key), (h, is_del) in updates.items():
            if is_del:
                state.v.pop((ns, _kb(key)), None)
            else:
                state.v[(ns, _kb(key))] = h
        for k, vp in kvops:
            if vp:
                state.kvmeta[k] = vp
            else:
                state.kvmeta.pop(k, None)
    return flags
