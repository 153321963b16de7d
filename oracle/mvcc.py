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
Range queries (phantom checks), metadata writes and a key written twice by one transaction
are outside the modelled state and raise Unsupported.
"""
import hashlib

from .protowire import DecodeError, decode
from .v20 import Unsupported, get_action_from_envelope, parse_rwset

MVCC_READ_CONFLICT, NIL_TXACTION, INVALID_OTHER_REASON = 11, 16, 255
_EMPTY_HASH = hashlib.sha256(b"").digest()


def hashed_ns(ns, coll):
    """privacyenabledstate.deriveHashedDataNs (privacyenabledstate/db.go:355-357)"""
    return ns + "$$h" + coll


def _kb(key):
    """state DB keys are bytes (public keys are UTF-8 strings, hashed keys raw hash bytes)"""
    return key.encode() if isinstance(key, str) else bytes(key)


class StateDB:
    """committed versions: {(ns, key bytes): (block_num, tx_num)}"""

    def __init__(self, versions=None):
        self.v = {(ns, _kb(k)): h for (ns, k), h in dict(versions or {}).items()}

    def get_version(self, ns, key):
        return self.v.get((ns, _kb(key)))


def _tx_rwsets(env_bytes):
    """-> list of (ns, reads[(key, ver|None)], writes[(key, is_delete)], hashed) or an int code."""
    try:
        cca, _ = get_action_from_envelope(env_bytes)
    except (DecodeError, ValueError, KeyError, IndexError):
        return NIL_TXACTION
    try:
        rw = parse_rwset(cca.get("results"))
    except DecodeError:
        return INVALID_OTHER_REASON
    out, kinds = [], []
    for ns in rw:
        kv = ns["kv"]
        if kv.get("range_queries_info") or kv.get("metadata_writes"):
            raise Unsupported("range queries / metadata writes")
        if any(c["hashed"].get("metadata_writes") for c in ns["coll"]):
            raise Unsupported("private-data metadata writes")
        reads = []
        for r in kv.get("reads", []):
            v = r.get("version")
            reads.append((r.get("key", ""), None if v is None else (v.get("block_num", 0), v.get("tx_num", 0))))
        writes = [(w.get("key", ""), bool(w.get("is_delete", False)) or not w.get("value"))
                  for w in kv.get("writes", [])]
        out.append((ns["namespace"], reads, writes))
        kinds.append(False)
        for c in ns["coll"]:
            hns, h = hashed_ns(ns["namespace"], c["name"]), c["hashed"]
            hreads = []
            for r in h.get("hashed_reads", []):
                v = r.get("version")
                hreads.append((bytes(r.get("key_hash") or b""),
                               None if v is None else (v.get("block_num", 0), v.get("tx_num", 0))))
            hwrites = []
            for w in h.get("hashed_writes", []):
                vh = bytes(w.get("value_hash") or b"")
                hwrites.append((bytes(w.get("key_hash") or b""),
                                bool(w.get("is_delete", False)) or not vh or vh == _EMPTY_HASH))
            out.append((hns, hreads, hwrites))
            kinds.append(True)
    # a key written twice by one transaction: txOps adds the operation flags
    # (validation/tx_ops.go:183-191), a state the engine does not model
    seen = set()
    for hashed, (nsname, _, writes) in zip(kinds, out):
        for key, _ in writes:
            if (hashed, nsname, key) in seen:
                raise Unsupported("key written twice by one transaction")
            seen.add((hashed, nsname, key))
    # public and hashed updates are separate maps (privacyenabledstate.UpdateBatch); committed
    # versions of both live under the flattened namespace (one state DB key space)
    return [(ns, reads, writes, hashed) for hashed, (ns, reads, writes) in zip(kinds, out)]


def validate_block(state, block_bytes, flags, block_num, commit=False, updates_out=None):
    """flags: committer TxValidationFlags (list of ints) -> new flags list.  updates_out (dict):
    receives the block's update batch {(hashed, ns, key bytes): (height, is_delete)}."""
    blk = decode("Block", block_bytes)
    data = (blk.get("data") or {}).get("data", [])
    flags = list(flags)
    updates = {}  # (ns, key) -> (height, is_delete)
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
        ok = True
        for ns, reads, _, hashed in sets:
            for key, ver in reads:
                if (hashed, ns, _kb(key)) in updates or state.get_version(ns, key) != ver:
                    ok = False
                    break
            if not ok:
                break
        if not ok:
            flags[i] = MVCC_READ_CONFLICT
            continue
        for ns, _, writes, hashed in sets:
            for key, is_del in writes:
                updates[(hashed, ns, _kb(key))] = ((block_num, i), is_del)
    if updates_out is not None:
        updates_out.update(updates)
    if commit:
        for (_, ns, key), (h, is_del) in updates.items():
            if is_del:
                state.v.pop((ns, _kb(key)), None)
            else:
                state.v[(ns, _kb(key))] = h
    return flags
