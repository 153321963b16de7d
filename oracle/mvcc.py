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
Range queries (phantom checks) and metadata writes are outside the modelled state and raise
Unsupported.
"""
import hashlib

from .protowire import DecodeError, decode
from .v20 import Unsupported, get_action_from_envelope, parse_rwset

MVCC_READ_CONFLICT, NIL_TXACTION, INVALID_OTHER_REASON = 11, 16, 255
_EMPTY_HASH = hashlib.sha256(b"").digest()


def hashed_ns(ns, coll):
    """privacyenabledstate.deriveHashedDataNs (privacyenabledstate/db.go:355-357)"""
    return ns + "$$h" + coll


class StateDB:
    """committed versions: {(ns, key): (block_num, tx_num)}"""

    def __init__(self, versions=None):
        self.v = dict(versions or {})

    def get_version(self, ns, key):
        return self.v.get((ns, key))


def _tx_rwsets(env_bytes):
    """-> list of (ns, reads[(key, ver|None)], writes[(key, is_delete)]) or an int code."""
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
    return out


def validate_block(state, block_bytes, flags, block_num, commit=False):
    """flags: committer TxValidationFlags (list of ints) -> new flags list."""
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
        for ns, reads, _ in sets:
            for key, ver in reads:
                if (ns, key) in updates or state.get_version(ns, key) != ver:
                    ok = False
                    break
            if not ok:
                break
        if not ok:
            flags[i] = MVCC_READ_CONFLICT
            continue
        for ns, _, writes in sets:
            for key, is_del in writes:
                updates[(ns, key)] = ((block_num, i), is_del)
    if commit:
        for k, (h, is_del) in updates.items():
            if is_del:
                state.v.pop(k, None)
            else:
                state.v[k] = h
    return flags
