"""Restated ledger commit hash (TEST INFRASTRUCTURE ONLY -- the oracle).

Follows (citations under /root/reference):
  core/ledger/kvledger/kv_ledger.go:806-817   addBlockCommitHash: commitHash = SHA-256(
        varint(len(TRANSACTIONS_FILTER)) || TRANSACTIONS_FILTER || updateBatchBytes || prevCommitHash),
        stored as Metadata{value} in Metadata[COMMIT_HASH]; computed for block 1 on and whenever a
        previous commit hash exists (kv_ledger.go:647-652)
  core/ledger/kvledger/txmgmt/txmgr/update_batch_bytes.go:29-105  deterministicBytesForPubAndHashUpdates:
        namespaces of the public and hashed updates deduplicated and sorted, "" (channel config)
        skipped; per namespace its public writes sorted by key, then per collection (sorted) its
        hashed writes sorted by key hash; the first write of a namespace carries the namespace and the
        first of a collection the collection; KVWrite{namespace 1, collection 2, key 3, isDelete 4,
        value 5, version_bytes 6} (txmgr/updates.proto) in an Updates{kvwrites 1} message
  core/ledger/internal/version/version.go:50-54 + common/ledger/util/util.go:32-52  Height.ToBytes =
        EncodeOrderPreservingVarUint64(blockNum) || ...(txNum)
  validation/types.go:81-112 + tx_ops.go   the update batch: puts / deletes of the VALID endorser
        transactions at Height{blockNum, txIdx}, a later transaction's write of a key replacing an
        earlier one; CONFIG transactions write only namespace "" (core/peer/configtx_processor.go:19-39)
Metadata writes (their merged values come from the state DB) are outside the model -> Unsupported.
"""
import hashlib

from .protowire import decode
from .v20 import Unsupported, get_action_from_envelope, parse_rwset

_EMPTY_HASH = hashlib.sha256(b"").digest()


def _pvarint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _fld(num, payload):
    return _pvarint(num << 3 | 2) + _pvarint(len(payload)) + payload


def order_preserving_varuint64(n):
    b = n.to_bytes(8, "big")
    for i, x in enumerate(b):
        if x:
            return bytes([8 - i]) + b[i:]
    return b"\x00"


def height_bytes(block_num, tx_num):
    return order_preserving_varuint64(block_num) + order_preserving_varuint64(tx_num)


def update_batch(block_bytes, flags, block_num):
    """-> (pub {ns: {key bytes: (value|None, (blk, tx))}}, hashed {ns: {coll: {keyhash: ...}}})"""
    blk = decode("Block", block_bytes)
    data = (blk.get("data") or {}).get("data", [])
    pub, hashed = {}, {}
    for i, d in enumerate(data):
        if flags[i] != 0:
            continue
        env = decode("Envelope", d)
        pl = decode("Payload", env.get("payload"))
        chdr = decode("ChannelHeader", (pl.get("header") or {}).get("channel_header"))
        t = chdr.get("type", 0)
        if t == 1:
            continue  # CONFIG: the channel config under namespace "" (skipped by the hash)
        if t != 3:
            raise Unsupported("valid non-endorser transaction type %d" % t)
        cca, _ = get_action_from_envelope(d)
        for ns in parse_rwset(cca.get("results")):
            kv = ns["kv"]
            if kv.get("metadata_writes") or any(c["hashed"].get("metadata_writes") for c in ns["coll"]):
                raise Unsupported("metadata writes")
            seen = set()
            for w in kv.get("writes", []):
                k = (w.get("key") or "").encode()
                if ("", k) in seen:
                    raise Unsupported("key written twice by one transaction")
                seen.add(("", k))
                v = w.get("value")
                dl = bool(w.get("is_delete")) or not v
                pub.setdefault(ns["namespace"], {})[k] = (None if dl else bytes(v), (block_num, i))
            for c in ns["coll"]:
                for w in c["hashed"].get("hashed_writes", []):
                    k = bytes(w.get("key_hash") or b"")
                    if (c["name"], k) in seen:
                        raise Unsupported("key written twice by one transaction")
                    seen.add((c["name"], k))
                    vh = bytes(w.get("value_hash") or b"")
                    dl = bool(w.get("is_delete")) or not vh or vh == _EMPTY_HASH
                    hashed.setdefault(ns["namespace"], {}).setdefault(c["name"], {})[k] = (None if dl else vh, (block_num, i))
    return pub, hashed


def _kvwrite(ns, coll, key, value, height):
    m = b""
    if ns:
        m += _fld(1, ns.encode())
    if coll:
        m += _fld(2, coll.encode())
    if key:
        m += _fld(3, key)
    if value is None:
        m += b"\x20\x01"  # isDelete = true
    elif value:
        m += _fld(5, value)
    return m + _fld(6, height_bytes(*height))


def update_batch_bytes(pub, hashed):
    out = b""
    for ns in sorted(set(pub) | set(hashed)):
        if ns == "":
            continue
        items = [("", k, pub[ns][k]) for k in sorted(pub.get(ns, {}))]
        for coll in sorted(hashed.get(ns, {})):
            items += [(coll if j == 0 else "", k, hashed[ns][coll][k]) for j, k in enumerate(sorted(hashed[ns][coll]))]
        for j, (coll, k, (v, h)) in enumerate(items):
            out += _fld(1, _kvwrite(ns if j == 0 else "", coll, k, v, h))
    return out


def commit_hash(flags, batch_bytes, prev):
    return hashlib.sha256(_pvarint(len(flags)) + bytes(flags) + batch_bytes + (prev or b"")).digest()


def block_commit_hash(block_bytes, flags, block_num, prev):
    pub, hashed = update_batch(block_bytes, flags, block_num)
    return commit_hash(flags, update_batch_bytes(pub, hashed), prev)
