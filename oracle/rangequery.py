"""Restated phantom-read validation of range queries (TEST INFRASTRUCTURE ONLY -- the oracle).

Follows (citations under /root/reference/core/ledger/kvledger/txmgmt):
  validation/validator.go:205-244        validateRangeQueries / validateRangeQuery: a combined
        iterator over the committed state and the block's update batch; raw KVReads or a
        merkle summary decide which validator runs (GetReadsMerkleHashes() != nil -> hashes)
  validation/combined_iterator.go:43-177 the merge of the DB range scan [start, end) and the
        updates' range scan; the updates win on equal keys, deletes are skipped, and the end key
        is served once more at the end when the simulation did not exhaust the iterator
  validation/rangequery_validator.go     rangeQueryResultsValidator (raw KVReads, first
        mismatch fails, extra results fail) and rangeQueryHashValidator (incremental merkle
        tree compared level by level, merkleSummariesEqual at the end)
  rwsetutil/query_results_helper.go      RangeQueryResultsHelper / merkleTree: leaves are the
        SHA-256 of proto.Marshal(QueryReads{kv_reads}) of maxDegree+1 results
  statedb/stateleveldb/stateleveldb.go:152-173  DB scan: start inclusive, end exclusive, end ""
        = to the end of the namespace; statedb/statedb.go:281-300 the same for the updates
The hash function is the ledger's SHA-256 (the tests' testHashFunc is SHA-256 too).
"""
import hashlib


class RangeQueryError(Exception):
    """the reference returns an error (not a validation code): the peer would stop"""


def _pb_varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _pb_len(field, payload):
    return _pb_varint(field << 3 | 2) + _pb_varint(len(payload)) + payload


def marshal_query_reads(kv_reads):
    """proto.Marshal(&kvrwset.QueryReads{KvReads: kv_reads}); kv_reads [(key bytes, (blk, tx))].
    KVRead{key = 1 (omitted when empty), version = 2 (always present: NewKVRead of a committed or
    updated height)}; Version{block_num = 1, tx_num = 2} (zero fields omitted)."""
    out = b""
    for key, (blk, tx) in kv_reads:
        ver = (_pb_varint(1 << 3) + _pb_varint(blk) if blk else b"") + (_pb_varint(2 << 3) + _pb_varint(tx) if tx else b"")
        msg = (_pb_len(1, key) if key else b"") + _pb_len(2, ver)
        out += _pb_len(1, msg)
    return out


def sha256(b):
    return hashlib.sha256(b).digest()


class MerkleTree:
    """rwsetutil/query_results_helper.go:146-262"""

    def __init__(self, max_degree):
        if max_degree < 2:
            raise RangeQueryError("maxDegree [%d] should not be less than 2 in the merkle tree" % max_degree)
        self.tree = {}
        self.max_level = 1
        self.max_degree = max_degree

    def update(self, h):
        self.tree.setdefault(1, []).append(h)
        level = 1
        while True:
            hashes = self.tree.get(level, [])
            if len(hashes) <= self.max_degree:
                return
            nxt = sha256(b"".join(hashes))
            del self.tree[level]
            level += 1
            self.tree.setdefault(level, []).append(nxt)
            if level > self.max_level:
                self.max_level = level

    def done(self):
        level = 1
        h = None
        while level < self.max_level:
            hashes = self.tree.get(level, [])
            if len(hashes) == 0:
                level += 1
                continue
            h = hashes[0] if len(hashes) == 1 else sha256(b"".join(hashes))
            self.tree.pop(level, None)
            level += 1
            self.tree.setdefault(level, []).append(h)
        final = self.tree.get(self.max_level, [])
        if len(final) > self.max_degree:
            del self.tree[self.max_level]
            self.max_level += 1
            self.tree[self.max_level] = [sha256(b"".join(final))]

    def summary(self):
        return (self.max_degree, self.max_level, list(self.tree.get(self.max_level, [])))

    def is_empty(self):
        return self.max_level == 1 and len(self.tree.get(1, [])) == 0


class ResultsHelper:
    """RangeQueryResultsHelper with hashing enabled"""

    def __init__(self, max_degree):
        self.pending = []
        self.max_degree = max_degree
        self.mt = MerkleTree(max_degree)

    def add(self, kv):
        self.pending.append(kv)
        if len(self.pending) > self.max_degree:
            self._process()

    def _process(self):
        b = marshal_query_reads(self.pending)
        self.pending = []
        self.mt.update(sha256(b))

    def summary(self):
        return self.mt.summary()

    def done(self):
        if self.mt.is_empty():
            return None
        if self.pending:
            self._process()
        self.mt.done()
        return self.mt.summary()


def combined_iterator(db_items, upd_items, end_key, include_end, end_lookup):
    """combined_iterator.go: db_items / upd_items sorted [(key bytes, version, is_delete)] of the
    range; end_lookup() -> (version, is_delete) or None for the served end key."""
    i = j = 0
    while i < len(db_items) or j < len(upd_items):
        if j >= len(upd_items) or (i < len(db_items) and db_items[i][0] < upd_items[j][0]):
            sel = db_items[i]
            i += 1
        elif i >= len(db_items) or upd_items[j][0] < db_items[i][0]:
            sel = upd_items[j]
            j += 1
        else:  # equal keys: the update (latest) wins, both advance
            sel = upd_items[j]
            i += 1
            j += 1
        if not sel[2]:
            yield sel[0], sel[1]
    if include_end:
        r = end_lookup()
        if r is not None and not r[1]:
            yield end_key, r[0]


def validate_range_query(rq, itr):
    """rangeQueryResultsValidator / rangeQueryHashValidator.  rq: dict(raw=[(key, ver|None)] or
    None, merkle=(max_degree, max_level, [hashes]) or None); itr: the combined iterator."""
    if rq.get("merkle") is not None:
        max_degree, max_level, in_hashes = rq["merkle"]
        helper = ResultsHelper(max_degree)  # (raises RangeQueryError for max_degree < 2)
        last = -1
        for key, ver in itr:
            helper.add((key, ver))
            _, lvl, hashes = helper.summary()
            if lvl < max_level:
                continue
            if last == len(hashes) - 1:
                continue
            if len(hashes) > len(in_hashes):
                return False
            last += 1
            if hashes[last] != in_hashes[last]:
                return False
        got = helper.done()
        return got is not None and got[0] == max_degree and got[1] == max_level and got[2] == list(in_hashes)
    raw = rq.get("raw") or []
    results = iter(itr)
    cur = next(results, None)
    if not raw:
        return cur is None
    for key, ver in raw:
        if cur is None or cur[0] != key:
            return False
        if ver is None:  # convertToVersionHeight(nil) dereferences nil: the reference panics
            raise RangeQueryError("range query raw read without a version")
        if cur[1] != ver:
            return False
        cur = next(results, None)
    return cur is None
