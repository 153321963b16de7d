"""CPU: the restated phantom-read validation (oracle/rangequery.py, oracle/mvcc.py) pinned by the
reference's own tests and fixtures:
  * rwsetutil/testdata/kvrwsetV1ProtoBytes (a KVRWSet with a raw-reads and a merkle range query,
    written by proto.Marshal in the reference's tests; tests/golden/kvrwset_v1_range_queries.bin)
    pins the QueryReads serialization the merkle leaves hash;
  * rwsetutil/query_results_helper_test.go: the tree shapes (one / two / three levels, the level
    increment and the first-level skip in Done) against their closed-form construction;
  * validation/{validator,rangequery_validator,combined_iterator}_test.go known answers
    (tests/rq_cases.py)."""
import hashlib
import os

import pytest

from oracle import mvcc as OM
from oracle.protowire import decode
from oracle.rangequery import ResultsHelper, marshal_query_reads
from tests import rq_cases as RQ

HERE = os.path.dirname(os.path.abspath(__file__))


def _field_bytes(buf, field):
    """raw payloads of the length-delimited occurrences of `field` in a message"""
    out, i = [], 0
    while i < len(buf):
        tag, i = _varint(buf, i)
        wt = tag & 7
        if wt == 2:
            n, i = _varint(buf, i)
            if tag >> 3 == field:
                out.append(buf[i:i + n])
            i += n
        elif wt == 0:
            _, i = _varint(buf, i)
        else:
            raise AssertionError("unexpected wire type")
    return out


def _varint(b, i):
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, i


def test_query_reads_serialization_matches_reference_fixture():
    b = open(os.path.join(HERE, "golden", "kvrwset_v1_range_queries.bin"), "rb").read()
    rq1 = _field_bytes(b, 2)[0]                  # KVRWSet.range_queries_info[0]
    raw = _field_bytes(rq1, 4)[0]                # RangeQueryInfo.raw_reads (QueryReads)
    assert marshal_query_reads([(b"k1", (1, 1)), (b"k2", (1, 2))]) == raw
    d = decode("KVRWSet", b)
    assert d["range_queries_info"][1]["reads_merkle_hashes"] == {
        "max_degree": 5, "max_level": 4, "max_level_hashes": [b"Hash-1", b"Hash-2"]}


def _leaf(kvs):
    return hashlib.sha256(marshal_query_reads(kvs)).digest()


def _comb(*hs):
    return hashlib.sha256(b"".join(hs)).digest()


def _kvs(n):
    """buildTestKVReads: key_i at Height{1, i}"""
    return [(b"key_%d" % i, (1, i)) for i in range(n)]


def _build(deg, kvs):
    h = ResultsHelper(deg)
    for kv in kvs:
        h.add(kv)
    return h.done()


@pytest.mark.parametrize("case", ["one", "two", "three", "increment", "skip", "small"])
def test_merkle_shapes_match_query_results_helper_test(case):
    if case == "small":  # TestQueryResultHelper_ResultsNoMoreThanMaxDegree: no summary
        assert _build(3, _kvs(3)) is None
        return
    if case == "one":
        k = _kvs(9)
        exp = (3, 1, [_leaf(k[0:4]), _leaf(k[4:8]), _leaf(k[8:])])
        assert _build(3, k) == exp
    elif case == "two":
        k = _kvs(25)
        l1 = [_leaf(k[i:i + 4]) for i in range(0, 24, 4)] + [_leaf(k[24:])]
        assert _build(3, k) == (3, 2, [_comb(*l1[0:4]), _comb(*l1[4:7])])
    elif case == "three":
        k = _kvs(65)
        l1 = [_leaf(k[i:i + 4]) for i in range(0, 64, 4)] + [_leaf(k[64:])]
        l2 = [_comb(*l1[i:i + 4]) for i in range(0, 16, 4)]
        assert _build(3, k) == (3, 3, [_comb(*l2), l1[16]])
    elif case == "increment":
        k = _kvs(24)
        l1 = [_leaf(k[i:i + 3]) for i in range(0, 24, 3)]
        l2 = [_comb(*l1[0:3]), _comb(*l1[3:6]), _comb(*l1[6:8])]
        assert _build(2, k) == (2, 3, [_comb(*l2)])
    elif case == "skip":
        k = _kvs(45)
        l1 = [_leaf(k[i:i + 3]) for i in range(0, 45, 3)]
        l2 = [_comb(*l1[i:i + 3]) for i in range(0, 15, 3)]
        assert _build(2, k) == (2, 3, [_comb(*l2[0:3]), _comb(*l2[3:5])])


@pytest.mark.parametrize("case", RQ.known_answer_cases(), ids=lambda c: c[0])
def test_reference_known_answers(case):
    name, db, envs, expected, blk = case
    out = OM.validate_block(OM.StateDB(db), _blk(envs), [0] * len(envs), blk)
    assert out == expected, name


def _blk(envs):
    from tests.blockfix import block_from_envs
    return block_from_envs(envs)


def test_unsupported_merkle_degree_and_versionless_raw_read():
    from oracle.v20 import Unsupported
    db = RQ.phantom_db()
    with pytest.raises(Unsupported):  # NewRangeQueryResultsHelper: maxDegree < 2 is an error
        OM.validate_block(OM.StateDB(db), _blk([RQ.tx(rqs=[RQ.rqi("key1", "key3", True, merkle=(1, 1, [b"x"]))])]),
                          [0], 7)
    with pytest.raises(Unsupported):  # convertToVersionHeight(nil): the reference panics
        OM.validate_block(OM.StateDB(db), _blk([RQ.tx(rqs=[RQ.rqi("key1", "key3", True, raw=[("key1", None)])])]),
                          [0], 7)
    # a versionless raw read that is never compared (key mismatch first) is just a phantom
    out = OM.validate_block(OM.StateDB(db), _blk([RQ.tx(rqs=[RQ.rqi("key1", "key3", True, raw=[("key0", None)])])]),
                            [0], 7)
    assert out == [12]


def test_random_blocks_mix_outcomes():
    db, blocks = RQ.random_blocks(3, nblocks=2, ntx=80)
    st = OM.StateDB(db)
    seen = set()
    for blk, flags, number in blocks:
        seen |= set(OM.validate_block(st, blk, flags, number, commit=True))
    assert {0, 11, 12} <= seen
