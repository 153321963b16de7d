"""GPU parity of MVCC: flags and the committed state after each block match the oracle."""
import numpy as np
import pytest

from fabric_amd import _lib
from fabric_amd.synth import mvcc as M
from oracle import mvcc as OM
from tests.test_oracle_mvcc import _blk, _db, _tx

pytestmark = pytest.mark.gpu


def _engine(st, slots=1 << 20):
    eng = _lib.Engine(0)
    eng.statedb_init(slots, 32 << 20)
    keys, blk, txn = st.items()
    eng.statedb_load("mycc", keys, blk, txn)
    return eng


def test_blocks_match_oracle_and_labels():
    st = M.MvccState(100_000, seed=4)
    db = _db(st)
    eng = _engine(st)
    for b in range(4):
        blk, labels, flags = M.make_block(st, 3000, number=1001 + b, seed=10 + b)
        exp = OM.validate_block(db, blk, flags, 1001 + b, commit=True)
        got = eng.mvcc_validate(blk, 1001 + b, flags, commit=True)
        assert list(got) == list(exp) == list(labels)
    eng.close()


def test_next_block_presplit_matches():
    """fgv_mvcc_validate_block_next (block k+1's framing walked while block k validates) and a
    pre-split of an unrelated block left pending: same codes as the oracle and the labels."""
    st = M.MvccState(50_000, seed=5)
    db = _db(st)
    eng = _engine(st)
    blks = [M.make_block(st, 1500, number=1001 + b, seed=20 + b) for b in range(4)]
    stray = eng.block_batch([M.make_block(st, 50, number=9999, seed=99)[0]])
    for b, (blk, labels, flags) in enumerate(blks):
        if b == 2:
            eng.presplit(stray)  # not this block's: must be ignored
        nxt = blks[b + 1][0] if b + 1 < len(blks) else None
        exp = OM.validate_block(db, blk, flags, 1001 + b, commit=True)
        got = eng.mvcc_validate(blk, 1001 + b, flags, commit=True, next_block=nxt)
        assert list(got) == list(exp) == list(labels), b
    eng.close()


def test_known_answers_and_chains():
    db = OM.StateDB({("ns1", "key%d" % i): (1, i - 1) for i in range(1, 6)})
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 1 << 20)
    eng.statedb_load("ns1", ["key%d" % i for i in range(1, 6)], [1] * 5, list(range(5)))
    envs = [
        _tx([("key1", (1, 0)), ("key2", (1, 1))], [("key2", b"v", False)]),
        _tx([("key2", (1, 1))], []),
        _tx([("key3", (1, 0))], []),
        _tx([("key9", None)], [("key4", b"v", False)]),
        _tx([("key4", (1, 3))], []),
        _tx([("key5", None)], []),
        # chain: tx7 writes k, tx8 (invalid: stale) writes m, tx9 reads m -> valid, tx10 reads k -> 11
        _tx([("key1", (1, 0))], [("kk", b"v", False)]),
        _tx([("key3", (9, 9))], [("mm", b"v", False)]),
        _tx([("mm", None)], [("nn", b"v", True)]),
        _tx([("kk", None)], []),
        _tx([("nn", None)], []),   # nn deleted by tx 8 (valid) -> in updates -> 11
    ]
    blk = _blk(envs)
    exp = OM.validate_block(db, blk, [0] * len(envs), 2, commit=True)
    got = eng.mvcc_validate(blk, 2, [0] * len(envs), commit=True)
    assert list(got) == exp
    # second block reads the committed heights written by block 2
    envs2 = [_tx([("key2", (2, 0)), ("key4", (2, 3)), ("kk", (2, 6))], []), _tx([("key2", (1, 1))], []),
             _tx([("nn", None)], [])]
    blk2 = _blk(envs2)
    assert list(eng.mvcc_validate(blk2, 3, [0] * 3)) == OM.validate_block(db, blk2, [0] * 3, 3, commit=True)
    eng.close()


def test_long_dependency_chain():
    """tx i reads the key written by tx i-1: alternating validity -> many fixpoint rounds."""
    db = OM.StateDB({("ns1", "c0"): (1, 0)})
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 1 << 20)
    eng.statedb_load("ns1", ["c0"], [1], [0])
    envs = [_tx([("c%d" % i, (1, 0) if i == 0 else None)], [("c%d" % (i + 1), b"v", False)]) for i in range(40)]
    blk = _blk(envs)
    exp = OM.validate_block(db, blk, [0] * 40, 2, commit=False)
    got = eng.mvcc_validate(blk, 2, [0] * 40, commit=False)
    assert list(got) == exp
    assert eng.mvcc_stats()["rounds"] >= 10
    eng.close()


def test_hashed_reads_and_delete_rules():
    """Private-data hashed reads/writes (ns + "$$h" + coll) and the empty-value / empty-hash
    delete rules: same flags and committed state as the oracle over two blocks."""
    from tests.test_oracle_mvcc import hashed_case
    committed, blocks, expected = hashed_case()
    db = OM.StateDB(committed)
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 1 << 20)
    by_ns = {}
    for (ns, k), (b, t) in committed.items():
        by_ns.setdefault(ns, []).append((k, b, t))
    for ns, items in by_ns.items():
        eng.statedb_load(ns, [k for k, _, _ in items], [b for _, b, _ in items], [t for _, _, t in items])
    for n, (envs, exp) in enumerate(zip(blocks, expected)):
        blk = _blk(envs)
        want = OM.validate_block(db, blk, [0] * len(envs), 2 + n, commit=True)
        got = eng.mvcc_validate(blk, 2 + n, [0] * len(envs), commit=True)
        assert list(got) == want == exp, n
    eng.close()


def test_private_data_blocks_match_oracle_and_labels():
    """C3 shape with every 8th key private-data (hashed namespace mycc$$hpvt): flags and the
    committed state over consecutive blocks match the oracle and the generator's labels."""
    from tests.test_oracle_mvcc import _db_with_private
    st = M.MvccState(60_000, seed=6, private_every=8)
    db = _db_with_private(st)
    eng = _engine(st)
    hk, hb, ht = st.items_hashed()
    eng.statedb_load(M.HASHED_NS, hk, hb, ht)
    for b in range(3):
        blk, labels, flags = M.make_block(st, 3000, number=1001 + b, seed=40 + b)
        assert blk.count(b"pvt") > 500  # private reads/writes are really in the block
        exp = OM.validate_block(db, blk, flags, 1001 + b, commit=True)
        got = eng.mvcc_validate(blk, 1001 + b, flags, commit=True)
        assert list(got) == list(exp) == list(labels), b
    eng.close()


def test_hashed_metadata_write_unsupported():
    from tests.test_oracle_mvcc import hashed_metadata_block
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 1 << 20)
    blk = hashed_metadata_block()
    with pytest.raises(_lib.Unsupported):
        eng.mvcc_validate(blk, 2, [0, 0], commit=False)
    assert list(eng.mvcc_validate(blk, 2, [0, 10], commit=False)) == [0, 10]
    eng.close()


def test_reference_bulkload_known_answers():
    from tests.test_oracle_mvcc import bulkload_case
    committed, blk, exp = bulkload_case()
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 1 << 20)
    for (ns, k), (b, t) in committed.items():
        eng.statedb_load(ns, [k], [b], [t])
    assert list(eng.mvcc_validate(blk, 2, [0, 0, 0], commit=False)) == exp
    eng.close()
