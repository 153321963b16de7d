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


def test_metadata_write_known_answers():
    """metadata writes go to the host path (fgv_mvcc.cpp): codes, unsupported cases and the
    committed versions equal the oracle's"""
    from tests import rq_cases as RQ
    from tests.test_gpu_rangequery import _engine as rq_engine
    for name, envs, flags, exp in RQ.meta_cases():
        eng = rq_engine(RQ.meta_db())
        blk = _blk(envs)
        if exp == "unsupported":
            with pytest.raises(_lib.Unsupported):
                eng.mvcc_validate(blk, 5, flags, commit=True)
            eng.close()
            continue
        st = OM.StateDB(RQ.meta_db())
        assert list(eng.mvcc_validate(blk, 5, flags, commit=True)) == exp == OM.validate_block(st, blk, flags, 5,
                                                                                               commit=True), name
        # the next block reads every key at the oracle's committed version
        keys = sorted({k for (ns, k) in st.v if ns == "ns1"} | {b"key1", b"key2", b"key9"})
        reads = [(k.decode(), st.get_version("ns1", k)) for k in keys]
        nxt = _blk([_tx(reads, [])])
        assert list(eng.mvcc_validate(nxt, 6, [0], commit=False)) == [0], name
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


def test_duplicate_write_unsupported_and_kind_separation():
    """A key written twice by one tx -> Unsupported, nothing committed; public vs hashed update
    maps stay separate while sharing the committed key space."""
    from tests.test_oracle_mvcc import dup_write_blocks, kind_separation_case
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 1 << 20)
    a, b, c = dup_write_blocks()
    for blk in (a, b):
        with pytest.raises(_lib.Unsupported):
            eng.mvcc_validate(blk, 2, [0], commit=True)
    assert eng.statedb_stats()["keys"] == 0
    assert list(eng.mvcc_validate(c, 2, [0], commit=True)) == [0]
    assert eng.statedb_stats()["keys"] == 2  # public "k1" and hashed (ns1, c1, "k1")
    committed, blk, exp = kind_separation_case()
    eng2 = _lib.Engine(0)
    eng2.statedb_init(1 << 12, 1 << 20)
    for (ns, k), (bn, t) in committed.items():
        eng2.statedb_load(ns, [k], [bn], [t])
    assert list(eng2.mvcc_validate(blk, 2, [0, 0, 0], commit=False)) == exp
    eng.close()
    eng2.close()


def test_fallback_block_applied_then_gpu_matches_oracle():
    """Block 1 validated + committed by the engine, block 2 committed by the reference path (the
    oracle stands in) and handed over with fgv_statedb_apply, block 3 by the engine again: the
    flags of block 3 equal the oracle's, i.e. the GPU cache did not go stale."""
    st = M.MvccState(30_000, seed=11)
    db = _db(st)
    eng = _engine(st, slots=1 << 17)
    b1, l1, f1 = M.make_block(st, 1500, number=1001, seed=1)
    assert list(eng.mvcc_validate(b1, 1001, f1, commit=True)) == list(OM.validate_block(db, b1, f1, 1001, commit=True))
    b2, l2, f2 = M.make_block(st, 1500, number=1002, seed=2)
    upd = {}
    OM.validate_block(db, b2, f2, 1002, commit=True, updates_out=upd)
    by_ns = {}
    for (_, ns, key), ((bn, t), dl) in upd.items():
        by_ns.setdefault(ns, []).append((key, bn, t, dl))
    for ns, items in by_ns.items():
        eng.statedb_apply(ns, [k for k, *_ in items], [x[1] for x in items], [x[2] for x in items],
                          [1 if x[3] else 0 for x in items])
    b3, l3, f3 = M.make_block(st, 1500, number=1003, seed=3)
    exp = OM.validate_block(db, b3, f3, 1003, commit=True)
    got = eng.mvcc_validate(b3, 1003, f3, commit=True)
    assert list(got) == list(exp) == list(l3)
    # the same block 3 without the hand-over would have read stale versions
    eng.close()


def test_many_blocks_commit_exact_arena_accounting():
    """300 consecutive committed blocks over a fixed key set: overwrites reuse their entries, so
    the arena and slot counts stay where the load left them (no ENOMEM after N blocks)."""
    st = M.MvccState(20_000, seed=12)
    eng = _lib.Engine(0)
    keys, blk, txn = st.items()
    eng.statedb_init(1 << 16, 20_000 * 16 + (64 << 10))   # the loaded keys + one block of writes
    eng.statedb_load("mycc", keys, blk, txn)
    s0 = eng.statedb_stats()
    for b in range(300):
        blkb, labels, flags = M.make_block(st, 400, number=1001 + b, seed=100 + b)
        assert list(eng.mvcc_validate(blkb, 1001 + b, flags, commit=True)) == list(labels), b
    s1 = eng.statedb_stats()
    assert s1["keys"] == s0["keys"] == 20_000 and s1["arena_used"] == s0["arena_used"]
    eng.close()


def test_c3_full_size_matches_oracle():
    """BASELINE configs[2] at its size: 10k-tx blocks against a 1M-key state DB, two consecutive
    committed blocks, flags == oracle == generator labels."""
    st = M.MvccState(1_000_000, seed=4)
    db = _db(st)
    eng = _lib.Engine(0)
    keys, blk, txn = st.items()
    eng.statedb_init(1 << 22, 64 << 20)
    eng.statedb_load("mycc", keys, blk, txn)
    for b in range(2):
        blkb, labels, flags = M.make_block(st, 10_000, number=1001 + b, seed=500 + b)
        exp = OM.validate_block(db, blkb, flags, 1001 + b, commit=True)
        got = eng.mvcc_validate(blkb, 1001 + b, flags, commit=True)
        assert list(got) == list(exp) == list(labels), b
        assert 11 in list(got)
    eng.close()


def test_load_semantics():
    """re-loading a key updates it in place; duplicate keys in one call -> EINVAL; an arena
    beyond 32 GiB -> EINVAL; apply deletes a key (a later nil read is valid)"""
    eng = _lib.Engine(0)
    with pytest.raises(_lib.FgvError):
        eng.statedb_init(1 << 12, 33 << 30)
    eng.statedb_init(1 << 12, 1 << 20)
    eng.statedb_load("ns1", ["a", "b"], [1, 1], [0, 1])
    eng.statedb_load("ns1", ["a"], [5], [7])
    with pytest.raises(_lib.FgvError):
        eng.statedb_load("ns1", ["c", "c"], [1, 1], [0, 0])
    assert eng.statedb_stats()["keys"] == 2
    from tests.test_oracle_mvcc import _tx, _blk
    envs = [_tx([("a", (5, 7)), ("b", (1, 1))], []), _tx([("a", (1, 0))], [])]
    assert list(eng.mvcc_validate(_blk(envs), 9, [0, 0], commit=False)) == [0, 11]
    eng.statedb_apply("ns1", ["b"], [0], [0], [1])
    envs = [_tx([("b", None)], []), _tx([("b", (1, 1))], [])]
    assert list(eng.mvcc_validate(_blk(envs), 9, [0, 0], commit=False)) == [0, 11]
    eng.close()


def test_extraction_scratch_spill_and_envelope_sizes():
    """k_mvx_extract's record scratch (LDS by default, 8 records of each kind per transaction) and
    its staging cap (768 B per transaction with the LDS scratch): transactions with more than 8
    reads or writes take the second walk, envelopes past the cap are walked from global memory,
    beside ordinary small ones in the same workgroups -- flags and the committed state over two
    blocks match the oracle."""
    import random
    rng = random.Random(7)
    keys = ["k%d" % i for i in range(200)]
    db = OM.StateDB({("ns1", k): (1, i) for i, k in enumerate(keys)})
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 4 << 20)
    eng.statedb_load("ns1", keys, [1] * len(keys), list(range(len(keys))))
    envs = [
        _tx([(keys[i], (1, i)) for i in range(12)], [("w%d" % i, b"x" * 5, False) for i in range(10)]),  # spill both
        _tx([("w3", None)], []),                                      # written by tx 0 -> 11
        _tx([(keys[20], (1, 20))], [("big1", b"y" * 1000, False)]),   # envelope past 768 B
        _tx([(keys[21], (1, 21))], [("big2", b"z" * 2000, False)]),   # past 1,536 B
        _tx([], [("m%d" % i, b"v", i % 3 == 0) for i in range(9)]),   # 9 writes, some deletes
        _tx([("m4", None)], []),                                      # written by tx 4 -> 11
        _tx([(keys[i], (1, i)) for i in range(30, 39)], []),          # 9 reads
        _tx([(keys[40], (7, 7))], [("big3", b"q" * 900, False)]),     # stale read, big envelope -> 11
    ]
    for i in range(56):  # small transactions around them
        k = rng.randrange(50, 200)
        envs.append(_tx([(keys[k], (1, k))], [(keys[k], b"s", False)] if i % 2 else []))
    blk = _blk(envs)
    n = len(envs)
    want = OM.validate_block(db, blk, [0] * n, 2, commit=True)
    got = eng.mvcc_validate(blk, 2, [0] * n, commit=True)
    assert list(got) == want
    assert want[1] == 11 and want[5] == 11 and want[7] == 11 and want[0] == 0
    # the next block reads what block 2 committed (versions Height{2, tx})
    envs2 = [_tx([("w%d" % i, (2, 0)) for i in range(10)], []), _tx([("big2", (2, 3)), ("m1", (2, 4))], []),
             _tx([("m0", None), ("big3", None)], []), _tx([("big1", (1, 0))], [])]
    blk2 = _blk(envs2)
    assert list(eng.mvcc_validate(blk2, 3, [0] * 4)) == OM.validate_block(db, blk2, [0] * 4, 3, commit=True)
    eng.close()
