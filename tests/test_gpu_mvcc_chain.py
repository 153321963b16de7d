"""GPU parity of fgv_mvcc_validate_blocks (consecutive blocks as one device chain): every block's
flags equal the oracle validating and committing the blocks one at a time, and the committed
state after the chain equals that of one fgv_mvcc_validate_block call per block -- including
blocks the chain hands to the single-block path (range queries / metadata writes, a fixpoint
longer than the rounds enqueued, unsupported blocks, empty blocks)."""
import numpy as np
import pytest
import torch

from fabric_amd import _lib
from fabric_amd.synth import mvcc as M
from oracle import mvcc as OM
from tests import rq_cases as RQ
from tests.test_gpu_rangequery import _engine as db_engine, block_from_envs
from tests.test_oracle_mvcc import _blk, _db, _tx, dup_write_blocks

pytestmark = pytest.mark.gpu


def _engine(st, slots=1 << 20):
    eng = _lib.Engine(0)
    eng.statedb_init(slots, 32 << 20)
    keys, blk, txn = st.items()
    eng.statedb_load("mycc", keys, blk, txn)
    return eng


def _probe_state(eng, keys, versions, number):
    """one block reading every key at `versions`: all valid iff the engine's committed state agrees"""
    envs = [_tx([(k, v)], []) for k, v in zip(keys, versions)]
    return list(eng.mvcc_validate(_blk(envs), number, [0] * len(envs), commit=False))


def test_chain_matches_oracle_labels_and_single_path():
    st = M.MvccState(100_000, seed=21)
    db = _db(st)
    a, b = _engine(st), _engine(st)
    blocks = [M.make_block(st, 2000, number=1001 + i, seed=60 + i) for i in range(7)]
    exp = [OM.validate_block(db, blk, flags, 1001 + i, commit=True) for i, (blk, _, flags) in enumerate(blocks)]
    single = [list(a.mvcc_validate(blk, 1001 + i, flags, commit=True)) for i, (blk, _, flags) in enumerate(blocks)]
    # two chains (4 + 3 blocks): the second starts from the state the first committed
    got = []
    for lo, hi in ((0, 4), (4, 7)):
        nxt = [x[0] for x in blocks[4:7]] if lo == 0 else None  # the second call's walks run meanwhile
        fl, rc, done = b.mvcc_validate_blocks([x[0] for x in blocks[lo:hi]], range(1001 + lo, 1001 + hi),
                                              [x[2] for x in blocks[lo:hi]], commit=True, next_blocks=nxt)
        assert rc == 0 and done == hi - lo
        got += [list(f) for f in fl]
    for i in range(7):
        assert got[i] == single[i] == list(exp[i]) == list(blocks[i][1]), i
    assert a.statedb_stats() == b.statedb_stats()
    assert b.mvcc_stats()["reads"] > 0
    a.close()
    b.close()


def test_chain_device_copies_and_empty_blocks():
    """device-resident blocks (d_blocks), a mix of given and missing device copies, and empty
    blocks (no transactions) inside the chain"""
    st = M.MvccState(40_000, seed=22)
    db = _db(st)
    eng = _engine(st, slots=1 << 17)
    blocks = [M.make_block(st, 1200, number=2001 + i, seed=70 + i) for i in range(4)]
    exp = [list(OM.validate_block(db, blk, flags, 2001 + i, commit=True)) for i, (blk, _, flags) in enumerate(blocks)]
    dev = [torch.frombuffer(bytearray(b + bytes(64)), dtype=torch.uint8).cuda() for b, _, _ in blocks]
    torch.cuda.synchronize()
    empty = _blk([])
    bl = [blocks[0][0], empty, blocks[1][0], blocks[2][0], empty, blocks[3][0]]
    fl = [blocks[0][2], [], blocks[1][2], blocks[2][2], [], blocks[3][2]]
    nums = [2001, 2001, 2002, 2003, 2003, 2004]
    dptr = [dev[0].data_ptr(), None, None, dev[2].data_ptr(), None, dev[3].data_ptr()]
    out, rc, done = eng.mvcc_validate_blocks(bl, nums, fl, commit=True, d_blocks=dptr)
    assert rc == 0 and done == 6
    got = [list(out[i]) for i in (0, 2, 3, 5)]
    assert got == exp
    assert list(out[1]) == [] and list(out[4]) == []
    eng.close()


def test_chain_with_phantom_path_blocks():
    """device-path blocks and range-query blocks (the host phantom path) alternate inside one
    chain; each sees the other's commits"""
    st = M.MvccState(2000, seed=7)
    db = {("mycc", k): (int(b), int(t)) for k, b, t in zip(*st.items())}
    ost = OM.StateDB(db)
    blks, flags, nums, exp = [], [], [], []
    for b in range(6):
        number = 2001 + b
        if b % 2 == 0:
            blk, _, fl = M.make_block(st, 300, number=number, seed=30 + b)
        else:
            keys = sorted(k for (ns, k) in db if ns == "mycc")[:40]
            cur = {k.decode() if isinstance(k, bytes) else k: v for (ns, k), v in ost.v.items() if ns == "mycc"}
            res = sorted((k, v) for k, v in cur.items() if keys[0] <= k < keys[-1])
            envs = [RQ.env([("mycc", RQ.B.kv_rwset([], [(keys[3 + b], b"new", False)], []))], 0, number),
                    RQ.env([("mycc", RQ.B.kv_rwset([], [], [RQ.rqi(keys[0], keys[-1], True, raw=res)]))], 1, number),
                    RQ.env([("mycc", RQ.B.kv_rwset([], [], [RQ.rqi(keys[0], keys[2], True,
                                                                   raw=[r for r in res if r[0] < keys[2]])]))], 2, number)]
            blk, fl = block_from_envs(envs, number=number), [0, 0, 0]
        exp.append(list(OM.validate_block(ost, blk, fl, number, commit=True)))
        blks.append(blk)
        flags.append(fl)
        nums.append(number)
    eng = db_engine(db, slots=1 << 13)
    out, rc, done = eng.mvcc_validate_blocks(blks, nums, flags, commit=True)
    assert rc == 0 and done == 6
    assert [list(f) for f in out] == exp
    assert exp[1] == [0, 12, 0]
    eng.close()


@pytest.mark.parametrize("seed", [1, 2])
def test_chain_random_range_query_blocks(seed):
    db, blocks = RQ.random_blocks(seed, nblocks=4, ntx=150)
    st = OM.StateDB(db)
    exp = [list(OM.validate_block(st, blk, flags, number, commit=True)) for blk, flags, number in blocks]
    eng = db_engine(db)
    out, rc, done = eng.mvcc_validate_blocks([b[0] for b in blocks], [b[2] for b in blocks],
                                             [b[1] for b in blocks], commit=True)
    assert rc == 0 and done == len(blocks)
    assert [list(f) for f in out] == exp
    eng.close()


def test_chain_long_fixpoint_block():
    """a block whose conflict chain needs more fixpoint rounds than the chain enqueues: it and
    the blocks after it finish through the single-block path with the oracle's codes"""
    st = M.MvccState(20_000, seed=23)
    db = _db(st)
    db.v[("ns1", b"c0")] = (1, 0)
    eng = _engine(st, slots=1 << 16)
    eng.statedb_load("ns1", ["c0"], [1], [0])
    b0, _, f0 = M.make_block(st, 800, number=3001, seed=1)
    chain = _blk([_tx([("c%d" % i, (1, 0) if i == 0 else None)], [("c%d" % (i + 1), b"v", False)]) for i in range(40)])
    b2, _, f2 = M.make_block(st, 800, number=3003, seed=2)
    bl, fl, nums = [b0, chain, b2], [f0, [0] * 40, f2], [3001, 3002, 3003]
    exp = [list(OM.validate_block(db, b, f, n, commit=True)) for b, f, n in zip(bl, fl, nums)]
    out, rc, done = eng.mvcc_validate_blocks(bl, nums, fl, commit=True)
    assert rc == 0 and done == 3
    assert [list(f) for f in out] == exp
    assert exp[1].count(0) == 20 and exp[1].count(11) == 20
    # the state after the chain: c1..c40 at the versions the oracle committed
    keys = ["c%d" % i for i in range(41)]
    vers = [db.get_version("ns1", k.encode()) for k in keys]
    assert _probe_state(eng, keys, vers, 3004) == [0] * 41
    eng.close()


def test_chain_stops_at_unsupported_block():
    """[ok, duplicate write (unsupported), ok]: the first block is final and committed, the chain
    returns Unsupported with n_done = 1, nothing of the failing block is committed"""
    st = M.MvccState(20_000, seed=24)
    db = _db(st)
    eng = _engine(st, slots=1 << 16)
    b0, _, f0 = M.make_block(st, 600, number=4001, seed=3)
    dup = dup_write_blocks()[0]
    b2, _, f2 = M.make_block(st, 600, number=4003, seed=4)
    e0 = list(OM.validate_block(db, b0, f0, 4001, commit=True))
    s0 = None
    out, rc, done = eng.mvcc_validate_blocks([b0, dup, b2], [4001, 4002, 4003], [f0, [0], f2], commit=True)
    assert rc == _lib.FGV_EUNSUPPORTED and done == 1
    assert list(out[0]) == e0
    s0 = eng.statedb_stats()
    # the reference commits the failing block; here the caller resumes with the next one
    e2 = list(OM.validate_block(db, b2, f2, 4003, commit=True))
    out2, rc2, done2 = eng.mvcc_validate_blocks([b2], [4003], [f2], commit=True)
    assert rc2 == 0 and done2 == 1 and list(out2[0]) == e2
    assert eng.statedb_stats()["keys"] >= s0["keys"]
    eng.close()


def test_chain_next_batch_mismatch_is_ignored():
    """a pre-split of other blocks (or of a different batch) never changes the results"""
    st = M.MvccState(30_000, seed=25)
    db = _db(st)
    eng = _engine(st, slots=1 << 17)
    blocks = [M.make_block(st, 900, number=5001 + i, seed=80 + i) for i in range(5)]
    exp = [list(OM.validate_block(db, blk, flags, 5001 + i, commit=True)) for i, (blk, _, flags) in enumerate(blocks)]
    stray = [M.make_block(st, 50, number=9999, seed=99)[0]]
    fl, rc, done = eng.mvcc_validate_blocks([b[0] for b in blocks[:2]], [5001, 5002], [b[2] for b in blocks[:2]],
                                            commit=True, next_blocks=[blocks[2][0]])  # not the next call's batch
    assert rc == 0 and [list(f) for f in fl] == exp[:2]
    fl, rc, done = eng.mvcc_validate_blocks([b[0] for b in blocks[2:4]], [5003, 5004], [b[2] for b in blocks[2:4]],
                                            commit=True, next_blocks=stray)
    assert rc == 0 and [list(f) for f in fl] == exp[2:4]
    f, = eng.mvcc_validate_blocks([blocks[4][0]], [5005], [blocks[4][2]], commit=True)[0]
    assert list(f) == exp[4]
    eng.close()


def test_chain_empty_call():
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 1 << 20)
    out, rc, done = eng.mvcc_validate_blocks([], [], [], commit=True)
    assert rc == 0 and done == 0 and out == []
    eng.close()


def _random_batch(seed, nblocks, ntx, nkeys, committed, base_num, dels=0.15, hot=None):
    """blocks over a small key space: reads at the committed version, at an earlier block's
    height (right or wrong), nil, or a stale version; writes and deletes of few keys, so keys
    have several writers across and inside blocks.  `committed`: the version map a correct
    endorser would have seen before each block -- updated here by the ORACLE's own commit
    (reads are drawn from the true state half of the time)."""
    import random
    rng = random.Random(seed)
    out = []
    keys = ["k%03d" % i for i in range(nkeys)]
    for b in range(nblocks):
        envs = []
        for t in range(ntx):
            reads = []
            for _ in range(rng.randrange(0, 4)):
                k = hot if hot and rng.random() < 0.3 else rng.choice(keys)
                u = rng.random()
                if u < 0.5:
                    v = committed.get(k)
                elif u < 0.7:
                    v = (base_num + rng.randrange(max(1, b)), rng.randrange(ntx))
                elif u < 0.85:
                    v = None
                else:
                    v = (rng.randrange(1, 50), rng.randrange(20))
                reads.append((k, v))
            writes = []
            for k in rng.sample(keys, rng.randrange(0, 3)):
                writes.append((k, b"v%d" % t, rng.random() < dels))
            if hot and rng.random() < 0.5 and hot not in [w[0] for w in writes]:
                writes.append((hot, b"h", False))
            envs.append(_tx(reads, writes))
        out.append(_blk(envs))
    return out


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_batch_pass_cross_block_rules(seed):
    """fgv_mvcc_validate_blocks over blocks whose transactions read keys the batch's earlier
    blocks wrote or deleted (at those blocks' heights, stale heights, nil), with several writers
    of a key across and inside blocks: every block's flags and the committed state equal the
    oracle committing block after block"""
    import random
    rng = random.Random(seed)
    init = {("ns1", "k%03d" % i): (rng.randrange(1, 40), rng.randrange(10)) for i in range(40) if rng.random() < 0.7}
    db = OM.StateDB(dict(init))
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 1 << 20)
    ks = [k for (_, k) in init]
    eng.statedb_load("ns1", ks, np.array([init[("ns1", k)][0] for k in ks]), np.array([init[("ns1", k)][1] for k in ks]))
    base_num = 100
    for call in range(3):
        nb = 4
        # blocks drawn against the oracle's state as it evolves (half the reads current)
        committed = {k: v for (_, k), v in db.v.items()}
        blks = _random_batch(seed * 10 + call, nb, 30, 40, committed, base_num, hot=None if call < 2 else "k007")
        exp = [list(OM.validate_block(db, blk, [0] * 30, base_num + i, commit=True)) for i, blk in enumerate(blks)]
        fl, rc, done = eng.mvcc_validate_blocks(blks, range(base_num, base_num + nb), [[0] * 30] * nb, commit=True)
        assert rc == 0 and done == nb
        for i in range(nb):
            assert list(fl[i]) == exp[i], (call, i, [(t, int(fl[i][t]), exp[i][t]) for t in range(30) if fl[i][t] != exp[i][t]][:8])
        base_num += nb
    # the committed state: every key probed at the oracle's version
    keys = sorted({k.decode() for (_, k) in db.v} | set(ks))
    vers = [db.get_version("ns1", k) for k in keys]
    envs = [_tx([(k, v)], []) for k, v in zip(keys, vers)]
    assert list(eng.mvcc_validate(_blk(envs), base_num, [0] * len(envs), commit=False)) == [0] * len(envs)
    eng.close()
