"""GPU: the update-batch bytes built on the device (mvcc_ub.hip, fgv_mvcc_set_update_bytes) against
the restated deterministicBytesForPubAndHashUpdates (oracle/commithash.py), and the commit hashes
chained from them (fgv_commit_hashes_ub) against the host path and the oracle.

The blocks mix what the serialisation has to order and frame: two namespaces, public and hashed
writes in two collections, keys written again by later transactions of the same block (the last
valid writer wins), deletes (is_delete, an empty value, an empty value hash, SHA-256("")),
committer-invalid transactions and MVCC conflicts.  Paths: the batch pass (consecutive small
blocks), the per-block chain (blocks over FGV_MVCC_BATCH_TX transactions), the single-block call,
and a block over the device's limit (decoded on the host instead).

Reference: core/ledger/kvledger/kv_ledger.go:806-817, txmgr/update_batch_bytes.go:29-105,
validation/types.go:81-112, tx_ops.go:17-51."""
import hashlib

import numpy as np
import pytest

from fabric_amd import _lib
from fabric_amd.synth.blocks import f_msg, f_varint, f_bytes, hashed_rwset, kv_rwset, tx_rwset
from fabric_amd.synth.mvcc import _envelope
from oracle import commithash, mvcc

pytestmark = pytest.mark.gpu

EMPTY = hashlib.sha256(b"").digest()


def _block(rng, number, ntx, pool, state, wmax=3, invalid=0.05, lite=False):
    """(block bytes, committer flags): random reads / writes over `pool` keys per namespace
    (lite: one namespace, at most one public write and one collection write per tx)"""
    envs, flags = [], np.zeros(ntx, np.uint8)
    for i in range(ntx):
        sets = []
        for ns in ("mycc", "cc2"):
            if ns == "cc2" and (lite or rng.random() < 0.3):
                continue
            rd, wr, colls = [], [], []
            for _ in range(int(rng.integers(0, 3))):
                k = "k%05d" % rng.integers(pool)
                ver = state.get((ns, k.encode()))
                if rng.random() < 0.05:
                    ver = (1, 1)  # stale
                rd.append((k, ver))
            for k in rng.choice(pool, size=int(rng.integers(0, wmax + 1)), replace=False):
                u = rng.random()
                val = b"" if u < 0.05 else b"v%d-%d" % (number, i) * int(rng.integers(1, 40))
                wr.append(("k%05d" % k, val, u > 0.95))
            for coll in ("pvt", "apvt"):
                if rng.random() < (0.85 if lite else 0.5):
                    continue
                hw = []
                for k in rng.choice(pool, size=int(rng.integers(1, wmax + 1)), replace=False):
                    u = rng.random()
                    vh = EMPTY if u < 0.05 else b"" if u < 0.1 else hashlib.sha256(b"%d" % rng.integers(1 << 30)).digest()
                    hw.append((hashlib.sha256(b"k%05d" % k).digest(), vh, u > 0.95))
                colls.append((coll, hashed_rwset([], hw)))
            sets.append((ns, kv_rwset(rd, wr), colls))
        envs.append(_envelope(tx_rwset(sets), i, number))
        if rng.random() < invalid:
            flags[i] = 10  # committer-invalid: skipped by MVCC, its writes never apply
    header = f_varint(1, number) + f_bytes(2, b"\x00" * 32) + f_bytes(3, b"\x00" * 32)
    block = f_msg(1, header) + f_msg(2, b"".join(f_msg(1, e) for e in envs)) + \
        f_msg(3, b"".join(f_msg(1, b"") for _ in range(5)))
    return block, flags


def _setup(pool, seed):
    rng = np.random.default_rng(seed)
    keys = [b"k%05d" % k for k in range(0, pool, 2)]
    vers = {("mycc", k): (5, int(i)) for i, k in enumerate(keys)}
    return rng, keys, vers


def _check_call(eng, blks, nums, final, prev=b""):
    """the call's device bytes equal the oracle's update batches; the hashes equal both chains"""
    t = eng.mvcc_last_ticket()
    ub = eng.mvcc_update_bytes(t, len(blks))
    made = 0
    for b, blk in enumerate(blks):
        want = commithash.update_batch_bytes(*commithash.update_batch(blk, list(final[b]), nums[b]))
        if ub[b] is not None:
            made += 1
            assert ub[b] == want, (b, len(ub[b]), len(want))
    dev = _lib.CommitHashesDev(eng, blks, nums).run(final, prev, ticket=t)
    host = _lib.commit_hashes(blks, final, nums, prev)
    p, orc = prev, []
    for b, blk in enumerate(blks):
        p = commithash.block_commit_hash(blk, list(final[b]), nums[b], p)
        orc.append(p)
    assert dev == host == orc
    return made


@pytest.mark.parametrize("nblocks,ntx,path", [(3, 300, "batch"), (2, 4200, "chain"), (1, 500, "single")])
def test_update_bytes_match_oracle(nblocks, ntx, path):
    pool = 3000 if path != "chain" else 40000
    rng, keys, vers = _setup(pool, 7 + ntx)
    state = dict(vers)
    eng = _lib.Engine(0)
    try:
        eng.statedb_init(1 << 18, 32 << 20)
        eng.statedb_load("mycc", keys, [v[0] for v in vers.values()], [v[1] for v in vers.values()])
        eng.mvcc_set_update_bytes(True)
        sdb = mvcc.StateDB({k: v for k, v in vers.items()})
        nums = list(range(3001, 3001 + nblocks))
        blks, fin = [], []
        cfl = []
        for b in range(nblocks):
            blk, cf = _block(rng, nums[b], ntx, pool, state, wmax=3 if path != "chain" else 1, lite=path == "chain")
            blks.append(blk)
            cfl.append(cf)
        if path == "single":
            fin = [eng.mvcc_validate(blks[0], nums[0], cfl[0], commit=True)]
        else:
            fin, rc, done = eng.mvcc_validate_blocks(blks, nums, cfl, commit=True)
            assert rc == 0 and done == nblocks
        for b in range(nblocks):
            of = mvcc.validate_block(sdb, blks[b], list(cfl[b]), nums[b], commit=True)
            assert list(fin[b]) == list(of), b
        assert any((f == 11).any() for f in fin) and any((f == 0).any() for f in fin)
        made = _check_call(eng, blks, nums, fin, prev=b"\x07" * 32)
        assert made == nblocks  # every block's bytes came from the device
    finally:
        eng.close()


def test_update_bytes_over_limit_falls_back():
    """a block with more valid writes than the device serialisation holds: no device bytes, the
    same hashes from the host decode"""
    pool = 60000
    rng, keys, vers = _setup(pool, 99)
    eng = _lib.Engine(0)
    try:
        eng.statedb_init(1 << 18, 32 << 20)
        eng.statedb_load("mycc", keys, [v[0] for v in vers.values()], [v[1] for v in vers.values()])
        eng.mvcc_set_update_bytes(True)
        blk, cf = _block(rng, 4001, 3000, pool, dict(vers), wmax=6, invalid=0.0)
        fin = [eng.mvcc_validate(blk, 4001, cf, commit=True)]
        t = eng.mvcc_last_ticket()
        assert eng.mvcc_update_bytes(t, 1) == [None]
        _check_call(eng, [blk], [4001], fin)
    finally:
        eng.close()


def test_update_bytes_tickets_two_generations():
    """two calls are kept: the older ticket stays readable until the second call after it"""
    pool = 3000
    rng, keys, vers = _setup(pool, 5)
    eng = _lib.Engine(0)
    try:
        eng.statedb_init(1 << 18, 32 << 20)
        eng.statedb_load("mycc", keys, [v[0] for v in vers.values()], [v[1] for v in vers.values()])
        eng.mvcc_set_update_bytes(True)
        state = dict(vers)
        got = []
        for k in range(3):
            blk, cf = _block(rng, 5001 + k, 200, pool, state)
            fin = eng.mvcc_validate(blk, 5001 + k, cf, commit=True)
            got.append((eng.mvcc_last_ticket(), blk, fin))
        t0, t1, t2 = (g[0] for g in got)
        assert t0 < t1 < t2
        with pytest.raises(_lib.FgvError):
            eng.mvcc_update_bytes(t0, 1)  # the third call reused its generation
        for k in (1, 2):
            t, blk, fin = got[k]
            want = commithash.update_batch_bytes(*commithash.update_batch(blk, list(fin), 5001 + k))
            assert eng.mvcc_update_bytes(t, 1)[0] == want
        eng.mvcc_set_update_bytes(False)
    finally:
        eng.close()


def test_update_bytes_phantom_path_block_falls_back():
    """a block with range queries goes through the host phantom path (fgv_mvcc.cpp): its update
    bytes are not produced on the device (NULL), the device-path blocks' are, and the chained
    hashes equal the host decode and the oracle either way"""
    from fabric_amd.synth import mvcc as M
    from tests import rq_cases as RQ
    from tests.blockfix import block_from_envs
    st = M.MvccState(2000, seed=7)
    db = {("mycc", k): (int(b), int(t)) for k, b, t in zip(*st.items())}
    ost = mvcc.StateDB(db)
    eng = _lib.Engine(0)
    try:
        eng.statedb_init(1 << 13, 8 << 20)
        keys0 = [k for (ns, k) in db]
        eng.statedb_load("mycc", keys0, [db[("mycc", k)][0] for k in keys0], [db[("mycc", k)][1] for k in keys0])
        eng.mvcc_set_update_bytes(True)
        prev = b""
        for b in range(4):
            number = 2001 + b
            if b % 2 == 0:
                blk, _, flags = M.make_block(st, 300, number=number, seed=30 + b)
            else:
                keys = sorted(k for (ns, k) in db if ns == "mycc")[:40]
                cur = {k.decode() if isinstance(k, bytes) else k: v for (ns, k), v in ost.v.items() if ns == "mycc"}
                res = sorted((k, v) for k, v in cur.items() if keys[0] <= k < keys[-1])
                envs = [RQ.env([("mycc", RQ.B.kv_rwset([], [(keys[3], b"new", False)], []))], 0, number),
                        RQ.env([("mycc", RQ.B.kv_rwset([], [], [RQ.rqi(keys[0], keys[-1], True, raw=res)]))], 1, number)]
                blk, flags = block_from_envs(envs, number=number), [0, 0]
            exp = mvcc.validate_block(ost, blk, list(flags), number, commit=True)
            got = eng.mvcc_validate(blk, number, flags, commit=True)
            assert list(got) == list(exp), b
            t = eng.mvcc_last_ticket()
            ub = eng.mvcc_update_bytes(t, 1)[0]
            want = commithash.update_batch_bytes(*commithash.update_batch(blk, list(got), number))
            if b % 2 == 0:
                assert ub == want, b  # the device path
            else:
                assert ub is None, b  # the phantom path: decoded on the host
            h = _lib.CommitHashesDev(eng, [blk], [number]).run([got], prev, ticket=t)[0]
            assert h == _lib.commit_hash(blk, got, number, prev) == commithash.commit_hash(list(got), want, prev)
            prev = h
    finally:
        eng.close()
