"""GPU parity of range-query (phantom read) validation: the engine's phantom path (device
lookups + range scans of the committed-state table, host combined iterator and raw / merkle
validators; fgv_mvcc.cpp) against the oracle on the reference's known answers and on
randomized multi-block workloads with commits."""
import numpy as np
import pytest

from fabric_amd import _lib
from fabric_amd.synth import mvcc as M
from oracle import mvcc as OM
from tests import rq_cases as RQ
from tests.blockfix import block_from_envs

pytestmark = pytest.mark.gpu


def _engine(db, slots=1 << 14):
    eng = _lib.Engine(0)
    eng.statedb_init(slots, 8 << 20)
    by_ns = {}
    for (ns, k), v in db.items():
        by_ns.setdefault(ns, []).append((k, v))
    for ns, items in by_ns.items():
        eng.statedb_load(ns, [k for k, _ in items], [v[0] for v in (x[1] for x in items)],
                         [v[1] for v in (x[1] for x in items)])
    return eng


@pytest.mark.parametrize("case", RQ.known_answer_cases(), ids=lambda c: c[0])
def test_reference_known_answers(case):
    name, db, envs, expected, blk = case
    eng = _engine(db)
    got = eng.mvcc_validate(block_from_envs(envs), blk, [0] * len(envs), commit=False)
    assert list(got) == expected, name
    eng.close()


def test_unsupported_when_the_reference_errors_out():
    db = RQ.phantom_db()
    eng = _engine(db)
    for q in (RQ.rqi("key1", "key3", True, merkle=(1, 1, [b"x"])), RQ.rqi("key1", "key3", True, raw=[("key1", None)])):
        with pytest.raises(_lib.Unsupported):
            eng.mvcc_validate(block_from_envs([RQ.tx(rqs=[q])]), 7, [0], commit=True)
    # nothing was committed: a read at the loaded version is still valid
    got = eng.mvcc_validate(block_from_envs([RQ.tx(reads=[("key1", (1, 0))])]), 8, [0], commit=False)
    assert list(got) == [0]
    eng.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_blocks_match_oracle_with_commits(seed):
    db, blocks = RQ.random_blocks(seed, nblocks=4, ntx=150)
    st = OM.StateDB(db)
    eng = _engine(db)
    for b, (blk, flags, number) in enumerate(blocks):
        exp = OM.validate_block(st, blk, flags, number, commit=True)
        got = eng.mvcc_validate(blk, number, flags, commit=True)
        assert list(got) == list(exp), (seed, b, [(i, int(g), e) for i, (g, e) in enumerate(zip(got, exp)) if g != e][:8])
    eng.close()


def test_device_and_phantom_paths_share_the_committed_state():
    """device-path blocks (no range queries) and phantom-path blocks alternate; each sees the
    other's commits"""
    st = M.MvccState(2000, seed=7)
    db = {("mycc", k): (int(b), int(t)) for k, b, t in zip(*st.items())}
    ost = OM.StateDB(db)
    eng = _engine(db, slots=1 << 13)
    for b in range(4):
        number = 2001 + b
        if b % 2 == 0:
            blk, _, flags = M.make_block(st, 300, number=number, seed=30 + b)
        else:
            keys = sorted(k for (ns, k) in db if ns == "mycc")[:40]
            cur = {k.decode() if isinstance(k, bytes) else k: v for (ns, k), v in ost.v.items() if ns == "mycc"}
            res = sorted((k, v) for k, v in cur.items() if keys[0] <= k < keys[-1])
            envs = [RQ.env([("mycc", RQ.B.kv_rwset([], [(keys[3], b"new", False)], []))], 0, number),
                    RQ.env([("mycc", RQ.B.kv_rwset([], [], [RQ.rqi(keys[0], keys[-1], True, raw=res)]))], 1, number),
                    RQ.env([("mycc", RQ.B.kv_rwset([], [], [RQ.rqi(keys[0], keys[2], True,
                                                                   raw=[r for r in res if r[0] < keys[2]])]))], 2, number)]
            blk, flags = block_from_envs(envs, number=number), [0, 0, 0]
        exp = OM.validate_block(ost, blk, flags, number, commit=True)
        got = eng.mvcc_validate(blk, number, flags, commit=True)
        assert list(got) == list(exp), b
        if b % 2 == 1:
            assert list(exp) == [0, 12, 0]
        else:  # the generator's own commit view follows the oracle's
            pass
    eng.close()
