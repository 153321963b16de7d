"""CPU, world_size 2 (gloo): the multi-GPU exchange (shard ranges -> all-gather ->
re-order -> fgv_finalize_flags) reproduces single-process flags on synthetic records."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from fabric_amd import _lib, shard


def _records(seed, ntx):
    rng = np.random.default_rng(seed)
    n = int(sum(ntx))
    res = np.zeros((n, 68), np.uint8)
    res[:, 0] = rng.choice([0, 0, 0, 0, 4, 10, 8], size=n)
    reached = rng.random(n) < 0.9
    res[:, 1] = reached * 1 + (rng.random(n) < 0.95) * 2
    ids = rng.integers(0, 40, size=n)  # small id space -> many duplicates
    for i in range(n):
        res[i, 4:36] = ids[i]
        res[i, 36:68] = ids[i] if rng.random() < 0.8 else 255
    return res


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ntx, seed, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = _records(seed, ntx)
    plan = shard.plan(ntx, world, mode)
    cnt = shard.plan_counts(*plan)
    lo = np.where(cnt[rank] > 0, plan[0][rank], 0).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(ntx)])
    local = np.concatenate([full[offs[b] + lo[b]: offs[b] + lo[b] + cnt[rank, b]] for b in range(len(ntx))])
    got = shard.allgather_results(local, ntx, world, plan_=plan)
    flags = _lib.finalize_flags(ntx, got)
    q.put((rank, bool(np.array_equal(got, full)), flags.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["tx", "block"])
def test_allgather_finalize_world2(mode):
    ntx = [37, 0, 64, 5]
    world, seed = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ntx, seed, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    single = _lib.finalize_flags(ntx, _records(seed, ntx)).tolist()
    for rank, same, flags in out:
        assert same, rank
        assert flags == single
    assert 9 in single  # the duplicate logic was exercised


def test_finalize_semantics_cpu():
    """fgv_finalize_flags: batch index precedes everything; markTXIdDuplicates on VALID only."""
    def rec(code, reached, tid, idx):
        r = np.zeros(68, np.uint8)
        r[0] = code
        r[1] = (1 if reached else 0) | (2 if idx is not None else 0)
        r[4:36] = tid
        if idx is not None:
            r[36:68] = idx
        return r
    b1 = [rec(0, True, 1, 1), rec(4, False, 0, 2)]               # indexes txids 1 and 2
    b2 = [rec(10, True, 1, 1), rec(0, True, 2, 2), rec(0, True, 3, 3), rec(0, True, 3, 3), rec(5, False, 3, 3)]
    flags = _lib.finalize_flags([2, 5], np.stack(b1 + b2))
    assert flags.tolist() == [0, 4, 9, 9, 0, 9, 5]


def _outcome_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ntx = [3, 2, 4, 1]
    flags = np.array([0, 0, 10, 0xFD, 0, 0, 0, 0, 0, 0xFD], np.uint8)  # undecided: blocks 1 and 3
    # rank 0's key-level walk found no wait; rank 1's makes block 3 wait (its n_final = 3)
    q.put((rank, shard.block_outcomes(flags, ntx, 4 if rank == 0 else 3)))
    dist.destroy_process_group()


def test_block_outcomes_world2():
    """shard.block_outcomes: n_final is the minimum over the ranks (all-reduce), the statuses come
    from the final flags (0xFD -> unsupported) and are the same on every rank"""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_outcome_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, (st, n_final) in out:
        assert n_final == 3, rank
        assert st == [0, shard.UNSUPPORTED, 0, shard.LATER], (rank, st)
    # one process: no all-reduce
    assert shard.block_outcomes(np.zeros(3, np.uint8), [1, 1, 1], 3) == ([0, 0, 0], 3)
