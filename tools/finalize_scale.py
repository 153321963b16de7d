"""The N>1 finalize's cost at N ranks, measured on one GPU (profiling aid): every
rank of the shard protocol finalizes the whole batch's all-gathered records (N x 16k for C2), so
its step grows with N by the finalize's growth.  This validates one C2 shard (32 x 500 tx),
replicates its records N times as the all-gather would deliver N ranks' shards, and times
fgv_finalize_flags_dev_plan over them for N = 1, 2, 4, 8 (the replicated txids make the flags
meaningless -- duplicates everywhere -- but the kernels do the work of N distinct shards).

python tools/finalize_scale.py [--steps 20]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fabric_amd import _lib, shard, txvalidator  # noqa: E402
from fabric_amd.synth import blocks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    B, T = 32, 500
    net = blocks.Network(seed=3, orgs=3, clients=100)
    blks = []
    prev = b"\x00" * 32
    for i in range(B):
        blk, _, envs = blocks.make_block(net, T, number=1 + i, seed=i, threads=8, prev_hash=prev)
        prev = blocks.header_hash(1 + i, prev, envs)
        blks.append(blk)
    dev = torch.device("cuda:0")
    eng = _lib.Engine(0)
    txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes, hot_clients=True)
    sizes = [(len(b) + 64 + 255) // 256 * 256 for b in blks]
    arena = torch.zeros(sum(sizes), dtype=torch.uint8, device=dev)
    dptr, o = [], 0
    for b in blks:
        arena[o:o + len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
        dptr.append(arena.data_ptr() + o)
        o += (len(b) + 64 + 255) // 256 * 256
    pad = torch.zeros(256, dtype=torch.uint8, device=dev)  # (other ranks' blocks: empty placeholders)
    out = {}
    for N in (1, 2, 4, 8):
        # N ranks, each with its own 32 blocks: rank 0's shard validated here, replicated
        ntx = np.array([T] * (N * B), dtype=np.int64)
        plan = shard.plan(ntx, N, "block")
        rows = shard.plan_rows(*plan)
        send = torch.zeros((rows, shard.REC), dtype=torch.uint8, device=dev)
        recv = torch.zeros((N * rows, shard.REC), dtype=torch.uint8, device=dev)
        flags = np.empty(N * B * T, dtype=np.uint8)
        lo, hi = plan[0][0], plan[1][0]
        batch = eng.block_batch(blks + [b""] * ((N - 1) * B), dptr + [pad.data_ptr()] * ((N - 1) * B))
        bs = _lib.BlockStep(eng, batch, lo, hi, send.data_ptr(), rows, ntx, N, recv.data_ptr(), flags, plan=plan,
                            presplit=False)
        bs.validate()
        torch.cuda.synchronize()
        for r in range(N):
            recv[r * rows:(r + 1) * rows].copy_(send)
        torch.cuda.synchronize()
        for _ in range(3):
            bs.finalize()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            bs.finalize()
        torch.cuda.synchronize()
        out[N] = round((time.perf_counter() - t) / a.steps * 1e3, 4)
        print(f"[finalize_scale] N={N}: {N * B * T} records, {out[N]} ms per finalize", file=sys.stderr)
    print({"finalize_ms_by_ranks": out})
    eng.close()


if __name__ == "__main__":
    main()
