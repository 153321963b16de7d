"""Host commit-hash throughput (profiling aid): fgv_commit_hashes over 32
pipeline blocks (500 tx, C2 shape, 4 writes x 200 B per tx) on the caller only and on the pool,
and fgv_commit_hash one block at a time.  python tools/commit_hash_bench.py [--blocks 32]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fabric_amd import _lib  # noqa: E402
from fabric_amd.synth import blocks, pipeline  # noqa: E402
from fabric_amd.synth.mvcc import MvccState  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=32)
    a = ap.parse_args()
    net = blocks.Network(seed=3, orgs=3, clients=20)
    st = MvccState(200_000, seed=9)
    blks, _, fexp, _ = pipeline.make_blocks(net, st, a.blocks, 500, 2001, seed=5)
    out = {"cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    for th in (1, 0):
        ch = _lib.CommitHashes(blks, range(2001, 2001 + a.blocks), threads=th)
        ch.run(fexp)
        t = time.perf_counter()
        for _ in range(5):
            ch.run(fexp)
        out["pool" if th == 0 else "one_thread"] = round((time.perf_counter() - t) / 5 * 1e3, 3)
    t = time.perf_counter()
    prev = b""
    for b in range(a.blocks):
        prev = _lib.commit_hash(blks[b], fexp[b], 2001 + b, prev)
    out["per_block_calls"] = round((time.perf_counter() - t) * 1e3, 3)
    print({"ms_per_%d_blocks" % a.blocks: out})


if __name__ == "__main__":
    main()
