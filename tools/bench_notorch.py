"""Torch-free C2 harness: the headline workload driven through the
C ABI alone, as a Go peer through cgo would -- no torch in the process, so no other HIP stream
exists before the engine's own (the torch bench's first stream is torch's); the blocks live in
HBM allocated and filled through the engine (fgv_dev_alloc / fgv_dev_upload).  Same generator,
seeds, rotation and pipelined call (fgv_validate_blocks_pipelined, the next batch pre-split and
its front half ahead) as bench.py's default line.

--contexts 2: two channel contexts on the one GPU, each with its own batches, driven from two
host threads at once (a peer serving two channels); value = their aggregate validated tx/s.

python tools/bench_notorch.py [--steps 40] [--warmup 5] [--contexts 1|2]"""
import argparse
import json
import os
import sys
import threading
import time

os.environ["FGV_NO_TORCH"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from fabric_amd import _lib, txvalidator  # noqa: E402
from fabric_amd.synth import blocks  # noqa: E402


def make_batches(net, nb, B, T, rank=0):
    """bench.py run_block's batches (world 1): NB x B hash-chained blocks"""
    out = []
    for k in range(nb):
        prev, cur = b"\x00" * 32, []
        for i in range(B):
            num = 1 + k * B + i
            blk, lab, envs = blocks.make_block(net, T, number=num, seed=7919 * rank + 100003 * k + i, threads=8,
                                               endorse_dist=((2, 0.6), (3, 0.4)), prev_hash=prev)
            cur.append((blk, lab))
            prev = blocks.header_hash(num, prev, envs)
        out.append(cur)
    return out


class Channel:
    """one context, its HBM-resident rotation and the bound pipelined calls"""

    def __init__(self, net, batches, T):
        self.eng = _lib.Engine(0)
        txvalidator.setup_channel(self.eng, net.channel, net.identities(), net.chaincodes, hot_clients=True)
        self.blks = [[b for b, _ in cur] for cur in batches]
        self.labels = [[lab for _, lab in cur] for cur in batches]
        sizes = [(len(b) + 64 + 255) // 256 * 256 for bl in self.blks for b in bl]
        self.arena = self.eng.dev_alloc(sum(sizes))
        dptrs, o = [], 0
        for bl in self.blks:
            cur = []
            for b in bl:
                self.eng.dev_upload(self.arena, b, o)
                cur.append(self.arena + o)
                o += (len(b) + 64 + 255) // 256 * 256
            dptrs.append(cur)
        NB = len(self.blks)
        self.NB = NB
        self.hb = [self.eng.block_batch(self.blks[k], dptrs[k]) for k in range(NB)]
        B = len(self.blks[0])
        self.flags = np.empty(B * T, dtype=np.uint8)
        ntx = np.array([T] * B, dtype=np.int64)
        self.steps = [_lib.BlockStep(self.eng, self.hb[k], [0] * B, [T] * B, 0, B * T, ntx, 1, 0, self.flags,
                                     presplit=True, next_batch=self.hb[(k + 1) % NB], fused=True) for k in range(NB)]

    def step(self, s):
        st = self.steps[s % self.NB]
        st.validate()
        # as bench.py: batches k+2 and k+3 pre-split once call k returns (fgv_presplit)
        self.eng.presplit(self.hb[(s + 2) % self.NB])
        self.eng.presplit(self.hb[(s + 3) % self.NB])
        return st.flags

    def parity(self, k, flags):
        exp = np.array([e if e is not None else 255 for bl in self.labels[k] for e in blocks.expected_codes(bl)], np.int64)
        known = np.array([e is not None for bl in self.labels[k] for e in blocks.expected_codes(bl)])
        return int(((flags.astype(np.int64) != exp) & known).sum())

    def close(self):
        self.eng.dev_free(self.arena)
        self.eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--contexts", type=int, default=1, choices=[1, 2])
    ap.add_argument("--batches", type=int, default=6)
    a = ap.parse_args()
    B, T = 32, 500
    assert "torch" not in sys.modules
    t0 = time.time()
    nets = [blocks.Network(seed=3 + c, orgs=3, clients=100) for c in range(a.contexts)]
    nb = a.batches if a.contexts == 1 else max(3, a.batches // 2)
    chans = [Channel(nets[c], make_batches(nets[c], nb, B, T, rank=c), T) for c in range(a.contexts)]
    print(f"[notorch] {a.contexts} context(s) x {nb} batches ready in {time.time() - t0:.1f}s", file=sys.stderr)
    mism = 0
    for ch in chans:
        for k in range(ch.NB):
            mism += ch.parity(k, ch.step(k).copy())
        for s in range(a.warmup):
            ch.step(s)
    K = a.steps
    start = a.warmup
    el = [0.0] * a.contexts
    go = threading.Barrier(a.contexts)

    def run(c):
        ch = chans[c]
        go.wait()
        t = time.perf_counter()
        for s in range(start, start + K):
            ch.step(s)
        el[c] = time.perf_counter() - t

    th = [threading.Thread(target=run, args=(c,)) for c in range(a.contexts)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    wall = max(el)
    assert "torch" not in sys.modules
    out = dict(metric="validated tx/s, torch-free harness", value=round(a.contexts * K * B * T / wall, 1),
               unit="validated tx/s", contexts=a.contexts, steps=K, warmup=a.warmup,
               ms_per_step=round(wall / K * 1e3, 3), per_context_ms_per_step=[round(e / K * 1e3, 3) for e in el],
               parity_vs_labels=mism == 0, torch_loaded=False,
               config=dict(workload="C2 (bench.py default): 32 x 500-tx blocks per step, HBM-resident via "
                                    "fgv_dev_alloc, %d distinct batches per context" % nb))
    for ch in chans:
        ch.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
