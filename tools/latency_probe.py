"""Single-block latency probe (profiling aid, not the bench): one C2 block (500 tx) HBM-resident,
validated + finalized one call at a time (fgv_validate_blocks, no pre-split, nothing ahead), the
median of --reps calls; run under rocprofv3 --kernel-trace to see the per-block chain.
python tools/latency_probe.py [--reps 40] [--tx 500]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fabric_amd import _lib, txvalidator  # noqa: E402
from fabric_amd.synth import blocks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--tx", type=int, default=500)
    ap.add_argument("--churn", action="store_true", help="client keys on the variable-base kernels (no combs)")
    a = ap.parse_args()
    net = blocks.Network(seed=3, orgs=3, clients=100)
    blk, lab, _ = blocks.make_block(net, a.tx, number=1, seed=7)
    exp = np.array([e if e is not None else 255 for e in blocks.expected_codes(lab)])
    known = np.array([e is not None for e in blocks.expected_codes(lab)])
    eng = _lib.Engine(0)
    # the bench's headline setup: the 100 clients hold comb tables (--churn: variable-base)
    txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes, hot_clients=not a.churn)
    dev = torch.device("cuda", 0)
    d = torch.zeros(len(blk) + 256, dtype=torch.uint8, device=dev)
    d[:len(blk)].copy_(torch.frombuffer(bytearray(blk), dtype=torch.uint8))
    torch.cuda.synchronize()
    ts = []
    for i in range(a.reps + 3):
        t = time.perf_counter()
        f = eng.validate_blocks([blk], d_blocks=[d.data_ptr()])[0]
        ts.append((time.perf_counter() - t) * 1e3)
        assert ((f.astype(np.int64) != exp) & known).sum() == 0
    ts = np.array(ts[3:])
    print(f"single block ({a.tx} tx, HBM-resident): median {np.median(ts):.3f} ms, min {ts.min():.3f}, "
          f"p90 {np.percentile(ts, 90):.3f}")
    eng.close()


if __name__ == "__main__":
    main()
