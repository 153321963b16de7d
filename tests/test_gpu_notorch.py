"""GPU: the engine driven through the C ABI alone, in a process without torch (a Go peer through
cgo has no other GPU runtime): blocks placed in HBM with fgv_dev_alloc / fgv_dev_upload, two
channel contexts on the one device validating from two host threads at once, flags equal the
restated committer's (oracle/v20.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, threading
sys.path.insert(0, %(root)r)
import numpy as np
from fabric_amd import _lib, txvalidator
from fabric_amd.synth import blocks
from oracle import v20
res = {}
def run(c):
    net = blocks.Network(seed=30 + c, orgs=3, clients=20)
    blks = [blocks.make_block(net, 60 + 10 * i, number=1 + i, seed=500 + 10 * c + i)[0] for i in range(3)]
    exp = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), blks)
    eng = _lib.Engine(0)
    txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
    sizes = [(len(b) + 64 + 255) // 256 * 256 for b in blks]
    arena = eng.dev_alloc(sum(sizes))
    d, o = [], 0
    for b, sz in zip(blks, sizes):
        eng.dev_upload(arena, b, o)
        d.append(arena + o)
        o += sz
    ok = True
    for it in range(3):
        got = eng.validate_blocks(blks, d_blocks=d)
        ok &= all(list(g) == list(e) for g, e in zip(got, exp))
    eng.dev_free(arena)
    eng.close()
    res[c] = ok
th = [threading.Thread(target=run, args=(c,)) for c in range(2)]
[t.start() for t in th]
[t.join() for t in th]
assert "torch" not in sys.modules, "torch was loaded"
print("NOTORCH", res[0], res[1])
"""


def test_two_contexts_without_torch():
    env = dict(os.environ, FGV_NO_TORCH="1")
    p = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "NOTORCH True True" in p.stdout, (p.stdout[-500:], p.stderr[-1000:])
