"""GPU, two processes on the one GPU of the box (gloo for the exchange): the multi-process
protocol of fabric_amd/shard.py with REAL engine shards -- each rank validates its plan's
transactions of a C2 batch with fgv_validate_shard, the ranks all-gather the records, each rank
finalizes -- and every rank's flags equal the oracle's.  (The 8-GPU RCCL run is the driver's.)"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, pems, blks, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    from fabric_amd import _lib, shard, txvalidator
    from fabric_amd.synth import blocks
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net = blocks.Network(seed=3, orgs=3, clients=40, pems=pems)
        eng = _lib.Engine(0, host_threads=4)
        txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
        from oracle.protowire import decode
        ntx = np.array([len(decode("Block", b)["data"].get("data", [])) for b in blks], np.int64)
        lo, hi = shard.plan(ntx, world, mode)
        res, got_ntx = eng.validate_shard(blks, lo[rank], hi[rank])
        cnt = shard.plan_counts(lo, hi)
        assert len(res) == int(cnt[rank].sum())
        full = shard.allgather_results(res, ntx, world, plan_=(lo, hi))
        flags = _lib.finalize_flags(ntx, full)
        q.put((rank, flags.tolist(), None))
        eng.close()
    except Exception as e:  # reported to the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["block", "tx"])
def test_two_process_engine_shards_match_oracle(mode):
    from fabric_amd.synth import blocks
    from oracle import v20
    net = blocks.Network(seed=3, orgs=3, clients=40)
    txs = []
    blks = [blocks.make_block(net, 60, number=1, seed=41, out_txs=txs)[0]]
    blks.append(blocks.make_block(net, 45, number=2, seed=42, reuse={3: (txs[5].creator, txs[5].nonce)})[0])
    blks.append(blocks.make_block(net, 30, number=3, seed=43)[0])
    exp = [f for fl in v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), blks)
           for f in fl]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, net.export_pems(), blks, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, flags, err in out:
        assert err is None, (rank, err)
        assert flags == exp, rank


RCCL_CHILD = r"""
import os, sys, socket
sys.path.insert(0, %(root)r)
import numpy as np, torch, torch.distributed as dist
from fabric_amd import _lib, shard, txvalidator
from fabric_amd.synth import blocks
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
net = blocks.Network(seed=3, orgs=3, clients=40)
blks = [blocks.make_block(net, 50 + 7 * i, number=1 + i, seed=71 + i)[0] for i in range(3)]
eng = _lib.Engine(0)
txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
fused = eng.validate_blocks(blks)
ntx = np.array([len(f) for f in fused], np.int64)
lo, hi = shard.plan(ntx, 1, "block")
rows = shard.plan_rows(lo, hi)
send = torch.zeros((rows, shard.REC), dtype=torch.uint8, device=dev)
recv = torch.zeros((rows, shard.REC), dtype=torch.uint8, device=dev)
ok = True
for it in range(3):
    eng.validate_shard_dev(blks, lo[0], hi[0], send.data_ptr(), rows)
    recv.zero_()
    shard.allgather_device(send, recv, eng=eng)   # RCCL on torch's stream; the engine waits by an event
    flags = eng.finalize_flags_dev(ntx, 1, rows, recv.data_ptr(), plan=(lo, hi))
    ok &= list(flags) == [x for f in fused for x in f]
dist.destroy_process_group()
eng.close()
print("RCCL_OK", ok)
"""


def test_rccl_allgather_event_wait_world1():
    """the N > 1 device protocol's exchange over RCCL (backend "nccl", one rank on the box's GPU):
    the all-gather runs on torch's stream and the engine's finalize waits for it by an event
    (fgv_stream_wait_external, no host synchronisation); flags equal the fused single-GPU call"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", RCCL_CHILD % {"root": root}], capture_output=True, text=True,
                       timeout=240, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert p.returncode == 0, p.stderr[-2000:]
    assert "RCCL_OK True" in p.stdout, (p.stdout[-500:], p.stderr[-1500:])
