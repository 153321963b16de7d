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
