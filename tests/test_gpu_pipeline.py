"""GPU: the end-to-end commit pipeline on the same blocks -- committer validation
(fgv_validate_blocks), then MVCC validation and commit of consecutive blocks in one device chain
(fgv_mvcc_validate_blocks, committer flags in), then the commit hash (fgv_commit_hash) -- against
the restated committer (oracle/v20.py), txmgmt validation (oracle/mvcc.py) and commit hash
(oracle/commithash.py), and the generator's own expectation.

Reference: gossip/privdata/coordinator.go:152-184 (StoreBlock: Validate, then CommitLegacy),
core/ledger/kvledger/kv_ledger.go:612-652 (ValidateAndPrepare, commit), :806-817 (commit hash)."""
import numpy as np
import pytest

from fabric_amd import _lib, txvalidator
from fabric_amd.synth import blocks, pipeline
from fabric_amd.synth.mvcc import MvccState
from oracle import commithash, mvcc, v20

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nblocks,ntx", [(3, 120), (2, 500)])
def test_pipeline_blocks_match_oracles(nblocks, ntx):
    net = blocks.Network(seed=3, orgs=3, clients=40)
    st = MvccState(50_000, seed=11)
    keys, kb, kt = st.items()
    sdb = mvcc.StateDB({("mycc", k): (int(x), int(y)) for k, x, y in zip(keys, kb, kt)})
    blks, cexp, fexp, _ = pipeline.make_blocks(net, st, nblocks, ntx, 2001, seed=nblocks)
    eng = _lib.Engine(0)
    try:
        txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
        eng.statedb_init(1 << 18, 16 << 20)
        eng.statedb_load("mycc", keys, kb, kt)
        # stage 1: committer
        cf = eng.validate_blocks(blks)
        m = v20.ChannelModel(net.channel, net.identities(), net.chaincodes)
        ocf = v20.validate_blocks(m, blks)
        for b in range(nblocks):
            assert list(cf[b]) == list(ocf[b]) == list(cexp[b]), b
        # stage 2: MVCC of the consecutive blocks, committed on the device
        fl, rc, done = eng.mvcc_validate_blocks(blks, range(2001, 2001 + nblocks), cf, commit=True)
        assert rc == 0 and done == nblocks
        prev_e = prev_o = b""
        for b in range(nblocks):
            of = mvcc.validate_block(sdb, blks[b], list(ocf[b]), 2001 + b, commit=True)
            assert list(fl[b]) == list(of) == list(fexp[b]), (b, [i for i in range(ntx) if fl[b][i] != fexp[b][i]][:8])
            # stage 3: commit hash over the final flags
            he = _lib.commit_hash(blks[b], fl[b], 2001 + b, prev_e)
            ho = commithash.block_commit_hash(blks[b], list(of), 2001 + b, prev_o)
            assert he == ho, b
            prev_e, prev_o = he, ho
        # the batched, parallel commit-hash entry point gives the same chain
        assert _lib.commit_hashes(blks, fl, range(2001, 2001 + nblocks))[-1] == prev_e
        assert any((f == 11).any() for f in fl)  # MVCC conflicts were exercised
        assert eng.statedb_stats()["keys"] >= len(keys)
    finally:
        eng.close()


def test_pipeline_32x500_device_update_batches():
    """the bench's step shape -- 32 x 500-tx blocks through the committer and one
    MVCC chain call with the update batches built on the device (mvcc_ub.hip) -- every block's
    bytes equal oracle.commithash's update batch and the chained hashes equal the oracle's."""
    net = blocks.Network(seed=3, orgs=3, clients=40)
    st = MvccState(200_000, seed=12)
    keys, kb, kt = st.items()
    blks, cexp, fexp, _ = pipeline.make_blocks(net, st, 32, 500, 4001, seed=21)
    nums = list(range(4001, 4033))
    eng = _lib.Engine(0)
    try:
        txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
        eng.statedb_init(1 << 20, 64 << 20)
        eng.statedb_load("mycc", keys, kb, kt)
        eng.mvcc_set_update_bytes(True)
        cf = eng.validate_blocks(blks)
        for b in range(32):
            assert list(cf[b]) == list(cexp[b]), b
        fl, rc, done = eng.mvcc_validate_blocks(blks, nums, cf, commit=True)
        assert rc == 0 and done == 32
        ticket = eng.mvcc_last_ticket()
        ub = eng.mvcc_update_bytes(ticket, 32)
        prev, want = b"\x05" * 32, []
        for b in range(32):
            assert list(fl[b]) == list(fexp[b]), b
            want_ub = commithash.update_batch_bytes(*commithash.update_batch(blks[b], list(fl[b]), nums[b]))
            assert ub[b] == want_ub, b
            prev = commithash.commit_hash(list(fl[b]), want_ub, prev)
            want.append(prev)
        assert _lib.CommitHashesDev(eng, blks, nums).run(fl, b"\x05" * 32, ticket=ticket) == want
    finally:
        eng.close()
