"""GPU parity of whole-block validation: TxValidationFlags from libfgv (HIP engine) must be
bit-identical to the oracle's restated v20 committer on the same blocks."""
import numpy as np
import pytest

from fabric_amd import _lib, txvalidator
from fabric_amd.synth import blocks
from oracle import v20
from tests.blockfix import C5_ENDORSE, SPECIAL, block_from_envs, corrupt_envelopes, network, network_c5

pytestmark = pytest.mark.gpu


def _engine_for(net, committed=(), mode=0):
    """mode 0: device-resident parse (default), 1: host parser."""
    eng = _lib.Engine(0)
    eng.set_parse_mode(mode)
    txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes, committed)
    return eng


MODES = pytest.mark.parametrize("mode", [0, 1], ids=["devparse", "hostparse"])


def _oracle(net, blks, committed=()):
    m = v20.ChannelModel(net.channel, net.identities(), net.chaincodes, committed)
    return v20.validate_blocks(m, blks)


def _check(eng, net, blks, committed=()):
    got = eng.validate_blocks(blks)
    exp = _oracle(net, blks, committed)
    for b, (g, e) in enumerate(zip(got, exp)):
        mism = [(i, int(g[i]), e[i]) for i in range(len(e)) if g[i] != e[i]]
        assert len(g) == len(e) and not mism, (b, mism[:10])
    return exp


@MODES
def test_c2_blocks_and_fault_classes(mode):
    net = network()
    eng = _engine_for(net, mode=mode)
    blks = [blocks.make_block(net, 500, number=1 + i, seed=i)[0] for i in range(2)]
    blks.append(blocks.make_block(net, len(SPECIAL), number=3, seed=3, faults=(), force=SPECIAL)[0])
    exp = _check(eng, net, blks)
    assert exp[2] == blocks.expected_codes(blocks.make_block(net, len(SPECIAL), number=3, seed=3, faults=(),
                                                              force=SPECIAL)[1])
    eng.close()


@MODES
@pytest.mark.parametrize("seed", [11, 12, 13])
def test_corruption_fuzz(seed, mode):
    """Mutated envelopes exercise every protobuf rule and code-precedence branch."""
    net = network()
    eng = _engine_for(net, mode=mode)
    _, _, envs = blocks.make_block(net, 60, number=1, seed=seed)
    bad = corrupt_envelopes(envs, seed, 300)
    # a mutated certificate of a known MSP is outside the engine (the MSP layer would parse it):
    # those envelopes are checked alone for Unsupported on both sides, the rest form the block
    m = v20.ChannelModel(net.channel, net.identities(), net.chaincodes)
    keep, unsup = [], []
    for e in bad:
        try:
            v20.validate_block(m, block_from_envs([e], number=2))
            keep.append(e)
        except v20.Unsupported:
            unsup.append(e)
    assert len(keep) >= 200
    # envelopes whose dependency extraction fails go last: an earlier one would leave every later
    # writer's key-level check waiting forever in the reference (oracle: Unsupported)
    keep.sort(key=lambda e: v20.extract_dependencies(e)[0] != v20.EXTRACT_OK)
    _check(eng, net, [block_from_envs(envs + keep, number=2)])
    for e in unsup[:8]:
        with pytest.raises(_lib.Unsupported):
            eng.validate_blocks([block_from_envs([e], number=3)])
    eng.close()


@MODES
def test_multi_block_txid_index_and_ledger(mode):
    net = network()
    txs = []
    b1, _, envs1 = blocks.make_block(net, 20, number=1, seed=21, faults=(), out_txs=txs)
    b2, _, _ = blocks.make_block(net, 20, number=2, seed=22, faults=(), reuse={5: (txs[7].creator, txs[7].nonce),
                                                                                 9: (txs[7].creator, txs[7].nonce)})
    committed = [v20.index_txid(envs1[0])]
    b3, _, _ = blocks.make_block(net, 5, number=3, seed=23, faults=(), reuse={1: (txs[0].creator, txs[0].nonce)})
    eng = _engine_for(net, committed, mode=mode)
    exp = _check(eng, net, [b1, b2, b3], committed)
    assert exp[0][0] == 9 and exp[1][5] == 9 and exp[1][9] == 9 and exp[2][1] == 9
    eng.close()


@MODES
def test_empty_and_degenerate_blocks(mode):
    net = network()
    eng = _engine_for(net, mode=mode)
    _, _, envs = blocks.make_block(net, 3, number=1, seed=31, faults=())
    # (the degenerate envelopes last: an empty Envelope has no actions, and the key-level
    # validator's dependency extraction panics on it when a later tx reaches a vscc,
    # validator_keylevel.go:203 -- that block is Unsupported on both sides)
    blks = [block_from_envs([]), block_from_envs([envs[0], b"", b"\x0a\x00", b"\x12\x00"]),
            block_from_envs([envs[1]] * 3)]
    exp = _check(eng, net, blks)
    assert len(exp[0]) == 0 and exp[2] == [0, 9, 9]
    panics = block_from_envs([b"", b"\x0a\x00", envs[0], b"\x12\x00"])
    with pytest.raises(v20.Unsupported):
        _oracle(net, [panics])
    with pytest.raises(_lib.Unsupported):
        eng.validate_blocks([panics])
    eng.close()


@MODES
def test_policy_variants(mode):
    for n in (1, 3):
        net = network(policy_n=n)
        eng = _engine_for(net, mode=mode)
        blk, _, _ = blocks.make_block(net, 50, number=1, seed=40 + n)
        _check(eng, net, [blk])
        eng.close()


@MODES
def test_unsupported_is_reported_not_guessed(mode):
    net = network()
    eng = _lib.Engine(0)
    eng.set_parse_mode(mode)
    txvalidator.setup_channel(eng, net.channel, net.identities(), {"mycc": blocks.f_str(2, "/Channel/Application/E")})
    blk, _, _ = blocks.make_block(net, 4, number=1, seed=50, faults=())
    with pytest.raises(_lib.Unsupported):
        eng.validate_blocks([blk])
    eng.close()


def test_device_resident_blocks_match_host_upload():
    import torch
    net = network()
    eng = _engine_for(net)
    blks = [blocks.make_block(net, 100, number=1 + i, seed=60 + i)[0] for i in range(3)]
    dev = [torch.zeros(len(b) + 64, dtype=torch.uint8, device="cuda:0") for b in blks]
    for d, b in zip(dev, blks):
        d[:len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
    torch.cuda.synchronize()
    a = eng.validate_blocks(blks)
    b = eng.validate_blocks(blks, [d.data_ptr() for d in dev])
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    eng.close()


def test_batch_duplicate_precedes_dispatch_failure():
    """A later block's tx re-using an earlier txid gets 9 even when its endorsements would
    fail the policy (checkTxIdDupsLedger runs before Dispatch, validator.go:365-373)."""
    net = network()
    txs = []
    b1, _, _ = blocks.make_block(net, 6, number=1, seed=71, faults=(), out_txs=txs)
    force = [None, "policy_unsatisfied", None, "unknown_cc", None]
    b2, labels, _ = blocks.make_block(net, 5, number=2, seed=72, faults=(), force=force,
                                      reuse={1: (txs[2].creator, txs[2].nonce), 3: (txs[3].creator, txs[3].nonce)})
    eng = _engine_for(net)
    exp = _check(eng, net, [b1, b2])
    assert exp[1][1] == 9 and exp[1][3] == 9
    eng.close()


@pytest.mark.parametrize("shards", [2, 3])
def test_sharded_validation_matches_single(shards):
    """Multi-GPU protocol on one device: per-shard results + finalize == whole-batch flags."""
    net = network()
    txs = []
    b1, _, _ = blocks.make_block(net, 40, number=1, seed=81, out_txs=txs)
    b2, _, _ = blocks.make_block(net, 37, number=2, seed=82, reuse={2: (txs[5].creator, txs[5].nonce),
                                                                     30: (txs[9].creator, txs[9].nonce)})
    blks = [b1, b2]
    eng = _engine_for(net)
    whole = eng.validate_blocks(blks)
    ntx = [40, 37]
    parts = []
    for r in range(shards):
        lo = [n * r // shards for n in ntx]
        hi = [n * (r + 1) // shards for n in ntx]
        res, nt = eng.validate_shard(blks, lo, hi)
        assert list(nt) == ntx
        parts.append((lo, hi, res))
    # reorder to block-major, tx order (what the all-gather + reshuffle produces)
    rows = []
    for b in range(2):
        for lo, hi, res in parts:
            off = sum(hi[k] - lo[k] for k in range(b))
            rows.append(res[off: off + hi[b] - lo[b]])
    flags = _lib.finalize_flags(ntx, np.concatenate(rows))
    assert np.array_equal(flags, np.concatenate(whole))
    exp = _oracle(net, blks)
    assert list(flags) == exp[0] + exp[1]
    eng.close()


@pytest.mark.parametrize("shards,mode", [(1, "tx"), (2, "tx"), (3, "tx"), (8, "tx"), (2, "block"), (3, "block")])
def test_device_sharded_protocol(shards, mode):
    """fgv_validate_shard_dev per rank into the rank-major gathered buffer (what
    all_gather_into_tensor produces) + fgv_finalize_flags_dev == whole-batch flags == oracle."""
    import torch
    from fabric_amd import shard
    net = network()
    txs = []
    b1, _, _ = blocks.make_block(net, 40, number=1, seed=91, out_txs=txs)
    b2, _, _ = blocks.make_block(net, 3, number=2, seed=92, reuse={1: (txs[5].creator, txs[5].nonce)})
    b3, _, _ = blocks.make_block(net, 29, number=3, seed=93, reuse={4: (txs[7].creator, txs[7].nonce),
                                                                    20: (txs[7].creator, txs[7].nonce)})
    blks = [b1, b2, b3]
    ntx = np.array([40, 3, 29], dtype=np.int64)
    eng = _engine_for(net)
    plan = shard.plan(ntx, shards, mode)
    rows = shard.plan_rows(*plan)
    recv = torch.zeros((shards * rows, shard.REC), dtype=torch.uint8, device="cuda")
    batch = eng.block_batch(blks)
    for r in range(shards):
        lo, hi = plan[0][r], plan[1][r]
        nt = eng.validate_shard_dev(batch, lo, hi, recv[r * rows:].data_ptr(), rows)
        assert list(nt) == [0 if lo[b] == shard.SKIP else ntx[b] for b in range(len(ntx))]
    flags = eng.finalize_flags_dev(ntx, shards, rows, recv.data_ptr(), plan=None if mode == "tx" else plan)
    exp = _oracle(net, blks)
    assert list(flags) == exp[0] + exp[1] + exp[2]
    assert np.array_equal(flags, np.concatenate(eng.validate_blocks(blks)))
    eng.close()


@pytest.mark.parametrize("shards,mode", [(1, "tx"), (3, "tx"), (2, "block")])
def test_presplit_is_used_only_for_its_batch(shards, mode):
    """fgv_presplit (the batch's framing walked ahead on a host thread): a validation of the
    same batch and shard range uses it, any other call ignores it; flags identical to the
    oracle either way."""
    import torch
    from fabric_amd import shard
    net = network()
    blks = [blocks.make_block(net, n, number=1 + i, seed=95 + i)[0] for i, n in enumerate([40, 7, 29])]
    ntx = np.array([40, 7, 29], dtype=np.int64)
    eng = _engine_for(net)
    plan = shard.plan(ntx, shards, mode)
    rows = shard.plan_rows(*plan)
    batch = eng.block_batch(blks)
    other = eng.block_batch([blocks.make_block(net, 12, number=9, seed=99)[0]])
    exp = _oracle(net, blks)
    exp = exp[0] + exp[1] + exp[2]
    for presplit_plan in ("same", "other_rank", "other_batch"):
        recv = torch.zeros((shards * rows, shard.REC), dtype=torch.uint8, device="cuda")
        for r in range(shards):
            lo, hi = plan[0][r], plan[1][r]
            if presplit_plan == "same":
                eng.presplit(batch, lo, hi)
            elif presplit_plan == "other_rank":
                q = (r + 1) % shards
                eng.presplit(batch, plan[0][q], plan[1][q])
            else:
                eng.presplit(other)
            nt = eng.validate_shard_dev(batch, lo, hi, recv[r * rows:].data_ptr(), rows)
            used = eng.last_presplit()
            assert used == (presplit_plan == "same" or (presplit_plan == "other_rank" and shards == 1)), presplit_plan
            assert list(nt) == [0 if lo[b] == shard.SKIP else ntx[b] for b in range(len(ntx))]
        flags = eng.finalize_flags_dev(ntx, shards, rows, recv.data_ptr(), plan=None if mode == "tx" else plan)
        assert list(flags) == exp, presplit_plan
    eng.presplit(batch)  # left pending at close
    eng.close()


@pytest.mark.parametrize("shards,mode", [(1, "tx"), (3, "tx"), (2, "block")])
def test_validate_next_presplits_the_following_call(shards, mode):
    """fgv_validate_shard_dev_next: rank r's call pre-splits rank r+1's range during its own
    GPU work; every following call uses it; flags identical to the oracle."""
    import torch
    from fabric_amd import shard
    net = network()
    blks = [blocks.make_block(net, n, number=1 + i, seed=95 + i)[0] for i, n in enumerate([40, 7, 29])]
    ntx = np.array([40, 7, 29], dtype=np.int64)
    eng = _engine_for(net)
    plan = shard.plan(ntx, shards, mode)
    rows = shard.plan_rows(*plan)
    batch = eng.block_batch(blks)
    exp = _oracle(net, blks)
    recv = torch.zeros((shards * rows, shard.REC), dtype=torch.uint8, device="cuda")
    for rep in range(2):
        for r in range(shards):
            q = (r + 1) % shards
            eng.validate_shard_dev_next(batch, plan[0][r], plan[1][r], recv[r * rows:].data_ptr(), rows, batch,
                                        plan[0][q], plan[1][q])
            assert eng.last_presplit() == (rep > 0 or r > 0)
        flags = eng.finalize_flags_dev(ntx, shards, rows, recv.data_ptr(), plan=None if mode == "tx" else plan)
        assert list(flags) == exp[0] + exp[1] + exp[2]
    eng.close()


@pytest.mark.parametrize("pinned", [True, False], ids=["pinned", "pageable"])
def test_host_resident_rotation_prefetches_next_batch(pinned):
    """Host-resident batches A, B, C, A, ... through fgv_validate_shard_dev_next: every call
    after the first finds its blocks already copied by the previous call's prefetch (copy
    stream, second staging arena); a call whose batch was not the announced one copies itself.
    Flags equal the oracle's on every call."""
    import torch
    net = network()
    sizes = [[23, 5], [31], [9, 17, 3]]
    sets, exps = [], []
    for k, sz in enumerate(sizes):
        blks = [blocks.make_block(net, n, number=1 + i, seed=300 + 10 * k + i)[0] for i, n in enumerate(sz)]
        sets.append(blks)
        exps.append([f for fl in _oracle(net, blks) for f in fl])
    eng = _engine_for(net)
    bufs = []
    batches = []
    for blks in sets:
        if pinned:
            pb = eng.host_alloc(sum(len(b) for b in blks))
            views, o = [], 0
            for b in blks:
                pb.a[o:o + len(b)] = np.frombuffer(b, np.uint8)
                views.append(pb.a[o:o + len(b)])
                o += len(b)
            bufs.append(pb)
            batches.append(eng.block_batch(views))
        else:
            batches.append(eng.block_batch(blks))
    order = [0, 1, 2, 0, 2, 1, 1]
    res = torch.zeros((64, _lib.TX_RESULT_BYTES), dtype=torch.uint8, device="cuda")
    for i, k in enumerate(order):
        nxt = order[i + 1] if i + 1 < len(order) else 0
        ntx_b = eng.validate_shard_dev_next(batches[k], [0] * batches[k].nb, [1 << 30] * batches[k].nb,
                                            res.data_ptr(), 64, batches[nxt])
        copied, hits = eng.last_h2d()
        assert hits == (batches[k].nb if i > 0 else 0), (i, hits)
        assert (copied == 0) == (i > 0), (i, copied)
        flags = eng.finalize_flags_dev(ntx_b, 1, 64, res.data_ptr())
        assert list(flags) == exps[k], (i, k)
    # a call that is not the announced batch copies itself; the rotation then resumes
    eng.validate_shard_dev_next(batches[2], [0] * 3, [1 << 30] * 3, res.data_ptr(), 64, batches[1])
    assert eng.last_h2d()[1] == 0 and eng.last_h2d()[0] > 0
    ntx_b = eng.validate_shard_dev_next(batches[1], [0], [1 << 30], res.data_ptr(), 64, batches[0])
    assert eng.last_h2d() == (0, 1)
    assert list(eng.finalize_flags_dev(ntx_b, 1, 64, res.data_ptr())) == exps[1]
    for pb in bufs:
        pb.close()
    eng.close()


@pytest.mark.parametrize("where", ["hbm", "pinned", "pageable"])
def test_single_gpu_pipelined_rotation(where):
    """fgv_validate_blocks_pipelined (validation + finalize queued back to back, one
    synchronisation; the next batch pre-split -- and, host-resident, pre-copied -- during the
    call) over a rotation A, B, C, A, C, B, B: flags equal the oracle's on every call, the
    pre-split is used exactly when the call's batch was the announced one, host-resident calls
    find their blocks prefetched, and a mid-rotation call of an unannounced batch still matches."""
    import torch
    net = network()
    sizes = [[23, 5], [31], [9, 17, 3]]
    sets, exps = [], []
    for k, sz in enumerate(sizes):
        blks = [blocks.make_block(net, n, number=1 + i, seed=700 + 10 * k + i)[0] for i, n in enumerate(sz)]
        sets.append(blks)
        exps.append([f for fl in _oracle(net, blks) for f in fl])
    eng = _engine_for(net)
    bufs, batches, keep = [], [], []
    for blks in sets:
        if where == "hbm":
            arena = torch.zeros(sum((len(b) + 64 + 255) // 256 * 256 for b in blks), dtype=torch.uint8, device="cuda")
            dp, o = [], 0
            for b in blks:
                arena[o:o + len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
                dp.append(arena.data_ptr() + o)
                o += (len(b) + 64 + 255) // 256 * 256
            keep.append(arena)
            batches.append(eng.block_batch(blks, dp))
        elif where == "pinned":
            pb = eng.host_alloc(sum(len(b) for b in blks))
            views, o = [], 0
            for b in blks:
                pb.a[o:o + len(b)] = np.frombuffer(b, np.uint8)
                views.append(pb.a[o:o + len(b)])
                o += len(b)
            bufs.append(pb)
            batches.append(eng.block_batch(views))
        else:
            batches.append(eng.block_batch(blks))
    torch.cuda.synchronize()
    order = [0, 1, 2, 0, 2, 1, 1]
    for i, k in enumerate(order):
        nxt = batches[order[i + 1]] if i + 1 < len(order) else None
        flags = eng.validate_blocks_pipelined(batches[k], nxt)
        assert list(flags) == exps[k], (i, k)
        assert eng.last_presplit() == (i > 0), i
        if where != "hbm":
            assert eng.last_h2d()[1] == (batches[k].nb if i > 0 else 0), (i, eng.last_h2d())
    # an unannounced batch (announced: 0, called: 2), then the plain single-batch call
    eng.validate_blocks_pipelined(batches[1], batches[0])
    assert list(eng.validate_blocks_pipelined(batches[2])) == exps[2] and not eng.last_presplit()
    assert [f for fl in eng.validate_blocks(sets[0]) for f in fl] == exps[0]
    if where == "pinned":  # fgv_prefetch: batch k stages batch k+2 beside its pipelined next batch
        order = [0, 1, 2, 1, 0, 2, 0, 1]
        eng.prefetch(batches[order[0]])
        eng.prefetch(batches[order[1]])
        for i, k in enumerate(order):
            if i + 2 < len(order):
                eng.prefetch(batches[order[i + 2]])
            nxt = batches[order[i + 1]] if i + 1 < len(order) else None
            assert list(eng.validate_blocks_pipelined(batches[k], nxt)) == exps[k], (i, k)
            assert eng.last_h2d()[1] == batches[k].nb, (i, eng.last_h2d())
        # three staged batches fill the ring; a call of a fourth batch (batch 0's blocks in another
        # pinned buffer) drops the oldest staged one, whose call then copies its blocks itself
        pb = eng.host_alloc(sum(len(b) for b in sets[0]))
        views, o = [], 0
        for b in sets[0]:
            pb.a[o:o + len(b)] = np.frombuffer(b, np.uint8)
            views.append(pb.a[o:o + len(b)])
            o += len(b)
        bufs.append(pb)
        extra = eng.block_batch(views)
        for k in (1, 2, 0):
            eng.prefetch(batches[k])
        assert list(eng.validate_blocks_pipelined(extra)) == exps[0] and eng.last_h2d()[1] == 0
        assert list(eng.validate_blocks_pipelined(batches[1])) == exps[1] and eng.last_h2d()[1] == 0
        assert list(eng.validate_blocks_pipelined(batches[2])) == exps[2] and eng.last_h2d()[1] == batches[2].nb
        assert list(eng.validate_blocks_pipelined(batches[0])) == exps[0] and eng.last_h2d()[1] == batches[0].nb
    for pb in bufs:
        pb.close()
    eng.close()


@pytest.mark.parametrize("where", ["hbm", "pinned"])
def test_pipelined_rotation_presplit_after_next(where):
    """The caller pre-splits the batch after next once a call returns (fgv_presplit, the
    deliver-side walk): the following call finds that walk done and queues the next batch's head
    upload, parse and payload hashes at its top (front_launch_a, FGV_FRONT_EARLY), the rest behind
    its back half.  Flags equal the oracle's on every call of a rotation that also announces
    batches it then does not call (the early half is drained and forgotten) and pre-splits batches
    that are never announced."""
    import time
    import torch
    net = network()
    sizes = [[23, 5], [31], [9, 17, 3]]
    sets, exps = [], []
    for k, sz in enumerate(sizes):
        blks = [blocks.make_block(net, n, number=1 + i, seed=900 + 10 * k + i)[0] for i, n in enumerate(sz)]
        sets.append(blks)
        exps.append([f for fl in _oracle(net, blks) for f in fl])
    eng = _engine_for(net)
    bufs, batches, keep = [], [], []
    for blks in sets:
        if where == "hbm":
            arena = torch.zeros(sum((len(b) + 64 + 255) // 256 * 256 for b in blks), dtype=torch.uint8, device="cuda")
            dp, o = [], 0
            for b in blks:
                arena[o:o + len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
                dp.append(arena.data_ptr() + o)
                o += (len(b) + 64 + 255) // 256 * 256
            keep.append(arena)
            batches.append(eng.block_batch(blks, dp))
        else:
            pb = eng.host_alloc(sum(len(b) for b in blks))
            views, o = [], 0
            for b in blks:
                pb.a[o:o + len(b)] = np.frombuffer(b, np.uint8)
                views.append(pb.a[o:o + len(b)])
                o += len(b)
            bufs.append(pb)
            batches.append(eng.block_batch(views))
    torch.cuda.synchronize()
    # (called, announced next, pre-split after the call); the announced batch is called next
    # except at steps 5 (announced 0, calls 1) and 8 (announced 2, calls 0)
    script = [(0, 1, 2), (1, 2, 0), (2, 0, 1), (0, 1, 2), (1, 0, 2), (1, 2, 0), (2, 0, 0), (0, 2, 1),
              (0, 1, 1), (1, None, None)]
    for i, (k, nx, after) in enumerate(script):
        flags = eng.validate_blocks_pipelined(batches[k], None if nx is None else batches[nx])
        assert list(flags) == exps[k], (i, k)
        if after is not None:
            eng.presplit(batches[after])
            time.sleep(0.05)  # (the walk is done when the next call starts: the early path runs)
    # the bench's pattern: after call k, pre-split k+2 and k+3 (both slots), no waiting
    rot = [0, 1, 2, 0, 1, 2, 0, 1, 2, 0]
    for i, k in enumerate(rot):
        nx = batches[rot[i + 1]] if i + 1 < len(rot) else None
        assert list(eng.validate_blocks_pipelined(batches[k], nx)) == exps[k], (i, k)
        for d in (2, 3):
            if i + d < len(rot):
                eng.presplit(batches[rot[i + d]])
    assert [f for fl in eng.validate_blocks(sets[2]) for f in fl] == exps[2]
    for pb in bufs:
        pb.close()
    eng.close()


def _random_records(rng, ntx, pool):
    """fgv_tx_result records honouring the engine's invariants: VALID => REACHED;
    REACHED => INDEXED with index_txid == txid."""
    n = int(sum(ntx))
    rec = np.zeros((n, 68), np.uint8)
    keys = rng.integers(0, 256, size=(pool, 32), dtype=np.uint8)
    code = rng.choice(np.array([0, 0, 0, 0, 9, 10, 8, 4, 255], np.uint8), size=n)
    reached = (code == 0) | (rng.random(n) < 0.3)
    indexed = reached | (rng.random(n) < 0.5)
    tid = rng.integers(0, pool, size=n)
    iid = np.where(reached, tid, rng.integers(0, pool, size=n))
    rec[:, 0] = code
    rec[:, 1] = reached.astype(np.uint8) | (indexed.astype(np.uint8) << 1)
    rec[:, 4:36] = keys[tid]
    rec[:, 36:68] = keys[iid]
    return rec


@pytest.mark.parametrize("seed,pool,world", [(1, 7, 1), (2, 50, 3), (3, 3000, 8), (4, 2, 2)])
def test_device_finalize_matches_host_finalize(seed, pool, world):
    """Device finalize (hash table in HBM) == host finalize on adversarially colliding txids,
    with the rank-major gathered layout built by hand."""
    import torch
    from fabric_amd import shard
    rng = np.random.default_rng(seed)
    ntx = np.array([int(x) for x in rng.integers(0, 400, size=12)] + [0, 1], dtype=np.int64)
    rec = _random_records(rng, ntx, pool)
    host = _lib.finalize_flags(ntx, rec)
    rows = shard.padded_rows(ntx, world)
    g = np.zeros((world * rows, 68), np.uint8)
    starts = np.concatenate([[0], np.cumsum(ntx)])
    for r in range(world):
        lo, hi = shard.shard_ranges(ntx, r, world)
        o = r * rows
        for b in range(len(ntx)):
            k = int(hi[b]) - int(lo[b])
            g[o:o + k] = rec[starts[b] + int(lo[b]): starts[b] + int(hi[b])]
            o += k
    eng = _lib.Engine(0)
    d = torch.from_numpy(g).to("cuda")
    dev = eng.finalize_flags_dev(ntx, world, rows, d.data_ptr())
    assert np.array_equal(dev, host)
    eng.close()


@MODES
def test_c5_mixed_ed25519_blocks_match_oracle(mode):
    """C5 shape at oracle-sized blocks: 8 orgs, 5-of-8, 5-6 endorsements, Ed25519 identities."""
    net = network_c5()
    eng = _engine_for(net, mode=mode)
    blks = [blocks.make_block(net, 300, number=1 + i, seed=100 + i, endorse_dist=C5_ENDORSE)[0] for i in range(2)]
    _check(eng, net, blks)
    eng.close()


def test_c5_full_size_block_and_integrity():
    """A 20k-tx C5 block at full size: flags equal the generator's labels (size-independent
    property), and the deliver-side integrity pass (data hash over ~110 MB) verifies it."""
    net = network_c5()
    eng = _engine_for(net)
    blk, labels, envs = blocks.make_block(net, 20000, number=1, seed=7, endorse_dist=C5_ENDORSE)
    got = eng.validate_blocks([blk])[0]
    exp = blocks.expected_codes(labels)
    known = [i for i, e in enumerate(exp) if e is not None]
    assert len(got) == 20000 and all(int(got[i]) == exp[i] for i in known)
    chk = eng.blocks_verify([blk, blk])
    assert chk[0][0] == _lib.BLK_OK and chk[0][3] == blocks.hashlib.sha256(b"".join(envs)).digest()
    chain = _lib.ChainState(number=0, valid=1, has_hash=0)
    chk = eng.blocks_verify([blk, blk], chain)
    assert [c[0] for c in chk] == [_lib.BLK_OK, _lib.BLK_NUMBER] and chain.number == 1
    eng.close()


def test_device_capacity_overflow_falls_back_to_host_parser():
    """17 endorsements exceed the device parser's capacity (BD_MAX_END): the batch is parsed
    by the host parser and the flags still equal the oracle's."""
    net = network()
    _, _, envs = blocks.make_block(net, 4, number=1, seed=111, faults=())
    import fabric_amd.synth.blocks as B
    txs = []
    blocks.make_block(net, 3, number=2, seed=112, faults=(), out_txs=txs)
    # a tx with 17 copies of one endorsement (dedup -> 1 identity -> policy failure, code 10)
    t = txs[0]
    e = B.f_msg(2, B.f_bytes(1, t.endorsers[0].serialized) + B.f_bytes(2, t.esigs[0]))
    big = B.f_bytes(1, t.prp) + e * 17
    cap = B.f_bytes(1, t.ccpp) + B.f_msg(2, big)
    action = B.f_msg(1, B.f_bytes(1, t.shdr) + B.f_bytes(2, cap))
    payload = B.f_msg(1, B.f_bytes(1, t.chdr) + B.f_bytes(2, t.shdr)) + B.f_bytes(2, action)
    from fabric_amd import synth
    sig = synth.sign(t.creator.key, blocks.hashlib.sha256(payload).digest())
    env = B.f_bytes(1, payload) + B.f_bytes(2, sig)
    eng = _engine_for(net)
    exp = _check(eng, net, [block_from_envs(envs + [env], number=1)])
    assert exp[0][-1] == 10
    eng.close()


def _device_copies(blks):
    import torch
    sizes = [(len(b) + 64 + 255) // 256 * 256 for b in blks]
    arena = torch.zeros(max(1, sum(sizes)), dtype=torch.uint8, device="cuda")
    ptrs, o = [], 0
    for b, sz in zip(blks, sizes):
        if len(b):
            arena[o:o + len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
        ptrs.append(arena.data_ptr() + o)
        o += sz
    return arena, ptrs


def _flags(eng, batch, ntx, res, cap, nxt, lo=None, hi=None):
    lo = [0] * batch.nb if lo is None else lo
    hi = [1 << 30] * batch.nb if hi is None else hi
    nt = eng.validate_shard_dev_pipelined(batch, lo, hi, res.data_ptr(), cap, nxt, [0] * nxt.nb,
                                          [1 << 30] * nxt.nb)
    return list(eng.finalize_flags_dev(nt, 1, cap, res.data_ptr()))


def test_pipelined_front_half_ahead_rotation():
    """fgv_validate_shard_dev_pipelined over HBM-resident batches A, B, C, A, ...: each call
    enqueues the next batch's front half (parse, identities, hashes) while its own back half
    runs; every following call continues from it (fgv_last_ahead) and the flags equal the
    oracle's.  A call for a batch other than the announced one discards the front half."""
    import torch
    net = network()
    sizes = [[23, 5], [31], [9, 17, 3]]
    sets, exps, keep = [], [], []
    eng = _engine_for(net)
    for k, sz in enumerate(sizes):
        blks = [blocks.make_block(net, n, number=1 + i, seed=400 + 10 * k + i)[0] for i, n in enumerate(sz)]
        arena, ptrs = _device_copies(blks)
        keep.append(arena)
        sets.append(eng.block_batch(blks, ptrs))
        exps.append([f for fl in _oracle(net, blks) for f in fl])
    res = torch.zeros((64, _lib.TX_RESULT_BYTES), dtype=torch.uint8, device="cuda")
    order = [0, 1, 2, 0, 0, 2, 1, 1, 2]
    for mode in (0, 3, 1, 2):  # 0: never ahead; 2 (the default) at once; the others place it differently
        eng.set_ahead(mode)
        for i, k in enumerate(order):
            nxt = order[i + 1] if i + 1 < len(order) else 0
            got = _flags(eng, sets[k], None, res, 64, sets[nxt])
            assert eng.last_ahead() == (mode > 0 and i > 0), (mode, i)
            assert got == exps[k], (mode, i, k)
    # the announced batch is 0; a call for batch 1 discards it and starts its own
    assert _flags(eng, sets[1], None, res, 64, sets[2]) == exps[1]
    assert not eng.last_ahead()
    # a shard range other than the announced one is another batch too
    lo, hi = [0, 4, 0], [9, 17, 3]
    nt = eng.validate_shard_dev_pipelined(sets[2], lo, hi, res.data_ptr(), 64, sets[2], lo, hi)
    assert not eng.last_ahead()
    nt = eng.validate_shard_dev_pipelined(sets[2], lo, hi, res.data_ptr(), 64, sets[0])
    assert eng.last_ahead()
    assert list(nt) == [9, 17, 3]
    eng.close()


def test_pipelined_ahead_and_channel_or_ledger_changes():
    """Between two pipelined calls: ledger txids added (fgv_ledger_add_txids) keep the front
    half enqueued ahead (only the back half reads them) and its duplicates come out as 9; a
    chaincode redefinition discards it and the new policy applies -- both equal the oracle."""
    import torch
    net = network()
    a = [blocks.make_block(net, n, number=1 + i, seed=500 + i)[0] for i, n in enumerate([20, 11])]
    b = [blocks.make_block(net, n, number=3 + i, seed=510 + i)[0] for i, n in enumerate([15, 8])]
    eng = _engine_for(net)
    eng.set_ahead(2)
    aa, ap = _device_copies(a)
    ba, bp = _device_copies(b)
    A, Bt = eng.block_batch(a, ap), eng.block_batch(b, bp)
    res = torch.zeros((64, _lib.TX_RESULT_BYTES), dtype=torch.uint8, device="cuda")
    assert _flags(eng, A, None, res, 64, Bt) == [f for fl in _oracle(net, a) for f in fl]
    # the ledger already holds some of B's txids
    txids = []
    for blk in b:
        for env in v20.decode("Block", blk)["data"]["data"][:4]:
            pl = v20.decode("Payload", v20.decode("Envelope", env)["payload"])
            txids.append(v20.decode("ChannelHeader", pl["header"]["channel_header"])["tx_id"])
    eng.ledger_add_txids(txids)
    got = _flags(eng, Bt, None, res, 64, A)
    assert eng.last_ahead()
    exp = [f for fl in _oracle(net, b, committed=txids) for f in fl]
    assert got == exp and exp.count(9) >= 4
    # the chaincode's policy changes: 3-of-3 -> the front half enqueued for A is discarded
    pol = blocks.out_of_policy(3, net.mspids)
    eng.chaincode_define("mycc", pol)
    got = _flags(eng, A, None, res, 64, A)
    assert not eng.last_ahead()
    m = v20.ChannelModel(net.channel, net.identities(), dict(net.chaincodes, mycc=pol), txids)
    assert got == [f for fl in v20.validate_blocks(m, a) for f in fl]
    eng.close()
