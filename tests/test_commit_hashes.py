"""CPU (host code of libfgv.so): fgv_commit_hashes -- the update batches of consecutive blocks
hashed on host threads in parallel, then chained in block order -- reproduces every commit hash
stored in the reference's sample ledgers (kv_ledger.go:806-817; tests/golden/sample_ledgers.*),
and equals block-by-block fgv_commit_hash on the end-to-end pipeline generator's blocks."""
import numpy as np
import pytest

from fabric_amd import _lib
from tests.test_oracle_ledgers import ledgers


@pytest.mark.parametrize("name", ["v20_testchannel", "v11_ledger1", "v11_ledger2"])
@pytest.mark.parametrize("threads", [0, 1, 3])
def test_commit_hashes_reference_ledgers(name, threads):
    bl = [b for b in ledgers()[name] if b["commit_hash"] is not None]
    assert bl[0]["number"] == 1
    got = _lib.commit_hashes([b["block"] for b in bl], [np.array(b["flags"], np.uint8) for b in bl],
                             [b["number"] for b in bl], b"", threads=threads)
    assert [h.hex() for h in got] == [b["commit_hash"] for b in bl]
    # a chain resumed in the middle: the previous block's hash as `prev`
    k = len(bl) // 2
    tail = _lib.commit_hashes([b["block"] for b in bl[k:]], [np.array(b["flags"], np.uint8) for b in bl[k:]],
                              [b["number"] for b in bl[k:]], bytes.fromhex(bl[k - 1]["commit_hash"]), threads=threads)
    assert [h.hex() for h in tail] == [b["commit_hash"] for b in bl[k:]]


def test_commit_hashes_pipeline_blocks():
    from fabric_amd.synth import blocks, pipeline
    from fabric_amd.synth.mvcc import MvccState
    net = blocks.Network(seed=3, orgs=3, clients=10)
    st = MvccState(5000, seed=2)
    blks, _, fexp, _ = pipeline.make_blocks(net, st, 4, 40, 3001, seed=1)
    got = _lib.commit_hashes(blks, fexp, range(3001, 3005), b"\x07" * 32)
    prev = b"\x07" * 32
    for b in range(4):
        prev = _lib.commit_hash(blks[b], fexp[b], 3001 + b, prev)
        assert got[b] == prev, b


def test_commit_hashes_ub_given_bytes():
    """fgv_commit_hashes_ub (the device update-batch path's host half): blocks whose update bytes
    are given hash them as they are (here the oracle's deterministicBytesForPubAndHashUpdates),
    the others are decoded -- the same chain as fgv_commit_hashes and the reference ledgers"""
    from oracle import commithash
    bl = [b for b in ledgers()["v20_testchannel"] if b["commit_hash"] is not None]
    blks = [b["block"] for b in bl]
    fl = [np.array(b["flags"], np.uint8) for b in bl]
    nums = [b["number"] for b in bl]
    ub = [commithash.update_batch_bytes(*commithash.update_batch(b, list(f), n)) if i % 2 == 0 else None
          for i, (b, f, n) in enumerate(zip(blks, fl, nums))]
    got = _lib.commit_hashes_ub(ub, blks, fl, nums)
    assert [h.hex() for h in got] == [b["commit_hash"] for b in bl]
    # bytes that differ from the block's update batch change the hash (they are what is hashed)
    if any(u for u in ub if u):
        k = next(i for i, u in enumerate(ub) if u)
        bad = list(ub)
        bad[k] = ub[k] + b"\x00"
        assert _lib.commit_hashes_ub(bad, blks, fl, nums)[k] != got[k]


def _bulk_block(nwrites, dup_at=None):
    """Two transactions: a bulk load of `nwrites` keys (one key written twice when dup_at is
    set) and an ordinary one; flags all VALID (the commit hash does not validate)."""
    from fabric_amd.synth import blocks
    net = blocks.Network(seed=5, orgs=3, clients=4)
    keys = ["bulk%06d" % i for i in range(nwrites)]
    if dup_at is not None:
        keys[dup_at] = keys[dup_at // 2]
    bulk = blocks.tx_rwset([("mycc", blocks.kv_rwset([], [(k, b"v%d" % i, False) for i, k in enumerate(keys)]))])
    other = blocks.tx_rwset([("mycc", blocks.kv_rwset([], [("bulk000001", b"later", False), ("z", b"", True)]))])
    blk, _, _ = blocks.make_block(net, 2, number=9, seed=1, faults=(("clean", 1.0),), rwsets=[bulk, other])
    return blk


def test_commit_hash_bulk_transaction():
    """one VALID transaction writing 50k keys -- the twice-written-key check
    is O(w log w), not pairwise; the hash equals the oracle's."""
    import time

    import oracle.commithash as och
    blk = _bulk_block(50_000)
    flags = np.zeros(2, np.uint8)
    t0 = time.perf_counter()
    got = _lib.commit_hash(blk, flags, 9, b"\x01" * 32)
    dt = time.perf_counter() - t0
    assert dt < 1.0, dt  # pairwise: ~1.25e9 comparisons, several seconds
    assert got == och.block_commit_hash(blk, [0, 0], 9, b"\x01" * 32)


def test_commit_hash_bulk_transaction_dup_key():
    """A key written twice inside one bulk transaction stays outside the model (tx_ops.go:183-191
    flag arithmetic), as in the oracle."""
    import oracle.commithash as och
    blk = _bulk_block(5_000, dup_at=4_321)
    with pytest.raises(Exception):
        och.block_commit_hash(blk, [0, 0], 9, b"")
    with pytest.raises(_lib.FgvError):
        _lib.commit_hash(blk, np.zeros(2, np.uint8), 9, b"")
