"""Multi-GPU committer protocol: transaction-index sharding + one all-gather.

Every rank holds the block batch (bytes in host memory and HBM) and validates a contiguous
range of the batch's transactions with fgv_validate_shard[_dev]; the ranks all-gather their
fgv_tx_result records (68 B/tx; RCCL over xGMI with backend "nccl", gloo on CPU) and each
rank runs fgv_finalize_flags[_dev] -- the only cross-transaction steps of the reference
(block-store txid index of earlier blocks, validator.go:460-481; markTXIdDuplicates,
validator.go:279-295).  No other collective touches the data path.

Shard plans (`plan`): with at least as many blocks as ranks, the ranges fall on block
boundaries ("block": rank r takes blocks [B r / W, B (r+1) / W) whole, so it splits and parses
only its own blocks -- the host block split does not grow with W); otherwise every block is
split by transaction index ("tx": [n r / W, n (r+1) / W) of each block).  Either way a
transaction's creator and endorsements stay on one GPU.
"""
import numpy as np
import torch
import torch.distributed as dist

REC = 68  # sizeof(fgv_tx_result)
SKIP = 0xFFFFFFFF  # FGV_SHARD_SKIP: another rank's block


def plan(ntx, world, mode="auto"):
    """(lo, hi): uint32 [world, nblocks]; rank r validates transactions [lo[r,b], hi[r,b]) of
    block b (SKIP: none, block not parsed)."""
    ntx = np.asarray(ntx, dtype=np.int64)
    B = len(ntx)
    if mode == "auto":
        mode = "block" if B >= world else "tx"
    lo = np.zeros((world, B), np.uint32)
    hi = np.zeros((world, B), np.uint32)
    for r in range(world):
        if mode == "tx":
            lo[r] = (ntx * r) // world
            hi[r] = (ntx * (r + 1)) // world
        else:
            b0, b1 = (B * r) // world, (B * (r + 1)) // world
            lo[r, :] = SKIP
            hi[r, :] = SKIP
            lo[r, b0:b1] = 0
            hi[r, b0:b1] = ntx[b0:b1]
    return lo, hi


def plan_counts(lo, hi):
    """transactions per (rank, block)"""
    return np.where(lo == SKIP, 0, hi.astype(np.int64) - lo.astype(np.int64))


def plan_rows(lo, hi):
    """rows per rank after padding (the largest shard)"""
    return int(plan_counts(lo, hi).sum(axis=1).max()) if lo.size else 0


def shard_ranges(ntx, rank, world):
    ntx = np.asarray(ntx, dtype=np.int64)
    lo = (ntx * rank) // world
    hi = (ntx * (rank + 1)) // world
    return lo.astype(np.uint32), hi.astype(np.uint32)


def padded_rows(ntx, world):
    """rows per rank after padding (the largest shard)"""
    ntx = np.asarray(ntx, dtype=np.int64)
    return int(max(((ntx * (r + 1)) // world - (ntx * r) // world).sum() for r in range(world)))


def allgather_results(local, ntx, world, device=None, group=None, out=None, plan_=None):
    """local: (rows, 68) uint8 results of this rank's shard.  Returns (sum(ntx), 68) uint8 in
    block-major transaction order, identical on every rank."""
    rows = padded_rows(ntx, world) if plan_ is None else plan_rows(*plan_)
    if dist.get_backend(group) == "gloo":
        device = "cpu"
        out = None
    send = torch.zeros((rows, REC), dtype=torch.uint8, device=device)
    send[: len(local)].copy_(torch.as_tensor(local).to(device))
    recv = torch.empty((world * rows, REC), dtype=torch.uint8, device=device) if out is None else out
    dist.all_gather_into_tensor(recv, send, group=group)
    g = recv.cpu().numpy() if recv.device.type != "cpu" else recv.numpy()
    return reorder(g, ntx, world, rows, plan_)


def allgather_device(send, recv, group=None, eng=None):
    """All-gather the per-rank device record buffers (rows x 68 each) into `recv`
    (world*rows x 68, rank-major -- the layout fgv_finalize_flags_dev reads).  With `eng` the
    engine's stream waits for the collective's stream by an event (fgv_stream_wait_external: no
    host synchronisation; the finalize kernels queue behind it), else the host waits for it.
    gloo (CPU rehearsal) gathers through host memory."""
    if dist.get_backend(group) == "gloo":
        tmp = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_gather_into_tensor(tmp, send.cpu(), group=group)
        recv.copy_(tmp)
    else:
        dist.all_gather_into_tensor(recv, send, group=group)
    if eng is not None:
        eng.wait_stream(torch.cuda.current_stream(recv.device).cuda_stream)
    else:
        torch.cuda.current_stream(recv.device).synchronize()


def reorder(gathered, ntx, world, rows, plan_=None):
    """rank-major padded rows -> block-major transaction order"""
    ntx = np.asarray(ntx, dtype=np.int64)
    lo, hi = plan_ if plan_ is not None else plan(ntx, world, "tx")
    cnt = plan_counts(lo, hi)
    parts = []
    for b in range(len(ntx)):
        for r in sorted(range(world), key=lambda r: (0 if cnt[r, b] == 0 else int(lo[r, b]))):
            off = int(cnt[r, :b].sum())
            parts.append(gathered[r * rows + off: r * rows + off + int(cnt[r, b])])
    return np.concatenate(parts) if parts else np.zeros((0, REC), np.uint8)


UNSUPPORTED = -6  # FGV_EUNSUPPORTED
LATER = 1  # FGV_BLOCK_LATER


def block_outcomes(flags, ntx, n_final_local, group=None):
    """Per-block outcomes of the shard protocol (each rank's engine with fgv_set_block_outcomes
    on; include/fgv.h): n_final = the minimum over ranks of each rank's fgv_last_block_status
    n_final (an all-reduce when torch.distributed is initialised; a rank's key-level walk sees only
    its own transactions of a block), then per block of the final flags: LATER from n_final on,
    FGV_EUNSUPPORTED where an undecided transaction (0xFD) remains, else 0 (final).  The same
    rules as the single-GPU call (oracle/v20.py validate_blocks_outcomes)."""
    n_final = int(n_final_local)
    if dist.is_available() and dist.is_initialized():
        t = torch.tensor([n_final], dtype=torch.int64)
        if dist.get_backend(group) != "gloo":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        n_final = int(t.item())
    flags = np.asarray(flags, dtype=np.uint8)
    st, o = [], 0
    for b, n in enumerate(np.asarray(ntx, dtype=np.int64)):
        n = int(n)
        if b >= n_final:
            st.append(LATER)
        elif n and (flags[o:o + n] == 0xFD).any():
            st.append(UNSUPPORTED)
        else:
            st.append(0)
        o += n
    return st, n_final
