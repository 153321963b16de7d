"""Multi-GPU committer protocol: transaction-index sharding + one all-gather.

Every rank holds the block batch (bytes in host memory and HBM), validates transactions
[lo_b, hi_b) of every block b with fgv_validate_shard, then the ranks all-gather their
fgv_tx_result records (68 B/tx; RCCL over xGMI with backend "nccl", gloo on CPU) and each
rank runs fgv_finalize_flags -- the only cross-transaction steps of the reference
(block-store txid index of earlier blocks, validator.go:460-481; markTXIdDuplicates,
validator.go:279-295).  No other collective touches the data path.
"""
import numpy as np
import torch
import torch.distributed as dist

REC = 68  # sizeof(fgv_tx_result)


def shard_ranges(ntx, rank, world):
    ntx = np.asarray(ntx, dtype=np.int64)
    lo = (ntx * rank) // world
    hi = (ntx * (rank + 1)) // world
    return lo.astype(np.uint32), hi.astype(np.uint32)


def padded_rows(ntx, world):
    """rows per rank after padding (the largest shard)"""
    ntx = np.asarray(ntx, dtype=np.int64)
    return int(max(((ntx * (r + 1)) // world - (ntx * r) // world).sum() for r in range(world)))


def allgather_results(local, ntx, world, device=None, group=None, out=None):
    """local: (rows, 68) uint8 results of this rank's shard.  Returns (sum(ntx), 68) uint8 in
    block-major transaction order, identical on every rank."""
    rows = padded_rows(ntx, world)
    if dist.get_backend(group) == "gloo":
        device = "cpu"
        out = None
    send = torch.zeros((rows, REC), dtype=torch.uint8, device=device)
    send[: len(local)].copy_(torch.as_tensor(local).to(device))
    recv = torch.empty((world * rows, REC), dtype=torch.uint8, device=device) if out is None else out
    dist.all_gather_into_tensor(recv, send, group=group)
    g = recv.cpu().numpy() if recv.device.type != "cpu" else recv.numpy()
    return reorder(g, ntx, world, rows)


def allgather_device(send, recv, group=None):
    """All-gather the per-rank device record buffers (rows x 68 each) into `recv`
    (world*rows x 68, rank-major -- the layout fgv_finalize_flags_dev reads), and wait for it
    so the engine's own stream may read `recv`.  gloo (CPU rehearsal) gathers through host
    memory."""
    if dist.get_backend(group) == "gloo":
        tmp = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_gather_into_tensor(tmp, send.cpu(), group=group)
        recv.copy_(tmp)
    else:
        dist.all_gather_into_tensor(recv, send, group=group)
    torch.cuda.current_stream(recv.device).synchronize()


def reorder(gathered, ntx, world, rows):
    """rank-major padded rows -> block-major transaction order"""
    ntx = np.asarray(ntx, dtype=np.int64)
    parts = []
    for b in range(len(ntx)):
        for r in range(world):
            lo, hi = shard_ranges(ntx, r, world)
            off = int((hi[:b].astype(np.int64) - lo[:b]).sum())
            parts.append(gathered[r * rows + off: r * rows + off + int(hi[b]) - int(lo[b])])
    return np.concatenate(parts) if parts else np.zeros((0, REC), np.uint8)
