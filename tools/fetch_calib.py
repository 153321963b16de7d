"""FETCH_SIZE calibration on gfx950 for the two access shapes the traffic figures mix (profiling
aid): a wide streaming read and random 64-byte row gathers from a table far larger
than the Infinity Cache.  Run under rocprofv3 --pmc FETCH_SIZE (tools/gpu_round.sh fetchcalib);
tools/fetch_calib_report.py divides each kernel's counter by the bytes it must read.

Kernels (torch's own, on purpose: no engine code is measured here):
  stream  -- table.sum() over a 1 GiB fp32 table (1 GiB read once)
  gather  -- table.index_select(0, rows) of 1M random distinct 64 B rows of a 2 GiB table
             (64 MiB of rows; each row sits in its own 128 B line), then the same with 32 B and
             128 B rows (the table viewed with 8 / 32 words per row): the counter per row tells
             the fetch granularity apart from the counter's scale
"""
import torch

dev = torch.device("cuda:0")
torch.manual_seed(0)
ROW = 16  # fp32 words per row: 64 B
big = torch.empty((2 << 30) // 64, ROW, dtype=torch.float32, device=dev).uniform_()
n = 1 << 20
rows = torch.randperm(big.shape[0], device=dev)[:n]
stream = big[: (1 << 30) // 64]
b32, b128 = big.view(-1, 8), big.view(-1, 32)
r32 = torch.randperm(b32.shape[0], device=dev)[:n]
r128 = torch.randperm(b128.shape[0], device=dev)[:n]
for _ in range(3):
    s = stream.sum()
    g = big.index_select(0, rows)
torch.cuda.synchronize()
for _ in range(2):
    g32 = b32.index_select(0, r32)  # 32 B rows
    torch.cuda.synchronize()
    g128 = b128.index_select(0, r128)  # 128 B rows
    torch.cuda.synchronize()
print("stream bytes", stream.numel() * 4, "gather rows", n, "row bytes", ROW * 4, "sum", float(s), float(g.sum()))
