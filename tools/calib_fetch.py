"""FETCH_SIZE calibration for k_proc's access mix (MI355X_MICROARCH.md §HBM:
only 16-B/lane streaming reads are calibrated; "calibrate on a known byte count
in your own access pattern").  Run under one rocprofv3 --pmc pass, e.g.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o calib --output-format csv -- python tools/calib_fetch.py

Three known-count kernels, each launched three times (the last is read):
  stream   x.sum() over 1 GiB of float32 (16-B/lane streaming reads: expect
           FETCH = 1/2 of the bytes)
  rand4    4-byte gathers at 16M distinct random 128-B lines of a 4 GiB table
           (plus the int64 index stream); random narrow reads that miss L2 —
           k_proc's destination lookups
  rand4s   the same gathers confined to a 2 MiB table (k_proc's vertex table
           size): what L2 / Infinity-Cache residency leaves to the counter
tools/calib_summary.py turns the counters into bytes-per-access factors.
"""
import torch

torch.manual_seed(0)
dev = torch.device("cuda", 0)
M = 16 << 20
x = torch.ones(1 << 28, dtype=torch.float32, device=dev)           # 1 GiB
big = torch.ones(1 << 30, dtype=torch.float32, device=dev)         # 4 GiB
small = torch.ones(1 << 19, dtype=torch.float32, device=dev)       # 2 MiB
idx_big = (torch.randperm(1 << 25, device=dev)[:M] * 32).to(torch.int64)   # distinct 128-B lines
idx_small = torch.randint(0, 1 << 19, (M,), device=dev, dtype=torch.int64)
torch.cuda.synchronize()
for _ in range(3):
    s = x.sum()
for _ in range(3):
    g = big[idx_big]
for _ in range(3):
    h = small[idx_small]
torch.cuda.synchronize()
print("calib done", float(s), float(g[0]), float(h[0]), flush=True)
