#!/usr/bin/env python3
"""Known-byte calibration run for rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950.

crdt_vv_max_async over two 512 MiB u64 arrays (8 B per lane, the width of the
join kernel's key/counter streams): algorithmic reads 1 GiB, writes 512 MiB per
launch.  tools/traffic.py divides the counters by these to get the correction.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-crdt-playground_amd"))
import torch  # noqa: E402

import crdtgpu  # noqa: E402

N = 64 << 20  # u64 elements = 512 MiB per array
a = torch.randint(0, 1 << 62, (N,), dtype=torch.int64, device="cuda")
b = torch.randint(0, 1 << 62, (N,), dtype=torch.int64, device="cuda")
eng = crdtgpu.Engine(0)
for _ in range(4):
    eng.vv_max_async(a, b, N)
eng.sync()
print("calib: vv_max_kernel reads %d B writes %d B per launch" % (16 * N, 8 * N))
