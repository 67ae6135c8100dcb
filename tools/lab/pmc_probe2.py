#!/usr/bin/env python3
"""Kernels for the round-2 latency PMC passes (tools/lab/pmc_latency.sh), not
part of the product: config 2 (k_xxh3_fixed<4096>), config 3 (k_xxh3_desc),
16 KiB pages (k_xxh3_split<16384>) and the plain streaming read, 3 launches
each, same buffers throughout."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import eloqstore_amd as pcs  # noqa: E402

torch.cuda.set_device(0)
w2 = bench.Workload(2, 0, 0, None, "cuda:0")
w3 = bench.Workload(3, 0, 0, None, "cuda:0")
w7 = bench.Workload(7, 0, 0, None, "cuda:0")
scratch = torch.empty(1 << 20, dtype=torch.int64, device="cuda:0")
for _ in range(3):
    w2.step("digest")
    w3.step("digest")
    w7.step("digest")
    pcs.stream_read(w2.pages, w2.bytes, scratch)
torch.cuda.synchronize()
print("ok")
