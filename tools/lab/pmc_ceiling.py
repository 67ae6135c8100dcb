#!/usr/bin/env python3
"""Kernels for tools/lab/pmc_ceiling.sh, not part of the product: the
headline hash kernel (k_xxh3_fixed<4096>, config 2) and the streaming-read
ceiling (k_stream_read, same buffer), 4 launches each, interleaved."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import eloqstore_amd as pcs  # noqa: E402

torch.cuda.set_device(0)
w2 = bench.Workload(2, 0, 0, None, "cuda:0")
scratch = torch.empty(w2.bytes // 4096, dtype=torch.int64, device="cuda:0")
for _ in range(4):
    w2.step("digest")
    pcs.stream_read(w2.pages, w2.bytes, scratch)
torch.cuda.synchronize()
print("ok")
