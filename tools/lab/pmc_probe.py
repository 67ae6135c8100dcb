#!/usr/bin/env python3
"""Run each hot kernel a few times for rocprofv3 --pmc passes (not part of the product)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import eloqstore_amd as pcs  # noqa: E402

P, n = 4096, 1 << 20
pages = torch.empty(n * P, dtype=torch.uint8, device="cuda:0")
pcs.gen_pages(pages, P, n, 0x5EED0002, 0)
out = torch.empty(n, dtype=torch.int64, device="cuda:0")
for _ in range(3):
    pcs.pages_digest(pages, P, n, pcs.XXH3_64, out=out)
    pcs.pages_digest(pages, P, n, pcs.XXH64, out=out)
    pcs.stream_read(pages, n * P, out)
torch.cuda.synchronize()
print("ok")
