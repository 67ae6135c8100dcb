#!/usr/bin/env python3
"""Per-kernel timing of the manifest checksum forms (run under rocprofv3 --kernel-trace).  Not part of the product."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import eloqstore_amd as pcs  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
buf = torch.empty(L, dtype=torch.uint8, device="cuda:0")
pcs.gen_pages(buf, 4096, L // 4096, 99, 0)
d_out = torch.empty(1, dtype=torch.int64, device="cuda:0")
for wide in (2, 0):
    pcs.set_tuning(pcs.TUNE_MANIFEST_WIDE, wide)
    for _ in range(5):
        pcs._call("pcs_manifest_checksum_dev", buf.data_ptr(), L, d_out.data_ptr(), pcs._stream(None))
torch.cuda.synchronize()
print("ok")
