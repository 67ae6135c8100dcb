#!/usr/bin/env python3
"""XXH64 kernels for rocprofv3 --pmc passes (not part of the product): config 3
(1 M mixed 4/8/16 KiB descriptor pages) and config 2 (1 M x 4 KiB), each with
the register-staged LDS kernel (k_xxh64_lds) and the direct-to-LDS ring
(k_xxh64_glds, PCS_TUNE_XXH64_GLDS = 2 on config 3, 3 on config 2), three
launches each; the kernel name tells the two apart in the counter CSV."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import eloqstore_amd as pcs  # noqa: E402

for cfg, depth in ((3, 2), (2, 3)):
    w = bench.Workload(cfg, pcs.XXH64, 0, None, "cuda:0")
    for d in (0, depth):
        pcs.set_tuning(pcs.TUNE_XXH64_GLDS, d)
        for _ in range(3):
            w.step("digest")
        torch.cuda.synchronize()
    pcs.set_tuning(pcs.TUNE_XXH64_GLDS, 0)
    w.free()
    del w
print("ok")
