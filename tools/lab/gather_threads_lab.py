#!/usr/bin/env python3
"""Gather threads of the host pipeline (PCS_GATHER_THREADS, read once per
process).  Not part of the product.  1 GiB of 4 KiB pages: pageable
contiguous and scattered (a random permutation), through
pcs_pages_digest_host (gather into pinned staging -> H2D -> kernel -> D2H),
digests checked against the device run.  Run once per thread count:
  PCS_GATHER_THREADS=8 python tools/lab/gather_threads_lab.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import eloqstore_amd as pcs  # noqa: E402

P, n = 4096, 1 << 18
dev = torch.empty(n * P, dtype=torch.uint8, device="cuda:0")
pcs.gen_pages(dev, P, n, 0x5EED0002, 0)
want = pcs.pages_digest(dev, P, n).cpu().numpy().view(np.uint64)
host = dev.cpu().numpy()
perm = np.random.default_rng(7).permutation(n).astype(np.uint64)
out = np.empty(n, dtype=np.uint64)
res = {}
for name, idx in (("contiguous", np.arange(n, dtype=np.uint64)), ("scattered", perm)):
    ptrs = idx * np.uint64(P) + np.uint64(host.ctypes.data)
    fn = pcs.lib().pcs_pages_digest_host
    assert fn(ptrs.ctypes.data, P, n, 0, out.ctypes.data) == 0
    assert np.array_equal(out, want[idx.astype(np.int64)])
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or time.perf_counter() - t0 < 2.0:
        fn(ptrs.ctypes.data, P, n, 0, out.ctypes.data)
        reps += 1
    res[name] = n * P / ((time.perf_counter() - t0) / reps) / 2**30
print(f"gather threads {os.environ.get('PCS_GATHER_THREADS', 'default')}: "
      + "  ".join(f"{k} {v:.2f} GiB/s" for k, v in res.items()), flush=True)
