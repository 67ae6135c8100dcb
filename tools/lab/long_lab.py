#!/usr/bin/env python3
"""Throughput of raw-range XXH3 (long-range kernel) and the manifest API (not part of the product)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import eloqstore_amd as pcs  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda._sleep(1_000_000)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3)
    return sorted(ts)[len(ts) // 2]


total = 4 << 30
buf = torch.empty(total, dtype=torch.uint8, device="cuda:0")
pcs.gen_pages(buf, 4096, total // 4096, 99, 0)
for chunk in (1 << 20, 64 << 10, 8 << 10):
    n = total // chunk
    off = torch.arange(n, dtype=torch.int64, device="cuda:0") * chunk
    ln = torch.full((n,), chunk, dtype=torch.int32, device="cuda:0")
    out = torch.empty(n, dtype=torch.int64, device="cuda:0")
    t = timeit(lambda: pcs.xxh3_64_ranges(buf, off, ln, n, out=out))
    print(f"raw XXH3 ranges of {chunk >> 10} KiB x {n}: {t*1e3:.3f} ms  {total / t / 1e9:.1f} GB/s", flush=True)
d_out = torch.empty(1, dtype=torch.int64, device="cuda:0")
for wide in (1, 0):
    pcs.set_tuning(pcs.TUNE_MANIFEST_WIDE, wide)
    for L in (64 << 10, 1 << 20, 4 << 20, 64 << 20, 256 << 20, 1 << 30, 4 << 30):
        t = timeit(lambda: pcs._call("pcs_manifest_checksum_dev", buf.data_ptr(), L, d_out.data_ptr(), pcs._stream(None)), 5)
        print(f"wide={wide} manifest checksum of {L >> 10} KiB: {t*1e6:9.1f} us  {L / t / 1e9:7.1f} GB/s", flush=True)
import time
content = bytes(np.random.default_rng(1).integers(0, 256, size=1 << 20, dtype=np.uint8))
pcs.set_tuning(pcs.TUNE_MANIFEST_WIDE, 1)
for L in (64 << 10, 1 << 20):
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        pcs.manifest_checksum_host(content[:L])
        ts.append(time.perf_counter() - t0)
    print(f"host API manifest checksum of {L >> 10} KiB: {sorted(ts)[25] * 1e6:.1f} us (H2D included)", flush=True)
