#!/usr/bin/env python3
"""Validate throughput on all-valid vs all-corrupt batches (not part of the product)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import eloqstore_amd as pcs  # noqa: E402

P, n = 4096, 1 << 20
pages = torch.empty(n * P, dtype=torch.uint8, device="cuda:0")
pcs.gen_pages(pages, P, n, 7, 0)
ok = torch.empty(n, dtype=torch.uint8, device="cuda:0")
fb = torch.empty(1, dtype=torch.int64, device="cuda:0")


def t(fn, reps=10):
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
        ts.append(a.elapsed_time(b))
    return sorted(ts)[reps // 2]


for algo in (pcs.XXH3_64, pcs.XXH64):
    ms_bad = t(lambda: pcs.pages_validate(pages, P, n, algo, ok=ok, first_bad=fb))
    assert int(fb.item()) == 0 and int(ok.sum()) == 0
    pcs.pages_stamp(pages, P, n, algo)
    ms_good = t(lambda: pcs.pages_validate(pages, P, n, algo, ok=ok, first_bad=fb))
    assert int(ok.sum()) == n
    print(f"algo {algo}: all-corrupt {n*P/ms_bad/1e6:.0f} GB/s, all-valid {n*P/ms_good/1e6:.0f} GB/s")
    pcs.gen_pages(pages, P, n, 7, 0)
