#!/usr/bin/env python3
"""A/B of the validate call's first_bad forms in one process (config 2:
1 M x 4 KiB pages, XXH3, stamped): PCS_TUNE_FIRST_BAD 0 (fill launch in front,
round 2) vs 1 (leased self-resetting slot, written by the last block).  Each
form runs R rounds of K back-to-back validate calls bracketed by HIP events,
interleaved, and the medians per call are printed with the frac against the
8 TB/s spec (algorithmic bytes = n * (P + 1))."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import eloqstore_amd as pcs  # noqa: E402

P, n = 4096, 1 << 20
K, R = int(os.environ.get("K", "100")), int(os.environ.get("R", "7"))
buf = torch.empty(n * P, dtype=torch.uint8, device="cuda")
pcs.gen_pages(buf, P, n, 0x5EED0002, 0)
pcs.pages_stamp(buf, P, n)
ok = torch.empty(n, dtype=torch.uint8, device="cuda")
fb = torch.empty(1, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
res = {0: [], 1: []}
for r in range(R):
    for mode in (0, 1) if r % 2 == 0 else (1, 0):
        pcs.set_tuning(pcs.TUNE_FIRST_BAD, mode)
        for _ in range(5):
            pcs.pages_validate(buf, P, n, ok=ok, first_bad=fb)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            pcs.pages_validate(buf, P, n, ok=ok, first_bad=fb)
        e1.record()
        torch.cuda.synchronize()
        assert int(fb.item()) == -1 and bool(ok.all())
        res[mode].append(e0.elapsed_time(e1) / K * 1e3)
alg = n * (P + 1)
for mode, name in ((0, "fill launch (round 2)"), (1, "leased slot, last block writes")):
    m = statistics.median(res[mode])
    print(f"first_bad {mode} {name:32s} median {m:8.2f} us/call  frac {alg / (m * 1e-6) / 8e12:.4f}  "
          f"all {[round(x, 1) for x in res[mode]]}")
