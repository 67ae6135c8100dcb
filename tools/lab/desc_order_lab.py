#!/usr/bin/env python3
"""Does the ORDER in which a mixed-size descriptor batch is walked matter?

Config 3 (1 M pages of 4/8/16 KiB packed in random order): the product walks
the descriptors in the caller's order, so every 16-page group of a wave holds
mixed sizes and walks its longest page.  Here the same pages (same arena,
same bytes) are handed to the unchanged C ABI (pcs_desc_digest_dev) with the
descriptor arrays permuted: sorted by length descending (longest first, so
the launch's last round of workgroups is short-lived), ascending, and grouped
into size-homogeneous 64-page tiles in the original tile order.  Kernel time
only (the permutation is built outside the clock): an upper bound on what a
device-side binning pass could gain before paying for itself.  Digests are
un-permuted and checked against the caller-order run.  Interleaved rounds,
medians (env R, K)."""
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import eloqstore_amd as pcs  # noqa: E402

K, R = int(os.environ.get("K", "20")), int(os.environ.get("R", "5"))
w = bench.Workload(3, pcs.XXH3_64, 0, None, "cuda:0")
lens = w.lens.astype(np.int64)
n = w.n
orders = {
    "caller": np.arange(n),
    "desc": np.argsort(-lens, kind="stable"),
    "asc": np.argsort(lens, kind="stable"),
}
# size-homogeneous 64-page tiles, tiles interleaved in round-robin over sizes
by = [np.flatnonzero(lens == L) for L in sorted(set(lens.tolist()), reverse=True)]
tiles = [b[i:i + 64] for b in by for i in range(0, len(b), 64)]
orders["tiles_desc"] = np.concatenate(tiles)
variants = {}
for name, perm in orders.items():
    p = torch.from_numpy(perm.astype(np.int64)).to("cuda:0")
    variants[name] = (p, w.d_off[p].contiguous(), w.d_len[p].contiguous())
out = torch.empty(n, dtype=torch.int64, device="cuda:0")
alg = w.algorithmic_bytes("digest")
for algo in (pcs.XXH64, pcs.XXH3_64):
    ref = None
    times = {k: [] for k in variants}
    for r in range(R):
        for name in (list(variants) if r % 2 == 0 else list(variants)[::-1]):
            p, off, ln = variants[name]
            for _ in range(3):
                pcs.desc_digest(w.pages, off, ln, n, algo, out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                pcs.desc_digest(w.pages, off, ln, n, algo, out=out)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / K * 1e3)
            got = torch.empty_like(out)
            got[p] = out
            if ref is None:
                ref = got.clone()
            assert torch.equal(got, ref), f"{name}: digests differ"
    base = statistics.median(times["caller"])
    for name in variants:
        m = statistics.median(times[name])
        print(f"{'xxh64' if algo else 'xxh3'} {name:10s} median {m:8.1f} us  frac {alg / (m * 1e-6) / 8e12:.4f}  "
              f"vs caller {base / m - 1:+.2%}  rounds {[round(x, 1) for x in times[name]]}", flush=True)
