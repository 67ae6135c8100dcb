#!/usr/bin/env python3
"""region_lab.py — on boxes where the 32 GiB config-5 batch reads at ~0.81 of
spec while 4 GiB batches read at ~0.92 (profiles/r02/drift_lab.txt,
blocksize_lab.txt), is the slowness in some REGION of the buffer (placement)
or in its SIZE (translation reach)?

Times k_xxh3_fixed<4096> (pcs_pages_digest_dev) over: the whole 32 GiB
buffer; each of its eight 4 GiB eighths; the first 4, 8, 16 GiB; and a
separately allocated 4 GiB buffer.  Medians of 7 interleaved rounds.

    python tools/lab/region_lab.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import eloqstore_amd as pcs  # noqa: E402

P = 4096
GI = 1 << 30


def main():
    torch.cuda.set_device(0)
    big = torch.empty(32 * GI, dtype=torch.uint8, device="cuda:0")
    small = torch.empty(4 * GI, dtype=torch.uint8, device="cuda:0")
    pcs.gen_pages(big, P, (32 * GI) // P, 0x5EED0005, 0)
    pcs.gen_pages(small, P, (4 * GI) // P, 0x5EED0002, 0)
    out = torch.empty((32 * GI) // P, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    base = big.data_ptr()
    views = [("whole 32 GiB", base, 32)]
    views += [(f"eighth {k} ({4 * k}-{4 * k + 4} GiB)", base + k * 4 * GI, 4) for k in range(8)]
    views += [("first 8 GiB", base, 8), ("first 16 GiB", base, 16), ("separate 4 GiB buffer", small.data_ptr(), 4)]
    res = {v[0]: [] for v in views}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(7):
        for name, ptr, gib in views:
            n = gib * GI // P
            pcs.pages_digest(ptr, P, n, 0, out=out)
            e0.record()
            for _ in range(5):
                pcs.pages_digest(ptr, P, n, 0, out=out)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 1e3 / 5
            res[name].append(n * (P + 8) / t / 8e12)
    print("# region                      frac of 8 TB/s (median of 7)   min    max")
    for name, fr in res.items():
        print(f"# {name:28s} {statistics.median(fr):.4f}                      {min(fr):.4f} {max(fr):.4f}")


if __name__ == "__main__":
    main()
