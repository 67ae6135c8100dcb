"""Per-launch fixed cost of the XXH3 page kernel: time vs batch size, fit
t = a + b * bytes (experiment harness, not part of the product)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import eloqstore_amd as pcs  # noqa: E402


def main():
    P = 4096
    nmax = 1 << 23
    pages = torch.empty(nmax * P, dtype=torch.uint8, device="cuda:0")
    pcs.gen_pages(pages, P, nmax, 0x5EED0005, 0)
    out = torch.empty(nmax, dtype=torch.int64, device="cuda:0")
    sizes = [1 << k for k in range(16, 24)]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for rnd in range(7):
        for n in sizes:
            torch.cuda._sleep(1_000_000)
            ev0.record()
            pcs.pages_digest(pages, P, n, out=out)
            ev1.record()
            torch.cuda.synchronize()
            res.setdefault(n, []).append(ev0.elapsed_time(ev1) * 1e3)
    xs, ys = [], []
    for n in sizes:
        t = sorted(res[n])[len(res[n]) // 2]
        xs.append(n * P)
        ys.append(t)
        print(f"{n:9d} pages {n * P / 2**30:6.2f} GiB  {t:9.1f} us  {n * P / t / 1e3:8.1f} GB/s", flush=True)
    b, a = np.polyfit(np.array(xs, dtype=float), np.array(ys), 1)
    print(f"fit: t = {a:.1f} us + bytes / {1e-3 / b:.1f} GB/s")


if __name__ == "__main__":
    main()
