#!/usr/bin/env python3
"""stride_lab.py — does the page stride matter at a fixed page size?  Not part of the product.

Uniform pages of P bytes described by descriptors (pcs_desc_digest_dev) and
laid out at a stride of P (power-of-two aligned, the normal case) or P + pad
bytes (page starts spread over the low address bits).  Same kernels, same
bytes hashed; only where the pages sit differs.  Interleaved rounds, K
launches back to back per sample.

    python tools/lab/stride_lab.py [--sizes 4096,16384,65536] [--pads 0,256,4096]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import eloqstore_amd as pcs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,16384,65536")
    ap.add_argument("--pads", default="0,256,4096")
    ap.add_argument("--algos", default="xxh64,xxh3")
    ap.add_argument("--bytes", type=int, default=4 << 30)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--k", type=int, default=5)
    args = ap.parse_args()
    dev = "cuda:0"
    for P in [int(x) for x in args.sizes.split(",")]:
        n = args.bytes // P
        out = torch.empty(n, dtype=torch.int64, device=dev)
        vs = []
        for pad in [int(x) for x in args.pads.split(",")]:
            stride = P + pad
            base = torch.empty(n * stride, dtype=torch.uint8, device=dev)
            off = torch.arange(n, dtype=torch.int64, device=dev) * stride
            ln = torch.full((n,), P, dtype=torch.int32, device=dev)
            pcs.gen_desc(base, off, ln, n, 0x5EED0007, 0)
            for algo_name in args.algos.split(","):
                algo = pcs.XXH3_64 if algo_name == "xxh3" else pcs.XXH64
                vs.append((f"P={P} stride=P+{pad} {algo_name}", base, off, ln, algo))
        ref = {}
        for name, base, off, ln, algo in vs:  # same page contents at every stride
            pcs.desc_digest(base, off, ln, n, algo, out=out)
            torch.cuda.synchronize()
            d = out.clone()
            assert torch.equal(ref.setdefault(algo, d), d), name
        times = {v[0]: [] for v in vs}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.rounds):
            for name, base, off, ln, algo in vs:
                torch.cuda.synchronize()
                e0.record()
                for _k in range(args.k):
                    pcs.desc_digest(base, off, ln, n, algo, out=out)
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / args.k)
        for name, t in times.items():
            t = sorted(t)
            print(f"  {name:32s} med {t[len(t) // 2]:8.4f} ms  {n * P / t[len(t) // 2] / 1e6:8.1f} GB/s", flush=True)
        del vs, times
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
