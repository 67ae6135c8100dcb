#!/usr/bin/env python3
"""odd_size_lab.py — rate of the fixed-size page entry points at page sizes
off the fast kernels' shapes (not part of the product).

EloqStore's `data_page_size` is any uint16_t the options file parses
(kv_options.h:185, kv_options.cpp:272-277); the fast XXH3 kernels take
P % 256 == 0 on a 16-byte-aligned base, the XXH64 LDS kernel P % 64 == 0.
Everything else goes to the generic lanes.  This times ~2 GiB batches of each
size (and a 4 KiB batch at an 8-byte-misaligned base) for both hashes.

    python tools/lab/odd_size_lab.py [--gib 2] [--rounds 3]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import eloqstore_amd as pcs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--sizes", default="4096,6144,4352,4160,4104,4000,5000,8000,16000,4095")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    nbytes = args.gib << 30
    buf = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda:0")
    out = torch.empty(nbytes // 4000 + 1, dtype=torch.int64, device="cuda:0")
    cases = [(int(P), 0) for P in args.sizes.split(",")] + [(4096, 8)]
    pcs.gen_pages(buf, 4096, nbytes // 4096, 0x5EED0006, 0)  # content only; any page size reads it
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for r in range(args.rounds):
        for P, shift in cases:
            n = nbytes // P
            ptr = buf.data_ptr() + shift
            for algo in (pcs.XXH3_64, pcs.XXH64):
                pcs.pages_digest(ptr, P, n, algo, out=out)
                e0.record()
                for _ in range(args.steps):
                    pcs.pages_digest(ptr, P, n, algo, out=out)
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 1e3 / args.steps
                res.setdefault((P, shift, algo), []).append(n * (P + 8) / t / 1e12)
                print(f"round {r} P {P:6d} base+{shift} {'xxh3 ' if algo == 0 else 'xxh64'} {res[(P, shift, algo)][-1]:7.3f} TB/s",
                      flush=True)
    print("# page size  base  xxh3 TB/s  xxh64 TB/s   (median)")
    for P, shift in cases:
        a = statistics.median(res[(P, shift, pcs.XXH3_64)])
        b = statistics.median(res[(P, shift, pcs.XXH64)])
        print(f"# {P:9d}  +{shift:<3d} {a:9.3f}  {b:9.3f}")


if __name__ == "__main__":
    main()
