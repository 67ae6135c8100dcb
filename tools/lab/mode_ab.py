#!/usr/bin/env python3
"""Digest against validate on the same resident batch, interleaved in one
process.  Not part of the product.

    python tools/lab/mode_ab.py CONFIG [CONFIG ...]

Both modes read the same bytes; digest writes 8 bytes per page (the digest
array), validate 1 byte (the verdicts) plus the first-bad word.  A box where
digest runs measurably slower than validate is paying for the result writes.
Every variant runs R rounds (env R, default 7) of K back-to-back steps (env K,
default 50) bracketed by HIP events, ABAB then BABA.  Prints the median
per-step time and frac vs 8 TB/s (algorithmic bytes of each mode)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import eloqstore_amd as pcs  # noqa: E402


def main():
    K, R = int(os.environ.get("K", "50")), int(os.environ.get("R", "7"))
    for cfg in (int(c) for c in sys.argv[1:]):
        w = bench.Workload(cfg, pcs.XXH3_64, 0, None, "cuda:0")
        w.step("stamp")
        modes = ["digest", "validate"]
        times = {m: [] for m in modes}
        for r in range(R):
            for m in (modes if r % 2 == 0 else modes[::-1]):
                times[m].append(bench.timed_launches(w, m, K, 3))
        for m in modes:
            t = statistics.median(times[m])
            frac = w.algorithmic_bytes(m) / t / 8e12
            print(f"config{cfg} {m:9s} median {t * 1e6:9.1f} us  frac {frac:.4f}  rounds "
                  f"{[round(x * 1e6, 1) for x in times[m]]}", flush=True)
        del w


if __name__ == "__main__":
    main()
