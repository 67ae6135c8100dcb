#!/usr/bin/env python3
"""Interleaved in-process A/B of tuning knobs on a bench workload.

    python tools/lab/knob_ab.py CONFIG ALGO MODE 'label:key=val,key=val' ...

CONFIG is a bench.py config (2..7), ALGO xxh3|xxh64, MODE digest|validate|
stamp.  Every variant runs R rounds (env R, default 7) of K back-to-back
steps (env K, default 50) bracketed by HIP events, rounds interleaved (ABAB,
then BABA) so that drift hits every variant alike; digests are checked equal
across variants.  Prints the median per-step time and frac vs 8 TB/s."""
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


def parse(spec):
    label, _, kv = spec.partition(":")
    knobs = {}
    for item in filter(None, kv.split(",")):
        k, v = item.split("=")
        knobs[int(k)] = int(v)
    return label, knobs


def main():
    cfg, algo, mode = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    variants = [parse(s) for s in sys.argv[4:]]
    K, R = int(os.environ.get("K", "50")), int(os.environ.get("R", "7"))
    w = bench.Workload(cfg, pcs.XXH3_64 if algo == "xxh3" else pcs.XXH64, 0, None, "cuda:0")
    if mode == "validate":
        w.step("stamp")
    keys = sorted({k for _, kn in variants for k in kn})
    base = {k: pcs.get_tuning(k) for k in keys}
    times = {lab: [] for lab, _ in variants}
    ref = None
    for r in range(R):
        order = variants if r % 2 == 0 else variants[::-1]
        for lab, kn in order:
            for k in keys:
                pcs.set_tuning(k, kn.get(k, base[k]))
            times[lab].append(bench.timed_launches(w, mode, K, 3))
            if mode == "digest":
                d = w.out.cpu().numpy()
                if ref is None:
                    ref = d
                assert np.array_equal(d, ref), f"{lab}: digests differ"
    for k in keys:
        pcs.set_tuning(k, base[k])
    alg = w.algorithmic_bytes(mode)
    b0 = None
    for lab, _ in variants:
        m = statistics.median(times[lab])
        b0 = b0 or m
        print(f"config{cfg} {algo} {mode} {lab:24s} median {m * 1e6:9.1f} us  frac {alg / m / 8e12:.4f}  "
              f"vs first {b0 / m - 1:+.2%}  rounds {[round(x * 1e6, 1) for x in times[lab]]}", flush=True)


if __name__ == "__main__":
    main()
