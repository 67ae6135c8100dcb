#!/usr/bin/env python3
"""sweep_alloc_lab.py — why do bench sweep entries time 3-5 % below the same
kernels in the in-process labs?

The sweep (bench.py, round 2 first version) allocated each entry's buffer,
timed it, freed it and emptied torch's cache before the next entry, so every
entry ran on memory just handed back by the previous (up to 32 GiB) one.  The
labs allocate once.  This times every sweep entry three ways in one process:
  A  headline-style: the config-2 buffer allocated first thing and kept;
  B  the sweep's churn: allocate, time, free + empty_cache, next entry;
  C  all entries allocated up front, kept resident, timed in turn;
and repeats B and C once more, so position and allocation history separate.

    python tools/lab/sweep_alloc_lab.py [--steps 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

ENTRIES = [("c3x3", 3, 0, "digest"), ("c3x64", 3, 1, "digest"), ("c4", 4, 0, "digest"), ("c5", 5, 0, "digest"),
           ("c7", 7, 0, "digest"), ("c2v", 2, 0, "validate"), ("c2s", 2, 0, "stamp")]


def timed(w, mode, steps):
    if mode == "validate":
        w.step("stamp")
    torch.cuda.synchronize()
    time.sleep(0.1)
    t = bench.timed_launches(w, mode, steps, 5)
    return t, w.algorithmic_bytes(mode) / t / 1e9 / bench.HBM_PEAK_GBPS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    dev = "cuda:0"
    torch.cuda.set_device(0)
    head = bench.Workload(2, 0, 0, None, dev)
    rows = []

    def rec(phase, key, t, f):
        r = {"phase": phase, "entry": key, "us": round(t * 1e6, 1), "frac": round(f, 4)}
        rows.append(r)
        print(json.dumps(r), flush=True)

    rec("A", "c2d", *timed(head, "digest", 400))
    for rep in range(2):
        for key, cfg, algo, mode in ENTRIES:  # B: the churn
            w = bench.Workload(cfg, algo, 0, None, dev)
            rec(f"B{rep}", key, *timed(w, mode, args.steps))
            w.free()
            del w
            torch.cuda.empty_cache()
        wl = {}
        for key, cfg, algo, mode in ENTRIES:  # C: all resident
            wl[key] = bench.Workload(cfg, algo, 0, None, dev)
        for key, cfg, algo, mode in ENTRIES:
            rec(f"C{rep}", key, *timed(wl[key], mode, args.steps))
        for w in wl.values():
            w.free()
        del wl
        torch.cuda.empty_cache()
        rec(f"A{rep}", "c2d", *timed(head, "digest", 400))
    print("# entry   " + "  ".join(f"{p:>7s}" for p in ("B0", "C0", "B1", "C1")))
    for key, *_ in ENTRIES:
        vals = {r["phase"]: r["frac"] for r in rows if r["entry"] == key}
        print(f"# {key:7s} " + "  ".join(f"{vals.get(p, 0):7.4f}" for p in ("B0", "C0", "B1", "C1")))
    print("# headline c2 digest: " + " ".join(f"{r['phase']} {r['frac']:.4f}" for r in rows if r["entry"] == "c2d"))


if __name__ == "__main__":
    main()
