#!/usr/bin/env python3
"""drift_lab.py — does a sweep entry's launch time depend on what ran before it?

Round-2's sweep (profiles/r02a_sweep.json) put the same k_xxh3_fixed<4096>
kernel at 584.9 us as the headline and at ~601 us inside the later validate /
stamp entries.  This runs every sweep workload resident at once and times
them (bench.py's timed_launches: warmup + K launches bracketed by HIP events)
in a forward order, the reverse order and a repeat of config 2 between heavy
entries, so position effects show up as the same entry timing differently.

    python tools/lab/drift_lab.py [--steps 50] [--rounds 2]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--gap", type=float, default=0.1)
    args = ap.parse_args()
    dev = "cuda:0"
    torch.cuda.set_device(0)
    specs = {"c2": (2, 0), "c3x3": (3, 0), "c3x64": (3, 1), "c4": (4, 0), "c5": (5, 0), "c7": (7, 0)}
    wl = {}
    for k, (cfg, algo) in specs.items():
        if cfg == 3 and algo == 1:
            w = bench.Workload.__new__(bench.Workload)
            w.__dict__.update(wl["c3x3"].__dict__)
            w.algo = 1
            wl[k] = w
        else:
            wl[k] = bench.Workload(cfg, algo, 0, None, dev)
    wl["c2"].step("stamp")
    torch.cuda.synchronize()
    entries = [("c2", "digest"), ("c2", "validate"), ("c2", "stamp"), ("c3x3", "digest"), ("c3x64", "digest"),
               ("c4", "digest"), ("c5", "digest"), ("c7", "digest")]
    orders = {"forward": entries, "reverse": entries[::-1],
              "c2_between": [e for x in entries[3:] for e in (("c2", "digest"), x)] + [("c2", "digest")]}
    rows = []
    for r in range(args.rounds):
        for oname, order in orders.items():
            for pos, (k, mode) in enumerate(order):
                w = wl[k]
                if mode == "validate":
                    w.step("stamp")
                torch.cuda.synchronize()
                time.sleep(args.gap)
                avg = bench.timed_launches(w, mode, args.steps, args.warmup)
                frac = w.algorithmic_bytes(mode) / avg / 1e9 / bench.HBM_PEAK_GBPS
                row = {"round": r, "order": oname, "pos": pos, "entry": f"{k}:{mode}", "us": round(avg * 1e6, 1),
                       "frac": round(frac, 4)}
                rows.append(row)
                print(json.dumps(row), flush=True)
    # summary: per entry, min / median / max us over all positions
    import statistics
    print("# entry                 n    min_us    med_us    max_us   frac(med)")
    by = {}
    for row in rows:
        by.setdefault(row["entry"], []).append(row)
    for e, rs in by.items():
        us = sorted(x["us"] for x in rs)
        med = statistics.median(us)
        f = [x["frac"] for x in rs]
        print(f"# {e:20s} {len(us):3d} {us[0]:9.1f} {med:9.1f} {us[-1]:9.1f}   {statistics.median(f):.4f}")


if __name__ == "__main__":
    main()
