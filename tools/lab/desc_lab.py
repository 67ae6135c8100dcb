#!/usr/bin/env python3
"""desc_lab.py — in-process A/B of a tuning knob (default:  the XXH3 descriptor kernels on config 3)
(1 M mixed 4/8/16 KiB pages, 9.33 GiB): one group per page in 16-page tiles
(k_xxh3_desc, PCS_TUNE_XXH3_DESC_WAVE_LIST = 0) against pages dealt to a
wave's groups as they free up (k_xxh3_desc_wave, lists of 16/32/64 pages).
Every variant must give the same digests and verdicts; rounds interleave the
variants so box drift hits them alike.

    python tools/lab/desc_lab.py [--rounds 7] [--steps 20] [--modes digest,validate]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import eloqstore_amd as pcs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lists", default="0,16,32,64")
    ap.add_argument("--modes", default="digest,validate")
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--knob", type=int, default=16, help="tuning key to A/B (default PCS_TUNE_XXH3_DESC_WAVE_LIST)")
    ap.add_argument("--algo", type=int, default=0)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    w = bench.Workload(args.config, args.algo, 0, None, "cuda:0")
    lists = [int(x) for x in args.lists.split(",")]
    modes = args.modes.split(",")
    saved = pcs.get_tuning(args.knob)
    w.step("stamp")
    torch.cuda.synchronize()
    ref = None
    for lst in lists:  # parity across variants (digests and verdicts)
        pcs.set_tuning(args.knob, lst)
        w.step("digest")
        w.step("validate")
        torch.cuda.synchronize()
        cur = (w.out.clone(), w.ok.clone(), int(w.fb.item()))
        if ref is None:
            ref = cur
        same = torch.equal(cur[0], ref[0]) and torch.equal(cur[1], ref[1]) and cur[2] == ref[2]
        print(f"# list {lst:3d}: digests/verdicts {'identical' if same else 'DIFFER'}; "
              f"all valid {bool(cur[1].all().item())}, first_bad {cur[2]}", flush=True)
        if not same:
            sys.exit(1)
    res = {}
    for r in range(args.rounds):
        for mode in modes:
            for lst in lists:
                pcs.set_tuning(args.knob, lst)
                t = bench.timed_launches(w, mode, args.steps, 3)
                res.setdefault((mode, lst), []).append(t)
                frac = w.algorithmic_bytes(mode) / t / 1e9 / bench.HBM_PEAK_GBPS
                print(f"round {r} {mode:8s} list {lst:3d}: {t * 1e6:8.1f} us  frac {frac:.4f}", flush=True)
    pcs.set_tuning(args.knob, saved)
    print(f"# knob {args.knob}, algo {args.algo}, config {args.config}, {w.n} pages, {w.bytes / 2**30:.2f} GiB; medians over {args.rounds} rounds")
    print("# mode      list     med_us   TB/s    frac")
    for (mode, lst), ts in res.items():
        m = statistics.median(ts)
        a = w.algorithmic_bytes(mode) / m
        print(f"# {mode:8s} {lst:5d} {m * 1e6:10.1f} {a / 1e12:6.3f} {a / 1e9 / bench.HBM_PEAK_GBPS:7.4f}")


if __name__ == "__main__":
    main()
