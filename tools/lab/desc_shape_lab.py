#!/usr/bin/env python3
"""desc_shape_lab.py — where does config 3 lose against fixed-size pages?
(not part of the product)

Times the descriptor entry point (pcs_desc_digest_dev: k_xxh3_desc + the
generic pass) over one 9.33 GiB arena laid out several ways, all packed:
  uniform 4 / 8 / 16 KiB pages           (the descriptor kernel without mixing)
  config 3                                (sizes drawn per page, BASELINE order)
  config 3, tile-homogeneous              (the same sizes regrouped so every 16
                                           consecutive pages share one size;
                                           tiles of different sizes interleave)
  config 3, window-sorted (W pages)       (sizes sorted inside windows of W pages)
  config 3, sorted                        (all 4 KiB, then 8, then 16: 3 runs)
and the fixed-size kernels on the uniform layouts for reference.  Rounds
interleave the layouts; medians.

    python tools/lab/desc_shape_lab.py [--rounds 5] [--algo 0]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import eloqstore_amd as pcs  # noqa: E402
from workload import mixed_sizes  # noqa: E402

N3 = 1 << 20
SEED3 = 0x5EED0003


def packed(lens):
    offs = np.zeros(len(lens), dtype=np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    return offs, lens.astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--algo", type=int, default=0)
    ap.add_argument("--knob", type=int, default=None, help="tuning key to sweep per layout")
    ap.add_argument("--values", default="0")
    ap.add_argument("--layouts", default=None, help="comma-separated layout name prefixes to keep")
    args = ap.parse_args()
    values = [int(v) for v in args.values.split(",")] if args.knob is not None else [None]
    torch.cuda.set_device(0)
    lens3 = mixed_sizes(SEED3, 0, N3).astype(np.uint64)
    total = int(lens3.sum())
    arena = torch.empty(total, dtype=torch.uint8, device="cuda:0")
    pcs.gen_pages(arena, 4096, total // 4096, 0x5EED0006, 0)  # content only
    layouts = {}
    for P in (4096, 8192, 16384):
        n = total // P
        layouts[f"uniform {P // 1024:2d} KiB"] = packed(np.full(n, P, dtype=np.uint64))
    layouts["config 3"] = packed(lens3)
    # tile-homogeneous: the same multiset of sizes, 16 equal sizes per tile,
    # tiles in a seeded random order
    rng = np.random.default_rng(3)
    srt = np.sort(lens3)
    tiles = srt[: (len(srt) // 16) * 16].reshape(-1, 16)
    tiles = tiles[rng.permutation(len(tiles))]
    layouts["config 3 tile-homog."] = packed(np.concatenate([tiles.reshape(-1), srt[len(tiles) * 16:]]))
    for W in (64, 256, 4096):
        w = lens3[: (N3 // W) * W].reshape(-1, W)
        layouts[f"config 3 sorted in {W}"] = packed(np.sort(w, axis=1).reshape(-1))
    layouts["config 3 sorted"] = packed(srt)
    if args.layouts:
        keep = [k.strip() for k in args.layouts.split(",")]
        layouts = {k: v for k, v in layouts.items() if any(k.startswith(p) for p in keep)}
    dev = {}
    for name, (offs, lens) in layouts.items():
        assert int(offs[-1]) + int(lens[-1]) <= total
        dev[name] = (torch.from_numpy(offs.view(np.int64)).to("cuda:0"),
                     torch.from_numpy(lens.view(np.int32)).to("cuda:0"), len(lens), int(lens.astype(np.uint64).sum()))
    out = torch.empty(max(v[2] for v in dev.values()), dtype=torch.int64, device="cuda:0")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        fn()
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / args.steps

    res = {}
    for r in range(args.rounds):
        for name, (d_off, d_len, n, nbytes) in dev.items():
            for v in values:
                if v is not None:
                    pcs.set_tuning(args.knob, v)
                t = timed(lambda: pcs.desc_digest(arena, d_off, d_len, n, args.algo, out=out))
                key = name if v is None else f"{name} [{args.knob}={v}]"
                res.setdefault(key, []).append((nbytes + 8 * n) / t / 8e12)
            if args.knob is not None:
                pcs.set_tuning(args.knob, values[0])
        for P in (4096, 16384):
            n = total // P
            t = timed(lambda: pcs.pages_digest(arena, P, n, args.algo, out=out))
            res.setdefault(f"fixed kernel {P // 1024:2d} KiB", []).append(n * (P + 8) / t / 8e12)
        print(f"round {r}: " + "  ".join(f"{k} {v[-1]:.4f}" for k, v in res.items()), flush=True)
    print(f"# algo {args.algo}, {total / 2**30:.2f} GiB arena; frac of 8 TB/s, median of {args.rounds}")
    for k, v in res.items():
        print(f"# {k:28s} {statistics.median(v):.4f}   (min {min(v):.4f} max {max(v):.4f})")


if __name__ == "__main__":
    main()
