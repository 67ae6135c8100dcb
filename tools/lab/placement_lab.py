#!/usr/bin/env python3
"""Does config 3's rate depend on where its arena lands?  Not part of the product.

Config 3 (1 M mixed 4/8/16 KiB pages, 9.33 GiB arena) runs 1,400 us on some
boxes and 1,485 us on others with the same code, while config 2 runs the same
everywhere (tools/lab/slowbox_diag.sh).  Here one process builds config 3's
arena several times at different points of the device heap — first, after a
4 GiB and after a 16 GiB allocation, and twice side by side — and times the
kernel on each (digest, R rounds of K steps, interleaved), with the digests
compared across arenas.  The tile-order comparison of DESIGN.md §6a
(profiles/r03/placement_*.txt) ran this with a temporary tuning key that
selected the kernels' tile order; the key was removed with the chunked order
it chose.

    [ALGO=xxh64] python tools/lab/placement_lab.py [CONFIG]   (default 3)
"""
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import eloqstore_amd as pcs  # noqa: E402


def main():
    K, R = int(os.environ.get("K", "30")), int(os.environ.get("R", "5"))
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    algo = pcs.XXH64 if os.environ.get("ALGO") == "xxh64" else pcs.XXH3_64
    dev = "cuda:0"
    arenas = {}
    arenas["first"] = bench.Workload(cfg, algo, 0, None, dev)
    pad4 = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
    arenas["after_4G"] = bench.Workload(cfg, algo, 0, None, dev)
    pad16 = torch.empty(16 << 30, dtype=torch.uint8, device=dev)
    arenas["after_20G"] = bench.Workload(cfg, algo, 0, None, dev)
    arenas["next"] = bench.Workload(cfg, algo, 0, None, dev)
    for name, w in arenas.items():
        print(f"{name:10s} arena at {w.pages.data_ptr():#x}", flush=True)
    times = {a: [] for a in arenas}
    ref = None
    names = list(arenas)
    for r in range(R):
        for a in (names if r % 2 == 0 else names[::-1]):
            w = arenas[a]
            times[a].append(bench.timed_launches(w, "digest", K, 3))
            d = w.out.cpu().numpy()
            if ref is None:
                ref = d
            assert np.array_equal(d, ref), a
    for a in names:
        t = statistics.median(times[a])
        frac = arenas[a].algorithmic_bytes("digest") / t / 8e12
        print(f"config{cfg} {os.environ.get('ALGO', 'xxh3')} {a:10s} median {t * 1e6:8.1f} us  frac {frac:.4f}  rounds "
              f"{[round(x * 1e6, 1) for x in times[a]]}", flush=True)
    del pad4, pad16


if __name__ == "__main__":
    main()
