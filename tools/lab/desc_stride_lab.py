"""Config 3 (1 M mixed 4/8/16 KiB pages, XXH3 descriptor digest): does the
packed address pattern or the size mix hold k_xxh3_desc under the
fixed-size kernels?

The same 1 M descriptors, same sizes in the same order, placed
  packed     offset = prefix sum of sizes (config 3 as bench.py runs it)
  stride16k  offset = i * 16 KiB (every page on its own 16 KiB slot; 4 and
             8 KiB pages leave a gap behind them)
  shuffled   16 KiB slots in a random order (the page order no longer follows
             the address order)
and, for the size mix alone, uniform pages packed (4, 8 and 16 KiB, the same
kernel).  Then the channel question: at a 16 KiB stride every group of a
wave reads the same 4 KiB sub-block offset of its page at the same step
(address bits 12-13 equal across the wave); at a 20 KiB stride (stride20k,
uniform16k_s20k) the page starts rotate through those bits.  Each layout: 5 rounds x 20 launches bracketed by HIP events, the
layouts interleaved round by round (A B C ... A B C ...), median round.
frac = (sum of page bytes + 8 B digest per page) / time / 8 TB/s.

    python tools/lab/desc_stride_lab.py [--n 1048576] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import eloqstore_amd as pcs  # noqa: E402
from workload import mixed_layout  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()
n = args.n
dev = "cuda:0"
seed = 0x5EED0003
_, lens, total = mixed_layout(seed, 0, n)
packed = np.zeros(n, dtype=np.uint64)
np.cumsum(lens[:-1], dtype=np.uint64, out=packed[1:])
stride = np.arange(n, dtype=np.uint64) * np.uint64(16384)
perm = np.random.default_rng(5).permutation(n).astype(np.uint64)
shuffled = perm * np.uint64(16384)

layouts = {}
arena_bytes = n * 20480
arena = torch.empty(arena_bytes, dtype=torch.uint8, device=dev)


def add(name, offs, ls):
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(ls.astype(np.uint32).view(np.int32)).to(dev)
    layouts[name] = (d_off, d_len, int(ls.astype(np.uint64).sum()) + 8 * n)


add("packed", packed, lens)
add("stride16k", stride, lens)
add("shuffled", shuffled, lens)
add("stride20k", np.arange(n, dtype=np.uint64) * np.uint64(20480), lens)
for P in (4096, 8192, 16384):
    ls = np.full(n, P, dtype=np.uint32)
    add(f"uniform{P // 1024}k", np.arange(n, dtype=np.uint64) * np.uint64(P), ls)
add("uniform16k_s20k", np.arange(n, dtype=np.uint64) * np.uint64(20480), np.full(n, 16384, dtype=np.uint32))
add("uniform8k_s12k", np.arange(n, dtype=np.uint64) * np.uint64(12288), np.full(n, 8192, dtype=np.uint32))
pcs.gen_pages(arena, 4096, arena_bytes // 4096, seed, 0)  # bytes only: every layout reads the same arena
out = torch.empty(n, dtype=torch.int64, device=dev)
torch.cuda.synchronize()

times = {k: [] for k in layouts}
for name, (o, l, _) in layouts.items():  # warm-up
    for _ in range(3):
        pcs.desc_digest(arena, o, l, n, pcs.XXH3_64, out=out)
torch.cuda.synchronize()
for r in range(args.rounds):
    for name, (o, l, _) in layouts.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            pcs.desc_digest(arena, o, l, n, pcs.XXH3_64, out=out)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 1e3 / args.steps)
print(f"{'layout':12s} {'bytes/launch':>14s} {'median us':>10s} {'TB/s':>6s} {'frac':>6s}  rounds(us)")
for name, (_, _, alg) in layouts.items():
    t = statistics.median(times[name])
    print(f"{name:12s} {alg:14d} {t * 1e6:10.1f} {alg / t / 1e12:6.3f} {alg / t / 8e12:6.4f}  "
          + " ".join(f"{x * 1e6:.1f}" for x in times[name]))
