"""bench_gap_lab.py — does the driver's short bench (--steps 20 --warmup 5)
read lower than the default 400-step run on the same box, and is it the 0.1 s
idle gap bench.py leaves before the timed region?

Times config 2 (1 M x 4 KiB, XXH3 digest) the way bench.py's headline does
(barrier-free here: one rank), for K in {20, 400} steps after W = 5 warmup
launches, with an idle gap of 0 or 0.1 s between warmup and the timed region.
Cases run in a shuffled order per repetition.  Prints per-case medians of the
wall-clock rate (bench.py's `value`) and of the HIP-event launch average.

    python tools/lab/bench_gap_lab.py [reps]
"""
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))

import torch  # noqa: E402

import bench  # noqa: E402
import eloqstore_amd as pcs  # noqa: E402


def one(w, steps, warmup, gap):
    for _ in range(warmup):
        w.step("digest")
    torch.cuda.synchronize()
    if gap:
        time.sleep(gap)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        w.step("digest")
    ev1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    wall = w.bytes * steps / (t1 - t0) / bench.GIB
    ev = w.bytes * steps / (ev0.elapsed_time(ev1) / 1e3) / bench.GIB
    return wall, ev


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.cuda.set_device(0)
    if pcs.lib().pcs_set_device(0) != 0:
        raise SystemExit("pcs_set_device failed")
    w = bench.Workload(2, pcs.XXH3_64, 0, None, "cuda:0")
    cases = [(k, g) for k in (20, 400) for g in (0.0, 0.1)]
    res = {c: ([], []) for c in cases}
    rng = random.Random(5)
    for r in range(reps):
        order = cases[:]
        rng.shuffle(order)
        for c in order:
            wall, ev = one(w, c[0], 5, c[1])
            res[c][0].append(wall)
            res[c][1].append(ev)
        print(f"rep {r} done", flush=True)
        time.sleep(0.2)
    out = []
    for c in cases:
        wall, ev = res[c]
        out.append({"steps": c[0], "gap_s": c[1], "wall_GiBps_median": round(statistics.median(wall), 2),
                    "wall_min": round(min(wall), 2), "wall_max": round(max(wall), 2),
                    "event_GiBps_median": round(statistics.median(ev), 2)})
        print(f"steps {c[0]:4d} gap {c[1]:.1f}s: wall {statistics.median(wall):8.2f} GiB/s "
              f"(min {min(wall):8.2f} max {max(wall):8.2f})  event {statistics.median(ev):8.2f} GiB/s", flush=True)
    print("GAPLAB " + json.dumps(out))


if __name__ == "__main__":
    main()
