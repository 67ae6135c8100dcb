"""x64_depth3_lab.py — XXH64 LDS kernel: segments in flight per step (DEPTH)
1, 2 (default), 3 and 4 on config 3 (1 M mixed 4/8/16 KiB pages) and config 2,
selected with PCS_TUNE_XXH64_LAYOUT (2/3/5/4).  One process, the depths in a
shuffled order per repetition, 20 launches each bracketed by HIP events; every
depth's digests are checked against the default's.

    python tools/lab/x64_depth3_lab.py [reps]
"""
import os
import random
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))

import torch  # noqa: E402

import bench  # noqa: E402
import eloqstore_amd as pcs  # noqa: E402

DEPTH_KEY = {1: 2, 2: 3, 3: 5, 4: 4}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.cuda.set_device(0)
    if pcs.lib().pcs_set_device(0) != 0:
        raise SystemExit("pcs_set_device failed")
    rng = random.Random(3)
    for cfg in (3, 2):
        w = bench.Workload(cfg, pcs.XXH64, 0, None, "cuda:0")
        pcs.set_tuning(pcs.TUNE_XXH64_LAYOUT, 0)
        w.step("digest")
        torch.cuda.synchronize()
        ref = w.out.clone()
        bench.settle(w, "digest", 1000)
        res = {d: [] for d in DEPTH_KEY}
        for _ in range(reps):
            order = list(DEPTH_KEY)
            rng.shuffle(order)
            for d in order:
                pcs.set_tuning(pcs.TUNE_XXH64_LAYOUT, DEPTH_KEY[d])
                for _ in range(3):
                    w.step("digest")
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    w.step("digest")
                e1.record()
                torch.cuda.synchronize()
                res[d].append(e0.elapsed_time(e1) / 20)
                assert torch.equal(w.out, ref), f"depth {d} digests differ"
        pcs.set_tuning(pcs.TUNE_XXH64_LAYOUT, 0)
        alg = w.algorithmic_bytes("digest")
        base = statistics.median(res[2])
        for d in DEPTH_KEY:
            m = statistics.median(res[d])
            print(f"config {cfg} XXH64 depth {d}: median {m * 1e3:8.1f} us  frac {alg / (m * 1e-3) / 8e12:.4f}  "
                  f"vs depth 2 {base / m - 1:+.2%}  (min {min(res[d]) * 1e3:.1f}, max {max(res[d]) * 1e3:.1f})",
                  flush=True)
        w.free()
        del w


if __name__ == "__main__":
    main()
