#!/usr/bin/env python3
"""degrade_lab.py — which step of a bench sweep slows a buffer that is never
touched by it?

tools/lab/sweep_alloc_lab.py: the config-2 buffer allocated first timed 0.925
of spec, then 0.893 after the sweep's allocate / run / free / empty_cache
phases, on the same buffer; tools/lab/cooldown_lab.py rules out heat.  Here
the config-2 digest (50 launches, 3 repeats) is timed after each candidate
step in turn, in one process, and once more in a second, fresh process.

    python tools/lab/degrade_lab.py [--child]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    child = "--child" in sys.argv
    dev = "cuda:0"
    torch.cuda.set_device(0)
    c2 = bench.Workload(2, 0, 0, None, dev)

    def meas(tag):
        fr = []
        for _ in range(3):
            t = bench.timed_launches(c2, "digest", 50, 3)
            fr.append(c2.algorithmic_bytes() / t / 1e9 / bench.HBM_PEAK_GBPS)
        print(json.dumps({"proc": "child" if child else "parent", "after": tag,
                          "frac": [round(x, 4) for x in fr]}), flush=True)

    meas("start")
    if child:
        return
    x = torch.empty(32 << 30, dtype=torch.uint8, device=dev)  # allocate, never touched
    meas("alloc 32 GiB (untouched)")
    x.fill_(1)
    torch.cuda.synchronize()
    meas("fill 32 GiB")
    del x
    meas("del (kept in torch cache)")
    torch.cuda.empty_cache()
    meas("empty_cache (hipFree 32 GiB)")
    w = bench.Workload(5, 0, 0, None, dev)
    for _ in range(50):
        w.step("digest")
    torch.cuda.synchronize()
    meas("config 5 workload + 50 digests (resident)")
    w.free()
    del w
    torch.cuda.empty_cache()
    meas("config 5 freed + empty_cache")
    for cfg in (3, 4, 7):
        w = bench.Workload(cfg, 0, 0, None, dev)
        for _ in range(20):
            w.step("digest")
        torch.cuda.synchronize()
        w.free()
        del w
        torch.cuda.empty_cache()
    meas("configs 3, 4, 7: alloc, 20 digests, free, empty_cache")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout.strip(), flush=True)
    meas("after the child process")


if __name__ == "__main__":
    main()
