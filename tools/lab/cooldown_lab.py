#!/usr/bin/env python3
"""cooldown_lab.py — does the part slow down under sustained load and recover
when idle?

tools/lab/sweep_alloc_lab.py timed the SAME config-2 buffer at 0.925 of the
HBM spec first thing in the process and at 0.892 after ~20 s of sweep
entries.  This heats the part with back-to-back config-5 digests (32 GiB) for
a few seconds, then times the config-2 digest (50 launches) after idle gaps
of 0 .. 8 s, twice, and reads temperature / power / clocks with amd-smi
between measurements (when the tool works on the box).

    python tools/lab/cooldown_lab.py
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def smi():
    try:
        r = subprocess.run(["amd-smi", "metric", "-g", "0", "-t", "-p", "-c", "--json"], capture_output=True,
                           text=True, timeout=20)
        d = json.loads(r.stdout)
        g = d[0] if isinstance(d, list) else d
        g = g.get("gpu_data", [g])[0] if isinstance(g, dict) and "gpu_data" in g else g
        t = g.get("temperature", {})
        p = g.get("power", {})
        c = g.get("clock", {})

        def val(x):
            return x.get("value") if isinstance(x, dict) else x
        return {"hotspot_C": val(t.get("hotspot")), "mem_C": val(t.get("mem")), "power_W": val(p.get("socket_power")),
                "gfx_MHz": val((c.get("gfx_0") or {}).get("clk")), "mem_MHz": val((c.get("mem_0") or {}).get("clk"))}
    except Exception as e:  # noqa: BLE001 - diagnostics only
        return {"smi": f"unavailable: {type(e).__name__}"}


def main():
    dev = "cuda:0"
    torch.cuda.set_device(0)
    c2 = bench.Workload(2, 0, 0, None, dev)
    c5 = bench.Workload(5, 0, 0, None, dev)

    def meas(tag):
        t = bench.timed_launches(c2, "digest", 50, 3)
        f = c2.algorithmic_bytes() / t / 1e9 / bench.HBM_PEAK_GBPS
        r = {"tag": tag, "us": round(t * 1e6, 1), "frac": round(f, 4), **smi()}
        print(json.dumps(r), flush=True)
        return f

    def heat(seconds):
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < seconds:
            for _ in range(20):
                c5.step("digest")
            torch.cuda.synchronize()
            k += 20
        return k

    time.sleep(5)
    meas("cold (after 5 s idle)")
    for rep, secs in enumerate((5, 15)):
        n = heat(secs)
        print(f"# heated {secs} s: {n} config-5 launches ({n * 32 / secs:.0f} GiB/s)", flush=True)
        meas(f"heat{rep} +0 s")
        for gap in (0.5, 1, 2, 4, 8):
            time.sleep(gap)
            meas(f"heat{rep} +{gap} s idle")


if __name__ == "__main__":
    main()
