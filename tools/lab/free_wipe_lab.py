"""free_wipe_lab.py — is the GPU slower for a while after another process
frees a lot of HBM (a driver-side wipe or clear of the freed memory)?

    python tools/lab/free_wipe_lab.py hog GIB     allocate and fill GIB GiB, exit
    python tools/lab/free_wipe_lab.py probe SECS  config-2 workload (1 M x 4 KiB
        XXH3 digests): batches of 8 steps, each timed with HIP events, for
        SECS seconds from the first batch; prints a time series of the
        per-step time, the device's free memory (hipMemGetInfo) and a summary (first 200 ms, 0.2-1 s, the rest)

tools/lab/r05_wipe.sh runs: probe alone; hog 80 GiB then probe at once; hog
then 5 s of sleep then probe.
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))

import torch  # noqa: E402


def hog(gib: float):
    bufs = []
    left = int(gib * (1 << 30))
    while left > 0:
        b = min(left, 8 << 30)
        t = torch.empty(b, dtype=torch.uint8, device="cuda:0")
        t.fill_(0x5A)
        bufs.append(t)
        left -= b
    torch.cuda.synchronize()
    print(f"hog: {gib} GiB allocated and filled", flush=True)


def probe(secs: float):
    import bench
    import eloqstore_amd as pcs
    t_proc = time.perf_counter()
    if pcs.lib().pcs_set_device(0) != 0:
        raise SystemExit("pcs_set_device failed")
    w = bench.Workload(2, pcs.XXH3_64, 0, None, "cuda:0")
    t_ready = time.perf_counter()
    series = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(8):
            w.step("digest")
        e1.record()
        torch.cuda.synchronize()
        free = torch.cuda.mem_get_info(0)[0]
        series.append(((time.perf_counter() - t0) * 1e3, e0.elapsed_time(e1) * 1e3 / 8, free))
    print(f"probe: workload ready {t_ready - t_proc:.2f} s after start; {len(series)} batches", flush=True)
    for t, us, free in series[:12] + series[12::25]:
        print(f"  t={t:8.1f} ms  {us:7.1f} us/step  free {free / 2**30:8.2f} GiB", flush=True)
    best = min(us for _, us, _ in series)

    def seg(a, b):
        v = [us for t, us, _ in series if a <= t < b]
        return (statistics.median(v), max(v), len(v)) if v else (float("nan"), float("nan"), 0)

    for a, b in ((0, 200), (200, 1000), (1000, 1e9)):
        m, mx, k = seg(a, b)
        print(f"SEG {a:>5}-{'end' if b > 1e8 else int(b):>5} ms: median {m:7.1f} us/step ({m / best:.4f} x best), "
              f"max {mx:7.1f}, {k} batches", flush=True)


def series_of(w, secs):
    out, t0 = [], time.perf_counter()
    while time.perf_counter() - t0 < secs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(8):
            w.step("digest")
        e1.record()
        torch.cuda.synchronize()
        out.append(((time.perf_counter() - t0) * 1e3, e0.elapsed_time(e1) * 1e3 / 8))
    return out


def probe2(secs: float):
    """Is the slow phase tied to the process or to fresh allocations?  One
    process: batch A for `secs`, then a freshly allocated batch B for `secs`,
    then A again; per phase the median step time in 0-200 ms, 0.2-1 s and
    the rest."""
    import bench
    import eloqstore_amd as pcs
    if pcs.lib().pcs_set_device(0) != 0:
        raise SystemExit("pcs_set_device failed")
    a = bench.Workload(2, pcs.XXH3_64, 0, None, "cuda:0")
    phases = [("A", series_of(a, secs))]
    b = bench.Workload(2, pcs.XXH3_64, 0, None, "cuda:0")
    phases.append(("B fresh", series_of(b, secs)))
    phases.append(("A again", series_of(a, secs)))
    best = min(us for _, s in phases for _, us in s)
    for name, s in phases:
        segs = []
        for lo, hi in ((0, 200), (200, 1000), (1000, 1e9)):
            v = [us for t, us in s if lo <= t < hi]
            segs.append(f"{statistics.median(v):7.1f}" if v else "      -")
        print(f"PHASE {name:8s} median us/step 0-200 ms {segs[0]}, 0.2-1 s {segs[1]}, rest {segs[2]} "
              f"(best {best:.1f})", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "hog":
        hog(float(sys.argv[2]))
    elif sys.argv[1] == "probe2":
        probe2(float(sys.argv[2]))
    else:
        probe(float(sys.argv[2]))
