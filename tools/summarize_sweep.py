#!/usr/bin/env python3
"""Summarise tools/profile_sweep.sh into profiles/<tag>_sweep.json.

Per bench entry (the headline line and every `sweep` entry of the default
N=1 bench.py run):
  * kernel trace (rocprofv3 --kernel-trace, per-dispatch CSV): the timed loop
    of each entry is one contiguous segment of dispatches (bench.py sleeps
    PHASE_GAP_S between phases; segments split on idle gaps > 20 ms).  For
    every kernel launched at least `steps` times in that segment: calls,
    median / mean / min / max duration.  The entry's profile launch time is
    the sum of those medians (config 3 launches a descriptor pre-pass per
    step; stamp launches the digest pass and the header scatter).
  * frac_profile = algorithmic bytes per launch / profile launch time / 8 TB/s,
    next to the bench's live frac (HIP events bracketing the timed steps);
    `agree_within_2pct` compares them.
  * HBM traffic from the PMC passes (FETCH_SIZE and WRITE_SIZE in separate
    runs), corrected as MI355X_MICROARCH.md prescribes for gfx950:
    read = FETCH_SIZE (KiB) * 1024 * 2, write = WRITE_SIZE (KiB) * 1024; median
    over the dispatches of each (kernel, grid), summed over the entry's kernels.

    python tools/summarize_sweep.py gpurun_out/prof_r02 r02
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8000.0  # GB/s
GAP_NS = 20_000_000


def rows(pattern):
    out = []
    for path in sorted(glob.glob(pattern, recursive=True)):
        with open(path) as f:
            out.extend(csv.DictReader(f))
    return out


def kname(r):
    n = r["Kernel_Name"]
    return n[5:] if n.startswith("void ") else n


def grid(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r.get("Grid_Size_X", 0)) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)


def segments(trace):
    trace = sorted(trace, key=lambda r: int(r["Start_Timestamp"]))
    segs, cur, last_end = [], [], None
    for r in trace:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur and s - last_end > GAP_NS:
            segs.append(cur)
            cur = []
        cur.append(r)
        last_end = e if last_end is None else max(last_end, e)
    if cur:
        segs.append(cur)
    return segs


def seg_kernels(seg, min_calls):
    by = {}
    for r in seg:
        by.setdefault((kname(r), grid(r)), []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = []
    for (name, g), d in by.items():
        if len(d) >= min_calls:
            out.append({"kernel": name, "grid": g, "calls": len(d), "median_ns": statistics.median(d),
                        "mean_ns": round(statistics.fmean(d), 1), "min_ns": min(d), "max_ns": max(d)})
    return out


def pmc_medians(path_glob):
    by = {}
    for r in rows(path_glob):
        by.setdefault((kname(r), grid(r)), []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in by.items()}


def pmc_by_counter(path_glob):
    by = {}
    for r in rows(path_glob):
        by.setdefault((kname(r), grid(r)), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in by.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    with open(os.path.join(src, "bench_trace.json")) as f:
        bench = json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])
    trace = rows(os.path.join(src, "trace", "**", "*kernel_trace.csv"))
    fetch = pmc_medians(os.path.join(src, "fetch", "**", "*counter_collection.csv"))
    write = pmc_medians(os.path.join(src, "write", "**", "*counter_collection.csv"))
    utcl = pmc_by_counter(os.path.join(src, "utcl", "**", "*counter_collection.csv"))
    segs = segments(trace)

    wanted = [{"key": "headline", "steps": bench["steps"], "frac": bench["roofline"]["frac"],
               "avg_launch_ms": bench["roofline"]["avg_launch_ms"],
               "alg": bench["roofline"]["algorithmic_bytes_per_launch"]}]
    for e in bench.get("sweep") or []:
        wanted.append({"key": e["key"], "steps": e["steps"], "frac": e["frac"], "avg_launch_ms": e["avg_launch_ms"],
                       "alg": e["algorithmic_bytes_per_launch"]})
    # Round 6 bench phases: the `cold` run (W + K launches) precedes the
    # headline's settle + warmup + timed segment, and the ceiling A/B
    # (k_stream_read beside the hash kernel) follows it.  The headline takes
    # the first segment with settle + K launches of a kernel; segments that
    # hold k_stream_read are skipped.
    settle_steps = (bench.get("settle") or {}).get("steps", 0) if bench.get("cold") else 0
    entries, si = [], 0
    for w in wanted:
        ks = []
        need = w["steps"] + (settle_steps if w["key"] == "headline" else 0)
        while si < len(segs):
            seg = segs[si]
            si += 1
            if any("k_stream_read" in kname(r) for r in seg):
                continue
            ks = seg_kernels(seg, need)
            if ks:
                break
        if not ks:
            entries.append({"key": w["key"], "error": "no timed segment found"})
            continue
        t_ns = sum(k["median_ns"] for k in ks)
        frac_p = w["alg"] / (t_ns * 1e-9) / 1e9 / PEAK
        rd = sum(fetch.get((k["kernel"], k["grid"]), float("nan")) for k in ks) * 1024 * 2
        wr = sum(write.get((k["kernel"], k["grid"]), float("nan")) for k in ks) * 1024
        traffic = rd + wr
        tr = {}
        for k in ks:
            for c, v in utcl.get((k["kernel"], k["grid"]), {}).items():
                tr[c] = tr.get(c, 0.0) + v
        if tr.get("TCP_UTCL1_REQUEST_sum"):
            tr["translation_miss_per_request"] = round(tr.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0.0)
                                                       / tr["TCP_UTCL1_REQUEST_sum"], 6)
            tr["translation_miss_per_MiB"] = round(tr.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0.0)
                                                   / (w["alg"] / 2**20), 3)
        entries.append({
            "key": w["key"], "kernels": ks, "profile_launch_ms": round(t_ns / 1e6, 4),
            "bench_avg_launch_ms": w["avg_launch_ms"], "algorithmic_bytes_per_launch": w["alg"],
            "frac_profile": round(frac_p, 4), "frac_bench": w["frac"],
            "frac_ratio": round(w["frac"] / frac_p, 4),
            "agree_within_2pct": abs(w["frac"] / frac_p - 1) <= 0.02,
            "hbm_read_bytes_per_launch": None if rd != rd else round(rd),
            "hbm_write_bytes_per_launch": None if wr != wr else round(wr),
            "traffic_bytes_per_launch": None if traffic != traffic else round(traffic),
            "traffic_over_algorithmic": None if traffic != traffic else round(traffic / w["alg"], 6),
            "utcl1_per_launch": tr or None,
        })
    out = {
        "tag": tag,
        "how": "tools/profile_sweep.sh: rocprofv3 --kernel-trace over the default bench run (headline + sweep), "
               "then --pmc FETCH_SIZE, --pmc WRITE_SIZE and --pmc TCP_UTCL1_* (address translation) in separate "
               "short runs; segments split on >20 ms idle "
               "gaps; per entry the kernels launched >= steps times in its timed segment; launch time = sum of "
               "their median durations; read = FETCH_SIZE*1024*2 (gfx950 half-count), write = WRITE_SIZE*1024",
        "entries": entries,
        "bench_line_during_trace": bench,
    }
    dst = os.path.join(ROOT, "profiles", f"{tag}_sweep.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for e in entries:
        print(f"{e['key']:24s} prof {e.get('profile_launch_ms')} ms  frac_prof {e.get('frac_profile')}  "
              f"bench {e.get('frac_bench')}  agree {e.get('agree_within_2pct')}  "
              f"traffic/alg {e.get('traffic_over_algorithmic')}  "
              f"utcl1 miss/MiB {(e.get('utcl1_per_launch') or {}).get('translation_miss_per_MiB')}")
    print("wrote", dst)


if __name__ == "__main__":
    main()
