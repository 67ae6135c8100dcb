#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/<tag>_pmc.json.

HBM bytes per launch of the bench's hot kernel from the rocprofv3 PMC passes,
corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950:
  read  = FETCH_SIZE (KiB) * 1024 * 2   (FETCH_SIZE reports exactly half of a
                                          wide coalesced streaming read)
  write = WRITE_SIZE (KiB) * 1024       (exact for wide streaming stores)
plus the kernel-trace average duration, so bench.py can put `traffic` on its
line and the judge can cross-check the live HIP-event timing.

    python tools/summarize_profile.py gpurun_out/prof_r01 r01 [config_key]
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(pattern):
    out = []
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            out.extend(csv.DictReader(f))
    return out


# the dominant page kernel of each bench workload (the descriptor paths also
# launch a small generic pass over the descriptors; it is not counted here)
HOT = ("k_xxh3_fixed<", "k_xxh3_split<", "k_xxh3_desc<", "k_xxh64_lds<", "k_xxh64_stride<")


def hot(name: str) -> bool:
    return any(h in name for h in HOT)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    key = sys.argv[3] if len(sys.argv) > 3 else "config2_xxh3"
    fetch = [r for r in rows(os.path.join(src, "fetch", "**", "*counter_collection.csv")) if hot(r["Kernel_Name"])]
    write = [r for r in rows(os.path.join(src, "write", "**", "*counter_collection.csv")) if hot(r["Kernel_Name"])]
    stats = [r for r in rows(os.path.join(src, "trace", "**", "*kernel_stats.csv")) if hot(r["Name"])]
    if not fetch or not write:
        sys.exit("no PMC rows for the hot kernel")
    # the timed kernel is the most frequent one (the bench's untimed drills
    # launch other modes of the same templates a few times)
    kname = statistics.mode(r["Kernel_Name"] for r in fetch)
    fetch = [r for r in fetch if r["Kernel_Name"] == kname]
    write = [r for r in write if r["Kernel_Name"] == kname]
    stats = [s for s in stats if s["Name"] == kname]
    rd = statistics.median(float(r["Counter_Value"]) for r in fetch) * 1024 * 2
    wr = statistics.median(float(r["Counter_Value"]) for r in write) * 1024
    bench = {}
    bj = os.path.join(src, "bench_trace.json")
    if os.path.exists(bj):
        with open(bj) as f:
            bench = json.loads(f.read().strip().splitlines()[-1])
    alg = bench.get("roofline", {}).get("algorithmic_bytes_per_launch")
    out = {
        "tag": tag,
        "kernel": kname,
        "how": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes (tools/profile_round.sh); "
               "read = FETCH_SIZE*1024*2 (gfx950 half-count correction), write = WRITE_SIZE*1024; median over launches",
        "fetch_size_kib_median": rd / 2048,
        "write_size_kib_median": wr / 1024,
        "hbm_read_bytes_per_launch": round(rd),
        "hbm_write_bytes_per_launch": round(wr),
        "traffic_bytes_per_launch": {key: round(rd + wr)},
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (rd + wr) / alg if alg else None,
        "kernel_trace": [{k: s[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs")} for s in stats],
        "bench_line_during_trace": bench,
    }
    dst = os.path.join(ROOT, "profiles", f"{tag}_pmc.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", dst, json.dumps(out["traffic_bytes_per_launch"]), out["traffic_over_algorithmic"])


if __name__ == "__main__":
    main()
