#!/bin/bash
# tools/profile_sweep.sh <tag> — rocprofv3 evidence for every bench entry.
# Run on the GPU box from the repo root.  Writes gpurun_out/prof_<tag>/:
#   trace/  kernel trace + stats of the default N=1 bench run (headline + sweep)
#   fetch/  --pmc FETCH_SIZE over a short run of the same entries
#   write/  --pmc WRITE_SIZE over a short run (separate pass: gfx950 PMC slots)
#   utcl/   --pmc UTCL1 address-translation counters (requests, hits, misses,
#           multi-miss stalls) over the same short run: every box's record
#           says whether large buffers (config 5, 32 GiB) miss in translation
#           more than config 2's 4 GiB (VERDICT r02 Next #6)
# Summarised by tools/summarize_sweep.py into profiles/<tag>_sweep.json.
set -euo pipefail
TAG=${1:-r02}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
# (host-inclusive legs off: PCIe-bound, measured in the bench line itself)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-live-traffic --no-host-inclusive > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
SHORT="--steps 5 --warmup 2 --sweep-steps 5 --sweep-warmup 1 --no-cpu-baseline --no-live-traffic --no-host-inclusive"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- \
    python3 bench.py $SHORT > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- \
    python3 bench.py $SHORT > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum \
    -d "$OUT/utcl" -o utcl --output-format csv -- \
    python3 bench.py $SHORT > "$OUT/bench_utcl.json" 2> "$OUT/bench_utcl.err"
find "$OUT" -name "*.csv" | sort
