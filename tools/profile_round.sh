#!/bin/bash
# tools/profile_round.sh <tag> — rocprofv3 evidence for the bench's hot kernel.
# Run on the GPU box from the repo root.  Writes gpurun_out/prof_<tag>/:
#   kernel-trace + stats of a bench run, and separate PMC passes for HBM
#   read/write bytes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950,
#   MI355X_MICROARCH.md §rocprofv3 PMC slots).  Summarised by
#   tools/summarize_profile.py into profiles/.
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- \
    python3 bench.py ${PMC_ARGS:-} --steps 5 --warmup 2 --no-cpu-baseline --no-live-traffic > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- \
    python3 bench.py ${PMC_ARGS:-} --steps 5 --warmup 2 --no-cpu-baseline --no-live-traffic > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
find "$OUT" -name "*.csv" | sort
