#!/bin/bash
# tools/lab/pmc_valu.sh — issue-side PMC counters for the config-2 page kernels
# (XXH3, XXH64, read ceiling; tools/lab/pmc_probe.py).  Not part of the product.
# One pass: 7 SQ + 1 GRBM counters (gfx950 allows 8 SQ, 2 GRBM per pass).
# Each name is checked against `rocprofv3 -L` first, so an unknown counter
# stops the script instead of reaching the profiler.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_valu
mkdir -p "$OUT"
CTRS="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
for c in $CTRS; do
    grep -qw "$c" "$OUT/avail.txt" || { echo "counter $c not listed by rocprofv3 -L"; exit 3; }
done
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d "$OUT" -o valu --output-format csv -- python3 tools/lab/pmc_probe.py
find "$OUT" -name "*counter_collection.csv"
