#!/bin/bash
# tools/lab/pmc_ceiling.sh — the headline hash kernel against the
# streaming-read ceiling on the memory side ("if the ceiling
# cannot be made higher than the hash kernel, say why with counters").  One
# rocprofv3 --pmc pass per block within gfx950's limits.  Not part of the product.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ceiling
mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 tools/lab/pmc_ceiling.py
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum \
    -d "$OUT/tcc" -o tcc --output-format csv -- python3 tools/lab/pmc_ceiling.py
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
    -d "$OUT/sq" -o sq --output-format csv -- python3 tools/lab/pmc_ceiling.py
find "$OUT" -name "*.csv"
