#!/bin/bash
# tools/lab/pmc_latency.sh — memory-side latency / queueing counters for the
# config-2, config-3, 16 KiB and stream-read kernels (tools/lab/pmc_probe2.py),
# one rocprofv3 --pmc pass per hardware block within gfx950's limits
# (4 TCC, 8 SQ + GRBM, 4 TCP).  Not part of the product.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_latency
mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum \
    -d "$OUT/tcc" -o tcc --output-format csv -- python3 tools/lab/pmc_probe2.py
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE \
    -d "$OUT/sq" -o sq --output-format csv -- python3 tools/lab/pmc_probe2.py
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum \
    -d "$OUT/tcp" -o tcp --output-format csv -- python3 tools/lab/pmc_probe2.py
find "$OUT" -name "*counter_collection.csv"
