#!/bin/bash
# tools/lab/pmc_x64.sh — why the XXH64 kernels sit below the read rate:
# issue/wait (SQ), reads in flight at L2 (TCC) and L1 latency (TCP) for the
# register-staged and direct-to-LDS XXH64 kernels (tools/lab/pmc_x64_probe.py).
# One rocprofv3 --pmc pass per block within gfx950's limits.  Not product.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_x64
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE \
    -d "$OUT/sq" -o sq --output-format csv -- python3 tools/lab/pmc_x64_probe.py
timeout -s KILL 120 rocprofv3 --pmc SQ_LEVEL_WAVES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_CYCLES GRBM_GUI_ACTIVE \
    -d "$OUT/sq2" -o sq2 --output-format csv -- python3 tools/lab/pmc_x64_probe.py
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum \
    -d "$OUT/tcc" -o tcc --output-format csv -- python3 tools/lab/pmc_x64_probe.py
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum \
    -d "$OUT/tcp" -o tcp --output-format csv -- python3 tools/lab/pmc_x64_probe.py
find "$OUT" -name "*counter_collection.csv"
