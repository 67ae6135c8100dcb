#!/bin/bash
# tools/lab/slowbox_diag.sh — classify the box (config 2 and config 3 digest
# and validate timed in one process, tools/lab/mode_ab.py) and record the
# memory-side and address-translation counters of the same kernels
# (tools/lab/pmc_probe2.py), one rocprofv3 --pmc pass per hardware block
# within gfx950's limits.  Config 3 runs 1,400 us on some boxes and 1,490 on
# others with the same code; this puts both kinds of box on record.  Not part
# of the product.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-diag}
OUT=gpurun_out/slowbox_${TAG}
mkdir -p "$OUT"
R=3 K=30 timeout -k 10 200 python3 tools/lab/mode_ab.py 2 3 > "$OUT/mode_ab.txt" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum \
    -d "$OUT/tcc" -o tcc --output-format csv -- python3 tools/lab/pmc_probe2.py > "$OUT/tcc.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum \
    -d "$OUT/tcp" -o tcp --output-format csv -- python3 tools/lab/pmc_probe2.py > "$OUT/tcp.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE \
    -d "$OUT/grbm" -o grbm --output-format csv -- python3 tools/lab/pmc_probe2.py > "$OUT/grbm.log" 2>&1
find "$OUT" -name "*counter_collection.csv"
