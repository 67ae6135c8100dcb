#!/bin/bash
# XXH64 direct-to-LDS ring (PCS_TUNE_XXH64_GLDS = 22) against the register-
# staged LDS kernel, in one process per config (tools/lab/knob_ab.py).
set -e
V="staged:22=0,15=4 glds2:22=2,15=4 glds3:22=3,15=4 glds4:22=4,15=4 glds2_w1:22=2,15=1 glds3_w2:22=3,15=2"
for cfg in 3 2 4; do
    timeout -k 10 300 python tools/lab/knob_ab.py $cfg xxh64 digest $V
done
