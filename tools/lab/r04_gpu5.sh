# XXH64 equal-byte runs (PCS_TUNE_XXH64_RUNS): parity first, then an
# interleaved A/B against k_xxh64_lds on config 3 (digest, validate, stamp),
# runs at depths 1 / 2 / 4 (PCS_TUNE_XXH64_LAYOUT 2 / 0 / 4).
# Result: profiles/r04/x64_runs_ab.txt (runs 18-28 % slower); the kernel and
# key 29 were retired after it (commit 473b0b4), so this reruns only at 9196877.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04g
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_variants.py -k "mixed or leftovers" > gpurun_out/r04g/variants.log 2>&1 &&
timeout -k 10 300 python tools/lab/knob_ab.py 3 xxh64 digest 'lds:' 'runs:29=1' 'runs_d1:29=1,6=2' 'runs_d4:29=1,6=4' > gpurun_out/r04g/ab_c3_digest.txt 2>&1 &&
timeout -k 10 200 python tools/lab/knob_ab.py 3 xxh64 validate 'lds:' 'runs:29=1' > gpurun_out/r04g/ab_c3_validate.txt 2>&1
echo "exit $?"
