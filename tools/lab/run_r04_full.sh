# Round-4 full check on one box: GPU suite, smoke, default bench line (with
# its live PMC traffic leg), native-thread service test, crossover, then the
# rocprofv3 sweep.  usage: bash tools/lab/run_r04_full.sh <tag>
set -o pipefail
TAG=${1:-r04e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 120 tests/cpp/service_threads_test > "$OUT/service_threads.txt" 2>&1 && \
timeout -k 10 300 tests/cpp/integration_snippets --crossover > "$OUT/crossover.txt" 2>&1 && \
bash tools/profile_sweep.sh "$TAG" > "$OUT/sweep.log" 2>&1
rc=$?
echo "rc=$rc"; tail -1 "$OUT/gpu_tests.log"
exit $rc
