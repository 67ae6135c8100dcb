# Round-5 full check on one box: GPU suite, smoke, default bench line (live
# PMC traffic leg, config 1 with the all-cores in-memory leg), native-thread
# service test + 60 s soak, crossover (shuffled columns + controls), then the
# rocprofv3 sweep.  usage: bash tools/lab/run_r05_full.sh <tag> [nosuite]
set -o pipefail
TAG=${1:-r05e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "${2:-}" != "nosuite" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > "$OUT/smoke.log" 2>&1 || { rc=$?; echo "rc=$rc"; tail -5 "$OUT/gpu_tests.log"; exit $rc; }
fi
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 120 tests/cpp/service_threads_test > "$OUT/service_threads.txt" 2>&1 && \
timeout -k 10 150 tests/cpp/service_threads_test --soak 60 > "$OUT/soak60.txt" 2>&1 && \
timeout -k 10 400 tests/cpp/integration_snippets --crossover > "$OUT/crossover.txt" 2>&1 && \
bash tools/profile_sweep.sh "$TAG" > "$OUT/sweep.log" 2>&1
rc=$?
echo "rc=$rc"; tail -1 "$OUT/gpu_tests.log" 2>/dev/null
exit $rc
