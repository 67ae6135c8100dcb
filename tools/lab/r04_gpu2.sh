# Round-4 service measurements: crossover with the async-service column,
# service_load with the contention gate, the native-thread service test's
# output, then the CU-mask lab (last: the one that may stall; it has its own
# watchdog and exits 3 on a stall).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 tests/cpp/service_threads_test > gpurun_out/r04_service_threads.txt 2>&1 &&
timeout -k 10 300 tests/cpp/integration_snippets --crossover > gpurun_out/r04_crossover.txt 2>&1 &&
timeout -k 10 200 tools/lab/service_load 0.5 s1g1 6,32,128 > gpurun_out/r04_service_load.txt 2>&1 &&
timeout -k 10 60 tools/lab/cumask_lab 4 > gpurun_out/r04_cumask_lab.txt 2> gpurun_out/r04_cumask_lab.err
echo "exit $?"
