# Multi-line service: tests first, then the native-thread test's output,
# service_load with 1/2/4/8 lines against the gated single line, the crossover.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04c
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_service.py tests/test_gpu_integration.py > gpurun_out/r04c/service_tests.log 2>&1 &&
timeout -k 10 120 tests/cpp/service_threads_test > gpurun_out/r04c/service_threads.txt 2>&1 &&
timeout -k 10 400 tools/lab/service_load 0.5 g1L2L4L8 6,32 > gpurun_out/r04c/service_load_lines.txt 2>&1
echo "exit $?"
