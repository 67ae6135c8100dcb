# Service soak (tests/cpp/service_threads_test --soak): a 60 s run, then the
# service test file with its 12 s soak.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04i
timeout -k 10 150 tests/cpp/service_threads_test --soak 60 > gpurun_out/r04i/soak60.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_service.py > gpurun_out/r04i/service_tests.log 2>&1
rc=$?
echo "exit $rc"; cat gpurun_out/r04i/soak60.txt; tail -2 gpurun_out/r04i/service_tests.log
exit $rc
