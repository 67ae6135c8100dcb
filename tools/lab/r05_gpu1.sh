# Round 5, call 1: the service re-arm fix on hardware.  The new re-post and
# line-shrink tests plus the whole service test file (12 s soak included),
# then a 60 s soak on its own.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05a
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_service.py > gpurun_out/r05a/service_tests.log 2>&1 &&
timeout -k 10 150 tests/cpp/service_threads_test --soak 60 > gpurun_out/r05a/soak60.txt 2>&1
rc=$?
echo "exit $rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r05a/service_tests.log | tail -40; cat gpurun_out/r05a/soak60.txt
exit $rc
