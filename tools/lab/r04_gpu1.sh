set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_service.py tests/test_gpu_integration.py "tests/test_gpu_parity.py::test_batch_api_beside_page_cpp_in_any_link_order" "tests/test_gpu_parity.py::test_cpp_dropin_program" > gpurun_out/r04_t1.log 2>&1
