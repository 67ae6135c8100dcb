# final-code check on one box: GPU suite, smoke, default bench line, rocprofv3 sweep
set -o pipefail; mkdir -p gpurun_out/final
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > gpurun_out/final/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err && \
bash tools/profile_sweep.sh r03i > gpurun_out/final/sweep.log 2>&1
echo rc=$?; tail -1 gpurun_out/final/gpu_tests.log
