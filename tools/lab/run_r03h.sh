set -o pipefail; mkdir -p gpurun_out/r03h gpurun_out/lab1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > gpurun_out/r03h/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r03h/bench.json 2> gpurun_out/r03h/bench.err && \
timeout -k 10 180 python tools/lab/knob_ab.py 2 xxh64 digest 'eighths:25=0' 'c128:25=128' 'c256:25=256' 'c512:25=512' 'c1024:25=1024' > gpurun_out/lab1/x64_order_c2.txt 2>&1 && \
timeout -k 10 180 python tools/lab/knob_ab.py 3 xxh64 digest 'eighths:25=0' 'c128:25=128' 'c256:25=256' 'c512:25=512' 'c1024:25=1024' > gpurun_out/lab1/x64_order_c3.txt 2>&1 && \
timeout -k 10 180 python tools/lab/knob_ab.py 4 xxh64 digest 'eighths:25=0' 'c128:25=128' 'c256:25=256' 'c512:25=512' 'c1024:25=1024' > gpurun_out/lab1/x64_order_c4.txt 2>&1 && \
timeout -k 10 180 ./tools/lab/stream_lab 9 chunk > gpurun_out/lab1/stream_chunk.txt 2>&1
echo rc=$?; tail -2 gpurun_out/r03h/gpu_tests.log
