export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_first_bad.py tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_integration.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/lab/first_bad_lab.py > gpurun_out/r03c_first_bad_lab.txt 2>&1 || exit 1
timeout -k 10 200 python tools/lab/knob_ab.py 3 xxh3 digest 'vector:24=0' 'scalar:24=1' > gpurun_out/r03c_ab.txt 2>&1 || exit 1
timeout -k 10 200 python tools/lab/knob_ab.py 3 xxh3 validate 'vector:24=0' 'scalar:24=1' >> gpurun_out/r03c_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/lab/knob_ab.py 5 xxh3 digest 'whole:23=0' 'win16G:23=262144' 'win4G:23=65536' 'win1G:23=16384' 'win256M:23=4096' >> gpurun_out/r03c_ab.txt 2>&1 || exit 1
timeout -k 10 200 python tools/lab/knob_ab.py 2 xxh3 digest 'whole:23=0' 'win1G:23=16384' 'win256M:23=4096' >> gpurun_out/r03c_ab.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03c_prof -o validate --output-format csv -- python3 bench.py --mode validate --steps 100 --warmup 5 --no-sweep --no-cpu-baseline > gpurun_out/r03c_validate.json 2>gpurun_out/r03c_validate.err
