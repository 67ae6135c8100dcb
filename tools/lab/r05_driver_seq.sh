# The driver's round-end order, back to back on one box: GPU suite, smoke(),
# then bench.py with the driver's arguments (twice), timing each step.
# Output: gpurun_out/dseq/
set -o pipefail
mkdir -p gpurun_out/dseq
D=gpurun_out/dseq
s=$(date +%s.%N)
timeout -k 10 700 python -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || exit 1
t1=$(date +%s.%N)
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
t2=$(date +%s.%N)
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_1.json 2> $D/bench_1.err || exit 1
t3=$(date +%s.%N)
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_2.json 2> $D/bench_2.err || exit 1
t4=$(date +%s.%N)
python3 -c "print('suite %.1f s, smoke %.1f s, bench %.1f s, bench %.1f s' % ($t1-$s, $t2-$t1, $t3-$t2, $t4-$t3))" > $D/times.txt
