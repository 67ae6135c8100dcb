# Short (driver: --steps 20 --warmup 5) vs default bench on one box, plus
# bench_gap_lab.py (idle gap before the timed region).  Output: gpurun_out/gap/
set -o pipefail
mkdir -p gpurun_out/gap
timeout -k 10 300 python -u tools/lab/bench_gap_lab.py 10 > gpurun_out/gap/gap.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-sweep --no-cpu-baseline --no-live-traffic > gpurun_out/gap/b20_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --no-sweep --no-cpu-baseline --no-live-traffic > gpurun_out/gap/b400_$i.json 2>/dev/null || exit 1
done
