# Driver-style bench (--steps 20 --warmup 5) with and without the settle
# phase, alternating (order reversed per cycle), then one default run.
# Output: gpurun_out/settle/
set -o pipefail
mkdir -p gpurun_out/settle
O="--steps 20 --warmup 5 --no-sweep --no-cpu-baseline --no-live-traffic"
for i in 1 2 3; do
  if [ $((i % 2)) = 1 ]; then order="0 200"; else order="200 0"; fi
  for s in $order; do
    timeout -k 10 200 python bench.py $O --settle-ms $s > gpurun_out/settle/b20_s${s}_$i.json 2>/dev/null || exit 1
  done
done
timeout -k 10 200 python bench.py --no-sweep --no-cpu-baseline --no-live-traffic > gpurun_out/settle/b400.json 2>/dev/null
