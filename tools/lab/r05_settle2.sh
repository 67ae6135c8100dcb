# Driver-style bench (--steps 20 --warmup 5) right after a process that
# filled and freed 80 GiB, with the settle phase at 200 ms and at 1500 ms
# (the default), alternating, order reversed per cycle.  Output: gpurun_out/settle2/
set -o pipefail
mkdir -p gpurun_out/settle2
O="--steps 20 --warmup 5 --no-sweep --no-cpu-baseline --no-live-traffic"
for i in 1 2 3; do
  if [ $((i % 2)) = 1 ]; then order="200 1500"; else order="1500 200"; fi
  for s in $order; do
    timeout -k 10 120 python tools/lab/free_wipe_lab.py hog 80 > /dev/null 2>&1 || exit 1
    timeout -k 10 200 python bench.py $O --settle-ms $s > gpurun_out/settle2/b20_s${s}_$i.json 2>/dev/null || exit 1
  done
done
