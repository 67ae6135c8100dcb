# free_wipe_lab.py probe2: slow phase per process or per fresh allocation?
set -o pipefail
mkdir -p gpurun_out/wipe2
O=gpurun_out/wipe2/wipe2.txt
: > $O
for i in 1 2; do
  echo "== hog 80 GiB, then probe2 ($i)" >> $O
  timeout -k 10 120 python -u tools/lab/free_wipe_lab.py hog 80 >> $O 2>&1 || exit 1
  timeout -k 10 120 python -u tools/lab/free_wipe_lab.py probe2 2 >> $O 2>&1 || exit 1
  echo "== probe2 after 5 s idle ($i)" >> $O
  sleep 5
  timeout -k 10 120 python -u tools/lab/free_wipe_lab.py probe2 2 >> $O 2>&1 || exit 1
done
