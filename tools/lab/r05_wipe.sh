# free_wipe_lab.py: GPU step time right after another process freed 80 GiB.
set -o pipefail
mkdir -p gpurun_out/wipe
O=gpurun_out/wipe/wipe.txt
echo "== probe alone" > $O
timeout -k 10 120 python -u tools/lab/free_wipe_lab.py probe 3 >> $O 2>&1 || exit 1
for i in 1 2; do
  echo "== hog 80 GiB, then probe at once ($i)" >> $O
  timeout -k 10 120 python -u tools/lab/free_wipe_lab.py hog 80 >> $O 2>&1 || exit 1
  timeout -k 10 120 python -u tools/lab/free_wipe_lab.py probe 3 >> $O 2>&1 || exit 1
done
echo "== hog 80 GiB, sleep 5 s, probe" >> $O
timeout -k 10 120 python -u tools/lab/free_wipe_lab.py hog 80 >> $O 2>&1 || exit 1
sleep 5
timeout -k 10 120 python -u tools/lab/free_wipe_lab.py probe 3 >> $O 2>&1 || exit 1
echo "== probe alone (end)" >> $O
timeout -k 10 120 python -u tools/lab/free_wipe_lab.py probe 3 >> $O 2>&1
