# Driver-style bench twice: once right after an 80 GiB process (the worst
# start seen), once after it.  Output: gpurun_out/dbench/<tag>_*.json
set -o pipefail
T=${1:-x}
mkdir -p gpurun_out/dbench
timeout -k 10 120 python tools/lab/free_wipe_lab.py hog 80 > /dev/null 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dbench/${T}_after_hog.json 2> gpurun_out/dbench/${T}_after_hog.err || exit 1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dbench/${T}_second.json 2> gpurun_out/dbench/${T}_second.err
