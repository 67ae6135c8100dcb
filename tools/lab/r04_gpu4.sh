# Workgroups per request line: 4 lines of 1 / 2 / 4 workgroups and 2 lines of
# 4, against the gated single line (4 workgroups), 6 / 32 / 128 pages.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04d
timeout -k 10 500 tools/lab/service_load 0.4 g1N2N4M4 6,32,128 > gpurun_out/r04d/service_load_hyst.txt 2>&1
echo "exit $?"
