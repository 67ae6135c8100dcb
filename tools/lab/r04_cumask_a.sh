# CU-mask lab, call A: the product's priority stream (expected to pass), then
# the CU-masked stream with no service kernel at all (mode 2), last.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 tools/lab/cumask_lab prio 0 > gpurun_out/r04_cumask_prio.txt 2> gpurun_out/r04_cumask_prio.err &&
timeout -k 10 60 tools/lab/cumask_lab cumask 2 4 > gpurun_out/r04_cumask_nokernel.txt 2> gpurun_out/r04_cumask_nokernel.err
echo "exit $?"
