# CU-mask lab, call B: the launch-path threads create their streams and
# staging before the service's first kernel on the CU-masked stream (mode 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 tools/lab/cumask_lab cumask 1 4 > gpurun_out/r04_cumask_precreate.txt 2> gpurun_out/r04_cumask_precreate.err
echo "exit $?"
