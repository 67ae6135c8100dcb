# Round 5: bisect the soak's stamp mismatches (gpurun_out/r05b): one 6 s soak
# per (ops, controller) mask.  A run exiting 1 is a mismatch report, not a
# fault; any other non-zero status ends the script.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c
mkdir -p $O
for cfg in "4 0" "4 1" "4 2" "4 4" "4 8" "7 0" "4 15" "3 15" "7 15"; do
  set -- $cfg
  echo "== ops $1 ctl $2" >> $O/bisect.txt
  PCS_SOAK_OPS=$1 PCS_SOAK_CTL=$2 timeout -k 10 60 tests/cpp/service_threads_test --soak 6 >> $O/bisect.txt 2>&1
  rc=$?
  echo "rc $rc" >> $O/bisect.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc $rc"; break; fi
done
cat $O/bisect.txt
