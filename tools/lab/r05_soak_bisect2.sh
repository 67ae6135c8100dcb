# Round 5: after the done-byte fix (system-scope header + done byte), the
# stamp soak per path: launch path only (no service), service only (a line
# per thread, gate off), then the full soak and the service test file.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05d
mkdir -p $O
for cfg in "4 0 off" "4 0 8,2,0" "4 0 8,1,0" "7 0 off" "7 15 2,2,2"; do
  set -- $cfg
  echo "== ops $1 ctl $2 start $3" >> $O/bisect.txt
  PCS_SOAK_OPS=$1 PCS_SOAK_CTL=$2 PCS_SOAK_START=$3 timeout -k 10 60 tests/cpp/service_threads_test --soak 8 >> $O/bisect.txt 2>&1
  rc=$?
  echo "rc $rc" >> $O/bisect.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc $rc"; cat $O/bisect.txt; exit $rc; fi
done
cat $O/bisect.txt
timeout -k 10 420 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_service.py > $O/service_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/service_tests.log | tail -30
exit $rc
