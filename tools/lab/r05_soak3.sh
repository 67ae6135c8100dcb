# Round 5: async stamps with their digests (soak op 8) on each path, the
# launch-path stamp test, then the full soak.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05m
mkdir -p $O
for cfg in "8 0 off" "12 0 off" "8 0 8,2,0" "15 15 2,2,2"; do
  set -- $cfg
  echo "== ops $1 ctl $2 start $3" >> $O/soak.txt
  PCS_SOAK_OPS=$1 PCS_SOAK_CTL=$2 PCS_SOAK_START=$3 timeout -k 10 60 tests/cpp/service_threads_test --soak 8 >> $O/soak.txt 2>&1
  rc=$?
  echo "rc $rc" >> $O/soak.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc $rc"; cat $O/soak.txt; exit $rc; fi
done
cat $O/soak.txt
