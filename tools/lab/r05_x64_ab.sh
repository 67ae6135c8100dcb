# Round 5: config 3 XXH64, round 4's two launches (tools/lab/ab/libpcs_r04.so,
# built from ff8f025) against round 5's one launch (eloqstore_amd/), in
# alternating processes on one box.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05u
mkdir -p $O
for i in 1 2 3 4; do
  for lib in tools/lab/ab/libpcs_r04.so eloqstore_amd/libeloqstore_pcs.so; do
    timeout -k 10 60 tools/lab/x64_ab_lab $lib >> $O/x64_ab.txt 2>&1 || { echo "rc $?"; cat $O/x64_ab.txt; exit 1; }
  done
done
cat $O/x64_ab.txt
