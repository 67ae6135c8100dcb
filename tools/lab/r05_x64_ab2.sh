# Round 5: config 3 XXH64 A/B/C in alternating processes with the order
# reversed every cycle (A B C, C B A, ...): round 4's build, the current
# build (round 4's two-launch XXH64 path restored) and the one-launch build.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w
mkdir -p $O
A=tools/lab/ab/libpcs_r04.so; B=eloqstore_amd/libeloqstore_pcs.so; C=tools/lab/ab/libpcs_r05_onelaunch.so
for cyc in 1 2 3 4 5 6; do
  if [ $((cyc % 2)) -eq 1 ]; then order="$A $B $C"; else order="$C $B $A"; fi
  for lib in $order; do
    timeout -k 10 60 tools/lab/x64_ab_lab $lib >> $O/x64_abc.txt 2>&1 || { echo "rc $?"; cat $O/x64_abc.txt; exit 1; }
  done
done
cat $O/x64_abc.txt
