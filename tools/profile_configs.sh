#!/bin/bash
# tools/profile_configs.sh — tools/profile_round.sh over the non-default bench workloads
# (configs 3/4/5, XXH64), one tag each; summarise with tools/summarize_profile.py.
export TMPDIR=/tmp
set -e
for spec in "c3:--config 3" "c3x64:--config 3 --algo xxh64" "c4:--config 4" "c5:--config 5" "c2x64:--config 2 --algo xxh64" "c4x64:--config 4 --algo xxh64"; do
  tag=r01_${spec%%:*}; args=${spec#*:}
  BENCH_ARGS="$args --steps 10 --warmup 3 --no-cpu-baseline" PMC_ARGS="$args" bash tools/profile_round.sh $tag > gpurun_out/prof_$tag.log 2>&1
  echo "done $tag"
done
