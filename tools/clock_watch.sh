#!/bin/bash
# Run a GPU command several times with the GPU's clocks sampled beside it (rocm-smi
# --showclocks every 0.5 s), to see whether the bimodal products-synth iteration time
# (7.77 vs 8.22 ms on the same box, profiles/README) follows a clock state.
# Temperatures (rocm-smi --showtemp: edge, junction, memory) are sampled too: HBM refresh
# doubles above its temperature threshold, which would show as a memory-bound slowdown.
# Usage: [CW_GAP=seconds idle before each run] tools/clock_watch.sh <runs> <command...>
set -u
runs=$1; shift
mkdir -p gpurun_out
tag=${CW_TAG:-}
for i in $(seq 1 "$runs"); do
  sleep "${CW_GAP:-0}"
  ( end=$((SECONDS + 40)); while [ $SECONDS -lt $end ]; do
      echo "t=$(date +%s.%N)"; rocm-smi --showclocks --showtemp 2>/dev/null | grep -E 'sclk|mclk|fclk|Temperature'
      sleep 0.5; done ) > "gpurun_out/clocks_$tag$i.txt" 2>&1 &
  sampler=$!
  timeout -k 10 120 "$@" > "gpurun_out/clock_run_$tag$i.txt" 2>&1
  rc=$?
  kill "$sampler" 2>/dev/null; wait "$sampler" 2>/dev/null
  echo "run $tag$i rc=$rc: $(grep -h ms_per_iter_median gpurun_out/clock_run_$tag$i.txt | head -1 | cut -c1-160)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
