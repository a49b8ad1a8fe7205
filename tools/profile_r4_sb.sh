#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Round 4: source-block size of the W16 / W8 passes now that they take a barrier every S blocks
# (APPNP_SB_ROWS rows per block, APPNP_REM_SYNC_W16 / _W8 = S).  gpurun_out/sb/.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
C8="--layout col --emulate 8:0"
specs=()
for cfg in "32768:32" "16384:32" "16384:64" "65536:8" "65536:16"; do
  rows=${cfg%%:*}; q=${cfg#*:}
  specs+=("c8_${rows}_$q::200::APPNP_SB_ROWS=$rows APPNP_REM_SYNC_W16=$q $S -d gpurun_out/sb/c8_${rows}_$q -- $B $C8")
done
for cfg in "32768:32" "16384:64"; do
  rows=${cfg%%:*}; q=${cfg#*:}
  specs+=("f40_${rows}_$q::200::APPNP_SB_ROWS=$rows APPNP_REM_SYNC_W8=$q $S -d gpurun_out/sb/f40_${rows}_$q -- $B --features 40")
done
tools/gpu_session.sh "${specs[@]}"
