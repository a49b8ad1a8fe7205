#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Round 4: the period S of the remainder pass's workgroup barrier (APPNP_REM_SYNC_W<w>=S: every S
# source blocks), per width, after tools/profile_r4_window.sh found S = 16 faster than free-running
# waves on the W16 pass (1.79 against 1.94 ms).  W16 (13-column slab of the 8-rank column layout),
# W4 (headline), W8 (F = 40); then the L2 hits of the W16 pass at S = 16.  gpurun_out/sync2/.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
P="timeout -s KILL 200 rocprofv3 -o run --output-format csv"
C8="--layout col --emulate 8:0"
specs=()
for q in 0 8 12 16 24 32 48; do specs+=("c8_s$q::200::APPNP_REM_SYNC_W16=$q $S -d gpurun_out/sync2/c8_s$q -- $B $C8"); done
for q in 0 8 16 32; do specs+=("w4_s$q::200::APPNP_REM_SYNC_W4=$q $S -d gpurun_out/sync2/w4_s$q -- $B"); done
for q in 0 8 16 32; do specs+=("f40_s$q::200::APPNP_REM_SYNC_W8=$q $S -d gpurun_out/sync2/f40_s$q -- $B --features 40"); done
specs+=("c8_s16_l2::200::APPNP_REM_SYNC_W16=16 $P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/sync2/c8_s16_l2 -- $B $C8")
tools/gpu_session.sh "${specs[@]}"
