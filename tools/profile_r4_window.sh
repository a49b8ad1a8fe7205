#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Round 4: pacing the remainder pass's waves inside their workgroup.  APPNP_REM_WINDOW_W<w>=D: a
# wave more than D source blocks ahead of its workgroup's slowest wave sleeps until it catches
# up (no barrier); APPNP_REM_SYNC_W<w>=S: a workgroup barrier every S blocks.  The W16 pass of
# the 8-rank column slab, the W4 pass of the headline and the W8 pass of F = 40, against the
# free-running waves; first the split-path parity tests with a window on every width.
# Results under gpurun_out/win/.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
C8="--layout col --emulate 8:0"
specs=("split_tests_win::600::APPNP_REM_WINDOW_W4=2 APPNP_REM_WINDOW_W8=2 APPNP_REM_WINDOW_W16=2 $T tests/test_gpu_split.py")
specs+=("c8_free::200::$S -d gpurun_out/win/c8_free -- $B $C8")
for d in 1 2 4 8; do specs+=("c8_w$d::200::APPNP_REM_WINDOW_W16=$d $S -d gpurun_out/win/c8_w$d -- $B $C8"); done
for q in 4 16; do specs+=("c8_s$q::200::APPNP_REM_SYNC_W16=$q $S -d gpurun_out/win/c8_s$q -- $B $C8"); done
specs+=("w4_free::200::$S -d gpurun_out/win/w4_free -- $B")
for d in 2 4 8; do specs+=("w4_w$d::200::APPNP_REM_WINDOW_W4=$d $S -d gpurun_out/win/w4_w$d -- $B"); done
specs+=("f40_free::200::$S -d gpurun_out/win/f40_free -- $B --features 40")
for d in 2 4; do specs+=("f40_w$d::200::APPNP_REM_WINDOW_W8=$d $S -d gpurun_out/win/f40_w$d -- $B --features 40"); done
tools/gpu_session.sh "${specs[@]}"
