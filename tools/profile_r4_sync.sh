#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Round 4: the remainder pass walking its source blocks in step (SYNC, a workgroup barrier
# per block; APPNP_REM_SYNC = mask of bit LPE: 2 W4, 4 W8, 16 W16) against the free-running
# waves, for the W16 pass of the 8-rank column slab, the W8 pass (F = 40 = 32 + 8) and the W4
# pass of the headline; W8 / W16 with 4 chunks in flight (the new default) against 2
# (tools/bin/uw2.so).  First the split-path parity tests with and without SYNC.  Results under
# gpurun_out/sync/.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
P="timeout -s KILL 200 rocprofv3 -o run --output-format csv"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
tools/gpu_session.sh \
 "split_tests::600::$T tests/test_gpu_split.py" \
 "split_tests_sync::600::APPNP_REM_SYNC=22 $T tests/test_gpu_split.py" \
 "c8_s0::300::$S -d gpurun_out/sync/c8_s0 -- $B --layout col --emulate 8:0" \
 "c8_s1::300::APPNP_REM_SYNC=16 $S -d gpurun_out/sync/c8_s1 -- $B --layout col --emulate 8:0" \
 "c8_s1_l2::300::APPNP_REM_SYNC=16 $P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/sync/c8_s1_l2 -- $B --layout col --emulate 8:0" \
 "f40_s0::300::$S -d gpurun_out/sync/f40_s0 -- $B --features 40" \
 "f40_s1::300::APPNP_REM_SYNC=4 $S -d gpurun_out/sync/f40_s1 -- $B --features 40" \
 "f40_uw2::300::PPNP_AMD_LIB=tools/bin/uw2.so $S -d gpurun_out/sync/f40_uw2 -- $B --features 40" \
 "w4_s0::300::$S -d gpurun_out/sync/w4_s0 -- $B" \
 "w4_s1::300::APPNP_REM_SYNC=2 $S -d gpurun_out/sync/w4_s1 -- $B" \
 "bench_default::400::python bench.py"
