#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Round 5: XCD-wide pacing of the W16 remainder pass on the 8-rank column slab
# (bench.py --layout col --emulate 8:0: 13 of products-synth's 100 columns, 4 row passes) and of
# the W8 pass (F = 40 = 32 + 8).  APPNP_REM_PACE_W<w>=p: at every barrier (every 32 blocks) a
# workgroup waits until its XCD's workgroups have finished all but p - 1 barrier periods.  The
# tools/bin/allhit.so variant gathers every row from source block 0 (wrong results, timing only):
# the pass's floor with no L2 misses.  First the parity tests of the split path with pacing on,
# and the new C-engine tests.  roofline.kernel_ms of each line gives the pass's time.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
C8="$B --layout col --emulate 8:0"
T="python -u -m pytest -x -q --timeout 150 --timeout-method thread"
tools/gpu_session.sh \
 "dist_new::400::$T tests/test_gpu_configs.py -k 'misaligned or poisoned'" \
 "split_pace::600::APPNP_REM_PACE_W16=1 APPNP_REM_PACE_W8=1 APPNP_REM_PACE_W4=1 APPNP_REM_SYNC_W4=32 $T tests/test_gpu_split.py" \
 "c8_p0::200::$C8" \
 "c8_p1::200::APPNP_REM_PACE_W16=1 $C8" \
 "c8_p2::200::APPNP_REM_PACE_W16=2 $C8" \
 "c8_p3::200::APPNP_REM_PACE_W16=3 $C8" \
 "c8_s16_p1::200::APPNP_REM_SYNC_W16=16 APPNP_REM_PACE_W16=1 $C8" \
 "c8_s8_p1::200::APPNP_REM_SYNC_W16=8 APPNP_REM_PACE_W16=1 $C8" \
 "c8_s8_p2::200::APPNP_REM_SYNC_W16=8 APPNP_REM_PACE_W16=2 $C8" \
 "c8_allhit::200::PPNP_AMD_LIB=tools/bin/allhit.so $C8" \
 "f40_p0::200::$B --features 40" \
 "f40_p1::200::APPNP_REM_PACE_W8=1 $B --features 40" \
 "f40_p2::200::APPNP_REM_PACE_W8=2 $B --features 40" \
 "f40_allhit::200::PPNP_AMD_LIB=tools/bin/allhit.so $B --features 40" \
 "w4_allhit::200::PPNP_AMD_LIB=tools/bin/allhit.so $B"
