#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Round 4: the W16 remainder pass the 8-rank column layout runs on its 13-column
# products-synth slab (bench.py --layout col --emulate 8:0).  Kernel stats of the shipped pass,
# of source blocks of 2^13 / 2^14 / 2^16 rows (APPNP_SB_ROWS) and of 1 / 4 / 8 chunks in flight
# (tools/build_variant.sh u<U> appnp_blocks -DAPPNP_REM_U=<U>), then the PMC passes of the
# shipped pass: L2 hit / miss, FETCH_SIZE, WRITE_SIZE.  Results under gpurun_out/w16/.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0 --layout col --emulate 8:0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
P="timeout -s KILL 200 rocprofv3 -o run --output-format csv"
tools/gpu_session.sh \
 "bench_default::400::python bench.py" \
 "w16_base::300::$S -d gpurun_out/w16/base -- $B" \
 "w16_sb13::300::APPNP_SB_ROWS=8192 $S -d gpurun_out/w16/sb13 -- $B" \
 "w16_sb14::300::APPNP_SB_ROWS=16384 $S -d gpurun_out/w16/sb14 -- $B" \
 "w16_sb16::300::APPNP_SB_ROWS=65536 $S -d gpurun_out/w16/sb16 -- $B" \
 "w16_u1::300::PPNP_AMD_LIB=tools/bin/u1.so $S -d gpurun_out/w16/u1 -- $B" \
 "w16_u4::300::PPNP_AMD_LIB=tools/bin/u4.so $S -d gpurun_out/w16/u4 -- $B" \
 "w16_u8::300::PPNP_AMD_LIB=tools/bin/u8.so $S -d gpurun_out/w16/u8 -- $B" \
 "w16_l2::300::$P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/w16/pmc_l2 -- $B" \
 "w16_fetch::300::$P --pmc FETCH_SIZE -d gpurun_out/w16/pmc_fetch -- $B" \
 "w16_write::300::$P --pmc WRITE_SIZE -d gpurun_out/w16/pmc_write -- $B"
