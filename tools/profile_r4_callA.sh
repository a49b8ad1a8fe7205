#!/bin/bash
# Round 4, final kernel sources: the split-path parity tests, the 12-waves-per-workgroup A/B of the
# W4 remainder pass (tools/bin/w12.so = tools/build_variant.sh w12 appnp_blocks
# -DAPPNP_REM_WAVES=12), then the per-rank PMC traffic of every candidate (tools/profile_r4_pmc.sh).
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
tools/gpu_session.sh \
 "split_tests::600::python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_split.py" \
 "w4_waves16::200::$S -d gpurun_out/waves/w16 -- $B" \
 "w4_waves12::200::PPNP_AMD_LIB=tools/bin/w12.so $S -d gpurun_out/waves/w12 -- $B" || exit $?
tools/profile_r4_pmc.sh
