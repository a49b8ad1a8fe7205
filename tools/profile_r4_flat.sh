#!/bin/bash
# Round 4: the flat lane mapping of the main SpMM (k_step_flat; APPNP_FLAT=1, APPNP_FLAT_U =
# groups of 3 instructions in flight) against k_step_wide's 24-of-32-lane groups, on the 96 main
# columns of products-synth F = 100 and on F = 48; first parity with the flat kernel forced on.
# Results under gpurun_out/flat/.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
tools/gpu_session.sh \
 "flat_tests::700::APPNP_FLAT=1 $T tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -k 'products_k10 or not configs'" \
 "f100_wide::200::APPNP_FLAT=0 $S -d gpurun_out/flat/f100_wide -- $B" \
 "f100_flat1::200::APPNP_FLAT=1 APPNP_FLAT_U=1 $S -d gpurun_out/flat/f100_flat1 -- $B" \
 "f100_flat2::200::APPNP_FLAT=1 APPNP_FLAT_U=2 $S -d gpurun_out/flat/f100_flat2 -- $B" \
 "f48_wide::200::APPNP_FLAT=0 $S -d gpurun_out/flat/f48_wide -- $B --features 48" \
 "f48_flat1::200::APPNP_FLAT=1 APPNP_FLAT_U=1 $S -d gpurun_out/flat/f48_flat1 -- $B --features 48" \
 "f48_flat2::200::APPNP_FLAT=1 APPNP_FLAT_U=2 $S -d gpurun_out/flat/f48_flat2 -- $B --features 48"
