#!/bin/bash
# Round 4: the wide SpMM pipelined across rows (k_step_wide_pipe: APPNP_PIPE = rows per wave; a
# wave has row r+1's first col/val chunk and row r+2's pointers in flight while it gathers for
# row r) against one row per wave (APPNP_PIPE=1, k_step_wide).  Parity first with PIPE=4 forced.
# Results under gpurun_out/pipe/.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
specs=("pipe_tests::700::APPNP_PIPE=4 $T tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -k 'products_k10 or powerlaw or not configs'")
for p in 1 2 4 8 16; do specs+=("f100_p$p::200::APPNP_PIPE=$p $S -d gpurun_out/pipe/f100_p$p -- $B"); done
for p in 1 4; do specs+=("f48_p$p::200::APPNP_PIPE=$p $S -d gpurun_out/pipe/f48_p$p -- $B --features 48"); done
for p in 1 4; do specs+=("pl_p$p::200::APPNP_PIPE=$p $S -d gpurun_out/pipe/pl_p$p -- $B --workload products-powerlaw"); done
tools/gpu_session.sh "${specs[@]}"
