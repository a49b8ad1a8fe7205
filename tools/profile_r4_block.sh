#!/bin/bash
# Round 4: workgroup size of the step kernels (kBlock: 256 threads shipped) -- 512 and 1024
# (tools/bin/b512.so / b1024.so: every source rebuilt with -DAPPNP_BLOCK=N on a temporary header
# switch).  gpurun_out/blk/.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
tools/gpu_session.sh \
 "b256::200::$S -d gpurun_out/blk/b256 -- $B" \
 "b512::200::PPNP_AMD_LIB=tools/bin/b512.so $S -d gpurun_out/blk/b512 -- $B" \
 "b1024::200::PPNP_AMD_LIB=tools/bin/b1024.so $S -d gpurun_out/blk/b1024 -- $B" \
 "b256_again::200::$S -d gpurun_out/blk/b256b -- $B"
