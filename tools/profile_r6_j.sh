#!/bin/bash
# Round 6: PMC of the pipelined 4 x 2 rank (group exchange) on the final sources.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0 --layout 4x2 --overlap --exchange group --emulate 8:0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
P="timeout -s KILL 200 rocprofv3 -o run --output-format csv"
tools/gpu_session.sh \
  "r4c2g_stats::300::$S -d gpurun_out/pmc/r4c2g/stats -- $B" \
  "r4c2g_fetch::300::$P --pmc FETCH_SIZE -d gpurun_out/pmc/r4c2g/fetch -- $B" \
  "r4c2g_write::300::$P --pmc WRITE_SIZE -d gpurun_out/pmc/r4c2g/write -- $B"
