#!/bin/bash
# Round 5: tools/spmm_ladder.hip on the box -- timings, then FETCH_SIZE / WRITE_SIZE passes.
set -u
mkdir -p /tmp/xp gpurun_out/ladder
hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/spmm_ladder.hip -o /tmp/xp/spmm_ladder || exit 1
tools/gpu_session.sh \
 "ladder::200::/tmp/xp/spmm_ladder" \
 "ladder_fetch::200::timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ladder/fetch -o run --output-format csv -- /tmp/xp/spmm_ladder" \
 "ladder_write::200::timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ladder/write -o run --output-format csv -- /tmp/xp/spmm_ladder"
