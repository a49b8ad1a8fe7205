#!/bin/bash
# Evidence for profiles/: default bench (with CPU baseline), rocprofv3 stats + separate PMC
# passes of the same command, single-GPU layout emulations, multi-rank dist checks, workloads.
# Afterwards (in the build container): python tools/collect_round.py <tag>
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29517"
G="PPNP_DIST_BACKEND=gloo $TR"
tools/gpu_session.sh \
 "bench_default::400::python bench.py" \
 "prof_stats::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- $B" \
 "pmc_fetch::300::rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B" \
 "pmc_write::300::rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B" \
 "emu_col2::200::$B --layout col --emulate 2:0" \
 "emu_col4::200::$B --layout col --emulate 4:0" \
 "emu_col8::200::$B --layout col --emulate 8:0" \
 "emu_row2::200::$B --layout row --emulate 2:0" \
 "emu_row8::200::$B --layout row --emulate 8:0" \
 "emu_r2c4::200::$B --layout 2x4 --emulate 8:0" \
 "emu_r2c4ov::200::$B --layout 2x4 --overlap --emulate 8:0" \
 "emu_r4c2::200::$B --layout 4x2 --emulate 8:0" \
 "dc_col::200::$TR --nproc-per-node 2 tests/dist_worker.py --layout col" \
 "dc_row_arxiv::300::$G --nproc-per-node 4 tests/dist_worker.py --layout row --overlap --workload arxiv-synth --oracle" \
 "dc_row::300::$G --nproc-per-node 2 tests/dist_worker.py --layout row" \
 "dc_row_ov::300::$G --nproc-per-node 2 tests/dist_worker.py --layout row --overlap --p-drop 0.3" \
 "dc_2x2::300::$G --nproc-per-node 4 tests/dist_worker.py --layout 2x2" \
 "dc_2x4_mp::300::$G --nproc-per-node 8 tests/dist_worker.py --layout 2x4 --overlap --p-drop 0.3" \
 "dc_4x2_mp::300::$G --nproc-per-node 8 tests/dist_worker.py --layout 4x2" \
 "w_pubmed::200::$B --workload pubmed-synth" \
 "w_msacad::200::$B --workload ms-academic-synth" \
 "w_arxiv::200::$B --workload arxiv-synth" \
 "w_cora::200::$B --workload cora-ml" \
 "w_powerlaw::200::$B --workload products-powerlaw" \
 "w_local::200::$B --workload products-local" \
 "w_bf16::200::$B --dtype bf16" \
 "dist2_auto::300::$G --nproc-per-node 2 bench.py --gpus 2 --steps 3 --warmup 1" \
 "dist4_auto::300::$G --nproc-per-node 4 bench.py --gpus 4 --steps 3 --warmup 1 --workload arxiv-synth"
