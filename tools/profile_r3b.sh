#!/bin/bash
# Round-3 closing evidence (second session) for profiles/: the default bench line, rocprofv3
# kernel stats and separate PMC passes (FETCH_SIZE, WRITE_SIZE, L2 hit/miss) of the same
# command under the final sources, the 8-rank layout emulations, the other workloads, and the
# timing-state check (tools/timing_ab.py with the clocks sampled, before and after the profiler
# runs).  Afterwards (in the build container): python tools/collect_round.py r3b
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
tools/gpu_session.sh \
 "ab_pre::200::tools/clock_watch.sh 2 python tools/timing_ab.py --calls 10" \
 "bench_default::400::python bench.py" \
 "prof_stats::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- $B" \
 "pmc_fetch::300::timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B" \
 "pmc_write::300::timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B" \
 "pmc_l2::300::timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o run --output-format csv -- $B" \
 "emu_col8::200::$B --layout col --emulate 8:0" \
 "emu_row8ov::200::$B --layout row --overlap --emulate 8:0" \
 "emu_r2c4::200::$B --layout 2x4 --emulate 8:0" \
 "emu_r4c2::200::$B --layout 4x2 --emulate 8:0" \
 "emu_col4::200::$B --layout col --emulate 4:0" \
 "emu_col2::200::$B --layout col --emulate 2:0" \
 "w_pubmed::200::$B --workload pubmed-synth" \
 "w_msacad::200::$B --workload ms-academic-synth" \
 "w_arxiv::200::$B --workload arxiv-synth" \
 "w_cora_real::200::$B --workload cora-ml-real" \
 "ab_post::200::tools/clock_watch.sh 2 python tools/timing_ab.py --calls 10"
