#!/bin/bash
# Round 6, final sources (after the entries-in-flight rule): PMC traffic of every case (both
# halves of profile_r6_pmc.sh and the relayed 4 x 2 rank), then smoke, the default bench line and
# the driver's bench command under rocprofv3.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
P="timeout -s KILL 200 rocprofv3 -o run --output-format csv"
bash tools/profile_r6_pmc.sh a && bash tools/profile_r6_pmc.sh b && tools/gpu_session.sh \
  "r4c2m_stats::300::$S -d gpurun_out/pmc/r4c2m/stats -- $B --layout 4x2 --overlap --emulate 8:0" \
  "r4c2m_fetch::300::$P --pmc FETCH_SIZE -d gpurun_out/pmc/r4c2m/fetch -- $B --layout 4x2 --overlap --emulate 8:0" \
  "r4c2m_write::300::$P --pmc WRITE_SIZE -d gpurun_out/pmc/r4c2m/write -- $B --layout 4x2 --overlap --emulate 8:0" \
  "f_smoke::200::python -c 'import __graft_entry__ as g; g.smoke()'" \
  "f_bench_default::300::python bench.py" \
  "f_driver_stats::300::rocprofv3 --kernel-trace --stats -o run --output-format csv -d gpurun_out/drv6 -- python bench.py"
