#!/bin/bash
# Round 4: PMC traffic of the kernels rank 0 runs in every candidate layout of
# the driver's N = 1 / 2 / 4 / 8 products-synth runs, each rank emulated on one MI355X
# (bench.py --emulate P:0: that rank's real kernels on its real share, no exchange).  Per case
# a kernel-stats run and separate FETCH_SIZE and WRITE_SIZE passes.  The traffic key names what
# the rank runs (bench.rank_traffic_key), so these entries are the traffic of the real ranks.
# Afterwards, in the build container: tools/collect_pmc_r4.sh (profiles/pmc_traffic.json).
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
P="timeout -s KILL 200 rocprofv3 -o run --output-format csv"
specs=()
while read -r tag args; do
  [ -z "$tag" ] && continue
  specs+=("${tag}_stats::300::$S -d gpurun_out/pmc/$tag/stats -- $B $args")
  specs+=("${tag}_fetch::300::$P --pmc FETCH_SIZE -d gpurun_out/pmc/$tag/fetch -- $B $args")
  specs+=("${tag}_write::300::$P --pmc WRITE_SIZE -d gpurun_out/pmc/$tag/write -- $B $args")
done <<'EOF'
single
col2 --layout col --emulate 2:0
col2l --layout col-lines --emulate 2:0
row2 --layout row --overlap --emulate 2:0
col4 --layout col --emulate 4:0
col4l --layout col-lines --emulate 4:0
r2c2 --layout 2x2 --overlap --emulate 4:0
row4 --layout row --overlap --emulate 4:0
col8 --layout col --emulate 8:0
r2c4 --layout 2x4 --overlap --emulate 8:0
r4c2 --layout 4x2 --overlap --emulate 8:0
row8 --layout row --overlap --emulate 8:0
EOF
tools/gpu_session.sh "${specs[@]}"
