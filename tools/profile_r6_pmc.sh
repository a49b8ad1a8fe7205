#!/bin/bash
# Round 6: PMC traffic of every kernel set the bench lines can print, on the final HIP sources
# (their digest keys profiles/pmc_traffic.json): the N = 1 headline, configs 2 and 3, and rank 0
# of every candidate layout of the driver's N = 2 / 4 / 8 products runs, each rank emulated on one
# MI355X (--emulate P:0); the pipelined 8-rank row layout also at rank 3 and without the pipeline.
# Per case a kernel-stats run and separate FETCH_SIZE and WRITE_SIZE passes; the W16 slab also
# TCC_HIT / TCC_MISS.  Argument: "a" or "b" (two halves).
# Afterwards, in the build container: tools/collect_pmc_r6.sh.
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
P="timeout -s KILL 200 rocprofv3 -o run --output-format csv"
specs=()
add() {
  local tag=$1; shift
  specs+=("${tag}_stats::300::$S -d gpurun_out/pmc/$tag/stats -- $B $*")
  specs+=("${tag}_fetch::300::$P --pmc FETCH_SIZE -d gpurun_out/pmc/$tag/fetch -- $B $*")
  specs+=("${tag}_write::300::$P --pmc WRITE_SIZE -d gpurun_out/pmc/$tag/write -- $B $*")
}
if [ "${1:-a}" = a ]; then
  add single
  add pubmed --workload pubmed-synth
  add msacad --workload ms-academic-synth
  add col8 --layout col --emulate 8:0
  specs+=("col8_l2::300::$P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc/col8/l2 -- $B --layout col --emulate 8:0")
  add col2l --layout col-lines --emulate 2:0
  add col4 --layout col --emulate 4:0
else
  add col2 --layout col --emulate 2:0
  add row2 --layout row --overlap --emulate 2:0
  add col4l --layout col-lines --emulate 4:0
  add r2c2 --layout 2x2 --overlap --emulate 4:0
  add row4 --layout row --overlap --emulate 4:0
  add r2c4 --layout 2x4 --overlap --emulate 8:0
  add r4c2 --layout 4x2 --overlap --emulate 8:0
  add r4c2g --layout 4x2 --overlap --exchange group --emulate 8:0
  add row8 --layout row --overlap --emulate 8:0
  add row8r3 --layout row --overlap --emulate 8:3
  add row8np --layout row --overlap --pipeline off --emulate 8:0
fi
T="python -u -m pytest -x -q --timeout 150 --timeout-method thread"
[ "${1:-a}" = a ] && specs=("probe_tests::300::$T tests/test_gpu_probe.py" "${specs[@]}")
tools/gpu_session.sh "${specs[@]}"
