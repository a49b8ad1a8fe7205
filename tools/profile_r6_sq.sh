#!/bin/bash
# Round 6: where the W16 remainder pass (8-rank column slab, 16-column sums) and the W4 pass
# (headline) spend their cycles: SQ wave-state and instruction counters, one pass each.
set -u
C="python bench.py --layout col --emulate 8:0 --steps 3 --warmup 1 --cpu-iters 0"
H="python bench.py --steps 3 --warmup 1 --cpu-iters 0"
P="timeout -s KILL 120 rocprofv3 -o run --output-format csv"
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
S2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
tools/gpu_session.sh \
  "sq1_c16::150::APPNP_TUNING=1 APPNP_SB_COLS=16 $P --pmc $S1 -d gpurun_out/pmc6/sq1_c16 -- $C" \
  "sq2_c16::150::APPNP_TUNING=1 APPNP_SB_COLS=16 $P --pmc $S2 -d gpurun_out/pmc6/sq2_c16 -- $C" \
  "sq1_head::150::$P --pmc $S1 -d gpurun_out/pmc6/sq1_head -- $H" \
  "sq2_head::150::$P --pmc $S2 -d gpurun_out/pmc6/sq2_head -- $H"
