#!/bin/bash
# Round 6: PMC of the relayed 4 x 2 rank (non-pipelined since the emulation follows the real
# exchange), and the driver's N = 2 and N = 8 products commands rehearsed on the one GPU over
# gloo (every candidate, pipelined row layouts included, with per-rank oracle parity).
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
S="rocprofv3 --kernel-trace --stats -o run --output-format csv"
P="timeout -s KILL 200 rocprofv3 -o run --output-format csv"
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
tools/gpu_session.sh \
  "r4c2m_stats::300::$S -d gpurun_out/pmc/r4c2m/stats -- $B --layout 4x2 --overlap --emulate 8:0" \
  "r4c2m_fetch::300::$P --pmc FETCH_SIZE -d gpurun_out/pmc/r4c2m/fetch -- $B --layout 4x2 --overlap --emulate 8:0" \
  "r4c2m_write::300::$P --pmc WRITE_SIZE -d gpurun_out/pmc/r4c2m/write -- $B --layout 4x2 --overlap --emulate 8:0" \
  "n2_products::500::PPNP_DIST_BACKEND=gloo $R --nproc-per-node 2 --master-port 29536 bench.py --gpus 2 --steps 2 --warmup 1" \
  "n8_products::900::PPNP_DIST_BACKEND=gloo $R --nproc-per-node 8 --master-port 29538 bench.py --gpus 8 --steps 2 --warmup 1"
