#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Grid-cap sweep (APPNP_MAX_BLOCKS: the SpMM grid-strides over rows when capped) on products-synth
# and arxiv-synth; one bench line per setting into gpurun_out/grid/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/grid
for w in products-synth arxiv-synth; do
  for mb in 4194304 1024 2048 4096 8192 32768; do
    APPNP_MAX_BLOCKS=$mb timeout -k 10 120 python bench.py --workload $w --steps 10 --warmup 2 --cpu-iters 0 \
      > gpurun_out/grid/$w.$mb.json 2> gpurun_out/grid/$w.$mb.err || { echo "failed $w $mb"; exit 1; }
    echo "$w $mb done"
  done
done
