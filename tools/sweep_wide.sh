#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Wide remainder pass (APPNP_GRAPH_SB_W8/_W16) against whole-row gathers (APPNP_SPLIT=0) on the
# shapes it targets; one bench line per case into gpurun_out/wide/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wide
B="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
run() {  # tag, env, args
  env $2 timeout -k 10 150 $B $3 > gpurun_out/wide/$1.json 2> gpurun_out/wide/$1.err || { echo "failed $1"; exit 1; }
  echo "$1 done"
}
for s in 1 0; do
  run "col8r0.split$s" "APPNP_SPLIT=$s" "--layout col --emulate 8:0"
  run "col8r7.split$s" "APPNP_SPLIT=$s" "--layout col --emulate 8:7"
  run "prod_f40.split$s" "APPNP_SPLIT=$s" "--features 40"
  run "prod_f47.split$s" "APPNP_SPLIT=$s" "--features 47"
  run "arxiv_f40.split$s" "APPNP_SPLIT=$s" "--workload arxiv-synth --features 40"
  run "prod_f16.split$s" "APPNP_SPLIT=$s" "--features 16"
done
run "prod_f100.default" "APPNP_SPLIT=1" ""
