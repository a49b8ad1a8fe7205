#!/bin/bash
# Round 5, final tree: the whole -m gpu suite, smoke(), and the default bench line (call "a");
# the driver's N = 2 and N = 4 products commands rehearsed on the one GPU with the gloo exchange,
# which exercises the candidate loop, the run budget and the per-rank parity (call "b").
set -u
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
if [ "${1:-a}" = a ]; then
tools/gpu_session.sh \
 "gpu_tests::1000::python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread" \
 "smoke::200::python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench_default::300::python bench.py"
else
tools/gpu_session.sh \
 "bench_box::200::python bench.py --cpu-iters 0" \
 "n2_products::600::PPNP_DIST_BACKEND=gloo $R --nproc-per-node 2 --master-port 29526 bench.py --gpus 2 --steps 2 --warmup 1" \
 "n4_products::600::PPNP_DIST_BACKEND=gloo $R --nproc-per-node 4 --master-port 29527 bench.py --gpus 4 --steps 2 --warmup 1"
fi
