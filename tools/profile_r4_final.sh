#!/bin/bash
# Round 4, final tree: the whole -m gpu suite, smoke(), the default bench line, and the driver's
# N = 8 products command rehearsed on the one GPU (gloo) with the round-4 candidate order.
set -u
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
tools/gpu_session.sh \
 "gpu_tests::1000::python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread" \
 "smoke::200::python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench_default::300::python bench.py" \
 "n8_products::600::PPNP_DIST_BACKEND=gloo $R --nproc-per-node 8 --master-port 29528 bench.py --gpus 8 --steps 2 --warmup 1"
