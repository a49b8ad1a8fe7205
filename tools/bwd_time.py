#!/usr/bin/env python
"""Time the adjoint (appnp_propagate_bwd) and the forward on a bench workload, per iteration,
with HIP events on the launch stream.  APPNP_TUNING=1 APPNP_SPLIT=0 in the environment gathers
whole rows.

    python tools/bwd_time.py [--workload products-synth] [--reps 5]
"""

import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="products-synth")
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    import ppnp_amd
    from ppnp_amd import synth

    n, m, F, K, alpha, dtype = synth.CONFIGS[a.workload]
    dev = torch.device("cuda", 0)
    indptr, indices = synth.graph_for(a.workload, device=dev)
    G = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=dev)
    X = synth.features(n, F, dtype=dtype, device=dev)
    out = {}
    for name, fn in (("forward", lambda: ppnp_amd.propagate_forward(G, X, K, alpha)),
                     ("adjoint", lambda: ppnp_amd.propagate_backward(G, X, K, alpha))):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / (a.reps * K)
    print(f"{a.workload} split_point={G.split_point(F, dtype)} "
          + " ".join(f"{k} {v:.3f} ms/iter" for k, v in out.items()))


if __name__ == "__main__":
    main()
