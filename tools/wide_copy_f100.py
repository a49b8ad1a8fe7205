"""a 1-4-column remainder on a W8 / W16 source-blocked copy runs the 2- or
4-lane pass with all-zero pieces.  Measure it: products-synth, F = 100 (remainder 4) and F = 36,
K = 10, propagated on a graph built with each copy width (W4 / W8 / W16) and on one without the
copy (whole-row gathers), HIP events on the launch stream, median of 5 calls after 2 warm-ups.
Each result is also checked against the W4 graph's Z (bitwise-equal sums are not expected:
only the remainder pass's piece layout differs; the bar is the fp32 1e-5 relative).

    python tools/wide_copy_f100.py [--workload products-synth] [--features 100 36]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="products-synth")
    ap.add_argument("--features", type=int, nargs="+", default=[100, 36])
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()

    import ppnp_amd
    from ppnp_amd import synth
    from ppnp_amd.dist import line_ld

    dev = torch.device("cuda", 0)
    n, _, _, K, alpha, _ = synth.CONFIGS[args.workload]
    indptr, indices = synth.graph_for(args.workload, device=dev)
    graphs = {"whole": ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=dev,
                                               source_blocks=False)}
    for w in (4, 8, 16):  # features=w builds the W-wide copy (remainder_width picks w)
        graphs[f"W{w}"] = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=dev,
                                                  features=w)
    stream = torch.cuda.current_stream(dev)
    for F in args.features:
        ld = line_ld(F, 4)
        H = torch.zeros(n, ld, device=dev)
        H[:, :F] = synth.features(n, F, device=dev)
        H = H[:, :F]
        Z = torch.empty(n, ld, device=dev)[:, :F]
        ref = None
        for name, g in graphs.items():
            times = []
            before = (g.source_block_layout() or {}).get("launches", 0)
            for i in range(args.reps + 2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                ppnp_amd.propagate_forward(g, H, K, alpha, out=Z)
                e1.record(stream)
                torch.cuda.synchronize()
                if i >= 2:
                    times.append(e0.elapsed_time(e1) / K)
            after = (g.source_block_layout() or {}).get("launches", 0)
            if ref is None:
                ref = Z.clone()
            err = float((Z - ref).abs().max())
            tol = 1e-5 * float(ref.abs().max()) + 1e-6
            times.sort()
            print(json.dumps({"workload": args.workload, "F": F, "graph": name,
                              "remainder_cols": g.remainder_cols(F),
                              "remainder_launches": after - before,
                              "ms_per_iter_median": times[len(times) // 2],
                              "ms_per_iter_min": times[0],
                              "max_abs_vs_whole": err, "ok": err <= tol}), flush=True)


if __name__ == "__main__":
    main()
