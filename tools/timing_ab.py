"""Why does the same products-synth F = 100 propagation take 7.77 ms per iteration in
tools/wide_copy_f100.py and 8.24 ms in bench.py on one box (and 8.22 ms in either under
rocprofv3)?  A/B of the candidate causes, HIP events on the launch stream, ms per iteration:

  * back-to-back: ``--calls`` propagations enqueued without a host sync (bench.py's loop);
  * synced: a synchronize after every call (wide_copy's loop);
  * ``--order``: the order of the big device allocations --
      graph-first   A_hat, then H and Z, then the workspace at the first call;
      bench         bench.py's order: H (through a temporary), A_hat, Z, workspace;
      ws-first      bench.py's order, but the workspace's block is allocated (and returned to
                    torch's cache, where the first call finds it) before anything else.

    python tools/timing_ab.py [--order graph-first|bench|ws-first] [--extra-graph]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--extra-graph", action="store_true")
    ap.add_argument("--order", default="graph-first", choices=["graph-first", "bench", "ws-first"])
    args = ap.parse_args()

    import ppnp_amd
    from ppnp_amd import _lib, synth
    from ppnp_amd.dist import line_ld

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, _, F, K, alpha, _ = synth.CONFIGS["products-synth"]
    ld = line_ld(F, 4)
    # workspace bytes of an F = 100 W4 split: two buffers [n, 96] + [n, 4] fp32, 256-B aligned
    ws_guess = 2 * ((n * 96 * 4 + 255) // 256 * 256 + n * 16 + 255) // 256 * 256
    if args.order == "ws-first":
        blk = torch.empty(ws_guess, dtype=torch.uint8, device=dev)
        del blk
    indptr, indices = synth.graph_for("products-synth", device=dev)
    keep = []
    if args.extra_graph:
        keep.append(ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=dev,
                                            source_blocks=False))
    if args.order == "graph-first":
        g = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=dev, features=F)
        H = torch.zeros(n, ld, device=dev)
        H[:, :F] = synth.features(n, F, device=dev)
        H = H[:, :F]
        Z = torch.empty(n, ld, device=dev)[:, :F]
    else:
        H0 = synth.features(n, F, device=dev)
        Hbuf = torch.zeros(n, ld, device=dev)
        Hbuf[:, :F] = H0
        H = Hbuf[:, :F]
        del H0
        torch.cuda.synchronize()
        g = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=dev, features=F)
        torch.cuda.synchronize()
        del indices
        Z = torch.empty(n, ld, device=dev)[:, :F]
    ws_bytes = int(_lib.load().appnp_workspace_bytes(g.handle, F, ld, _lib.F32))
    stream = torch.cuda.current_stream(dev)

    def run():
        ppnp_amd.propagate_forward(g, H, K, alpha, out=Z)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    for mode in ("back-to-back", "synced", "back-to-back", "synced"):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.calls + 1)]
        evs[0].record(stream)
        for i in range(args.calls):
            run()
            evs[i + 1].record(stream)
            if mode == "synced":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        per = sorted(evs[i].elapsed_time(evs[i + 1]) / K for i in range(args.calls))
        print(json.dumps({"order": args.order, "mode": mode, "extra_graph": args.extra_graph,
                          "ws_bytes": ws_bytes, "ws_guess": ws_guess,
                          "ms_per_iter_median": per[len(per) // 2], "min": per[0],
                          "max": per[-1]}), flush=True)


if __name__ == "__main__":
    main()
