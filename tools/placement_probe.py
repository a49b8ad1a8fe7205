"""Is the products-synth iteration time a property of where the gathered buffer sits?

One process, one W4 graph, one H and Z; then ``--trials`` fresh workspaces (the split buffers
the main SpMM gathers from, 1.96 GB), each allocated while the earlier ones stay alive (so each
gets new device memory), each timed over ``--calls`` propagations (HIP events, ms per
iteration).  Then the first workspace again, to separate placement from drift over time.

    python tools/placement_probe.py [--trials 6] [--calls 5]
"""

import argparse
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=6)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--hipmalloc", action="store_true",
                    help="allocate each workspace with its own hipMalloc (not torch's cache)")
    ap.add_argument("--flags", type=int, default=None,
                    help="allocate each workspace with hipExtMallocWithFlags(flags), e.g. 4 = "
                         "hipDeviceMallocContiguous (physically contiguous: largest TLB fragments)")
    args = ap.parse_args()

    import ppnp_amd
    from ppnp_amd import _lib, synth
    from ppnp_amd.dist import line_ld

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, _, F, K, alpha, _ = synth.CONFIGS["products-synth"]
    ld = line_ld(F, 4)
    indptr, indices = synth.graph_for("products-synth", device=dev)
    g = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=dev, features=F)
    del indices
    H = torch.zeros(n, ld, device=dev)
    H[:, :F] = synth.features(n, F, device=dev)
    Z = torch.empty(n, ld, device=dev)
    lib = _lib.load()
    ws_bytes = int(lib.appnp_workspace_bytes(g.handle, F, ld, _lib.F32))
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)

    hip = None
    if args.hipmalloc or args.flags is not None:
        hip = C.CDLL("libamdhip64.so")

    def alloc():
        if hip is None:
            t = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
            return t, t.data_ptr()
        p = C.c_void_p()
        if args.flags is not None:
            rc = hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(ws_bytes), C.c_uint(args.flags))
        else:
            rc = hip.hipMalloc(C.byref(p), C.c_size_t(ws_bytes))
        assert rc == 0, f"allocation failed: {rc}"
        return p, p.value

    def call(ptr):
        rc = lib.appnp_propagate(g.handle, C.c_void_p(H.data_ptr()), ld,
                                 C.c_void_p(Z.data_ptr()), ld, F, _lib.F32, K,
                                 C.c_float(alpha), C.c_float(0.0), C.c_uint64(0),
                                 C.c_void_p(ptr), C.c_size_t(ws_bytes), sp)
        assert rc == 0, rc

    def time_ws(ptr):
        call(ptr)  # warm-up on this workspace
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.calls + 1)]
        evs[0].record(stream)
        for i in range(args.calls):
            call(ptr)
            evs[i + 1].record(stream)
        torch.cuda.synchronize()
        per = sorted(evs[i].elapsed_time(evs[i + 1]) / K for i in range(args.calls))
        return per[len(per) // 2], per[0], per[-1]

    keep = []
    t0 = time.perf_counter()
    for trial in range(args.trials):
        buf, ptr = alloc()
        keep.append((buf, ptr))
        med, lo, hi = time_ws(ptr)
        print(json.dumps({"trial": trial, "ws_addr": hex(ptr), "ms_per_iter_median": med,
                          "min": lo, "max": hi, "t_s": time.perf_counter() - t0}), flush=True)
    med, lo, hi = time_ws(keep[0][1])
    print(json.dumps({"trial": "first-again", "ws_addr": hex(keep[0][1]),
                      "ms_per_iter_median": med, "min": lo, "max": hi,
                      "t_s": time.perf_counter() - t0}), flush=True)


if __name__ == "__main__":
    main()
