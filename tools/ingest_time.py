#!/usr/bin/env python
"""SURVEY.md 8(f) row 2 at products scale: the device ingest + standardize (appnp_standardize,
ppnp_amd.data.standardize_device: symmetrise, drop self loops, binary, LCC, renumber;
sparsegraph.py:191-222) against the oracle's host restatement (oracle.standardize: scipy, as the
reference's SparseGraph.standardize runs), on the RAW directed pairs of products-synth
(numpy default_rng(4), the bench's generator, before it symmetrises them).  Also the device
calc_A_hat build (appnp_graph_create) against oracle.calc_a_hat on the standardized graph.
Checks the device results bit for bit against the oracle's, and prints one JSON line.

    python tools/ingest_time.py [--workload products-synth] [--reps 3]
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="products-synth")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    import ppnp_amd
    from ppnp_amd import synth
    from ppnp_amd.data import standardize_device
    from oracle import ppnp_oracle as O

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, m, _, _, _, _ = synth.CONFIGS[args.workload]
    seed = synth.SEEDS[args.workload]
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, size=m, dtype=np.int64)
    dst = rng.integers(0, n, size=m, dtype=np.int64)
    # the raw directed adjacency as a CSR file would hold it (duplicates summed, sorted)
    raw = sp.csr_matrix((np.ones(m, dtype=np.float32), (src, dst)), shape=(n, n))
    raw.sum_duplicates()
    raw.sort_indices()
    del src, dst
    ip = torch.from_numpy(raw.indptr.astype(np.int32)).to(dev)
    ix = torch.from_numpy(raw.indices.astype(np.int32)).to(dev)
    torch.cuda.synchronize()

    times = []
    for _ in range(args.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o_ip, o_ix, o_map = standardize_device(ip, ix, None, n, select_lcc=True, device=dev)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    dev_s = sorted(times[1:])[len(times[1:]) // 2]

    t0 = time.perf_counter()
    std, keep = O.standardize(raw, select_lcc=True)
    host_s = time.perf_counter() - t0
    same = (np.array_equal(o_ip.cpu().numpy().astype(np.int64), std.indptr.astype(np.int64))
            and np.array_equal(o_ix.cpu().numpy(), std.indices.astype(np.int32))
            and np.array_equal(o_map.cpu().numpy(), keep.astype(np.int64)))

    # calc_A_hat on the standardized graph: device build against the host oracle
    ns = std.shape[0]
    gtimes = []
    for _ in range(args.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        G = ppnp_amd.Graph.from_csr(o_ip, o_ix, None, ns, mode="sym", device=dev)
        torch.cuda.synchronize()
        gtimes.append(time.perf_counter() - t0)
        last = G
    g_s = sorted(gtimes[1:])[len(gtimes[1:]) // 2]
    t0 = time.perf_counter()
    ahat = O.calc_a_hat(std, "sym")
    host_ahat_s = time.perf_counter() - t0
    rp, col, val, _ = last.csr()
    ahat_same = (np.array_equal(rp.cpu().numpy().astype(np.int64), ahat.indptr.astype(np.int64))
                 and np.array_equal(col.cpu().numpy(), ahat.indices.astype(np.int32))
                 and np.array_equal(val.cpu().numpy(), ahat.data.astype(np.float32)))
    print(json.dumps({
        "workload": args.workload, "raw_nodes": n, "raw_entries": int(raw.nnz),
        "lcc_nodes": int(ns), "lcc_entries": int(std.nnz),
        "device_standardize_s": dev_s, "host_oracle_standardize_s": host_s,
        "standardize_bit_exact": bool(same),
        "device_calc_a_hat_s": g_s, "host_oracle_calc_a_hat_s": host_ahat_s,
        "a_hat_bit_exact_f32": bool(ahat_same), "nnz_a_hat": int(ahat.nnz),
        "host_threads": torch.get_num_threads(),
        "note": "device times: median of reps after one warm-up, synchronised, inputs resident; "
                "host: oracle/ppnp_oracle.py standardize / calc_a_hat (scipy, the reference's "
                "sparsegraph.py:191-222 and helpers.py:58-66 restated), one run"}), flush=True)


if __name__ == "__main__":
    main()
