"""Seeded synthetic graphs for benchmarking.

The reference ships only Cora-ML and Citeseer (PubMed / MS-Academic are missing,
.MISSING_LARGE_BLOBS:1-2; ogbn-arxiv / -products were never part of it), so the larger
configs run on uniform random stand-ins with the published node / edge counts:
m (src, dst) pairs uniform in [0, N), A = A + A^T, data := 1, no self loops, duplicates
merged -- the reference's ``standardize`` semantics (sparsegraph.py:191-222) without LCC.

This is input synthesis (like torch.randn for H), generated directly on the GPU with torch
so a 62M-edge graph takes well under a second; it is not part of the measured path.
"""

from __future__ import annotations

import torch

CONFIGS = {
    # name: (nodes, undirected edges, F, K, alpha, dtype)
    "cora-ml": (2810, 7981, 7, 10, 0.1, torch.float32),
    "pubmed-synth": (19717, 44324, 3, 10, 0.1, torch.float32),
    "ms-academic-synth": (18333, 81894, 15, 20, 0.2, torch.bfloat16),
    "arxiv-synth": (169343, 1166243, 128, 10, 0.1, torch.float32),
    "products-synth": (2449029, 61859140, 100, 10, 0.1, torch.float32),
    # power-law stand-in (SURVEY 8(d) "optionally add a Chung-Lu power-law variant")
    "products-powerlaw": (2449029, 61859140, 100, 10, 0.1, torch.float32),
    # gather locality: communities of consecutive nodes (the order a locality-preserving
    # relabelling gives a real graph with community structure); not a headline config
    "products-local": (2449029, 61859140, 100, 10, 0.1, torch.float32),
    # the reference's own datasets (standardized LCC adjacency from tests/golden, which
    # tests/golden/make_golden.py took from the reference's SparseGraph.standardize)
    "cora-ml-real": (2810, 7981, 7, 10, 0.1, torch.float32),
    "citeseer-real": (2110, 3668, 6, 10, 0.1, torch.float32),
}
REAL = {"cora-ml-real": "cora_ml", "citeseer-real": "citeseer"}

SEEDS = {"pubmed-synth": 1, "ms-academic-synth": 2, "arxiv-synth": 3, "products-synth": 4,
         "products-powerlaw": 5, "products-local": 6}
POWERLAW = {"products-powerlaw"}
LOCAL = {"products-local"}
DESCRIPTIONS = {name: "synthetic (uniform random graph with the dataset's node/edge counts)"
                for name in CONFIGS}
DESCRIPTIONS["products-powerlaw"] = ("synthetic (Chung-Lu power-law graph with the dataset's "
                                     "node/edge counts)")
DESCRIPTIONS["products-local"] = ("synthetic (the dataset's node/edge counts; communities of "
                                  "4096 consecutive nodes hold 90 % of the edges)")
for _name in REAL:
    DESCRIPTIONS[_name] = "the reference's dataset (standardized LCC adjacency)"


def uniform_graph_device(n: int, m: int, seed: int, device="cuda"):
    """CSR (indptr int32 [n+1], indices int32 [nnz]) of the symmetrised uniform graph, on
    ``device``; columns sorted within each row, no duplicates, no self loops."""
    g = torch.Generator(device=device).manual_seed(seed)
    src = torch.randint(0, n, (m,), device=device, generator=g, dtype=torch.int64)
    dst = torch.randint(0, n, (m,), device=device, generator=g, dtype=torch.int64)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    key = torch.cat([src * n + dst, dst * n + src])
    del src, dst, keep
    key = torch.unique(key, sorted=True)
    row = torch.div(key, n, rounding_mode="floor")
    col = (key - row * n).to(torch.int32)
    del key
    counts = torch.bincount(row, minlength=n)
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    indptr[1:] = torch.cumsum(counts, 0)
    return indptr.to(torch.int32), col


def chung_lu_graph_device(n: int, m: int, seed: int, exponent: float = 3.2,
                          device="cuda"):
    """Power-law graph (Chung-Lu): endpoints drawn with probability proportional to
    w_i = (i + 1)^(-1/(exponent-1)) (inverse-CDF sampling), then the same symmetrise /
    de-duplicate / no-self-loop steps as ``uniform_graph_device``.  Exponent 3.2 gives a
    largest degree of ~20k at products scale (the real ogbn-products: ~17k, mean ~50)."""
    g = torch.Generator(device=device).manual_seed(seed)
    w = torch.arange(1, n + 1, device=device, dtype=torch.float64).pow(-1.0 / (exponent - 1.0))
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    u = torch.rand(2, m, device=device, generator=g, dtype=torch.float64)
    ends = torch.searchsorted(cdf, u).clamp_(max=n - 1)
    # scatter node ids so hubs are not all at low indices
    perm = torch.randperm(n, device=device, generator=g)
    src, dst = perm[ends[0]], perm[ends[1]]
    del ends, u, cdf, w
    keep = src != dst
    src, dst = src[keep], dst[keep]
    key = torch.cat([src * n + dst, dst * n + src])
    del src, dst, keep
    key = torch.unique(key, sorted=True)
    row = torch.div(key, n, rounding_mode="floor")
    col = (key - row * n).to(torch.int32)
    del key
    counts = torch.bincount(row, minlength=n)
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    indptr[1:] = torch.cumsum(counts, 0)
    return indptr.to(torch.int32), col


def community_graph_device(n: int, m: int, seed: int, block: int = 4096, p_in: float = 0.9,
                           device="cuda"):
    """Graph with gather locality: the source of each of the m pairs is uniform; with
    probability p_in its destination is uniform inside the source's community (``block``
    consecutive node ids), otherwise uniform over all nodes.  Then the same symmetrise /
    de-duplicate / no-self-loop steps as ``uniform_graph_device``.  A community's rows of an
    F = 100 fp32 Z are 1.6 MB, so the rows a wave front gathers stay in L2."""
    g = torch.Generator(device=device).manual_seed(seed)
    src = torch.randint(0, n, (m,), device=device, generator=g, dtype=torch.int64)
    far = torch.randint(0, n, (m,), device=device, generator=g, dtype=torch.int64)
    base = torch.div(src, block, rounding_mode="floor") * block
    near = (base + torch.randint(0, block, (m,), device=device, generator=g)).clamp_(max=n - 1)
    inside = torch.rand(m, device=device, generator=g) < p_in
    dst = torch.where(inside, near, far)
    del far, base, near, inside
    keep = src != dst
    src, dst = src[keep], dst[keep]
    key = torch.cat([src * n + dst, dst * n + src])
    del src, dst, keep
    key = torch.unique(key, sorted=True)
    row = torch.div(key, n, rounding_mode="floor")
    col = (key - row * n).to(torch.int32)
    del key
    counts = torch.bincount(row, minlength=n)
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    indptr[1:] = torch.cumsum(counts, 0)
    return indptr.to(torch.int32), col


def real_graph(name: str, device="cuda"):
    """CSR of a dataset the reference ships, standardized as its SparseGraph does."""
    import os

    import numpy as np

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = np.load(os.path.join(root, "tests", "golden", name + ".npz"), allow_pickle=False)
    indptr = torch.from_numpy(d["adj_indptr"].astype(np.int32)).to(device)
    indices = torch.from_numpy(d["adj_indices"].astype(np.int32)).to(device)
    return indptr, indices


def graph_for(workload: str, device="cuda"):
    if workload in REAL:
        return real_graph(REAL[workload], device=device)
    n, m = CONFIGS[workload][:2]
    if workload in POWERLAW:
        return chung_lu_graph_device(n, m, SEEDS[workload], device=device)
    if workload in LOCAL:
        return community_graph_device(n, m, SEEDS[workload], device=device)
    return uniform_graph_device(n, m, SEEDS.get(workload, 0), device=device)


def features(n: int, f: int, dtype=torch.float32, device="cuda", seed: int = 0):
    g = torch.Generator(device=device).manual_seed(seed)
    return torch.randn(n, f, device=device, generator=g, dtype=torch.float32).to(dtype)
