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
}

SEEDS = {"pubmed-synth": 1, "ms-academic-synth": 2, "arxiv-synth": 3, "products-synth": 4}


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


def features(n: int, f: int, dtype=torch.float32, device="cuda", seed: int = 0):
    g = torch.Generator(device=device).manual_seed(seed)
    return torch.randn(n, f, device=device, generator=g, dtype=torch.float32).to(dtype)
