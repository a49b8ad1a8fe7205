"""Seeded synthetic graphs for benchmarking.

The reference ships only Cora-ML and Citeseer (PubMed / MS-Academic are missing,
.MISSING_LARGE_BLOBS:1-2; ogbn-arxiv / -products were never part of it), so the larger
configs run on uniform random stand-ins with the published node / edge counts:
m (src, dst) pairs uniform in [0, N), A = A + A^T, data := 1, no self loops, duplicates
merged -- the reference's ``standardize`` semantics (sparsegraph.py:191-222) without LCC.

The graphs are drawn on the HOST with numpy ``default_rng(seed)`` -- the recipe of SURVEY.md
section 8(d) and BASELINE.md, so ``uniform_graph`` yields exactly ``oracle.synth_graph``'s
instance (tests/test_synth.py) -- and H with a CPU ``torch.Generator().manual_seed(seed)``.
Sorting and de-duplicating on the host (numpy's vectorised sort: ~10 s for products-synth's
124 M keys) also keeps generation independent of how processes share a GPU: the round-2 device
generator (torch.unique on the GPU) stalled for minutes when 8 ranks time-sliced one device.
This is input synthesis, not part of the measured path.
"""

from __future__ import annotations

import os

import numpy as np
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


def _csr_from_pairs(src, dst, n: int, device):
    """Symmetrised, de-duplicated, self-loop-free int32 CSR of the (src, dst) pairs: the
    pattern of A + A^T with data := 1, setdiag(0), eliminate_zeros (the reference's
    ``standardize`` semantics without LCC, sparsegraph.py:191-222), columns sorted in each row.
    Returned as torch tensors on ``device``."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    key = np.concatenate([src * n + dst, dst * n + src])
    del src, dst, keep
    key.sort()  # vectorised (x86-simd-sort) quicksort: ~3 s for 124 M int64 keys
    if key.size:
        first = np.empty(key.size, dtype=bool)
        first[0] = True
        np.not_equal(key[1:], key[:-1], out=first[1:])
        key = key[first]
        del first
    row = key // n
    col = (key - row * n).astype(np.int32)
    del key
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(row, minlength=n), out=indptr[1:])
    del row
    return (torch.from_numpy(indptr.astype(np.int32)).to(device),
            torch.from_numpy(col).to(device))


def uniform_graph(n: int, m: int, seed: int, device="cuda"):
    """CSR (indptr int32 [n+1], indices int32 [nnz]) of SURVEY.md 8(d)'s uniform graph: m pairs
    (src, dst) from ``numpy.random.default_rng(seed)`` (src first, then dst), symmetrised, no
    self loops, duplicates merged.  Identical to ``oracle.synth_graph(n, m, seed)``."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, size=m, dtype=np.int64)
    dst = rng.integers(0, n, size=m, dtype=np.int64)
    return _csr_from_pairs(src, dst, n, device)


def chung_lu_graph(n: int, m: int, seed: int, exponent: float = 3.2, device="cuda"):
    """Power-law graph (Chung-Lu): endpoints drawn with probability proportional to
    w_i = (i + 1)^(-1/(exponent-1)) (inverse-CDF sampling), node ids permuted so hubs are not
    all at low indices, then the same symmetrise / de-duplicate / no-self-loop steps as
    ``uniform_graph``.  Exponent 3.2 gives a largest degree of ~20k at products scale (the real
    ogbn-products: ~17k, mean ~50)."""
    rng = np.random.default_rng(seed)
    w = np.arange(1, n + 1, dtype=np.float64) ** (-1.0 / (exponent - 1.0))
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    # numpy's searchsorted semantics (first i with cdf[i] >= u) on torch's threads: the same
    # indices, ~10x faster for 124 M lookups
    u = torch.from_numpy(rng.random((2, m)))
    ends = torch.searchsorted(torch.from_numpy(cdf), u.reshape(-1)).reshape(2, m).numpy()
    del u
    ends = np.minimum(ends, n - 1)
    perm = rng.permutation(n)
    return _csr_from_pairs(perm[ends[0]], perm[ends[1]], n, device)


def community_graph(n: int, m: int, seed: int, block: int = 4096, p_in: float = 0.9,
                    device="cuda"):
    """Graph with gather locality: the source of each of the m pairs is uniform; with
    probability p_in its destination is uniform inside the source's community (``block``
    consecutive node ids), otherwise uniform over all nodes.  Then the same symmetrise /
    de-duplicate / no-self-loop steps as ``uniform_graph``.  A community's rows of an
    F = 100 fp32 Z are 1.6 MB, so the rows a wave front gathers stay in L2."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, size=m, dtype=np.int64)
    far = rng.integers(0, n, size=m, dtype=np.int64)
    near = np.minimum(src // block * block + rng.integers(0, block, size=m), n - 1)
    dst = np.where(rng.random(m) < p_in, near, far)
    del far, near
    return _csr_from_pairs(src, dst, n, device)


def real_graph(name: str, device="cuda"):
    """CSR of a dataset the reference ships, standardized as its SparseGraph does."""
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = np.load(os.path.join(root, "tests", "golden", name + ".npz"), allow_pickle=False)
    indptr = torch.from_numpy(d["adj_indptr"].astype(np.int32)).to(device)
    indices = torch.from_numpy(d["adj_indices"].astype(np.int32)).to(device)
    return indptr, indices


def _make(workload: str, device):
    if workload in REAL:
        return real_graph(REAL[workload], device=device)
    n, m = CONFIGS[workload][:2]
    if workload in POWERLAW:
        return chung_lu_graph(n, m, SEEDS[workload], device=device)
    if workload in LOCAL:
        return community_graph(n, m, SEEDS[workload], device=device)
    return uniform_graph(n, m, SEEDS.get(workload, 0), device=device)


def graph_for(workload: str, device="cuda"):
    """The workload's CSR (indptr, indices) on ``device``.  With PPNP_SYNTH_CACHE naming a
    directory (the GPU test session sets one, so the products-scale tests and their child ranks
    draw the 124 M-key graph once instead of once per module and rank), the int32 arrays are
    kept there as ``<workload>.npz`` -- written to a temporary name and renamed, so concurrent
    ranks never read a partial file -- and reloaded; the arrays are the generator's own either
    way.  The bench never sets it."""
    cache = os.environ.get("PPNP_SYNTH_CACHE")
    if not cache:
        return _make(workload, device)
    path = os.path.join(cache, f"{workload}.npz")
    if os.path.exists(path):
        with np.load(path, allow_pickle=False) as z:
            return (torch.from_numpy(z["indptr"]).to(device),
                    torch.from_numpy(z["indices"]).to(device))
    indptr, indices = _make(workload, "cpu")
    os.makedirs(cache, exist_ok=True)
    tmp = f"{path}.{os.getpid()}.tmp.npz"
    np.savez(tmp, indptr=indptr.numpy(), indices=indices.numpy())
    os.replace(tmp, path)
    return indptr.to(device), indices.to(device)


def features(n: int, f: int, dtype=torch.float32, device="cuda", seed: int = 0):
    """H ~ N(0, 1): fp32 from a CPU ``torch.Generator().manual_seed(seed)``,
    then stored as ``dtype`` on ``device``."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, f, generator=g, dtype=torch.float32).to(device=device, dtype=dtype)
