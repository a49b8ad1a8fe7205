"""CPU oracle for the APPNP propagation path -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product path
(``ppnp_amd``) never imports it and has no CPU fallback.

It restates, in numpy/scipy (fp64) and torch.sparse (fp32 CPU baseline), the reference
operator that the HIP path replaces:

* ``calc_a_hat``      -- /root/reference/helpers.py:58-66  (A+I, weighted row-sum degree,
                         ``sym``  D^-1/2 (A+I) D^-1/2   or   ``rw``  D^-1 (A+I))
* ``compute_ppr``     -- /root/reference/helpers.py:68-71  (dense alpha (I-(1-alpha)A_hat)^-1)
* ``appnp_propagate`` -- the K-truncated Neumann series of compute_ppr:
                         Z_0 = H, Z_{k+1} = (1-alpha) A_hat Z_k + alpha H
* ``ppnp_forward``    -- /root/reference/model.py:61-67 propagation step ``ppr[idx] @ H``
* ``standardize``     -- /root/reference/ppnp/data/sparsegraph.py:191-222 (+ helpers 300-395)
* ``synth_graph``     -- the seeded uniform generator of SURVEY.md section 8(d)
* ``edge_keep_mask``  -- the counter-hash edge-dropout mask the HIP kernel uses (no reference
                         oracle exists for edge dropout; this pins the
                         device mask bit-for-bit instead)

Parity pin: ``tests/test_oracle.py`` checks every function above against the golden vectors
in ``tests/golden/*.npz``, which ``tests/golden/make_golden.py`` produced by importing the
reference's own ``helpers``/``model``/``SparseGraph`` in the build container.
"""

from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.csgraph as csgraph

# --------------------------------------------------------------------------------------
# Operator construction (helpers.py:58-66)
# --------------------------------------------------------------------------------------


def _merge_self_loops(indptr, indices, data, n):
    """A + I on CSR arrays, scipy-canonical: sorted columns, diagonal merged (a_ii + 1),
    entries whose value is exactly 0 pruned (scipy's csr_binop_csr drops zero results).
    Follows helpers.py:59 ``adj + sp.eye(adj.shape[0])`` (fp32 + fp64 -> fp64)."""
    indptr = np.asarray(indptr, dtype=np.int64)
    indices = np.asarray(indices, dtype=np.int64)
    data = np.asarray(data, dtype=np.float64)
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
    same_row = rows[1:] == rows[:-1]
    if not np.any((indices[1:] <= indices[:-1]) & same_row):
        return _merge_self_loops_sorted(indptr, indices, data, rows, n)
    # canonicalise (sum duplicates, sort) exactly as scipy would before the add
    coo = sp.coo_matrix((data, (rows, indices)), shape=(n, n))
    coo.sum_duplicates()
    r = np.concatenate([coo.row.astype(np.int64), np.arange(n, dtype=np.int64)])
    c = np.concatenate([coo.col.astype(np.int64), np.arange(n, dtype=np.int64)])
    v = np.concatenate([coo.data.astype(np.float64), np.ones(n, dtype=np.float64)])
    key = r * n + c
    order = np.argsort(key, kind="stable")
    key, v = key[order], v[order]
    uniq, start = np.unique(key, return_index=True)
    vsum = np.add.reduceat(v, start)  # a_ii + 1 where the diagonal existed
    keep = vsum != 0.0
    uniq, vsum = uniq[keep], vsum[keep]
    rr, cc = uniq // n, uniq % n
    out_ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(out_ptr, rr + 1, 1)
    return np.cumsum(out_ptr), cc, vsum, rr


def _merge_self_loops_sorted(indptr, indices, data, rows, n):
    """``_merge_self_loops`` for a CSR whose columns already increase strictly in every row
    (no duplicates to sum): the same arrays without the sorts -- the diagonal entry of row i
    becomes a_ii + 1 in place, or a 1 inserted after the row's entries left of column i; then
    the exact zeros are pruned.  Linear time, so the products-scale parity tests do not spend
    minutes sorting 126 M keys that are sorted already."""
    nnz = indices.size
    on_diag = indices == rows
    has_diag = np.zeros(n, dtype=bool)
    has_diag[rows[on_diag]] = True
    ins = ~has_diag  # rows that get an inserted 1
    out_ptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.diff(indptr) + ins, out=out_ptr[1:])
    # an entry moves right by one when its row gets an insert to its left
    pos = out_ptr[rows] + (np.arange(nnz, dtype=np.int64) - indptr[rows])
    pos += (indices > rows) & ins[rows]
    left = np.bincount(rows[indices < rows], minlength=n).astype(np.int64)
    total = int(out_ptr[-1])
    cc = np.empty(total, dtype=np.int64)
    v = np.empty(total, dtype=np.float64)
    rr = np.empty(total, dtype=np.int64)
    cc[pos], rr[pos] = indices, rows
    v[pos] = np.where(on_diag, data + 1.0, data)
    ins_rows = np.flatnonzero(ins)
    ipos = out_ptr[ins_rows] + left[ins_rows]
    cc[ipos], rr[ipos], v[ipos] = ins_rows, ins_rows, 1.0
    keep = v != 0.0
    if not keep.all():
        cc, v, rr = cc[keep], v[keep], rr[keep]
        out_ptr = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(np.bincount(rr, minlength=n), out=out_ptr[1:])
    return out_ptr, cc, v, rr


def calc_a_hat(adj, mode: str = "sym"):
    """Restates helpers.py:58-66.  ``adj`` is a scipy CSR (any float dtype).

    Returns a scipy CSR in fp64 with sorted indices.  Degree D_i is the weighted row sum of
    A+I in column order (helpers.py:60); sym value = (dinv_i * a_ij) * dinv_j with
    dinv = 1/sqrt(D) (helpers.py:61-63, evaluated left-to-right as scipy does); rw value =
    (1/D_i) * a_ij (helpers.py:64-66)."""
    adj = sp.csr_matrix(adj)
    n = adj.shape[0]
    ptr, col, val, row = _merge_self_loops(adj.indptr, adj.indices, adj.data, n)
    # sequential per-row sum in column order (scipy: csr_matvec with a ones vector)
    deg = np.zeros(n, dtype=np.float64)
    nonempty = ptr[1:] > ptr[:-1]
    if nonempty.any():
        deg[nonempty] = np.add.reduceat(val, ptr[:-1][nonempty])
    if mode == "sym":
        dinv = 1.0 / np.sqrt(deg)
        out = (dinv[row] * val) * dinv[col]
    elif mode == "rw":
        dinv = 1.0 / deg
        out = dinv[row] * val
    else:
        raise ValueError(f"unknown mode {mode!r}")
    return sp.csr_matrix((out, col, ptr), shape=(n, n))


def compute_ppr(adj, alpha: float, mode: str = "sym") -> np.ndarray:
    """Restates helpers.py:68-71: alpha * inv(I - (1-alpha) A_hat), dense fp64."""
    a_hat = calc_a_hat(adj, mode)
    n = a_hat.shape[0]
    inner = np.eye(n) - (1.0 - alpha) * a_hat.toarray()
    return alpha * np.linalg.inv(inner)


# --------------------------------------------------------------------------------------
# Propagation (the APPNP loop)
# --------------------------------------------------------------------------------------


def appnp_propagate(a_hat, H, K: int, alpha: float, p_drop: float = 0.0, seed: int = 0):
    """Z_0 = H; Z_{k+1} = (1-alpha) * (M_k o A_hat) Z_k + alpha H, fp64.

    M_k is the edge-keep mask of ``edge_keep_mask`` scaled by 1/(1-p) (p_drop > 0 only)."""
    a_hat = sp.csr_matrix(a_hat, dtype=np.float64)
    H = np.asarray(H, dtype=np.float64)
    Z = H.copy()
    for k in range(K):
        if p_drop > 0.0:
            M = masked_operator(a_hat, k, p_drop, seed)
        else:
            M = a_hat
        Z = (1.0 - alpha) * (M @ Z) + alpha * H
    return Z


def appnp_backward(a_hat, dZ, K: int, alpha: float, p_drop: float = 0.0, seed: int = 0):
    """Adjoint of ``appnp_propagate`` w.r.t. H (dH = J^T dZ), fp64.

    G_K = dZ; dH = alpha G_K; G_k = (1-alpha) M_k^T G_{k+1} (k = K-1..0); dH += alpha G_k for
    k >= 1 and dH += G_0 at the end."""
    a_hat = sp.csr_matrix(a_hat, dtype=np.float64)
    G = np.asarray(dZ, dtype=np.float64).copy()
    if K == 0:
        return G
    dH = alpha * G
    for k in range(K - 1, -1, -1):
        M = masked_operator(a_hat, k, p_drop, seed) if p_drop > 0.0 else a_hat
        G = (1.0 - alpha) * (M.T @ G)
        dH = dH + (alpha * G if k >= 1 else G)
    return dH


def appnp_closed_form(a_hat, H, K: int, alpha: float):
    """Z_K = [alpha sum_{k<K} ((1-alpha)A)^k + ((1-alpha)A)^K] H."""
    a_hat = sp.csr_matrix(a_hat, dtype=np.float64)
    H = np.asarray(H, dtype=np.float64)
    term = H.copy()
    acc = alpha * term if K > 0 else np.zeros_like(H)
    for k in range(1, K):
        term = (1.0 - alpha) * (a_hat @ term)
        acc = acc + alpha * term
    term = (1.0 - alpha) * (a_hat @ term) if K > 0 else term
    return acc + term


def ppnp_forward(ppr, H, idx=None, ppr_sub=None):
    """Restates the propagation step of model.py:61-67 (``ppr[idx] @ H`` / ``ppr @ H``)."""
    if idx is not None:
        return np.asarray(ppr)[np.asarray(idx)] @ H
    if ppr_sub is not None:
        return np.asarray(ppr_sub) @ H
    raise Exception()


# --------------------------------------------------------------------------------------
# CPU baseline: the "reference's own CPU torch.sparse.mm path" named by north_star
# --------------------------------------------------------------------------------------


def torch_sparse_operator(a_hat):
    """fp32 torch CSR tensor of A_hat (CPU)."""
    import torch

    a = sp.csr_matrix(a_hat)
    return torch.sparse_csr_tensor(
        torch.from_numpy(a.indptr.astype(np.int64)),
        torch.from_numpy(a.indices.astype(np.int64)),
        torch.from_numpy(a.data.astype(np.float32)),
        size=a.shape,
    )


def appnp_propagate_torch_cpu(a_csr_t, H_t, K: int, alpha: float):
    """fp32 CPU torch.sparse.mm APPNP loop (SURVEY.md section 8(d) CPU baseline (i))."""
    import torch

    Z = H_t
    aH = alpha * H_t
    for _ in range(K):
        Z = torch.sparse.mm(a_csr_t, Z).mul_(1.0 - alpha).add_(aH)
    return Z


# --------------------------------------------------------------------------------------
# Edge dropout mask (counter hash; identical arithmetic to ppnp_amd/csrc/appnp_common.h)
# --------------------------------------------------------------------------------------

_M64 = (1 << 64) - 1
_GOLDEN = 0x9E3779B97F4A7C15


def _splitmix64(x):
    x = (x + _GOLDEN) & _M64 if isinstance(x, int) else (x + np.uint64(_GOLDEN))
    if isinstance(x, int):
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
        return x ^ (x >> 31)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def drop_threshold(p_drop: float) -> int:
    """24-bit threshold: an edge is dropped when its 24-bit hash < threshold.  p crosses the
    C ABI as a float, so the threshold is taken from float32(p) (0.3 -> 5033165, where the
    double 0.3 would give 5033164)."""
    p = float(np.float32(min(max(p_drop, 0.0), 1.0)))
    return int(p * (1 << 24))


def edge_keep_mask(rows, cols, k: int, p_drop: float, seed: int):
    """Boolean keep-mask for edges (row, col) at iteration k.  Keyed on (seed, k, row, col)
    only, so it is independent of partitioning and of the order edges are visited."""
    with np.errstate(over="ignore"):
        base = _splitmix64((seed + (k + 1) * _GOLDEN) & _M64)
        x = (np.asarray(rows, dtype=np.uint64) << np.uint64(32)) | np.asarray(
            cols, dtype=np.uint64
        )
        h = _splitmix64(x ^ np.uint64(base))
    u24 = (h >> np.uint64(40)).astype(np.int64)
    return u24 >= drop_threshold(p_drop)


def masked_operator(a_hat, k: int, p_drop: float, seed: int):
    """(M_k o A_hat) / (1-p) with the device mask (fp64 values; the 1/(1-p) factor is the
    fp32 value the kernel uses)."""
    a = sp.csr_matrix(a_hat, dtype=np.float64)
    n = a.shape[0]
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(a.indptr))
    keep = edge_keep_mask(rows, a.indices, k, p_drop, seed)
    scale = float(np.float32(1.0) / (np.float32(1.0) - np.float32(p_drop)))
    data = np.where(keep, a.data * scale, 0.0)
    return sp.csr_matrix((data, a.indices, a.indptr), shape=a.shape)


# --------------------------------------------------------------------------------------
# Graph preprocessing (sparsegraph.py) and synthetic graphs
# --------------------------------------------------------------------------------------


def standardize(adj, select_lcc: bool = True):
    """Restates SparseGraph.standardize (sparsegraph.py:191-222) on the adjacency only:
    unweighted (135-138), undirected (112-128), no self-loops (380-395), LCC (355-377).
    Returns (adj_csr_fp32, kept_node_index)."""
    a = sp.csr_matrix(adj, dtype=np.float32)
    a.sum_duplicates()
    a.data = np.ones_like(a.data)
    a = ((a + a.T) > 0).astype(np.float32).tocsr()
    a.setdiag(0)
    a.eliminate_zeros()
    keep = np.arange(a.shape[0])
    if select_lcc:
        _, comp = csgraph.connected_components(a)
        sizes = np.bincount(comp)
        big = np.argsort(sizes)[::-1][:1]
        keep = np.nonzero(np.isin(comp, big))[0]
        a = a[keep][:, keep].tocsr()
    a.sort_indices()
    return a, keep


def synth_graph(n_nodes: int, n_edges: int, seed: int):
    """Uniform random undirected graph of SURVEY.md section 8(d): m (src, dst) pairs drawn
    uniformly, A = A + A^T, data := 1, no self loops.  Isolated nodes are kept."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n_nodes, size=n_edges, dtype=np.int64)
    dst = rng.integers(0, n_nodes, size=n_edges, dtype=np.int64)
    a = sp.coo_matrix(
        (np.ones(n_edges, dtype=np.float32), (src, dst)), shape=(n_nodes, n_nodes)
    ).tocsr()
    a = a + a.T
    a.data = np.ones_like(a.data)
    a.setdiag(0)
    a.eliminate_zeros()
    a.sort_indices()
    return a.astype(np.float32)
