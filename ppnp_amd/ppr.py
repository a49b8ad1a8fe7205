"""Rows of the PPR matrix for minibatch training, without the dense N x N inverse.

Reference: batch-main.py:111-117 forms the dense ``compute_ppr`` (helpers.py:68-71),
sparsifies it with ``topk`` and indexes ``model.ppr[idx_batch]`` per minibatch
(batch-main.py:140-146).  Here the rows come from the APPNP propagation of one-hot columns:

* sym:  Pi = alpha (I - (1-alpha) A_hat)^-1 is symmetric (A_hat is), so
        Pi[idx, :] = (Pi e_idx)^T = APPNP_K(E_idx)^T
* rw:   Pi^T = D Pi D^-1 (A symmetric), so Pi[i, :] = D * APPNP_K(e_i) / d_i

with E_idx the N x B one-hot matrix; the K-step series converges to the exact rows
(``tests/test_gpu_parity.py::test_ppr_rows_match_compute_ppr``).  The propagation is the
same fused HIP kernel, with F = B columns.

``batch_topk_quirk`` reproduces batch-main.py:115-116 literally, including its broadcasting
quirk (``ppr < thresh[:, -1]`` compares entry (i, j) with the threshold of row j, so each
COLUMN keeps its top k).  It needs every row's k-th largest value,
i.e. all of Pi, which it streams in column chunks: O(N^2) work, small graphs only -- exactly
the reference's own limit.
"""

from __future__ import annotations

import torch

from .graph import Graph
from .ops import propagate_forward


def _degrees(graph: Graph):
    """D_i of A+I from the stored inverse degrees (rw: dinv = 1/D)."""
    _, _, _, dinv = graph.csr()
    return 1.0 / dinv


def ppr_columns(graph: Graph, idx: torch.Tensor, K: int = 10, alpha: float = 0.1):
    """Pi[:, idx] (N x B, fp32) = APPNP_K of the one-hot columns of idx."""
    idx = torch.as_tensor(idx, device=graph.device).long()
    B = int(idx.numel())
    E = torch.zeros(graph.n, B, dtype=torch.float32, device=graph.device)
    E[idx, torch.arange(B, device=graph.device)] = 1.0
    return propagate_forward(graph, E, K, alpha)


def ppr_rows(graph: Graph, idx, K: int = 10, alpha: float = 0.1, topk: int | None = None):
    """Pi[idx, :] as a dense B x N fp32 tensor (entries outside each row's top-k zeroed when
    ``topk`` is given)."""
    if not graph.symmetric:
        raise ValueError("ppr_rows needs an undirected graph (symmetric A)")
    idx = torch.as_tensor(idx, device=graph.device).long()
    cols = ppr_columns(graph, idx, K, alpha)  # N x B
    if graph.mode == "sym":
        rows = cols.t().contiguous()
    else:  # rw: Pi[i, :] = D * Pi[:, i] / d_i
        deg = _degrees(graph).float()
        rows = (cols * deg[:, None]).t() / deg[idx][:, None]
        rows = rows.contiguous()
    if topk is not None and topk < graph.n:
        thr = rows.topk(topk, dim=1).values[:, -1:]
        rows = torch.where(rows >= thr, rows, torch.zeros_like(rows))
    return rows


def dense_ppr(graph: Graph, K: int = 10, alpha: float = 0.1, chunk: int = 1024) -> torch.Tensor:
    """All of Pi (N x N fp32), row chunks of ``ppr_rows``: the truncated series of
    compute_ppr (helpers.py:68-71).  Small graphs only (materialises N x N)."""
    n = graph.n
    if n * n > 2**31:
        raise ValueError("dense_ppr materialises N x N: N too large")
    P = torch.empty(n, n, dtype=torch.float32, device=graph.device)
    for s in range(0, n, chunk):
        idx = torch.arange(s, min(n, s + chunk), device=graph.device)
        P[s:s + len(idx)] = ppr_rows(graph, idx, K, alpha)
    return P


def batch_topk_quirk(graph: Graph, topk: int, K: int = 10, alpha: float = 0.1,
                     chunk: int = 1024) -> torch.Tensor:
    """Dense sparsified Pi exactly as batch-main.py:115-116 builds it:
    ``thresh, _ = ppr.topk(k, axis=-1); ppr[ppr < thresh[:, -1]] = 0`` (column-wise top-k
    through broadcasting).  Small graphs only (materialises N x N)."""
    P = dense_ppr(graph, K, alpha, chunk)
    thresh, _ = P.topk(topk, dim=-1)
    P[P < thresh[:, -1]] = 0
    return P
