"""Model surface: the reference's PPNP plus the APPNP drop-in on the HIP propagation path.

Mirrors /root/reference/model.py:
  CustomLinear  model.py:13-38   (weight laid out (in, out), fan_out Kaiming init, addmm)
  PPNP          model.py:41-67   (dense precomputed PPR; kept unchanged for callers that pass
                                  ``ppr=``, e.g. batch-main.py:140-146)
  APPNP         new              same constructor/forward/get_norm surface as PPNP, but the
                                  propagation ``ppr[idx] @ H`` (model.py:63) is computed as
                                  Z_K[idx] by K fused HIP SpMM launches over A_hat built on
                                  the GPU (helpers.py:58-66) -- no N x N matrix exists.
"""

from __future__ import annotations

import math

import numpy as np
import torch
from torch import nn

from .graph import Graph
from .ops import propagate
from .sparse import SparseFeatures, sparse_linear


class CustomLinear(nn.Module):
    """model.py:13-38."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.Tensor(in_features, out_features))
        if bias:
            self.bias = nn.Parameter(torch.Tensor(out_features))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.kaiming_uniform_(self.weight, mode="fan_out", a=math.sqrt(5))
        if self.bias is not None:
            _, fan_out = nn.init._calculate_fan_in_and_fan_out(self.weight)
            bound = 1 / math.sqrt(fan_out)
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, input):
        if self.bias is None:
            return input @ self.weight
        return torch.addmm(self.bias, input, self.weight)


def _encoder(n_features, n_classes, hidden_dim, drop_prob, bias):
    # model.py:46-52
    return nn.Sequential(
        nn.Dropout(drop_prob),
        CustomLinear(n_features, hidden_dim, bias=bias),
        nn.ReLU(inplace=True),
        nn.Dropout(drop_prob),
        nn.Linear(hidden_dim, n_classes, bias=bias),
    )


def _encode(encoder, X, training):
    """encoder(X) (model.py:46-52); a SparseFeatures X takes the sparse path: the input
    Dropout + CustomLinear become one dropout-SpMM on the GPU (ppnp_amd/sparse.py)."""
    if not isinstance(X, SparseFeatures):
        return encoder(X)
    lin = encoder[1]
    p = encoder[0].p if training else 0.0
    seed = int(torch.randint(0, 2**62, (1,)).item()) if p > 0 else 0
    h = sparse_linear(X, lin.weight, p, seed)
    if lin.bias is not None:
        h = h + lin.bias
    return encoder[4](encoder[3](encoder[2](h)))


class PPNP(nn.Module):
    """model.py:41-67, unchanged semantics (dense ``ppr`` buffer)."""

    def __init__(self, n_features, n_classes, ppr, hidden_dim=64, drop_prob=0.5, bias=False):
        super().__init__()
        self.encoder = _encoder(n_features, n_classes, hidden_dim, drop_prob, bias)
        self.register_buffer("ppr", ppr)
        self._reg_params = list(self.encoder[1].parameters())

    def get_norm(self):
        return sum((torch.sum(param ** 2) for param in self._reg_params))

    def forward(self, X, idx=None, ppr=None):
        if idx is not None:
            return self.ppr[idx] @ _encode(self.encoder, X, self.training)
        elif ppr is not None:
            return ppr @ _encode(self.encoder, X, self.training)
        else:
            raise Exception()


class APPNP(nn.Module):
    """Drop-in for PPNP on the gfx950 propagation path.

    ``adj`` is the (standardized) adjacency as a scipy sparse matrix, exactly what the
    reference passes to ``compute_ppr`` (main.py:106).  It is stored as CSR buffers so
    ``.cuda()`` / ``.to()`` move it like the reference's ``ppr`` buffer; A_hat is built on
    the device at the first forward on that device.

    forward(X, idx)      -> Z_K[idx]          (model.py:63 semantics, PPR truncated at K)
    forward(X, ppr=P)    -> P @ encoder(X)    (model.py:65, batch mode, dense P unchanged)
    forward(X)           -> raises Exception() (model.py:66-67)

    ``edge_drop`` > 0 applies edge dropout inside the propagation kernel in training mode.
    """

    def __init__(self, n_features, n_classes, adj, alpha=0.1, K=10, hidden_dim=64,
                 drop_prob=0.5, bias=False, mode="sym", edge_drop=0.0, dtype=torch.float32):
        super().__init__()
        import scipy.sparse as sp

        self.encoder = _encoder(n_features, n_classes, hidden_dim, drop_prob, bias)
        self._reg_params = list(self.encoder[1].parameters())
        a = sp.csr_matrix(adj)
        if not a.has_sorted_indices:
            a = a.copy()
            a.sort_indices()
        self.n_nodes = int(a.shape[0])
        self.register_buffer("adj_indptr", torch.from_numpy(a.indptr.astype(np.int32)))
        self.register_buffer("adj_indices", torch.from_numpy(a.indices.astype(np.int32)))
        self.register_buffer("adj_data", torch.from_numpy(a.data.astype(np.float32)))
        self.n_classes = int(n_classes)
        self.alpha = float(alpha)
        self.K = int(K)
        self.mode = mode
        self.edge_drop = float(edge_drop)
        self.prop_dtype = dtype
        self.ppr_topk = None  # batch-main.py:113-117 sparsification of the lazy ``ppr``
        self._graph = None
        self._ppr = None  # (device, topk, dense Pi) built on first access of ``ppr``
        self._memo = None  # (key, Z_K) of the last no-grad eval-mode propagation
        self.memo_hits = 0

    def graph(self) -> Graph:
        dev = self.adj_indptr.device
        if self._graph is None or self._graph.device != dev:
            # the propagation carries n_classes columns: the source-blocked copy of A_hat is
            # built only when that width takes the split-row path (graph.splits_rows)
            self._graph = Graph.from_csr(self.adj_indptr, self.adj_indices, self.adj_data,
                                         self.n_nodes, mode=self.mode, device=dev,
                                         transpose=True, features=self.n_classes,
                                         dtype=self.prop_dtype)
        return self._graph

    # K of the series behind ``ppr``: (1-alpha)^K below fp32 resolution of the rows
    PPR_TOL = 1e-7

    @property
    def ppr(self) -> torch.Tensor:
        """The dense PPR matrix Pi = alpha (I - (1-alpha) A_hat)^-1 (helpers.py:68-71), for
        callers that index the reference model's ``ppr`` buffer directly -- batch-main.py:140
        ``model.ppr[idx_batch]``.  Built lazily on the graph's device from the K-step series
        of one-hot columns (ppr.ppr_rows; K chosen so (1-alpha)^K <= PPR_TOL), with the
        column-wise top-k of batch-main.py:115-116 applied when ``ppr_topk`` is set.  N x N:
        small graphs only, exactly as in the reference."""
        from .ppr import batch_topk_quirk, dense_ppr

        g = self.graph()
        key = (g.device, self.ppr_topk)
        if self._ppr is None or self._ppr[0] != key:
            K = int(math.ceil(math.log(self.PPR_TOL) / math.log(1.0 - self.alpha)))
            P = (batch_topk_quirk(g, self.ppr_topk, K, self.alpha) if self.ppr_topk
                 else dense_ppr(g, K, self.alpha))
            self._ppr = (key, P)
        return self._ppr[1]

    def get_norm(self):
        return sum((torch.sum(param ** 2) for param in self._reg_params))

    def propagate(self, H):
        p = self.edge_drop if self.training else 0.0
        seed = int(torch.randint(0, 2**62, (1,)).item()) if p > 0 else 0
        Hc = H.to(self.prop_dtype)
        return propagate(self.graph(), Hc, self.K, self.alpha, p, seed).to(H.dtype)

    def _memo_key(self, X):
        """Identity of everything Z_K depends on, for deterministic (eval, no-grad) calls:
        main.py evaluates the stopping and validation sets with two forwards of the same X
        and weights (main.py:138, 145); the second reuses the first's Z_K.

        The key holds the tensors themselves (strong references) and their versions: a hit
        needs the SAME tensor objects (``is``), unchanged in place (an optimizer step,
        load_state_dict or an edited X bumps ``_version``).  A new X that the caching
        allocator happens to place at a just-freed address is a different object, so it can
        never match a stale entry."""
        if self.training or torch.is_grad_enabled():
            return None
        xs = (X.indptr, X.indices, X.data) if isinstance(X, SparseFeatures) else (X,)
        state = (*xs, *self.parameters(), *self.buffers())
        return (state, tuple(t._version for t in state), self.K, self.alpha, self.mode,
                self.prop_dtype)

    @staticmethod
    def _memo_match(a, b) -> bool:
        return (a is not None and b is not None and len(a[0]) == len(b[0])
                and all(x is y for x, y in zip(a[0], b[0])) and a[1:] == b[1:])

    def forward(self, X, idx=None, ppr=None):
        """X: dense tensor (as the reference) or ppnp_amd.SparseFeatures (CSR on the GPU)."""
        if idx is not None:
            key = self._memo_key(X)
            if key is not None and self._memo is not None and self._memo_match(self._memo[0],
                                                                               key):
                self.memo_hits += 1
                return self._memo[1][idx]
            Z = self.propagate(_encode(self.encoder, X, self.training))
            self._memo = (key, Z) if key is not None else None
            return Z[idx]
        elif ppr is not None:
            return ppr @ _encode(self.encoder, X, self.training)
        else:
            raise Exception()
