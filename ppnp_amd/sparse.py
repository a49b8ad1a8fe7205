"""Sparse encoder input: Dropout(X) @ W1 on a device CSR X.

The reference densifies the attribute matrix (main.py:90-91) although it is 1.76 % dense on
Cora-ML, and then spends most of a CPU epoch drawing the dropout mask over all N x F_in
entries (model.py:47).  ``SparseFeatures`` keeps X as a CSR on the GPU;
``sparse_linear`` computes ``dropout(X) @ W`` with the gather SpMM kernel of the propagation
path (``appnp_spmm``): rows of X gather rows of W, the dropout mask is the per-entry counter
hash, kept entries are scaled by 1/(1-p).  The backward ``dW = dropout(X)^T @ dY`` runs the
same kernel over the transposed CSR (built once, ``appnp_csr_transpose``) with the
transposed hash key, so it replays the forward mask exactly.

Dropout on a sparse X only touches stored entries; zeros stay zero either way, so the
distribution of dropout(X) @ W is the reference's.  The random stream differs from torch's.
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib


def _vp(t):
    return C.c_void_p(t.data_ptr()) if t is not None and t.numel() > 0 else None


def _stream(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class SparseFeatures:
    """A CSR feature matrix X (N x F_in) held on one GPU, with its transpose."""

    def __init__(self, indptr, indices, data, shape, device="cuda"):
        self.device = torch.device(device)
        self.shape = (int(shape[0]), int(shape[1]))
        self.indptr = torch.as_tensor(indptr).to(self.device, torch.int32).contiguous()
        self.indices = torch.as_tensor(indices).to(self.device, torch.int32).contiguous()
        self.data = torch.as_tensor(data).to(self.device, torch.float32).contiguous()
        self._t = None

    @classmethod
    def from_scipy(cls, X, device="cuda"):
        X = sp.csr_matrix(X, dtype=np.float32)
        X.sort_indices()
        return cls(X.indptr.astype(np.int32), X.indices.astype(np.int32), X.data, X.shape,
                   device)

    @property
    def nnz(self):
        return int(self.indices.numel())

    def transpose(self):
        """(indptr, indices, data) of X^T on the device (cached)."""
        if self._t is None:
            lib = _lib.load()
            h = C.c_void_p()
            with torch.cuda.device(self.device):
                rc = lib.appnp_csr_transpose(_vp(self.indptr), _vp(self.indices), _vp(self.data),
                                             self.shape[0], self.shape[1], self.nnz,
                                             _stream(self.device), C.byref(h))
            _lib.check("appnp_csr_transpose", rc)
            try:
                ip = torch.empty(self.shape[1] + 1, dtype=torch.int32, device=self.device)
                ix = torch.empty(self.nnz, dtype=torch.int32, device=self.device)
                dv = torch.empty(self.nnz, dtype=torch.float32, device=self.device)
                with torch.cuda.device(self.device):
                    _lib.check("appnp_csr_copy", lib.appnp_csr_copy(h, _vp(ip), _vp(ix), None,
                                                                   _stream(self.device)))
                    if self.nnz:
                        _lib.check("appnp_csr_values",
                                   lib.appnp_csr_values(h, _vp(dv), _stream(self.device)))
                torch.cuda.current_stream(self.device).synchronize()
            finally:
                lib.appnp_csr_destroy(h)
            self._t = (ip, ix, dv)
        return self._t

    def to_dense(self):
        return torch.sparse_csr_tensor(self.indptr.long(), self.indices.long(), self.data,
                                       size=self.shape).to_dense()


def spmm(indptr, indices, data, rows, cols, B, p_drop=0.0, seed=0, transposed_key=False,
         out=None):
    """C = (M o A) @ B through ``appnp_spmm`` (fp32)."""
    if B.dtype != torch.float32 or B.dim() != 2 or B.shape[0] != cols:
        raise ValueError("B must be fp32 [cols, F]")
    if B.shape[1] > 0 and B.stride(1) != 1:
        B = B.contiguous()
    f = int(B.shape[1])
    Cm = torch.empty(rows, f, dtype=torch.float32, device=B.device) if out is None else out
    ld_b = int(B.stride(0)) if B.shape[0] > 1 else f
    ld_c = int(Cm.stride(0)) if Cm.shape[0] > 1 else f
    lib = _lib.load()
    with torch.cuda.device(B.device):
        rc = lib.appnp_spmm(_vp(indptr), _vp(indices), _vp(data), int(rows), int(cols), _vp(B),
                            max(ld_b, f), _vp(Cm), max(ld_c, f), f, float(p_drop),
                            int(seed) & (2**64 - 1), 1 if transposed_key else 0,
                            _stream(B.device))
    _lib.check("appnp_spmm", rc)
    return Cm


class _SparseLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, W, X, p_drop, seed):
        ctx.X, ctx.p_drop, ctx.seed = X, p_drop, seed
        return spmm(X.indptr, X.indices, X.data, X.shape[0], X.shape[1], W.contiguous(),
                    p_drop, seed)

    @staticmethod
    def backward(ctx, dY):
        X = ctx.X
        ip, ix, dv = X.transpose()
        dW = spmm(ip, ix, dv, X.shape[1], X.shape[0], dY.contiguous(), ctx.p_drop, ctx.seed,
                  transposed_key=True)
        return dW, None, None, None


def sparse_linear(X: SparseFeatures, W: torch.Tensor, p_drop: float = 0.0, seed: int = 0):
    """dropout(X, p) @ W with X a SparseFeatures (W: F_in x F_out, fp32)."""
    return _SparseLinear.apply(W, X, float(p_drop), int(seed))
