"""Device-resident A_hat: the MI355X replacement for helpers.calc_A_hat / compute_ppr.

Reference: /root/reference/helpers.py:58-66 (calc_A_hat) builds A_hat on the host in fp64
scipy; helpers.py:68-71 (compute_ppr) then forms the dense N x N PPR matrix with an O(N^3)
inverse.  Here the CSR of A is copied to the GPU once and ``appnp_graph_create`` builds
A_hat there (fp64 arithmetic, fp32 storage, bit-identical to float32 of the reference).
"""

from __future__ import annotations

import ctypes as C
import itertools
import warnings
import weakref

import numpy as np
import torch

from . import _lib


def _stream_ptr(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None and t.numel() > 0 else None


def remainder_width(n: int, features: int, dtype=torch.float32) -> int:
    """Columns per row (4, 8 or 16) of the source-blocked remainder pass that appnp_propagate
    would use for this shape (appnp_capi.hip remainder_cols), 0 for whole-row gathers: fp32 rows
    of F = 32q + r features with 1 <= r <= 8 and 32 < F <= 256, or narrow rows F <= 16, above the
    latency regime (n > 2^16 rows).  The narrowest width that holds r."""
    if dtype != torch.float32 or n <= (1 << 16) or not 1 <= features <= 256:
        return 0
    if 16 < features <= 32:
        return 0
    r = features % 32 if features > 32 else features
    if features > 32 and r > 8:
        return 0  # beside a main part, 9-16 columns cost their extra line (appnp_capi.hip)
    return next((w for w in (4, 8, 16) if 1 <= r <= w), 0)


def source_block_flags(n: int, features: int, dtype=torch.float32) -> int:
    """The ``mode`` bits of the source-blocked copy for this shape (0: rows gathered whole):
    APPNP_GRAPH_SOURCE_BLOCKS / _SB_W8 / _SB_W16 by ``remainder_width``."""
    w = remainder_width(n, features, dtype)
    return {0: 0, 4: _lib.GRAPH_SOURCE_BLOCKS, 8: _lib.GRAPH_SB_W8, 16: _lib.GRAPH_SB_W16}[w]


def splits_rows(n: int, features: int, dtype=torch.float32) -> bool:
    """Whether appnp_propagate takes the split path for this shape on a graph built with the
    matching source-blocked copy (``remainder_width`` > 0)."""
    return remainder_width(n, features, dtype) > 0


def source_block_layout_of(handle):
    """``Graph.source_block_layout`` for any graph handle (also an appnp_dist engine's)."""
    w, vf, rp = C.c_int(), C.c_int(), C.c_int()
    ent, launches = C.c_int64(), C.c_int64()
    _lib.check("appnp_graph_source_block_layout",
               _lib.load().appnp_graph_source_block_layout(
                   handle, C.byref(w), C.byref(ent), C.byref(vf), C.byref(rp),
                   C.byref(launches)))
    if w.value == 0:
        return None
    return {"width": w.value, "entries": ent.value, "value_free": bool(vf.value),
            "row_passes": rp.value, "launches": launches.value}


def split_layout_of(handle, f: int):
    """``Graph.split_layout`` for any graph handle."""
    fs, rw = C.c_int64(), C.c_int64()
    rc = _lib.load().appnp_split_layout(handle, int(f), C.byref(fs), C.byref(rw))
    if rc == _lib.APPNP_ENOTSUP:
        return None
    _lib.check("appnp_split_layout", rc)
    return fs.value, rw.value


class Graph:
    """A_hat = calc_A_hat(adj, mode) held on one GPU (all rows, or rows [row_lo, row_hi)).

    Build it with :meth:`from_scipy` (host CSR) or :meth:`from_csr` (torch CSR arrays).
    """

    # live graphs by integer key: the torch.library ops (ops.py) take the key, since a custom
    # op's schema cannot carry a Python object
    _registry: "weakref.WeakValueDictionary[int, Graph]" = weakref.WeakValueDictionary()
    _next_key = itertools.count(1)

    @classmethod
    def lookup(cls, key: int) -> "Graph":
        g = cls._registry.get(int(key))
        if g is None or g._h is None:
            raise RuntimeError(f"ppnp_amd: graph key {key} is not a live Graph")
        return g

    def __init__(self, handle, device):
        self._h = handle
        self.key = next(Graph._next_key)
        Graph._registry[self.key] = self
        self.device = torch.device(device)
        lib = _lib.load()
        n, lo, hi, nnz = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        mode, sym = C.c_int(), C.c_int()
        _lib.check(
            "appnp_graph_info",
            lib.appnp_graph_info(self._h, C.byref(n), C.byref(lo), C.byref(hi), C.byref(nnz),
                                 C.byref(mode), C.byref(sym)),
        )
        self.n, self.row_lo, self.row_hi, self.nnz_hat = n.value, lo.value, hi.value, nnz.value
        self.mode = {0: "sym", 1: "rw"}[mode.value]
        self.symmetric = bool(sym.value)

    # -- construction ---------------------------------------------------------------------
    @classmethod
    def from_csr(cls, indptr, indices, data, n, mode="sym", device=None, row_lo=0,
                 row_hi=None, split_local=False, transpose=False, source_blocks=None,
                 features=None, dtype=torch.float32):
        """indptr/indices (int32) and optional data (fp32) of A; tensors or arrays.
        ``transpose=True`` also builds A_hat^T when A_hat is not symmetric (rw mode or a
        directed graph), which the backward needs.  ``source_blocks`` keeps the copy of A_hat
        blocked by source rows that lets fp32 rows of F = 32q + r (r <= 4) features gather q
        cache lines instead of q + 1 (APPNP_GRAPH_SOURCE_BLOCKS).  Default: only when the
        caller names a feature width ``features`` (and storage ``dtype``) that takes that path
        on a full graph above the latency regime (``splits_rows``) -- the copy costs about as
        much memory as the CSR itself, so it is never built on speculation.  The build is
        best-effort: if the copy does not fit, the graph keeps whole-row gathers."""
        if mode not in _lib.NORM:
            raise ValueError(f"mode must be 'sym' or 'rw', got {mode!r}")
        device = torch.device(device if device is not None else "cuda")
        if device.type != "cuda":
            raise ValueError("ppnp_amd.Graph lives on a GPU (no CPU fallback)")
        ip = torch.as_tensor(np.asarray(indptr) if not torch.is_tensor(indptr) else indptr)
        ix = torch.as_tensor(np.asarray(indices) if not torch.is_tensor(indices) else indices)
        ip = ip.to(device=device, dtype=torch.int32).contiguous()
        ix = ix.to(device=device, dtype=torch.int32).contiguous()
        dv = None
        if data is not None:
            d = torch.as_tensor(np.asarray(data) if not torch.is_tensor(data) else data)
            dv = d.to(device=device, dtype=torch.float32).contiguous()
            if bool((dv == 1).all()):
                dv = None  # unweighted: the kernel substitutes 1.0
        n = int(n)
        if ip.numel() != n + 1:
            raise ValueError("indptr must have n+1 entries")
        nnz = int(ix.numel())
        row_hi = n if row_hi is None else int(row_hi)
        sb_flag = _lib.GRAPH_SOURCE_BLOCKS
        if features is not None:
            sb_flag = source_block_flags(n, int(features), dtype) or _lib.GRAPH_SOURCE_BLOCKS
        if source_blocks is None:
            # full graphs (appnp_propagate) and the held rows of a row partition
            # (appnp_step_split) alike
            source_blocks = features is not None and splits_rows(n, int(features), dtype)
        flags = ((_lib.GRAPH_TRANSPOSE if transpose else 0)
                 | (sb_flag if source_blocks else 0))
        lib = _lib.load()
        out = C.c_void_p()
        with torch.cuda.device(device):
            rc = lib.appnp_graph_create_rows(
                _ptr(ip), _ptr(ix), _ptr(dv), n, nnz,
                _lib.NORM[mode] | flags, int(row_lo), row_hi,
                1 if split_local else 0, C.c_void_p(_stream_ptr(device)), C.byref(out),
            )
        _lib.check("appnp_graph_create", rc)
        g = cls(out, device)
        if source_blocks and g.source_block_bytes() == 0:
            warnings.warn(f"ppnp_amd: the source-blocked copy of A_hat (n={n}) could not be "
                          "built; this graph gathers whole rows", RuntimeWarning, stacklevel=2)
        return g

    @classmethod
    def from_scipy(cls, adj, mode="sym", device=None, **kw):
        import scipy.sparse as sp

        a = sp.csr_matrix(adj)
        if not a.has_sorted_indices:
            a = a.copy()
            a.sort_indices()
        return cls.from_csr(a.indptr.astype(np.int32), a.indices.astype(np.int32),
                            a.data.astype(np.float32), a.shape[0], mode=mode, device=device, **kw)

    # -- inspection -----------------------------------------------------------------------
    @property
    def handle(self):
        return self._h

    @property
    def rows(self) -> int:
        return self.row_hi - self.row_lo

    def split_point(self, f: int, dtype=torch.float32) -> int:
        """Columns [0, fs) that appnp_propagate gathers as whole cache lines when the rest run
        the L2-blocked remainder pass (appnp_propagate_split_point); 0: rows gathered whole."""
        fs = C.c_int64()
        dt = _lib.BF16 if dtype == torch.bfloat16 else _lib.F32
        _lib.check("appnp_propagate_split_point",
                   _lib.load().appnp_propagate_split_point(self._h, int(f), dt, C.byref(fs)))
        return fs.value

    def remainder_cols(self, f: int, dtype=torch.float32) -> int:
        """Columns [F - r, F) that run the L2-blocked remainder pass (r = F for narrow rows on a
        W8 / W16 copy); 0: rows gathered whole (appnp_propagate_remainder_cols)."""
        r = C.c_int64()
        dt = _lib.BF16 if dtype == torch.bfloat16 else _lib.F32
        _lib.check("appnp_propagate_remainder_cols",
                   _lib.load().appnp_propagate_remainder_cols(self._h, int(f), dt, C.byref(r)))
        return r.value

    def source_block_bytes(self) -> int:
        """Device bytes of the source-blocked copy of A_hat (0: not built)."""
        b = C.c_int64()
        _lib.check("appnp_graph_source_blocks",
                   _lib.load().appnp_graph_source_blocks(self._h, C.byref(b)))
        return b.value

    def source_block_layout(self):
        """The source-blocked copy as built (appnp_graph_source_block_layout): dict(width=4/8/16
        remainder columns per row, entries incl. padding, value_free, row_passes, launches =
        remainder-pass launches enqueued on this graph so far), or None when it was not built."""
        return source_block_layout_of(self._h)

    def split_layout(self, f: int):
        """(fs, rem_width) of the split layout appnp_step_split uses on the held rows for F = f
        columns (appnp_split_layout), or None when f does not split on this graph."""
        return split_layout_of(self._h, f)

    def csr(self):
        """(row_ptr int32, col int32, val fp32, dinv fp64) as new device tensors."""
        lib = _lib.load()
        rp = torch.empty(self.rows + 1, dtype=torch.int32, device=self.device)
        col = torch.empty(self.nnz_hat, dtype=torch.int32, device=self.device)
        val = torch.empty(self.nnz_hat, dtype=torch.float32, device=self.device)
        dinv = torch.empty(self.n, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            rc = lib.appnp_graph_copy_csr(self._h, _ptr(rp), _ptr(col), _ptr(val), _ptr(dinv),
                                          C.c_void_p(_stream_ptr(self.device)))
        _lib.check("appnp_graph_copy_csr", rc)
        return rp, col, val, dinv

    def close(self):
        if getattr(self, "_h", None) is not None:
            try:
                _lib.load().appnp_graph_destroy(self._h)
            finally:
                self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __repr__(self):
        return (f"Graph(n={self.n}, rows=[{self.row_lo},{self.row_hi}), nnz_hat={self.nnz_hat}, "
                f"mode={self.mode!r}, symmetric={self.symmetric}, device={self.device})")
