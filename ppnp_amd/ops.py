"""APPNP propagation op on the gfx950 HIP kernels (no CPU fallback).

``propagate(graph, H, K, alpha)`` replaces the reference's propagation product
``self.ppr[idx] @ self.encoder(X)`` (/root/reference/model.py:63) by its K-truncated Neumann
series Z_K; ``Z_K[idx]`` is the drop-in for ``ppr[idx] @ H`` and
converges to it as K grows (K=100: 6e-7 max-abs on Cora-ML).

All calls are stream-ordered on ``torch.cuda.current_stream()``.
"""

from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from .graph import Graph

_DTYPES = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16}


def _check_dense(name, t, graph: Graph, rows: int):
    if not torch.is_tensor(t):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device != graph.device:
        raise ValueError(f"{name} is on {t.device}, graph on {graph.device}")
    if t.dtype not in _DTYPES:
        raise TypeError(f"{name} dtype {t.dtype} unsupported (float32 / bfloat16)")
    if t.dim() != 2 or t.shape[0] != rows:
        raise ValueError(f"{name} must be [{rows}, F], got {tuple(t.shape)}")
    if t.shape[1] > 0 and t.stride(1) != 1:
        raise ValueError(f"{name} must have unit column stride")


def _ld(t) -> int:
    return max(int(t.stride(0)), int(t.shape[1])) if t.shape[0] > 1 else int(t.shape[1])


def _stream(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _vp(t):
    return C.c_void_p(t.data_ptr()) if t is not None and t.numel() > 0 else None


def propagate_forward(graph: Graph, H: torch.Tensor, K: int, alpha: float, p_drop: float = 0.0,
                      seed: int = 0, out: torch.Tensor | None = None) -> torch.Tensor:
    """Z = APPNP_K(H) via ``appnp_propagate`` (one fused HIP launch per iteration)."""
    _check_dense("H", H, graph, graph.n)
    Z = torch.empty_like(H, memory_format=torch.contiguous_format) if out is None else out
    _check_dense("out", Z, graph, graph.n)
    if Z.dtype != H.dtype or Z.shape != H.shape:
        raise ValueError("out must match H in shape and dtype")
    lib = _lib.load()
    dt = _DTYPES[H.dtype]
    f = int(H.shape[1])
    ws_bytes = int(lib.appnp_workspace_bytes(graph.handle, f, _ld(Z), dt)) if K >= 2 else 0
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=graph.device) if ws_bytes else None
    with torch.cuda.device(graph.device):
        rc = lib.appnp_propagate(graph.handle, _vp(H), _ld(H), _vp(Z), _ld(Z), f, dt, int(K),
                                 float(alpha), float(p_drop), int(seed) & (2**64 - 1), _vp(ws),
                                 ws_bytes, _stream(graph.device))
    _lib.check("appnp_propagate", rc)
    return Z


def propagate_backward(graph: Graph, dZ: torch.Tensor, K: int, alpha: float, p_drop: float = 0.0,
                       seed: int = 0) -> torch.Tensor:
    """dH = J^T dZ via ``appnp_propagate_bwd`` (A_hat^T: A_hat itself for 'sym' on an
    undirected graph, else the transpose built with ``Graph(..., transpose=True)``)."""
    dZ = dZ.contiguous()
    _check_dense("dZ", dZ, graph, graph.n)
    dH = torch.empty_like(dZ)
    lib = _lib.load()
    dt = _DTYPES[dZ.dtype]
    f = int(dZ.shape[1])
    ws_bytes = int(lib.appnp_workspace_bytes(graph.handle, f, _ld(dH), dt)) if K >= 2 else 0
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=graph.device) if ws_bytes else None
    with torch.cuda.device(graph.device):
        rc = lib.appnp_propagate_bwd(graph.handle, _vp(dZ), _ld(dZ), _vp(dH), _ld(dH), f, dt,
                                     int(K), float(alpha), float(p_drop),
                                     int(seed) & (2**64 - 1), _vp(ws), ws_bytes,
                                     _stream(graph.device))
    _lib.check("appnp_propagate_bwd", rc)
    return dH


# ---- torch.library registration ---------------------------------------------------------
# ``ppnp_amd::propagate`` / ``ppnp_amd::propagate_bwd`` are real dispatcher ops: torch.compile
# traces through them without a graph break (fake kernels give the output metadata), and
# autograd is registered on the op itself.  A custom op cannot take a Python object, so the
# graph crosses the dispatcher as the integer key Graph.key (graph.py registry).
# Call sites served: the three propagations per epoch of main.py:121, 138, 145.


@torch.library.custom_op("ppnp_amd::propagate", mutates_args=(), device_types="cuda")
def _propagate_op(H: torch.Tensor, graph_key: int, K: int, alpha: float, p_drop: float,
                  seed: int) -> torch.Tensor:
    return propagate_forward(Graph.lookup(graph_key), H.contiguous(), K, alpha, p_drop, seed)


@_propagate_op.register_fake
def _(H, graph_key, K, alpha, p_drop, seed):
    return torch.empty(H.shape, dtype=H.dtype, device=H.device)


@torch.library.custom_op("ppnp_amd::propagate_bwd", mutates_args=(), device_types="cuda")
def _propagate_bwd_op(dZ: torch.Tensor, graph_key: int, K: int, alpha: float, p_drop: float,
                      seed: int) -> torch.Tensor:
    return propagate_backward(Graph.lookup(graph_key), dZ, K, alpha, p_drop, seed)


@_propagate_bwd_op.register_fake
def _(dZ, graph_key, K, alpha, p_drop, seed):
    return torch.empty(dZ.shape, dtype=dZ.dtype, device=dZ.device)


def _propagate_setup(ctx, inputs, output):
    ctx.args = inputs[1:]


def _propagate_grad(ctx, dZ):
    return (torch.ops.ppnp_amd.propagate_bwd(dZ, *ctx.args), None, None, None, None, None)


_propagate_op.register_autograd(_propagate_grad, setup_context=_propagate_setup)


def propagate(graph: Graph, H: torch.Tensor, K: int = 10, alpha: float = 0.1,
              p_drop: float = 0.0, seed: int = 0) -> torch.Tensor:
    """Differentiable APPNP propagation Z_K(H) on the GPU (the ``ppnp_amd::propagate`` op).
    The seed is taken mod 2^64 like everywhere else (propagate_forward, the oracle); it crosses
    the op's int64 schema reinterpreted as signed, and propagate_forward maps it back."""
    s = int(seed) & (2**64 - 1)
    return torch.ops.ppnp_amd.propagate(H, graph.key, int(K), float(alpha), float(p_drop),
                                        s - 2**64 if s >= 2**63 else s)


def step(graph: Graph, Zin: torch.Tensor, H: torch.Tensor, out: torch.Tensor, k: int,
         alpha: float, part: int = _lib.PART_ALL, partial: torch.Tensor | None = None,
         p_drop: float = 0.0, seed: int = 0) -> torch.Tensor:
    """One iteration on the held rows (``appnp_step``); Zin holds all n rows."""
    lib = _lib.load()
    _check_dense("Zin", Zin, graph, graph.n)
    dt = _DTYPES[Zin.dtype]
    f = int(Zin.shape[1])
    ld_h = _ld(H) if H is not None else 0
    ld_p = _ld(partial) if partial is not None else 0
    with torch.cuda.device(graph.device):
        rc = lib.appnp_step(graph.handle, int(part), _vp(Zin), _ld(Zin), _vp(H), ld_h, _vp(out),
                            _ld(out), _vp(partial), ld_p, f, dt, int(k), float(alpha),
                            float(p_drop), int(seed) & (2**64 - 1), _stream(graph.device))
    _lib.check("appnp_step", rc)
    return out


def shard_offsets(graph: Graph, nshards: int, shard_rows: int) -> None:
    """The held rows' entries grouped by source shard (``appnp_graph_shard_offsets``), for the
    pipelined row steps ``step_shards`` / ``step_split_shards``."""
    with torch.cuda.device(graph.device):
        rc = _lib.load().appnp_graph_shard_offsets(graph.handle, int(nshards), int(shard_rows),
                                                   _stream(graph.device))
    _lib.check("appnp_graph_shard_offsets", rc)


def step_shards(graph: Graph, s_lo: int, s_hi: int, mode: int, Zin: torch.Tensor,
                H: torch.Tensor | None, out: torch.Tensor | None, partial: torch.Tensor | None,
                k: int, alpha: float, p_drop: float = 0.0, seed: int = 0) -> None:
    """One iteration's product over source shards [s_lo, s_hi) of the held rows
    (``appnp_step_shards``): mode SHARDS_FIRST / _ACC into ``partial``, _LAST / _ONLY into
    ``out`` (fp32; Zin holds all n rows)."""
    _check_dense("Zin", Zin, graph, graph.n)
    f = int(Zin.shape[1])
    with torch.cuda.device(graph.device):
        rc = _lib.load().appnp_step_shards(
            graph.handle, int(s_lo), int(s_hi), int(mode), _vp(Zin), _ld(Zin), _vp(H),
            _ld(H) if H is not None else 0, _vp(out), _ld(out) if out is not None else 0,
            _vp(partial), _ld(partial) if partial is not None else 0, f, int(k), float(alpha),
            float(p_drop), int(seed) & (2**64 - 1), _stream(graph.device))
    _lib.check("appnp_step_shards", rc)


def step_split_shards(graph: Graph, s_lo: int, s_hi: int, mode: int,
                      zin_main: torch.Tensor | None, zin_rem: torch.Tensor | None,
                      H: torch.Tensor | None, f: int, k: int, alpha: float,
                      out_main: torch.Tensor | None = None, out_rem: torch.Tensor | None = None,
                      Z: torch.Tensor | None = None, partial: torch.Tensor | None = None,
                      p_drop: float = 0.0, seed: int = 0) -> None:
    """``step_shards`` on the split layout (``appnp_step_split_shards``): the main columns take
    the shard range and mode; _LAST / _ONLY then run the remainder pass."""
    with torch.cuda.device(graph.device):
        rc = _lib.load().appnp_step_split_shards(
            graph.handle, int(s_lo), int(s_hi), int(mode), _vp(zin_main), _vp(zin_rem), _vp(H),
            _ld(H) if H is not None else 0, _vp(out_main), _vp(out_rem), _vp(Z),
            _ld(Z) if Z is not None else 0, _vp(partial),
            _ld(partial) if partial is not None else 0, int(f), int(k), float(alpha),
            float(p_drop), int(seed) & (2**64 - 1), _stream(graph.device))
    _lib.check("appnp_step_split_shards", rc)


def split_copy(graph: Graph, H: torch.Tensor, main: torch.Tensor | None,
               rem: torch.Tensor) -> None:
    """Z_0 of the split layout on the held rows (``appnp_split_copy``): H [held rows, F] into
    rows [row_lo, row_hi) of the full-height parts main [*, fs] and rem [*, rem_width]."""
    with torch.cuda.device(graph.device):
        rc = _lib.load().appnp_split_copy(graph.handle, _vp(H), _ld(H), int(H.shape[1]),
                                          _vp(main), _vp(rem), _stream(graph.device))
    _lib.check("appnp_split_copy", rc)


def step_split(graph: Graph, part: int, zin_main: torch.Tensor | None, zin_rem: torch.Tensor,
               H: torch.Tensor | None, f: int, k: int, alpha: float,
               out_main: torch.Tensor | None = None, out_rem: torch.Tensor | None = None,
               Z: torch.Tensor | None = None, partial: torch.Tensor | None = None,
               p_drop: float = 0.0, seed: int = 0) -> None:
    """One iteration of the held rows on the split layout (``appnp_step_split``): from every row
    of zin_main / zin_rem into rows [row_lo, row_hi) of out_main / out_rem, or into Z (the held
    rows, all F columns) on the last iteration."""
    with torch.cuda.device(graph.device):
        rc = _lib.load().appnp_step_split(
            graph.handle, int(part), _vp(zin_main), _vp(zin_rem), _vp(H),
            _ld(H) if H is not None else 0, _vp(out_main), _vp(out_rem), _vp(Z),
            _ld(Z) if Z is not None else 0, _vp(partial),
            _ld(partial) if partial is not None else 0, int(f), int(k), float(alpha),
            float(p_drop), int(seed) & (2**64 - 1), _stream(graph.device))
    _lib.check("appnp_step_split", rc)


class PropagatePlan:
    """A captured propagation (``appnp_plan_create``): K launches recorded once into a hipGraph
    for fixed H / Z buffers, replayed with one graph launch.  Refill ``plan.H`` in place, call
    ``plan()``, read ``plan.Z``.  For small, launch-bound graphs and serving loops."""

    def __init__(self, graph: Graph, H: torch.Tensor, K: int = 10, alpha: float = 0.1,
                 p_drop: float = 0.0, seed: int = 0):
        _check_dense("H", H, graph, graph.n)
        self.graph, self.H = graph, H
        self.Z = torch.empty_like(H, memory_format=torch.contiguous_format)
        lib = _lib.load()
        dt = _DTYPES[H.dtype]
        f = int(H.shape[1])
        self._ws_bytes = int(lib.appnp_workspace_bytes(graph.handle, f, _ld(self.Z), dt))
        self._ws = torch.empty(max(self._ws_bytes, 1), dtype=torch.uint8, device=graph.device)
        self._p = C.c_void_p()
        torch.cuda.current_stream(graph.device).synchronize()  # buffers allocated before capture
        with torch.cuda.device(graph.device):
            rc = lib.appnp_plan_create(graph.handle, _vp(H), _ld(H), _vp(self.Z), _ld(self.Z), f,
                                       dt, int(K), float(alpha), float(p_drop),
                                       int(seed) & (2**64 - 1), _vp(self._ws), self._ws_bytes,
                                       C.byref(self._p))
        _lib.check("appnp_plan_create", rc)

    def __call__(self) -> torch.Tensor:
        with torch.cuda.device(self.graph.device):
            rc = _lib.load().appnp_plan_launch(self._p, _stream(self.graph.device))
        _lib.check("appnp_plan_launch", rc)
        return self.Z

    def close(self):
        if getattr(self, "_p", None):
            _lib.load().appnp_plan_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


KERNEL_KINDS = {_lib.KT_COPY: "copy", _lib.KT_STEP: "step", _lib.KT_REM: "rem",
                _lib.KT_LOCAL: "local", _lib.KT_REMOTE: "remote", _lib.KT_XCHG: "xchg"}


def kernel_times(fn, device, max_launches: int = 1024) -> list[tuple[str, float]]:
    """Call ``fn()`` with the library's per-launch timer on (``appnp_kernel_timer_begin`` /
    ``_end``) and return one (kind, ms) pair per launch it enqueued, in launch order: "copy"
    (the split copy), "step" (the SpMM kernel), "local" / "remote" (its two halves on a
    row-partitioned graph), "rem" (the remainder pass), "xchg" (an exchange of the library's
    own row loop).  Each interval is bracketed by events right before and after its launch on
    the launch stream, so no wait before it is counted; no profiler runs."""
    lib = _lib.load()
    with torch.cuda.device(device):
        # fn() runs even if the timer cannot start: at N > 1 it may hold collectives that every
        # rank must join
        rc0 = lib.appnp_kernel_timer_begin(int(max_launches), _stream(device))
        try:
            fn()
        finally:
            ms = (C.c_float * max_launches)()
            kinds = (C.c_int * max_launches)()
            n = C.c_int(0)
            rc = lib.appnp_kernel_timer_end(ms, kinds, max_launches, C.byref(n)) if rc0 == 0 else 0
        _lib.check("appnp_kernel_timer_begin", rc0)
        _lib.check("appnp_kernel_timer_end", rc)
    return [(KERNEL_KINDS.get(kinds[i], str(kinds[i])), float(ms[i]))
            for i in range(min(n.value, max_launches))]


def line_rate_probe(table: torch.Tensor, lines: int, seed: int = 0, reps: int = 3) -> dict:
    """The device's random 128-B line rate (``appnp_line_rate_probe``): ``lines`` random lines
    gathered from ``table``'s storage (read only) per launch, one warm-up launch, then the
    median of ``reps`` launches timed with HIP events on the current stream.  Returns
    {"G_lines_s", "ms", "lines", "table_MB"}."""
    if not table.is_cuda:
        raise ValueError("table must be a device tensor")
    lib = _lib.load()
    dev = table.device
    base = table.untyped_storage().data_ptr()
    nbytes = table.untyped_storage().nbytes()
    skip = (-base) % 128  # the kernel gathers whole 128-B lines from a 128-B aligned start
    tbytes = (nbytes - skip) // 128 * 128
    sink = torch.zeros(1, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    times = []
    with torch.cuda.device(dev):
        for r in range(reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            _lib.check("appnp_line_rate_probe", lib.appnp_line_rate_probe(
                C.c_void_p(base + skip), tbytes, int(lines), int(seed + r) & (2**64 - 1),
                C.c_void_p(sink.data_ptr()), C.c_void_p(stream.cuda_stream)))
            b.record(stream)
            times.append((a, b))
        torch.cuda.synchronize(dev)
    ms = sorted(a.elapsed_time(b) for a, b in times[1:])[reps // 2]
    return {"G_lines_s": lines / (ms * 1e-3) / 1e9, "ms": ms, "lines": int(lines),
            "table_MB": tbytes / 2**20}
