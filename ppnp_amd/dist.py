"""Multi-GPU APPNP propagation: one process per GPU, torch.distributed over RCCL (xGMI).

SURVEY.md section 8(e).  P ranks are laid out as R row groups x C column (feature) groups:

* row partition (the north_star design, R = P): rank r owns the A_hat rows and the H / Z rows
  of [lo_r, hi_r).  Every iteration needs all of Z_k, so the ranks of one column group
  all-gather their row shards of Z_{k+1} (RCCL all_gather_into_tensor, in place) -- the
  path's one real exchange step.  With ``overlap=True`` each rank's rows are stored as a
  local-column and a remote-column CSR (appnp_graph_create_rows split_local): the local
  product of the next iteration runs while the all-gather is in flight, the remote product
  after it lands (appnp_step PART_LOCAL / PART_REMOTE).
* column partition (C = P): propagation is column-separable, so rank r takes a slab of
  F/C features of H and Z and a full replica of A_hat; the K loop has no communication.
  Each slab is stored with a line-friendly leading dimension (a 25-float slab in one 128-B
  line), which is what makes this layout pay on MI355X: a random row gather costs cache-line
  requests, and the chip serves ~55 G random line requests/s (profiles/r1_gather_probe.txt).
* R x C mixes the two (e.g. 2 x 4 on 8 GPUs).

The edge-dropout mask is keyed on (seed, k, global row, global col), so it does not depend on
the layout.  The communication and per-step kernels are injectable (``comm``, ``step_fn``) so
the orchestration is tested on CPU with gloo against the oracle (tests/test_dist.py).
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.distributed as dist

from . import _lib


@dataclass(frozen=True)
class Layout:
    rows: int  # R row groups
    cols: int  # C column groups
    # column slabs cut at whole 128-B lines (``line_slab_cols``) instead of evenly; column
    # layouts only (R = 1)
    lines: bool = False

    @property
    def size(self) -> int:
        return self.rows * self.cols

    def coords(self, rank: int):
        """(row group, column group) of a rank; ranks of one column group are contiguous
        in row order so that a column group's all-gather is a plain ordered all-gather."""
        return rank % self.rows, rank // self.rows

    @staticmethod
    def parse(spec: str, world: int) -> "Layout":
        if spec in ("row", "rows"):
            return Layout(world, 1)
        if spec in ("col", "cols", "column"):
            return Layout(1, world)
        if spec in ("col-lines", "lines"):
            return Layout(1, world, True)
        r, c = (int(x) for x in spec.lower().split("x"))
        if r * c != world:
            raise ValueError(f"layout {spec} does not cover {world} ranks")
        return Layout(r, c)


def row_range(n: int, R: int, ri: int):
    """Equal-size row shards (all_gather_into_tensor needs equal counts): shard = ceil(n/R);
    the padded tail rows beyond n are never referenced by a column index."""
    shard = -(-n // R) if R > 0 else n
    lo = min(n, ri * shard)
    hi = min(n, lo + shard)
    return lo, hi, shard


def col_range(f: int, C: int, ci: int):
    base, rem = divmod(f, C)
    lo = ci * base + min(ci, rem)
    return lo, lo + base + (1 if ci < rem else 0)


def line_slab_cols(f: int, C: int, elem_bytes: int = 4):
    """Column bounds [(lo, hi)] of C slabs cut at whole 128-B lines: the q = F // L full lines
    of a row (L = 128 / elem_bytes columns) go out as evenly as possible, the first slabs taking
    the extra ones, and the r = F % L remainder columns join the last slab, which holds the
    fewest lines.  Every slab but the last then gathers whole lines, and the last takes its
    remainder through the split path: F = 100 fp32 on 2 ranks is 64 | 36 (= 32 + 4), on 3 ranks
    32 | 32 | 36, on 4 ranks 32 | 32 | 32 | 4, where the even split (50, 34 / 33, 25 columns)
    costs 2, 2 and 1 lines per gather on every rank.  None when a slab would be empty (more
    slabs than lines, plus one for a remainder)."""
    L = 128 // elem_bytes
    q, r = divmod(f, L)
    if C < 1 or C > q + (1 if r else 0):
        return None
    base, extra = divmod(q, C)
    out, lo = [], 0
    for i in range(C):
        hi = lo + L * (base + (1 if i < extra else 0)) + (r if i == C - 1 else 0)
        if hi <= lo:
            return None
        out.append((lo, hi))
        lo = hi
    return out


def slab_range(f: int, layout: Layout, ci: int, elem_bytes: int = 4):
    """Column bounds of column group ci: ``line_slab_cols`` for a lines layout, else even."""
    if layout.lines and layout.rows == 1:
        slabs = line_slab_cols(f, layout.cols, elem_bytes)
        if slabs is None:
            raise ValueError(f"{f} columns cannot be cut into {layout.cols} line slabs")
        return slabs[ci]
    return col_range(f, layout.cols, ci)


def _avg_lines(row_bytes: int, stride: int) -> float:
    """Average number of 128-B lines a row of ``row_bytes`` spans at row stride ``stride``."""
    period = 128 // math.gcd(128, stride % 128 or 128)
    return sum(((i * stride) % 128 + row_bytes - 1) // 128 + 1 for i in range(period)) / period


def line_ld(width: int, elem_bytes: int = 4) -> int:
    """Leading dimension (elements) for row gathers: rows padded to start on a 128-B line (next
    power of two up to a line, then whole lines) when that lowers the average lines a row
    spans; otherwise packed to a 16-B multiple.  Same rule as appnp_capi.hip line_ld."""
    if width <= 0:
        return 1
    line = 128 // elem_bytes
    padded = (1 << (width - 1).bit_length()) if width <= line else -(-width // line) * line
    v = 16 // elem_bytes
    packed = -(-width // v) * v
    if _avg_lines(width * elem_bytes, padded * elem_bytes) < _avg_lines(width * elem_bytes,
                                                                        packed * elem_bytes):
        return padded
    return packed


# The process group that carries the data-path exchange (RCCL all-gathers and P2P).  None: the
# default group.  bench.py keeps the default group on gloo -- the control plane: barriers,
# max-over-ranks, failure agreement, which no RCCL failure can poison -- and creates an RCCL
# group for the exchange only when the first exchange candidate runs (``ensure_data_group``),
# inside that candidate's deadline, so an RCCL that fails to come up costs that candidate and
# not the run.
_DATA_GROUP = None


def data_group():
    return _DATA_GROUP


def data_backend():
    """Backend of the data-path group ('nccl' = RCCL, 'gloo'), None without a process group."""
    if not dist.is_initialized():
        return None
    return dist.get_backend(_DATA_GROUP) if _DATA_GROUP is not None else dist.get_backend()


def ensure_data_group(backend: str, device) -> None:
    """Create the data-path group over every rank once (collective: every rank calls it at the
    same point), and bring its communicator up with a one-element all-reduce, so that a caller
    reading the RCCL communicator (NativeRowAPPNP) finds it built.  No-op when the default group
    already has that backend."""
    global _DATA_GROUP
    if _DATA_GROUP is not None or not dist.is_initialized() or dist.get_backend() == backend:
        return
    kw = {"device_id": torch.device(device)} if backend == "nccl" else {}
    pg = dist.new_group(backend=backend, **kw)
    t = torch.zeros(1, device=device if backend == "nccl" else "cpu")
    dist.all_reduce(t, group=pg)
    if t.is_cuda:
        torch.cuda.synchronize(t.device)
    _DATA_GROUP = pg


class _TorchComm:
    """In-place all-gather of equal row shards within a column group (RCCL for 'nccl'), on the
    data-path group (``data_group``)."""

    name = "group"

    def __init__(self, layout: Layout, rank: int):
        self.layout = layout
        self.groups = {}
        ri, ci = layout.coords(rank)
        self.ri, self.ci = ri, ci
        self.backend = data_backend()
        self.group = _DATA_GROUP
        if layout.rows > 1 and layout.cols > 1:
            for c in range(layout.cols):
                members = [c * layout.rows + r for r in range(layout.rows)]
                g = dist.new_group(members, backend=self.backend)
                if c == ci:
                    self.group = g

    def all_gather_rows(self, full: torch.Tensor, shard_rows: int, async_op: bool):
        """full: [R * shard_rows, ld]; this rank's shard already sits at row ri*shard_rows."""
        R = self.layout.rows
        if R == 1:
            return None
        mine = full[self.ri * shard_rows:(self.ri + 1) * shard_rows]
        if self.backend == "nccl":
            return dist.all_gather_into_tensor(full, mine, group=self.group, async_op=async_op)
        # gloo (CPU tests, single-GPU multi-process rehearsal): stage through host memory
        host = full.detach().to("cpu", copy=True) if full.is_cuda else full
        parts = list(host.split(shard_rows))
        dist.all_gather(parts, parts[self.ri].clone(), group=self.group)
        if full.is_cuda:
            full.copy_(host)
        return None

    supports_broadcast = True

    def broadcast_rows(self, full: torch.Tensor, shard_rows: int, root: int, async_op: bool):
        """In-place broadcast of row shard ``root`` (a row-group index) of ``full`` from its
        owner to the column group: one step of the pipelined exchange, whose R broadcasts land
        one shard at a time (roots in the same order on every rank).  RCCL: an async work whose
        wait() orders the caller's stream after it; gloo: synchronous, through host memory."""
        if self.layout.rows == 1:
            return None
        view = full[root * shard_rows:(root + 1) * shard_rows]
        src = self.ci * self.layout.rows + root  # global rank of that row group's member
        if self.backend == "nccl":
            return dist.broadcast(view, src=src, group=self.group, async_op=async_op)
        host = view.detach().to("cpu", copy=True) if view.is_cuda else view
        dist.broadcast(host, src=src, group=self.group)
        if view.is_cuda:
            view.copy_(host)
        return None


def _pieces(rows: int, parts: int):
    """Row bounds of ``parts`` near-equal pieces of a shard of ``rows`` rows."""
    return [col_range(rows, parts, t) for t in range(parts)]


class _StreamDone:
    """Handle of a side-stream exchange: wait() orders the caller's current stream after it."""

    def __init__(self, event):
        self.event = event

    def wait(self):
        if self.event is not None:
            torch.cuda.current_stream().wait_event(self.event)


class MultipathComm:
    """All-gather of row shards within each column group, routed over every rank (RCCL P2P).

    In an R x C layout (C > 1) the ranks of one column group only need each other's shards,
    so a plain group all-gather drives R-1 of a GPU's 7 xGMI links and leaves the others idle
    (2 x 4 on 8 GPUs: one link carries the whole shard).  Here every shard S is cut into P-1
    pieces, one per other rank (the relay), in two batched P2P stages:

    1. rank a sends piece_b(S_a) to every b != a.  A relay in a's column group keeps it in place;
       any other relay parks it in a staging buffer.
    2. every relay b forwards each parked piece_b(S_a) to the members of a's column group, and a
       relay inside that group forwards to the other members (R > 2).

    Per link and stage this moves S/(P-1) bytes (stage 2: (R-1) S/(P-1)) instead of S on R-1
    links: on 2 x 4, 2 S/7 over all seven links instead of S over one.  P2P messages carry the
    originating rank as tag, and both sides walk origins in ascending order (RCCL matches P2P
    in issue order per peer pair, gloo by tag).

    On 'nccl' the two stages run on a side stream that waits for the producer, so the caller's
    stream stays free for the local-column product (overlap mode); the returned handle's wait()
    orders the caller's stream after the exchange.  On 'gloo' (CPU tests, single-GPU
    rehearsal) the exchange is synchronous and stages CUDA data through host memory.
    """

    name = "multipath"

    def __init__(self, layout: Layout, rank: int, widths=None):
        self.layout, self.rank = layout, rank
        # valid columns of each column group's slab: a slab padded to a line-friendly leading
        # dimension (25 of 32 floats) travels packed, 22 % fewer bytes over the links.  None:
        # whole rows of the buffers (every rank's leading dimension must then agree).
        self.widths = widths
        self.P = layout.size
        self.ri, self.ci = layout.coords(rank)
        self.backend = data_backend()
        self.group = _DATA_GROUP  # every rank relays: the whole data-path group
        self._stream = None
        self._staging = None

    # ranks of a's column group
    def group_of(self, a: int):
        R = self.layout.rows
        c = a // R
        return [c * R + r for r in range(R)]

    def relays(self, a: int):
        return [b for b in range(self.P) if b != a]

    def plan(self, shard_rows: int):
        """(stage-1 ops, stage-2 ops) as lists of (kind, peer, origin, row range in the
        origin's shard, 'full' | ('stage', slot)) for this rank."""
        me, P = self.rank, self.P
        mygroup = set(self.group_of(me))
        pieces = _pieces(shard_rows, P - 1)
        slots = {}
        s1, s2 = [], []
        for t, b in enumerate(self.relays(me)):  # my shard, piece t -> relay b
            s1.append(("send", b, me, pieces[t], "full"))
        for a in range(P):
            if a == me:
                continue
            t = self.relays(a).index(me)  # the piece of S_a that I relay
            if a in mygroup:
                s1.append(("recv", a, a, pieces[t], "full"))
                for c in self.group_of(a):
                    if c not in (a, me):
                        s2.append(("send", c, a, pieces[t], "full"))
            else:
                slot = slots.setdefault(a, len(slots))
                s1.append(("recv", a, a, pieces[t], ("stage", slot)))
                for c in self.group_of(a):
                    if c != a:
                        s2.append(("send", c, a, pieces[t], ("stage", slot)))
        for a in sorted(mygroup - {me}):  # the rest of S_a reaches me through the relays
            for tb, b in enumerate(self.relays(a)):
                if b != me:
                    s2.append(("recv", b, a, pieces[tb], "full"))
        return s1, s2, len(slots), max((hi - lo for lo, hi in pieces), default=0)

    def _width(self, origin: int, full) -> int:
        """Columns of origin's slab a message carries: its column group's width (packed), or
        the whole buffer row when no widths are given (every rank's buffers then agree)."""
        if self.widths is None:
            return full.shape[1]
        return self.widths[origin // self.layout.rows]

    def _views(self, full, shard_rows, ops, nslots, pmax):
        R = self.layout.rows
        # staging slot s holds a piece of origin a's slab, packed at a's width -- which is not
        # this relay's own width when a is in another column group (F = 73 on 2 x 2: 37 | 36)
        slot_w = {}
        for kind, peer, origin, (lo, hi), where in ops:
            if where != "full":
                slot_w[where[1]] = self._width(origin, full)
        total = sum(pmax * w for w in slot_w.values())
        if total and (self._staging is None or self._staging.numel() < total
                      or self._staging.dtype != full.dtype
                      or self._staging.device != full.device):
            self._staging = torch.empty(total, dtype=full.dtype, device=full.device)
        offs, off = {}, 0
        for slot in sorted(slot_w):
            offs[slot] = off
            off += pmax * slot_w[slot]
        out = []
        for kind, peer, origin, (lo, hi), where in ops:
            if where == "full":  # origin is in this rank's column group: its own width
                base = (origin % R) * shard_rows
                t = full[base + lo:base + hi, :min(self._width(origin, full), full.shape[1])]
            else:
                w = slot_w[where[1]]
                o = offs[where[1]]
                t = self._staging[o:o + (hi - lo) * w].view(hi - lo, w)
            out.append((kind, peer, origin, t))
        return out

    def _run_stage(self, views, host):
        ops = []
        bufs = []
        for kind, peer, origin, t in views:
            if t.shape[0] == 0:
                continue
            buf = t
            if host:
                buf = t.detach().to("cpu", copy=True) if kind == "send" else torch.empty(
                    t.shape, dtype=t.dtype)
                bufs.append((kind, t, buf))
            elif not t.is_contiguous():  # packed: column view of a padded slab
                buf = t.contiguous() if kind == "send" else torch.empty(
                    t.shape, dtype=t.dtype, device=t.device)
                bufs.append((kind, t, buf))
            fn = dist.isend if kind == "send" else dist.irecv
            if self.backend == "nccl":
                ops.append(dist.P2POp(fn, buf, peer, group=self.group, tag=origin))
            else:
                ops.append(fn(buf, peer, group=self.group, tag=origin))
        if self.backend == "nccl":
            works = dist.batch_isend_irecv(ops) if ops else []
        else:
            works = ops
        for w in works:
            w.wait()
        for kind, t, buf in bufs:
            if kind == "recv":
                t.copy_(buf)

    def all_gather_rows(self, full: torch.Tensor, shard_rows: int, async_op: bool):
        if self.layout.rows == 1 or self.P == 1:
            return None
        s1, s2, nslots, pmax = self.plan(shard_rows)
        v1 = self._views(full, shard_rows, s1, nslots, pmax)
        v2 = self._views(full, shard_rows, s2, nslots, pmax)
        if self.backend != "nccl":
            host = full.is_cuda
            if host:
                torch.cuda.current_stream(full.device).synchronize()
            self._run_stage(v1, host)
            self._run_stage(v2, host)
            return None
        main = torch.cuda.current_stream(full.device)
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=full.device)
        self._stream.wait_stream(main)
        with torch.cuda.stream(self._stream):
            self._run_stage(v1, False)  # wait(): the side stream waits for stage 1
            self._run_stage(v2, False)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        done = _StreamDone(ev)
        if not async_op:
            done.wait()
            return None
        return done


class NullComm:
    """No exchange (emulation of one rank on one GPU; the gathered rows keep stale data).
    ``broadcast``: whether the exchange it stands in for can broadcast row shards (the relayed
    exchange cannot), which decides whether the emulated rank pipelines like the real one."""

    name = "none"

    def __init__(self, broadcast: bool = True):
        self.supports_broadcast = broadcast

    def all_gather_rows(self, full, shard_rows, async_op):
        return None

    def broadcast_rows(self, full, shard_rows, root, async_op):
        return None


def relayed(layout: Layout, exchange: str) -> bool:
    """Whether ``exchange`` runs as MultipathComm's relayed all-gather on ``layout`` (R x C with
    R, C > 1).  The relay moves whole iterates and cannot broadcast single row shards, so such a
    rank never pipelines (the autotuner then measures an R x C layout both ways: relayed under
    'multipath', pipelined under 'group')."""
    return exchange == "multipath" and layout.rows > 1 and layout.cols > 1


def shard_groups(R: int, ri: int):
    """The pipelined step's groups of REMOTE source shards for row group ri of R: shard ranges
    [a, b) in arrival order (the exchange broadcasts roots 0 .. R-1 in turn), sized 1, 2, 4, ...
    from the last to arrive backwards (7 remote shards: 4 + 2 + 1), cut where a group would
    span the rank's own shard (whose rows are not exchanged to it), and then, front first,
    adjacent groups merged until there are at most ceil(log2 R) of them.  Each group's product
    runs as soon as its last shard has landed, so after the exchange only the last group's --
    one shard's -- compute is left; every group past the first costs one more pass over the
    fp32 partial (ACC), so their number is kept at log2 R (3 on 8 ranks; one more where the own
    shard cuts the only mergeable pair), not R - 2."""
    arrival = [s for s in range(R) if s != ri]
    sizes, left, sz = [], len(arrival), 1
    while left > 0:
        take = min(sz, left)
        sizes.append(take)
        left -= take
        sz *= 2
    groups, pos = [], 0
    for take in reversed(sizes):
        chunk = arrival[pos:pos + take]
        pos += take
        start = chunk[0]
        for a, b in zip(chunk, chunk[1:] + [None]):
            if b is None or b != a + 1:
                groups.append((start, a + 1))
                start = b
    cap = max(1, (R - 1).bit_length())  # ceil(log2 R); the last group is never merged
    i = 0
    while len(groups) > cap and i + 2 < len(groups):
        if groups[i][1] == groups[i + 1][0]:
            groups[i:i + 2] = [(groups[i][0], groups[i + 1][1])]
        else:
            i += 1
    return groups


class PartitionedAPPNP:
    """K-iteration APPNP over a Layout of ranks.  Build with :meth:`create`."""

    def __init__(self, layout, rank, n, f, K, alpha, graph, H_slab, f_lo, f_hi, bufs, shard,
                 lo, hi, comm, step_fn, overlap, partial, p_drop=0.0, seed=0, split=None):
        self.layout, self.rank = layout, rank
        self.n, self.f, self.K, self.alpha = n, f, K, alpha
        self.graph = graph
        self.H = H_slab
        self.f_lo, self.f_hi = f_lo, f_hi
        self.bufs = bufs
        self.shard, self.lo, self.hi = shard, lo, hi
        self.comm, self.step_fn = comm, step_fn
        self.overlap, self.partial = overlap, partial
        self.p_drop, self.seed = p_drop, seed
        # split rows on the held rows (row groups, appnp_step_split): (fs, rem width), the two
        # full-height parts of both iterates and the held rows' output
        self.split = split
        self.smain = self.srem = self.zout = None
        self.out = None

    # -- construction ---------------------------------------------------------------------
    @classmethod
    def create(cls, indptr, indices, n, H, K, alpha, device, layout: Layout | None = None,
               overlap=False, data=None, mode="sym", comm=None, step_fn=None, graph_fn=None,
               p_drop=0.0, seed=0, rank=None, world=None, exchange="multipath", pipeline=None):
        """rank / world override the process group's (single-GPU emulation of one rank of a
        larger layout, with a ``NullComm``: measures that rank's kernel time only).
        exchange: 'multipath' (MultipathComm, R x C layouts with C > 1) or 'group' (one RCCL
        all-gather per column group); a pure row layout always uses the all-gather, or, with
        'native', the library's own loop (NativeRowRunner over appnp_dist_*).
        pipeline: with overlap and R >= 3 row groups, exchange the iterate by R broadcasts, one
        row shard each, and run the remote product one group of arrived shards at a time
        (``shard_groups``), so only the last shard's compute follows the exchange (VERDICT r5
        #2).  None: whenever it applies (the exchange supports broadcasts)."""
        if rank is None:
            rank = dist.get_rank() if dist.is_initialized() else 0
        if world is None:
            world = dist.get_world_size() if dist.is_initialized() else 1
        layout = layout or Layout(1, world)
        if layout.size != world:
            raise ValueError("layout does not match the world size")
        if exchange == "native":  # the library's own row loop (appnp_dist_*)
            if layout.cols != 1 or comm is not None or step_fn is not None or graph_fn is not None:
                raise ValueError("exchange='native' runs a pure row layout on the HIP path")
            return NativeRowRunner(indptr, indices, n, H, K, alpha, device, overlap=overlap,
                                   mode=mode, data=data, p_drop=p_drop, seed=seed,
                                   pipeline=pipeline)
        ri, ci = layout.coords(rank)
        f = int(H.shape[1])
        lo, hi, shard = row_range(n, layout.rows, ri)
        f_lo, f_hi = slab_range(f, layout, ci, H.element_size())
        width = f_hi - f_lo
        esz = H.element_size()
        ld = line_ld(width, esz)
        # the LOCAL / REMOTE halves and the pipelined shard steps keep an fp32 partial of fp32
        # rows (appnp_step: APPNP_ENOTSUP otherwise): bf16 storage exchanges without overlap
        overlap = bool(overlap and layout.rows > 1 and H.dtype == torch.float32)
        if graph_fn is None:
            from .graph import Graph

            # source blocks only where the rank's loop is one appnp_propagate call (column
            # layout) on a slab whose rows split (graph.remainder_width: fp32, width 32q + r
            # with r <= 16, or a narrow slab of <= 16 columns, e.g. 12-13 of F = 100 on 8
            # ranks); appnp_step gathers whole rows
            # a column-layout rank runs appnp_propagate on its slab, a row-group rank
            # appnp_step_split on its held rows: both split like one GPU when the slab's rows do
            # (graph.remainder_width: fp32, width 32q + r with r <= 8, or a narrow slab of <= 16
            # columns), from the source-blocked copy of the rows the rank holds
            graph = Graph.from_csr(indptr, indices, data, n, mode=mode, device=device,
                                   row_lo=lo, row_hi=hi, split_local=overlap, features=width,
                                   dtype=H.dtype)
        else:
            graph = graph_fn(lo, hi, overlap)
        rows_pad = shard * layout.rows
        H_slab = torch.zeros(max(hi - lo, 0), ld, dtype=H.dtype, device=device)
        H_slab[:, :width] = H[lo:hi, f_lo:f_hi].to(device)
        split = None
        if layout.rows > 1 and step_fn is None:
            if (K >= 2 and H.dtype == torch.float32 and ld % 4 == 0
                    and hasattr(graph, "split_layout")):
                split = graph.split_layout(width)
            # every rank must take the same path (the split exchanges two parts per iterate,
            # and the relayed exchange spans all ranks): the rule is the same everywhere (the
            # locality measure is the whole graph's), but slab widths can differ between column
            # groups and the regrouped copy is best-effort, so all ranks agree -- every rank
            # takes part, whatever it found
            if dist.is_initialized() and layout.size > 1:
                split = agree_split(split, device)
        if split is None:
            bufs = [torch.zeros(rows_pad, ld, dtype=H.dtype, device=device) for _ in range(2)]
            partial = (torch.zeros(max(hi - lo, 0), ld, dtype=torch.float32, device=device)
                       if overlap else None)
        else:
            bufs = []
            fs = split[0]
            partial = (torch.zeros(max(hi - lo, 0), max(fs, 4), dtype=torch.float32,
                                   device=device) if overlap and fs > 0 else None)
        if comm is None:
            if exchange not in ("multipath", "group"):
                raise ValueError(f"unknown exchange {exchange!r}")
            # split parts travel whole (their padding is zero on every rank)
            widths = None if split else [
                col_range(f, layout.cols, c)[1] - col_range(f, layout.cols, c)[0]
                for c in range(layout.cols)]
            comm = (MultipathComm(layout, rank, widths) if relayed(layout, exchange)
                    else _TorchComm(layout, rank))
        step_fn = step_fn or _hip_step
        obj = cls(layout, rank, n, f, K, alpha, graph, H_slab, f_lo, f_hi, bufs, shard, lo, hi,
                  comm, step_fn, overlap, partial, p_drop, seed, split)
        if split is not None:
            fs, rw = split
            obj.smain = ([torch.zeros(rows_pad, fs, dtype=torch.float32, device=device)
                          for _ in range(2)] if fs > 0 else [None, None])
            obj.srem = [torch.zeros(rows_pad, rw, dtype=torch.float32, device=device)
                        for _ in range(2)]
            obj.zout = torch.zeros(max(hi - lo, 0), ld, dtype=torch.float32, device=device)
        obj.exchange = getattr(comm, "name", "group")
        R = layout.rows
        can = (overlap and R >= 3 and getattr(comm, "supports_broadcast", False)
               and (split is None or split[0] > 0))
        if pipeline and not can:
            raise ValueError("pipeline needs overlap, >= 3 row groups and a broadcast exchange")
        obj.pipeline = bool(can if pipeline is None else pipeline)
        obj.groups = shard_groups(R, ri) if obj.pipeline else None
        if obj.pipeline:
            if hasattr(graph, "shard_offsets"):
                graph.shard_offsets(R, shard)
            else:
                from .ops import shard_offsets

                shard_offsets(graph, R, shard)
            if obj.partial is None:
                w = split[0] if split is not None else ld
                obj.partial = torch.zeros(max(hi - lo, 0), max(w, 4), dtype=torch.float32,
                                          device=device)
        return obj

    @property
    def nnz_hat_local(self) -> int:
        return self.graph.nnz_hat

    @property
    def remainder_cols(self) -> int:
        """Columns of this rank's slab that run the L2-blocked remainder pass per iteration (0:
        whole rows): a column-layout rank runs appnp_propagate on its slab, which splits like a
        single GPU (appnp_propagate_remainder_cols); a row-group rank runs appnp_step_split
        when its rows split."""
        if self.split is not None:
            return self.width - self.split[0]
        if self.layout.rows == 1 and self.step_fn is _hip_step and self.K >= 2:
            return self.graph.remainder_cols(self.width, self.H.dtype)
        return 0

    @property
    def width(self) -> int:
        return self.f_hi - self.f_lo

    # -- the K loop -----------------------------------------------------------------------
    def _exchange_split(self, b: int, async_op: bool):
        """All-gather both parts of split iterate ``b``; the handles to wait for."""
        works = []
        for t in (self.smain[b], self.srem[b]):
            if t is not None:
                w = self.comm.all_gather_rows(t, self.shard, async_op=async_op)
                if w is not None:
                    works.append(w)
        return works

    def _broadcast_shards(self, full):
        """The pipelined exchange of one iterate (main part on the split layout): R in-place
        broadcasts, root 0 .. R-1 in turn; handle per shard (None when synchronous)."""
        return [self.comm.broadcast_rows(full, self.shard, r, async_op=True)
                for r in range(self.layout.rows)]

    @staticmethod
    def _wait(handles, lo, hi):
        for r in range(lo, hi):
            if handles[r] is not None:
                handles[r].wait()
                handles[r] = None

    def _run_split_pipelined(self):
        """``_run_split`` with the pipelined exchange: the remainder part is all-gathered first
        (it lands before the main part's shards), the main part travels by R broadcasts, and the
        main product runs FIRST on the own shard, then one launch per group of arrived shards
        (appnp_step_split_shards), the last of which finishes the rows and runs the remainder
        pass."""
        from .ops import split_copy, step_split_shards

        K, w, g, R = self.K, self.width, self.graph, self.layout.rows
        ri = self.layout.coords(self.rank)[0]
        H = self.H[:, :w]
        kw = dict(p_drop=self.p_drop, seed=self.seed)
        part = self.partial[:, :self.split[0]]
        split_copy(g, H, self.smain[0], self.srem[0])

        def exchange(b):
            rem = self.comm.all_gather_rows(self.srem[b], self.shard, async_op=True)
            return rem, self._broadcast_shards(self.smain[b])

        rem, shards = exchange(0)
        for k in range(K):
            cur, nxt = k & 1, (k & 1) ^ 1
            last = k == K - 1
            zin = (self.smain[cur], self.srem[cur])
            step_split_shards(g, ri, ri + 1, _lib.SHARDS_FIRST, zin[0], None, None, w, k,
                              self.alpha, partial=part, **kw)
            for i, (a, b) in enumerate(self.groups):
                self._wait(shards, a, b)
                if i + 1 < len(self.groups):
                    step_split_shards(g, a, b, _lib.SHARDS_ACC, zin[0], None, None, w, k,
                                      self.alpha, partial=part, **kw)
                    continue
                if rem is not None:
                    rem.wait()
                    rem = None
                step_split_shards(g, a, b, _lib.SHARDS_LAST, zin[0], zin[1], H, w, k,
                                  self.alpha, out_main=None if last else self.smain[nxt],
                                  out_rem=None if last else self.srem[nxt],
                                  Z=self.zout[:, :w] if last else None, partial=part, **kw)
            # the own shard's send is the only handle left: it precedes the next exchange on
            # the communicator's stream, so waiting for it here costs nothing
            self._wait(shards, 0, R)
            if not last:
                rem, shards = exchange(nxt)
        self.out = self.zout[:, :w]
        return self.out

    def _run_split(self):
        """The row-group loop on the split layout (appnp_step_split): the main columns gather
        whole lines (local / remote parts with overlap), the remainder columns run the
        L2-blocked pass once the exchange of the iterate has landed."""
        from .ops import split_copy, step_split

        if self.pipeline:
            return self._run_split_pipelined()
        K, w, g = self.K, self.width, self.graph
        fs, _ = self.split
        H = self.H[:, :w]
        split_copy(g, H, self.smain[0], self.srem[0])
        works = self._exchange_split(0, async_op=False)
        kw = dict(p_drop=self.p_drop, seed=self.seed)
        for k in range(K):
            cur, nxt = k & 1, (k & 1) ^ 1
            last = k == K - 1
            outs = dict(out_main=None if last else self.smain[nxt],
                        out_rem=None if last else self.srem[nxt],
                        Z=self.zout[:, :w] if last else None)
            zin = (self.smain[cur], self.srem[cur])
            if self.overlap and fs > 0:
                step_split(g, _lib.PART_LOCAL, zin[0], zin[1], None, w, k, self.alpha,
                           partial=self.partial[:, :fs], **kw)
                for wk in works:
                    wk.wait()
                works = []
                step_split(g, _lib.PART_REMOTE, zin[0], zin[1], H, w, k, self.alpha,
                           partial=self.partial[:, :fs], **outs, **kw)
            else:
                for wk in works:
                    wk.wait()
                works = []
                step_split(g, _lib.PART_ALL, zin[0], zin[1], H, w, k, self.alpha, **outs, **kw)
            if not last:
                works = self._exchange_split(nxt, async_op=self.overlap)
        for wk in works:
            wk.wait()
        self.out = self.zout[:, :w]
        return self.out

    def run(self):
        """Z_K for this rank's rows x feature slab; returns a [hi-lo, width] view."""
        K, R = self.K, self.layout.rows
        w = self.width
        lo, hi, shard = self.lo, self.hi, self.shard
        if K == 0:
            self.out = self.H[:, :w]
            return self.out
        if self.split is not None:
            return self._run_split()
        if self.pipeline:
            return self._run_pipelined()
        if R == 1 and self.step_fn is _hip_step:
            # column layout: this rank holds every row of its slab, so the K iterations are one
            # appnp_propagate call (no per-iteration host work between the launches)
            from .ops import propagate_forward

            self.out = propagate_forward(self.graph, self.H[:, :w], K, self.alpha, self.p_drop,
                                         self.seed, out=self.bufs[1][:, :w])
            return self.out
        # Z_0 = H: the full Z_0 needs every row shard of H (iteration 0 gathers from it)
        cur = self.bufs[0]
        cur[lo:hi].copy_(self.H)
        work = self.comm.all_gather_rows(cur, shard, async_op=False) if R > 1 else None
        if R == 1:
            cur = None  # gather straight from H (all rows held)
        nxt_i = 1
        for k in range(K):
            src = self.H if cur is None else cur
            dst = self.bufs[nxt_i]
            out_rows = dst[lo:hi]
            if self.overlap:
                # local columns first (ready before the all-gather of src completes)
                self.step_fn(self, src, out_rows, k, _lib.PART_LOCAL)
                if work is not None:
                    work.wait()
                    work = None
                self.step_fn(self, src, out_rows, k, _lib.PART_REMOTE)
            else:
                if work is not None:
                    work.wait()
                    work = None
                self.step_fn(self, src, out_rows, k, _lib.PART_ALL)
            if k < K - 1 and R > 1:
                # async (overlap) returns a work handle waited on inside the next iteration;
                # sync collectives are stream-ordered and return None
                work = self.comm.all_gather_rows(dst, shard, async_op=self.overlap)
            cur = dst
            nxt_i ^= 1
        if work is not None:
            work.wait()
        self.out = cur[lo:hi, :w]
        return self.out


    def _run_pipelined(self):
        """The row loop with the pipelined exchange (whole rows): every iterate travels by R
        broadcasts, one row shard each; the product runs FIRST on the own shard (complete at
        once), then ACC per group of arrived remote shards, the last group LAST (partial +
        alpha H into the rank's rows)."""
        K, R, w = self.K, self.layout.rows, self.width
        lo, hi = self.lo, self.hi
        ri = self.layout.coords(self.rank)[0]
        cur = self.bufs[0]
        cur[lo:hi].copy_(self.H)
        shards = self._broadcast_shards(cur)
        nxt_i = 1
        for k in range(K):
            dst = self.bufs[nxt_i]
            out_rows = dst[lo:hi]
            self.step_fn(self, cur, out_rows, k, ("shards", ri, ri + 1, _lib.SHARDS_FIRST))
            for i, (a, b) in enumerate(self.groups):
                self._wait(shards, a, b)
                mode = _lib.SHARDS_ACC if i + 1 < len(self.groups) else _lib.SHARDS_LAST
                self.step_fn(self, cur, out_rows, k, ("shards", a, b, mode))
            self._wait(shards, 0, R)  # the own shard's send (see _run_split_pipelined)
            if k < K - 1:
                shards = self._broadcast_shards(dst)
            cur = dst
            nxt_i ^= 1
        self.out = cur[lo:hi, :w]
        return self.out


def agree_split(split, device, group=None):
    """The split layout every rank of the (default) process group takes: this rank's ``split``
    -- (fs, remainder width) or None -- if every rank found the SAME (fs, width), else None
    (whole rows everywhere).  Collective.

    Agreeing only on "split or not" is not enough: the exchanged parts are [rows, fs] and
    [rows, width] buffers, and the relayed exchange (MultipathComm) sizes its staging and its
    P2P messages from the rank's own buffers, so column groups whose slabs split differently --
    F = 73 on 2 x 2 is 37 | 36 columns, i.e. a W8 copy (32 + 5) beside a W4 copy (32 + 4) --
    would send and receive messages of different sizes.  One MIN all-reduce of
    (split, fs, -fs, width, -width) gives the minimum and maximum of both."""
    on_gpu = dist.get_backend(group) == "nccl"
    fs, rw = split if split else (0, 0)
    t = torch.tensor([1 if split else 0, fs, -fs, rw, -rw], dtype=torch.int64,
                     device=device if on_gpu else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    ok, fs_min, fs_max, rw_min, rw_max = (int(x) for x in t.tolist())
    if not ok or fs_min != -fs_max or rw_min != -rw_max:
        return None
    return split


def _hip_step(runner: PartitionedAPPNP, src, out_rows, k, part):
    """One iteration through the C ABI (appnp_step)."""
    from .ops import step

    w = runner.width
    Zin = src[:, :w] if src.shape[0] == runner.graph.n else src[: runner.graph.n, :w]
    H = runner.H[:, :w]
    if isinstance(part, tuple):  # ("shards", s_lo, s_hi, mode): a pipelined step
        from .ops import step_shards

        _, a, b, mode = part
        to_partial = mode in (_lib.SHARDS_FIRST, _lib.SHARDS_ACC)
        step_shards(runner.graph, a, b, mode, Zin, None if to_partial else H,
                    None if to_partial else out_rows[:, :w], runner.partial[:, :w], k,
                    runner.alpha, p_drop=runner.p_drop, seed=runner.seed)
        return
    if part == _lib.PART_LOCAL:
        step(runner.graph, Zin, None, runner.partial[:, :w], k, runner.alpha,
             part=_lib.PART_LOCAL, p_drop=runner.p_drop, seed=runner.seed)
    elif part == _lib.PART_REMOTE:
        step(runner.graph, Zin, H, out_rows[:, :w], k, runner.alpha, part=_lib.PART_REMOTE,
             partial=runner.partial[:, :w], p_drop=runner.p_drop, seed=runner.seed)
    else:
        step(runner.graph, Zin, H, out_rows[:, :w], k, runner.alpha, p_drop=runner.p_drop,
             seed=runner.seed)


class NativeRowAPPNP:
    """The north_star's row partition run by the library's own loop (appnp_dist_*,
    include/ppnp_amd.h): the engine a C/C++ caller gets from the ABI.  This class only drives it
    from Python.  It makes the same launches as ``PartitionedAPPNP`` on a ``Layout(P, 1)``, but
    the K loop, the overlap schedule and the exchange stream live in C++.

    exchange: 'rccl' -- appnp_allgather_rccl on torch's own communicator (the process group's
    ncclComm_t, so RCCL is called from C with no Python per iteration); 'gloo' -- a Python
    callback that stages the shards through host memory (tests: ranks sharing one GPU).
    Default: 'rccl' on an 'nccl' process group, else 'gloo'.  Collective: every rank builds
    and runs it with the same arguments."""

    def __init__(self, indptr, indices, n, device, overlap=True, mode="sym", data=None,
                 exchange=None, rank=None, world=None, features=None, dtype=torch.float32,
                 pipeline=None):
        """features: the F the engine will propagate; when fp32 rows of that width split
        (graph.remainder_width), the held rows get a source-blocked copy and the engine runs the
        split layout (appnp_step_split).  pipeline: the engine's pipelined exchange
        (appnp_dist_set_broadcast: one broadcast per row shard, the product per group of
        arrived shards); None: whenever it applies (overlap, >= 3 ranks)."""
        import ctypes as C

        from .graph import source_block_flags

        lib = _lib.load()
        self.device = torch.device(device)
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        backend = data_backend()
        self.exchange = exchange or ("rccl" if backend == "nccl" else "gloo")
        self._ws = None
        ctx = None
        if self.world == 1:
            fn = None
        elif self.exchange == "rccl":
            pg = _DATA_GROUP or dist.distributed_c10d._get_default_group()
            ctx = C.c_void_p(pg._get_backend(self.device)._comm_ptr())
            fn = _lib.ALLGATHER_FN(C.cast(lib.appnp_allgather_rccl, C.c_void_p).value)
        elif self.exchange == "gloo":
            fn = _lib.ALLGATHER_FN(self._gloo_allgather)
        else:
            raise ValueError(f"unknown exchange {exchange!r}")
        self._fn = fn  # the ctypes callback must outlive the handle
        self._ctx = ctx
        ip = indptr.to(self.device, torch.int32).contiguous()
        ix = indices.to(self.device, torch.int32).contiguous()
        val = None if data is None else data.to(self.device, torch.float32).contiguous()
        h = C.c_void_p()
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        sb = source_block_flags(n, int(features), dtype) if features else 0
        _lib.check("appnp_dist_create", lib.appnp_dist_create(
            C.c_void_p(ip.data_ptr()), C.c_void_p(ix.data_ptr()) if ix.numel() else None,
            C.c_void_p(val.data_ptr()) if val is not None and val.numel() else None, n,
            ix.numel(), _lib.NORM[mode] | sb, self.rank, self.world, int(bool(overlap)), fn, ctx,
            stream, C.byref(h)))
        self._h = h
        lo, hi, shard = C.c_int64(), C.c_int64(), C.c_int64()
        _lib.check("appnp_dist_rows", lib.appnp_dist_rows(h, C.byref(lo), C.byref(hi),
                                                          C.byref(shard)))
        self.n, self.lo, self.hi, self.shard = n, lo.value, hi.value, shard.value
        can = bool(overlap) and self.world >= 3
        if pipeline and not can:
            raise ValueError("pipeline needs overlap and >= 3 ranks")
        self.pipeline = bool(can if pipeline is None else pipeline)
        self._bfn = None
        if self.pipeline:
            if self.exchange == "rccl":
                bfn = _lib.BCAST_FN(C.cast(lib.appnp_bcast_rccl, C.c_void_p).value)
            else:
                bfn = _lib.BCAST_FN(self._gloo_bcast)
            self._bfn = bfn  # the ctypes callback must outlive the handle
            _lib.check("appnp_dist_set_broadcast", lib.appnp_dist_set_broadcast(
                h, bfn, ctx, stream))
        n_g = C.c_int(0)
        lo_g, hi_g = (C.c_int * 64)(), (C.c_int * 64)()
        _lib.check("appnp_dist_pipeline_groups",
                   lib.appnp_dist_pipeline_groups(h, lo_g, hi_g, 64, C.byref(n_g)))
        self.groups = [(lo_g[i], hi_g[i]) for i in range(min(n_g.value, 64))]

    def _gloo_bcast(self, buf, nbytes, root, nranks, stream, ctx):
        self.gloo_bcasts = getattr(self, "gloo_bcasts", 0) + 1  # tests: broadcasts made
        try:
            torch.cuda.synchronize(self.device)
            off = buf - self._ws.data_ptr()
            view = self._ws[off:off + nbytes]
            host = view.cpu()
            dist.broadcast(host, src=root)
            view.copy_(host)
            torch.cuda.synchronize(self.device)
            return 0
        except Exception:  # noqa: BLE001 -- no Python exception may cross the C frame
            return _lib.APPNP_EDEVICE

    def _gloo_allgather(self, buf, shard_bytes, rank, nranks, stream, ctx):
        self.gloo_calls = getattr(self, "gloo_calls", 0) + 1  # tests: exchanges the engine made
        try:
            torch.cuda.synchronize(self.device)
            off = buf - self._ws.data_ptr()
            view = self._ws[off:off + nranks * shard_bytes]
            host = view.cpu()
            parts = list(host.split(shard_bytes))
            dist.all_gather(parts, parts[rank].clone())
            view.copy_(host)
            torch.cuda.synchronize(self.device)
            return 0
        except Exception:  # noqa: BLE001 -- no Python exception may cross the C frame
            return _lib.APPNP_EDEVICE

    def run(self, H_rows, K, alpha, p_drop=0.0, seed=0, out=None):
        """This rank's rows of APPNP_K(H) from this rank's rows ``H_rows`` [hi - lo, F]."""
        import ctypes as C

        lib = _lib.load()
        dtype = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16}[H_rows.dtype]
        f = int(H_rows.shape[1])
        if H_rows.stride(1) != 1:
            H_rows = H_rows.contiguous()
        Z = out if out is not None else torch.empty_like(H_rows)
        need = lib.appnp_dist_workspace_bytes(self._h, f, dtype)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 1), dtype=torch.uint8, device=self.device)
        rows = self.hi - self.lo
        ptr = (lambda t: C.c_void_p(t.data_ptr()) if rows > 0 else None)
        _lib.check("appnp_dist_propagate", lib.appnp_dist_propagate(
            self._h, ptr(H_rows), max(H_rows.stride(0), f), ptr(Z), max(Z.stride(0), f), f,
            dtype, int(K), float(alpha), float(p_drop), int(seed) & (2**64 - 1),
            C.c_void_p(self._ws.data_ptr()), self._ws.numel(),
            C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))
        return Z

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().appnp_dist_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class _DistGraphInfo:
    """The held rows' sizes of an appnp_dist graph (what bench.py reads from runner.graph)."""

    def __init__(self, handle):
        import ctypes as C

        self._h = handle
        n, lo, hi, nnz = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        mode, sym = C.c_int(), C.c_int()
        _lib.check("appnp_graph_info", _lib.load().appnp_graph_info(
            handle, C.byref(n), C.byref(lo), C.byref(hi), C.byref(nnz), C.byref(mode),
            C.byref(sym)))
        self.n, self.row_lo, self.row_hi = n.value, lo.value, hi.value
        self.rows = hi.value - lo.value
        self.nnz_hat = nnz.value

    def source_block_layout(self):
        from .graph import source_block_layout_of

        return source_block_layout_of(self._h)

    def split_layout(self, f: int):
        from .graph import split_layout_of

        return split_layout_of(self._h, f)


class NativeRowRunner:
    """``PartitionedAPPNP``'s runner surface (run(), out, lo/hi, layout, graph) over
    ``NativeRowAPPNP``: how bench.py times the library's own row loop as a layout candidate
    (exchange 'native')."""

    exchange = "native"

    def __init__(self, indptr, indices, n, H, K, alpha, device, overlap=True, mode="sym",
                 data=None, p_drop=0.0, seed=0, pipeline=None):
        self.engine = NativeRowAPPNP(indptr, indices, n, device, overlap=overlap, mode=mode,
                                     data=data, features=int(H.shape[1]), dtype=H.dtype,
                                     pipeline=pipeline)
        self.pipeline = self.engine.pipeline
        self.layout = Layout(self.engine.world, 1)
        self.rank = self.engine.rank
        self.overlap = bool(overlap and self.engine.world > 1)
        self.lo, self.hi = self.engine.lo, self.engine.hi
        self.shard = self.engine.shard
        self.f_lo, self.f_hi = 0, int(H.shape[1])
        self.H = H[self.lo:self.hi].to(device).contiguous()
        self.K, self.alpha, self.p_drop, self.seed = K, alpha, p_drop, seed
        self.out = torch.empty_like(self.H)
        import ctypes as C

        self.graph = _DistGraphInfo(C.c_void_p(_lib.load().appnp_dist_graph(self.engine._h)))
        # the split the engine takes (appnp_dist_propagate: fp32, K >= 2, every rank's copy
        # built; a misaligned H / Z is staged through the workspace since round 5)
        sp = self.graph.split_layout(self.width) if H.dtype == torch.float32 else None
        self.remainder_cols = (self.width - sp[0]) if sp and K >= 2 else 0

    @property
    def width(self) -> int:
        return self.f_hi - self.f_lo

    def run(self):
        return self.engine.run(self.H, self.K, self.alpha, self.p_drop, self.seed, out=self.out)


INT32_MAX = 2**31 - 1


def rank_bytes(layout: Layout, n: int, f: int, nnz_hat: int, elem_bytes: int = 4,
               overlap: bool = False, width: int | None = None) -> int:
    """Device bytes one rank of ``layout`` holds for the K loop (upper estimate): its rows'
    CSR (int32 row_ptr, int32 col + fp32 val; doubled by the local/remote split of overlap
    mode; plus the source-blocked copy where a column slab takes the split-row path), dinv
    (fp64, all n), the H slab of its rows, two full-height Z slabs, and the fp32 partial of
    overlap mode.  ``width``: the widest slab when the cut is not even (line slabs)."""
    R, C = layout.rows, layout.cols
    shard = -(-n // R)
    nnz_r = -(-nnz_hat // R)
    width = width or -(-f // C)
    ld = line_ld(width, elem_bytes)
    csr = 4 * (shard + 1) + 8 * nnz_r
    if overlap:
        csr += 4 * 2 * (shard + 1) + 8 * nnz_r
    from .graph import remainder_width

    w = remainder_width(n, width, torch.float32) if R == 1 and elem_bytes == 4 else 0
    if w:
        # a column slab that takes the split path keeps the source-blocked copy of A_hat
        # (8 B per nonzero plus one int per 2^15-row block and 640 / (w / 4)-row group, and
        # padding: appnp_blocks.hip)
        csr += 9 * nnz_hat + 4 * (-(-n // (1 << 15))) * (-(-n // (640 * 4 // w)) + 1)
    dense = (shard + 2 * shard * R) * ld * elem_bytes + (shard * ld * 4 if overlap else 0)
    return csr + 8 * n + dense


def fits(layout: Layout, n: int, f: int, nnz_hat: int, elem_bytes: int = 4,
         overlap: bool = False, mem_bytes: int | None = None, headroom: float = 0.85,
         width: int | None = None) -> bool:
    """Whether a rank's share stays inside the int32 CSR index range and, given the device
    memory, inside ``headroom`` of it.  A feature-column layout replicates the whole CSR on
    every rank; only row groups split it (the north_star's 'graphs that outgrow one GPU')."""
    if -(-nnz_hat // layout.rows) > INT32_MAX:
        return False
    if mem_bytes is None:
        return True
    return rank_bytes(layout, n, f, nnz_hat, elem_bytes, overlap, width) <= headroom * mem_bytes


def candidate_layouts(world: int, f: int, n: int = 0, nnz_hat: int = 0, elem_bytes: int = 4,
                      mem_bytes: int | None = None):
    """(layout, overlap, exchange) variants ``bench.py --layout auto`` measures, the fastest of
    which it reports (max over ranks).  The first is ``choose_layout``'s: the column partition,
    which needs no exchange, whenever it fits (and its cut at whole lines where that differs).
    Then the north_star's pure row partition (overlapped all-gather) and, from 4 ranks on, the
    two 2-D layouts with 2 row groups or 2 column groups -- 2 x (P/2) (half of each rank's
    gathers for half a slab of exchange) and (P/2) x 2 (a quarter of the rows on 8 ranks,
    two-line gathers) -- which only an xGMI measurement can price.

    Order (round 4): by how standard the exchange is, since a candidate that stalls ends the
    run at its deadline with the best line so far (bench.run_candidates), so whatever comes
    after it is never measured: exchange-free layouts; the row partition's all-gather over all
    ranks; the 2-D layouts' all-gathers within column groups; the library's own row loop
    (RCCL called from C); last the relayed exchange (batched RCCL send/recv).  Candidates that
    do not fit (``fits``) are dropped; if none does, the row-heaviest layout that fits is used."""
    first = choose_layout(world, n, f, nnz_hat, elem_bytes, mem_bytes)
    row = Layout(world, 1)
    # the north_star's design -- a pure row partition, all-gather overlapped with the local
    # product -- is always timed when it fits, so the scaling run measures it next to the rest
    row_fits = world >= 2 and fits(row, n, f, nnz_hat, elem_bytes, True, mem_bytes)
    two_d = []
    if first.rows > 1:  # row groups forced by size: overlap the exchange, try both routes
        if first.cols > 1:
            two_d.append(first)
        cands = [(first, True, "group")]
    else:
        cands = [(first, False, "group")]
        # the column layout cut at whole lines (exchange-free too): fewer lines per gather on
        # the ranks that get whole lines, when that differs from the even cut
        lines = line_slab_cols(f, world, elem_bytes) if first == Layout(1, world) else None
        if (lines and lines != [col_range(f, world, c) for c in range(world)]
                and fits(Layout(1, world, True), n, f, nnz_hat, elem_bytes, False, mem_bytes,
                         width=max(hi - lo for lo, hi in lines))):
            cands.append((Layout(1, world, True), False, "group"))
        if world >= 4 and world % 2 == 0:
            seen = {first}
            for lay in (Layout(2, world // 2), Layout(world // 2, 2)):
                if lay in seen or lay.rows == world or f < lay.cols:
                    continue
                seen.add(lay)
                if fits(lay, n, f, nnz_hat, elem_bytes, True, mem_bytes):
                    two_d.append(lay)
    if row_fits and row != first:
        cands.append((row, True, "group"))
    cands += [(lay, True, "group") for lay in two_d if lay != first]
    if row_fits:
        cands.append((row, True, "native"))
    cands += [(lay, True, "multipath") for lay in two_d]
    return cands


def choose_layout(world: int, n: int, f: int, nnz: int, elem_bytes: int = 4,
                  mem_bytes: int | None = None) -> Layout:
    """Default layout: the column partition (no data-path collective) unless F is too narrow
    to split or a rank's share would not fit (``fits``): then the fewest row groups R (a
    divisor of world) whose shares fit.  Row groups split the CSR, column groups split Z: a
    row layout holds all n rows of Z, so the smallest share is usually a 2-D layout.  See DESIGN.md 'Multi-GPU' for the line-request model
    behind the preference."""
    if f >= world:
        pref = Layout(1, world)
    else:
        c = max(1, math.gcd(world, f))
        pref = Layout(world // c, c)
    if fits(pref, n, f, nnz, elem_bytes, False, mem_bytes):
        return pref
    options = [Layout(r, world // r) for r in range(pref.rows + 1, world + 1) if world % r == 0]
    for lay in options:
        if fits(lay, n, f, nnz, elem_bytes, False, mem_bytes):
            return lay
    # nothing fits the memory: the smallest share inside the index range (the build then
    # reports APPNP_ENOMEM if it really does not fit)
    ok = [lay for lay in [pref] + options if fits(lay, n, f, nnz, elem_bytes)] or [
        Layout(world, 1)]
    return min(ok, key=lambda lay: rank_bytes(lay, n, f, nnz, elem_bytes))
