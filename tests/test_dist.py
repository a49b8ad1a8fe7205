"""CPU, world_size 2-8 (gloo): the multi-GPU orchestration of ppnp_amd.dist against the oracle.

The per-iteration kernel is replaced by an oracle step on the same CSR rows (the GPU kernel
itself is covered by tests/test_gpu_parity.py); what is tested here is the layout, the row /
feature slab bookkeeping, the equal-shard all-gather and the local/remote split of the
overlap mode, for row, column and 2-D layouts.
"""

import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ppnp_oracle as O

N, F, K, ALPHA = 257, 10, 5, 0.15


class _FakeGraph:
    def __init__(self, a_hat, lo, hi, overlap):
        self.n = a_hat.shape[0]
        self.rows_csr = a_hat[lo:hi].tocsr()
        self.nnz_hat = self.rows_csr.nnz
        self.lo, self.hi = lo, hi
        if overlap:
            coo = self.rows_csr.tocoo()
            loc = (coo.col >= lo) & (coo.col < hi)
            shape = self.rows_csr.shape
            self.local = sp.csr_matrix((coo.data[loc], (coo.row[loc], coo.col[loc])), shape=shape)
            self.remote = sp.csr_matrix((coo.data[~loc], (coo.row[~loc], coo.col[~loc])),
                                        shape=shape)

    def shard_offsets(self, nshards, shard_rows):
        """The pipelined steps' source shards (appnp_graph_shard_offsets): the rows' entries by
        the shard of their column."""
        self.shard_rows = shard_rows

    def shard_part(self, s_lo, s_hi):
        coo = self.rows_csr.tocoo()
        m = (coo.col >= s_lo * self.shard_rows) & (coo.col < s_hi * self.shard_rows)
        return sp.csr_matrix((coo.data[m], (coo.row[m], coo.col[m])), shape=self.rows_csr.shape)


def _oracle_step(runner, src, out_rows, k, part):
    from ppnp_amd import _lib

    g = runner.graph
    w = runner.width
    Zin = src[: g.n, :w].double().numpy()
    H = runner.H[:, :w].double().numpy()
    a = 1.0 - runner.alpha
    if isinstance(part, tuple):  # a pipelined step over source shards [s_lo, s_hi)
        _, s_lo, s_hi, mode = part
        y = a * (g.shard_part(s_lo, s_hi) @ Zin)
        P = runner.partial[:, :w].double().numpy()
        if mode == _lib.SHARDS_FIRST:
            runner.partial[:, :w] = torch.from_numpy(y).float()
        elif mode == _lib.SHARDS_ACC:
            runner.partial[:, :w] = torch.from_numpy(y + P).float()
        elif mode == _lib.SHARDS_LAST:
            out_rows[:, :w] = torch.from_numpy(y + P + runner.alpha * H).float()
        else:
            out_rows[:, :w] = torch.from_numpy(y + runner.alpha * H).float()
        runner.shard_steps = getattr(runner, "shard_steps", 0) + 1
        return
    if part == _lib.PART_LOCAL:
        runner.partial[:, :w] = torch.from_numpy(a * (g.local @ Zin)).float()
    elif part == _lib.PART_REMOTE:
        y = a * (g.remote @ Zin) + runner.partial[:, :w].double().numpy() + runner.alpha * H
        out_rows[:, :w] = torch.from_numpy(y).float()
    else:
        out_rows[:, :w] = torch.from_numpy(a * (g.rows_csr @ Zin) + runner.alpha * H).float()


def _worker(rank, world, init, layout_spec, overlap, q, exchange="multipath", f=F,
            pipeline=None):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        from ppnp_amd.dist import Layout, PartitionedAPPNP

        adj = O.synth_graph(N, 4 * N, seed=5)
        a_hat = O.calc_a_hat(adj, "sym")
        H = torch.randn(N, f, generator=torch.Generator().manual_seed(0))
        layout = Layout.parse(layout_spec, world)
        runner = PartitionedAPPNP.create(
            None, None, N, H, K, ALPHA, "cpu", layout=layout, overlap=overlap,
            graph_fn=lambda lo, hi, ov: _FakeGraph(a_hat, lo, hi, ov), step_fn=_oracle_step,
            exchange=exchange, pipeline=pipeline)
        Z = runner.run()
        if pipeline:  # the pipelined schedule ran: FIRST + one launch per shard group per step
            assert runner.pipeline and runner.shard_steps == K * (1 + len(runner.groups))
        ref = O.appnp_propagate(a_hat, H.numpy(), K, ALPHA)
        sub = ref[runner.lo:runner.hi, runner.f_lo:runner.f_hi]
        err = float(np.abs(Z.double().numpy() - sub).max()) if sub.size else 0.0
        q.put((rank, runner.lo, runner.hi, runner.f_lo, runner.f_hi, err))
    finally:
        dist.destroy_process_group()


def _rendezvous():
    """A file:// init method, fresh per run: no TCP port to race for between picking it and
    the store binding it (torch's FileStore removes the file when the last rank is done)."""
    import tempfile
    import uuid

    d = os.path.join(tempfile.gettempdir(), "ppnp_rdv")
    os.makedirs(d, exist_ok=True)
    return "file://" + os.path.join(d, uuid.uuid4().hex)


@pytest.mark.parametrize("world,layout,overlap,exchange,f", [
    (2, "row", False, "group", F), (2, "row", True, "group", F), (2, "col", False, "group", F),
    (2, "1x2", False, "group", F),
    # R x C layouts: two-stage relayed exchange over every rank (MultipathComm) and the
    # plain column-group all-gather
    (8, "2x4", True, "multipath", F), (8, "2x4", False, "multipath", F),
    (8, "4x2", True, "multipath", F),
    (4, "2x2", False, "multipath", F), (8, "2x4", True, "group", F),
    # column slabs cut at whole lines: 40 = 32 | 8, 100 = 32 | 32 | 36
    (2, "col-lines", False, "group", 40), (3, "col-lines", False, "group", 100),
    # uneven slabs on a 2-D layout: F = 73 on 2 x 2 is 37 | 36 columns, so the
    # relayed exchange packs each origin's piece at its own column group's width
    (4, "2x2", False, "multipath", 73), (4, "2x2", True, "multipath", 73),
    (4, "2x2", True, "group", 73)])
def test_partitioned_matches_oracle(world, layout, overlap, exchange, f, pipeline=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(world, _rendezvous(), layout, overlap, q, exchange, f,
                                      pipeline),
                       nprocs=world, join=True, start_method="spawn")
    res = sorted(q.get() for _ in range(world))
    covered = np.zeros((N, f), dtype=bool)
    for rank, lo, hi, flo, fhi, err in res:
        assert err < 1e-5, (rank, err)
        covered[lo:hi, flo:fhi] = True
    assert covered.all()  # every (row, feature) of Z_K is produced exactly by some rank


@pytest.mark.parametrize("world,layout,exchange", [
    (3, "row", "group"), (4, "row", "group"), (8, "row", "group"), (8, "4x2", "group")])
def test_pipelined_row_steps_match_oracle(world, layout, exchange):
    """the iterate travels by R broadcasts, one row shard each, and the
    remote product runs per group of arrived shards (FIRST on the own shard, ACC, LAST); every
    rank's block still matches the oracle at world 3 / 4 / 8, pure rows and 4 x 2."""
    test_partitioned_matches_oracle(world, layout, True, exchange, F, pipeline=True)


def test_shard_groups():
    """Groups of remote shards in arrival order, sized 1, 2, 4 from the last, never spanning
    the own shard; every remote shard exactly once."""
    from ppnp_amd.dist import shard_groups

    assert shard_groups(2, 0) == [(1, 2)] and shard_groups(2, 1) == [(0, 1)]
    assert shard_groups(8, 0) == [(1, 5), (5, 7), (7, 8)]
    assert shard_groups(8, 7) == [(0, 4), (4, 6), (6, 7)]
    # the own shard cuts (0, 4) in two; merging (4, 5) + (5, 7) keeps 3 = log2(8) groups
    assert shard_groups(8, 3) == [(0, 3), (4, 7), (7, 8)]
    assert shard_groups(8, 5) == [(0, 5), (6, 7), (7, 8)]
    for R in range(2, 17):
        for ri in range(R):
            g = shard_groups(R, ri)
            covered = [s for a, b in g for s in range(a, b)]
            assert covered == [s for s in range(R) if s != ri]
            assert all(not (a <= ri < b) for a, b in g)
            assert g[-1][1] - g[-1][0] == 1  # only one shard's compute after the exchange
            assert len(g) <= max(1, (R - 1).bit_length()) + 1


def test_layout_helpers():
    from ppnp_amd.dist import Layout, choose_layout, col_range, line_ld, row_range

    assert Layout.parse("row", 8) == Layout(8, 1)
    assert Layout.parse("col", 8) == Layout(1, 8)
    assert Layout.parse("2x4", 8) == Layout(2, 4)
    with pytest.raises(ValueError):
        Layout.parse("3x3", 8)
    spans = [row_range(10, 3, r) for r in range(3)]
    assert spans == [(0, 4, 4), (4, 8, 4), (8, 10, 4)]
    cols = [col_range(100, 8, c) for c in range(8)]
    assert cols[0][0] == 0 and cols[-1][1] == 100
    assert all(b - a in (12, 13) for a, b in cols)
    # padded only where it lowers the lines per row: 100 fp32 (400 B) spans 4 lines either way
    assert line_ld(25) == 32 and line_ld(13) == 16 and line_ld(50) == 64 and line_ld(100) == 100
    assert line_ld(7) == 8 and line_ld(40, 2) == 64 and line_ld(100, 2) == 128
    assert choose_layout(8, 2_449_029, 100, 126_000_000) == Layout(1, 8)
    from ppnp_amd.dist import candidate_layouts

    # the north_star's pure row partition (overlapped all-gather) is timed at every N >= 2,
    # driven from Python and by the library's own loop (appnp_dist_*)
    # ... and the column layout cut at whole lines, where that differs from the even cut
    assert candidate_layouts(2, 100) == [(Layout(1, 2), False, "group"),
                                         (Layout(1, 2, True), False, "group"),
                                         (Layout(2, 1), True, "group"),
                                         (Layout(2, 1), True, "native")]
    assert (Layout(1, 2, True), False, "group") not in candidate_layouts(2, 128)  # 64 | 64
    c8 = candidate_layouts(8, 100)
    assert c8[0] == (Layout(1, 8), False, "group") and (Layout(2, 4), True, "multipath") in c8
    assert (Layout(8, 1), True, "group") in c8 and (Layout(8, 1), True, "native") in c8
    # both 2-D layouts the single-GPU emulation priced (2x4 1.24 ms, 4x2 1.21 ms
    # per rank-iteration), each with both exchanges; the exchange-free column layout first
    for lay in (Layout(2, 4), Layout(4, 2)):
        assert (lay, True, "multipath") in c8 and (lay, True, "group") in c8
    assert len(c8) == len(set(c8)) == 7
    c4 = candidate_layouts(4, 100)
    assert c4 == [(Layout(1, 4), False, "group"), (Layout(1, 4, True), False, "group"),
                  (Layout(4, 1), True, "group"), (Layout(2, 2), True, "group"),
                  (Layout(4, 1), True, "native"), (Layout(2, 2), True, "multipath")]


def test_line_slabs():
    """Column slabs cut at whole 128-B lines: whole lines first, the remainder on the last
    slab (which holds the fewest lines); None when a slab would be empty."""
    from ppnp_amd.dist import Layout, line_slab_cols, slab_range

    assert line_slab_cols(100, 2) == [(0, 64), (64, 100)]
    assert line_slab_cols(100, 3) == [(0, 32), (32, 64), (64, 100)]
    assert line_slab_cols(100, 4) == [(0, 32), (32, 64), (64, 96), (96, 100)]
    assert line_slab_cols(100, 5) is None and line_slab_cols(100, 8) is None
    assert line_slab_cols(128, 4) == [(0, 32), (32, 64), (64, 96), (96, 128)]
    assert line_slab_cols(128, 5) is None and line_slab_cols(13, 2) is None
    assert line_slab_cols(100, 2, 2) == [(0, 64), (64, 100)]  # bf16: 64 columns per line
    assert Layout.parse("col-lines", 4) == Layout(1, 4, True)
    assert [slab_range(100, Layout(1, 4, True), c) for c in range(4)] == line_slab_cols(100, 4)
    assert slab_range(100, Layout(1, 4), 3) == (75, 100)
    with pytest.raises(ValueError):
        slab_range(100, Layout(1, 8, True), 0)


def test_layout_memory_and_index_limits():
    """Graphs that outgrow one GPU: a column layout replicates the CSR, so a graph whose CSR
    does not fit a rank (or exceeds the int32 index range) gets row groups."""
    from ppnp_amd.dist import Layout, candidate_layouts, choose_layout, fits, rank_bytes

    gb = 1 << 30
    # products-synth on 288 GB: column layout, 2x4 also a candidate
    n, nnz = 2_449_029, 126_166_051
    assert choose_layout(8, n, 100, nnz, 4, 288 * gb) == Layout(1, 8)
    assert (Layout(2, 4), True, "multipath") in candidate_layouts(8, 100, n, nnz, 4, 288 * gb)
    # papers100M-sized: 111 M nodes, 3.2 G nnz -- over int32 unless split in two row groups
    n2, nnz2 = 111_059_956, 3_228_124_712
    assert not fits(Layout(1, 8), n2, 128, nnz2)
    assert choose_layout(8, n2, 128, nnz2, 4, 288 * gb) == Layout(2, 4)
    # ordered by how standard the exchange is (a stalled candidate ends the run): all-gathers
    # first, the library's own loop, the relayed send/recv last
    assert candidate_layouts(8, 128, n2, nnz2, 4, 288 * gb) == [
        (Layout(2, 4), True, "group"), (Layout(8, 1), True, "group"),
        (Layout(8, 1), True, "native"), (Layout(2, 4), True, "multipath")]
    assert candidate_layouts(8, 100, n, nnz, 4, 288 * gb) == [
        (Layout(1, 8), False, "group"), (Layout(8, 1), True, "group"),
        (Layout(2, 4), True, "group"), (Layout(4, 2), True, "group"),
        (Layout(8, 1), True, "native"), (Layout(2, 4), True, "multipath"),
        (Layout(4, 2), True, "multipath")]
    # row groups split the CSR, column groups split Z: 2x4 holds the smallest share here
    shares = {lay: rank_bytes(lay, n, 100, nnz) for lay in
              (Layout(1, 8), Layout(2, 4), Layout(4, 2), Layout(8, 1))}
    assert min(shares, key=shares.get) == Layout(2, 4)
    assert choose_layout(8, n, 100, nnz, 4, int(1.45 * gb)) == Layout(2, 4)
    assert choose_layout(8, n, 100, nnz, 4, gb // 2) == Layout(2, 4)  # nothing fits: smallest
    # a slab on the split-row path also holds the source-blocked copy of A_hat
    assert rank_bytes(Layout(1, 1), n, 100, nnz) - rank_bytes(Layout(1, 1), n, 96, nnz) >= 8 * nnz
    assert rank_bytes(Layout(1, 1), n, 100, nnz, elem_bytes=2) < rank_bytes(Layout(1, 1), n, 96, nnz)
    # the line-cut column layout is held to its WIDEST slab (F = 200 on 2 ranks: 96 | 104 against
    # the even 100 | 100): offered when that fits, dropped when only the even cut does
    lines2 = (Layout(1, 2, True), False, "group")
    assert lines2 in candidate_layouts(2, 200, n, nnz, 4, 288 * gb)
    even, wide = rank_bytes(Layout(1, 2), n, 200, nnz), rank_bytes(Layout(1, 2), n, 200, nnz,
                                                                   width=104)
    assert wide > even
    tight = int((even + wide) / 2 / 0.85)
    assert choose_layout(2, n, 200, nnz, 4, tight) == Layout(1, 2)
    assert lines2 not in candidate_layouts(2, 200, n, nnz, 4, tight)


@pytest.mark.parametrize("spec,world", [("2x4", 8), ("4x2", 8), ("2x2", 4), ("2x3", 6)])
def test_multipath_plan(spec, world):
    """Every send has a matching receive (same pair, origin, rows, in the same per-pair order),
    each rank ends up with every row of its column group's shards, and the per-link load of a
    stage is at most (R-1) pieces."""
    from collections import Counter, defaultdict

    from ppnp_amd.dist import Layout, MultipathComm

    layout = Layout.parse(spec, world)
    shard = 1000
    plans = {r: MultipathComm(layout, r).plan(shard) for r in range(world)}
    for stage in (0, 1):
        sends, recvs = defaultdict(list), defaultdict(list)
        load = Counter()
        for r, p in plans.items():
            for kind, peer, origin, rows, _ in p[stage]:
                if kind == "send":
                    sends[(r, peer)].append((origin, rows))
                    load[(r, peer)] += rows[1] - rows[0]
                else:
                    recvs[(peer, r)].append((origin, rows))
        assert sends == recvs
        piece = -(-shard // (world - 1))
        assert max(load.values()) <= (layout.rows - 1 if stage else 1) * piece
    for r, p in plans.items():
        got = defaultdict(int)
        for kind, peer, origin, rows, where in p[0] + p[1]:
            if kind == "recv" and where == "full":
                got[origin] += rows[1] - rows[0]
        group = MultipathComm(layout, r).group_of(r)
        assert dict(got) == {a: shard for a in group if a != r}


def _agree_worker(rank, world, init, splits, q):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        from ppnp_amd.dist import agree_split

        q.put((rank, agree_split(splits[rank], "cpu")))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("splits,agreed", [
    # every rank found the same split: kept
    ([(32, 4)] * 4, (32, 4)),
    # F = 73 on 2 x 2: column groups of 37 (32 + 5: a W8 copy) and 36 (32 + 4: W4) columns --
    # the exchanged remainder parts would differ in width: whole rows everywhere
    ([(32, 8), (32, 8), (32, 4), (32, 4)], None),
    # different main widths (e.g. 68 | 36): whole rows
    ([(64, 4), (64, 4), (32, 4), (32, 4)], None),
    # one rank's best-effort copy failed: whole rows
    ([(32, 4), None, (32, 4), (32, 4)], None)])
def test_split_agreement_needs_equal_parts(splits, agreed):
    """dist.agree_split, the collective decision of the row-group split layout: every rank
    takes the split only if every rank found the same (main width, remainder width), since
    the parts are exchanged between column groups as equal-size messages."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_agree_worker, args=(4, _rendezvous(), splits, q), nprocs=4, join=True,
                       start_method="spawn")
    res = dict(q.get() for _ in range(4))
    assert all(v == agreed for v in res.values()), res


def test_bf16_row_layout_exchanges_without_overlap():
    """The LOCAL / REMOTE halves and the pipelined shard steps are fp32-only (appnp_step returns
    APPNP_ENOTSUP for bf16 halves), so a bf16 row layout asked to overlap runs the plain
    exchange-then-step loop instead of failing in its first step."""
    from ppnp_amd.dist import Layout, NullComm, PartitionedAPPNP

    a_hat = O.calc_a_hat(O.synth_graph(N, 4 * N, seed=5), "sym")
    H = torch.zeros(N, F, dtype=torch.bfloat16)
    for dtype, want in ((torch.bfloat16, False), (torch.float32, True)):
        r = PartitionedAPPNP.create(None, None, N, H.to(dtype), K, ALPHA, "cpu",
                                    layout=Layout(4, 1), overlap=True, rank=1, world=4,
                                    comm=NullComm(),
                                    graph_fn=lambda lo, hi, ov: _FakeGraph(a_hat, lo, hi, ov),
                                    step_fn=_oracle_step)
        assert r.overlap is want and r.pipeline is want, (dtype, r.overlap, r.pipeline)

