"""CPU, world_size 2-3 (gloo): the split-row loop of a row-partitioned rank
(ppnp_amd.dist.PartitionedAPPNP._run_split) against the oracle.

The two C entry points it drives -- appnp_split_copy (Z_0's held rows into the two full-height
parts) and appnp_step_split (one iteration: the main columns through the SpMM kernel, ALL or
LOCAL then REMOTE, and the remainder columns through the L2-blocked pass) -- are replaced by an
oracle restatement of their contract (include/ppnp_amd.h) on the same CSR rows; the HIP kernels
themselves are checked by tests/test_gpu_configs.py::test_row_partition_split_rows_matches_oracle.
What is tested here is the bookkeeping: both parts exchanged every iteration, the overlap order
(LOCAL before the exchange of the iterate lands, REMOTE and the remainder pass after it), the
last iteration into the held rows of Z, and uneven shards.
"""

import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ppnp_oracle as O

N, F, K, ALPHA, FS, RW = 301, 100, 4, 0.1, 96, 4


class _SplitGraph:
    """What PartitionedAPPNP reads from a Graph on the split path, over an oracle CSR."""

    def __init__(self, a_hat, lo, hi, overlap):
        self.n = a_hat.shape[0]
        self.row_lo, self.row_hi = lo, hi
        self.rows_csr = a_hat[lo:hi].tocsr()
        self.nnz_hat = self.rows_csr.nnz
        coo = self.rows_csr.tocoo()
        loc = (coo.col >= lo) & (coo.col < hi)
        shape = self.rows_csr.shape
        self.local = sp.csr_matrix((coo.data[loc], (coo.row[loc], coo.col[loc])), shape=shape)
        self.remote = sp.csr_matrix((coo.data[~loc], (coo.row[~loc], coo.col[~loc])), shape=shape)
        self.split = bool(overlap)
        self.events = []  # (kind, k) in call order

    def split_layout(self, f):
        return (f - 4, RW) if f == F else None

    def shard_offsets(self, nshards, shard_rows):  # appnp_graph_shard_offsets
        self.shard_rows = shard_rows

    def shard_part(self, s_lo, s_hi):
        coo = self.rows_csr.tocoo()
        m = (coo.col >= s_lo * self.shard_rows) & (coo.col < s_hi * self.shard_rows)
        return sp.csr_matrix((coo.data[m], (coo.row[m], coo.col[m])), shape=self.rows_csr.shape)


def _split_copy(g, H, main, rem):
    r = H.shape[1] - FS
    main[g.row_lo:g.row_hi] = H[:, :FS]
    rem[g.row_lo:g.row_hi, :r] = H[:, FS:]
    g.events.append(("copy", -1))


def _step_split(g, part, zin_main, zin_rem, H, f, k, alpha, out_main=None, out_rem=None, Z=None,
                partial=None, p_drop=0.0, seed=0):
    from ppnp_amd import _lib

    r = f - FS
    a = 1.0 - alpha
    zm = zin_main[: g.n].double().numpy()
    g.events.append(({_lib.PART_ALL: "all", _lib.PART_LOCAL: "local",
                      _lib.PART_REMOTE: "remote"}[part], k))
    if part == _lib.PART_LOCAL:
        partial[:, :FS] = torch.from_numpy(a * (g.local @ zm)).float()
        return
    Hd = H.double().numpy()
    if part == _lib.PART_REMOTE:
        main = a * (g.remote @ zm) + partial[:, :FS].double().numpy() + alpha * Hd[:, :FS]
    else:
        main = a * (g.rows_csr @ zm) + alpha * Hd[:, :FS]
    zr = zin_rem[: g.n, :r].double().numpy()
    remv = a * (g.rows_csr @ zr) + alpha * Hd[:, FS:]
    if Z is not None:
        Z[:, :FS] = torch.from_numpy(main).float()
        Z[:, FS:f] = torch.from_numpy(remv).float()
    else:
        out_main[g.row_lo:g.row_hi] = torch.from_numpy(main).float()
        out_rem[g.row_lo:g.row_hi, :r] = torch.from_numpy(remv).float()


def _step_split_shards(g, s_lo, s_hi, mode, zin_main, zin_rem, H, f, k, alpha, out_main=None,
                       out_rem=None, Z=None, partial=None, p_drop=0.0, seed=0):
    """appnp_step_split_shards' contract: the main columns over source shards [s_lo, s_hi) in
    `mode`; LAST also finishes the rows and runs the remainder pass (every row of zin_rem)."""
    from ppnp_amd import _lib

    a = 1.0 - alpha
    zm = zin_main[: g.n].double().numpy()
    y = a * (g.shard_part(s_lo, s_hi) @ zm)
    name = {_lib.SHARDS_FIRST: "first", _lib.SHARDS_ACC: "acc", _lib.SHARDS_LAST: "last",
            _lib.SHARDS_ONLY: "only"}[mode]
    g.events.append((name, k, s_lo, s_hi))
    if mode == _lib.SHARDS_FIRST:
        partial[:, :FS] = torch.from_numpy(y).float()
        return
    if mode == _lib.SHARDS_ACC:
        partial[:, :FS] = torch.from_numpy(y + partial[:, :FS].double().numpy()).float()
        return
    r = f - FS
    Hd = H.double().numpy()
    main = y + partial[:, :FS].double().numpy() + alpha * Hd[:, :FS]
    zr = zin_rem[: g.n, :r].double().numpy()
    remv = a * (g.rows_csr @ zr) + alpha * Hd[:, FS:]
    if Z is not None:
        Z[:, :FS] = torch.from_numpy(main).float()
        Z[:, FS:f] = torch.from_numpy(remv).float()
    else:
        out_main[g.row_lo:g.row_hi] = torch.from_numpy(main).float()
        out_rem[g.row_lo:g.row_hi, :r] = torch.from_numpy(remv).float()


def _worker(rank, world, init, overlap, q, pipeline=None):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        from ppnp_amd import dist as pdist
        from ppnp_amd import ops

        ops.split_copy = _split_copy  # the loop imports them from ppnp_amd.ops at run time
        ops.step_split = _step_split
        ops.step_split_shards = _step_split_shards
        adj = O.synth_graph(N, 900, seed=3)
        a_hat = O.calc_a_hat(adj, "sym")
        g = torch.Generator().manual_seed(5)
        H = torch.randn(N, F, generator=g)
        made = {}

        def graph_fn(lo, hi, ov):
            made["g"] = _SplitGraph(a_hat, lo, hi, ov)
            return made["g"]

        runner = pdist.PartitionedAPPNP.create(adj.indptr, adj.indices, N, H, K, ALPHA, "cpu",
                                               layout=pdist.Layout(world, 1), overlap=overlap,
                                               graph_fn=graph_fn, pipeline=pipeline)
        assert runner.split == (FS, RW) and runner.remainder_cols == 4
        Z = runner.run()
        ref = O.appnp_propagate(a_hat, H.double().numpy(), K, ALPHA)[runner.lo:runner.hi]
        err = float(np.abs(Z.double().numpy() - ref).max()) if ref.size else 0.0
        q.put((rank, err, made["g"].events, runner.groups))
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


@pytest.mark.parametrize("world,overlap,pipeline", [(2, False, None), (2, True, None),
                                                    (3, True, False), (3, True, None),
                                                    (4, True, None)])
def test_row_split_loop_matches_oracle(world, overlap, pipeline):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(world, _rendezvous(), overlap, q, pipeline), nprocs=world,
                       join=True, start_method="spawn")
    res = sorted(q.get() for _ in range(world))
    piped = overlap and world >= 3 and pipeline is not False
    for rank, err, events, groups in res:
        assert err <= 1e-5, (rank, err)
        assert events[0] == ("copy", -1)
        if piped:
            # per iteration FIRST on the own shard, ACC per group of arrived
            # remote shards, LAST (with the remainder pass) on the last group
            want = []
            for k in range(K):
                want.append(("first", k, rank, rank + 1))
                want += [("acc", k, a, b) for a, b in groups[:-1]]
                want.append(("last", k, *groups[-1]))
            assert events[1:] == want, (rank, events[1:])
            continue
        # Z_0 copied once; per iteration LOCAL then REMOTE (overlap) or ALL
        per_k = ["local", "remote"] if overlap else ["all"]
        assert events[1:] == [(kind, k) for k in range(K) for kind in per_k]
