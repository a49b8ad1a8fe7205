"""GPU parity of the split layout on row-partitioned graphs (appnp_split_copy / appnp_step_split,
round 3): P "ranks" run in ONE process on one GPU, each with its own graph of held rows
[lo, hi) and its own source-blocked copy, sharing the two full-height parts of the iterate --
so every rank's rows land where the exchange would put them, and no exchange is needed.

Covered against the float64 oracle (oracle/ppnp_oracle.py appnp_propagate, the K-step series of
helpers.py:58-66): remainders of 4 (W4), 8 (W8) and narrow rows of 13 (W16, no main part);
ALL and LOCAL + REMOTE (split_local); edge dropout keyed on the global row; weighted (values in
the regrouped copy) and unit (value-free, dl/dr scaled) graphs; 'rw' normalisation; uneven
shards (P = 3).  Tolerance: the fp32 bar max|Z - Z_ref| <= 1e-5 max|Z_ref| + 1e-6.
"""

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import ppnp_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
N = 200_000  # above the 2^16-row latency regime; 7 source blocks of 2^15 rows


@pytest.fixture(scope="module")
def adj():
    return O.synth_graph(N, 900_000, seed=13)


@pytest.fixture(scope="module")
def weighted(adj):
    w = adj.copy()
    rng = np.random.default_rng(17)
    w.data = rng.uniform(0.5, 2.0, size=w.nnz).astype(np.float32)
    w = ((w + w.T) * 0.5).tocsr()
    w.sort_indices()
    return w


def _run(a, f, P, K, overlap, p_drop=0.0, mode="sym", alpha=0.1, seed=9):
    """Z_K of the P-rank split loop on one GPU, and the graphs' split layouts."""
    import ppnp_amd
    from ppnp_amd import _lib
    from ppnp_amd.dist import row_range

    shard = row_range(N, P, 0)[2]
    graphs = []
    for r in range(P):
        lo, hi, _ = row_range(N, P, r)
        g = ppnp_amd.Graph.from_csr(a.indptr, a.indices, a.data, N, mode=mode, device=DEV,
                                    row_lo=lo, row_hi=hi, split_local=overlap, features=f)
        graphs.append(g)
    lay = {g.split_layout(f) for g in graphs}
    assert len(lay) == 1 and None not in lay, lay
    fs, rw = lay.pop()
    g_ = torch.Generator().manual_seed(f * 7 + P)
    H = torch.randn(N, f, generator=g_)
    ld = (f + 3) // 4 * 4
    Hb = torch.zeros(N, ld, device=DEV)
    Hb[:, :f] = H.to(DEV)
    rows_pad = shard * P
    mains = [torch.zeros(rows_pad, max(fs, 1), device=DEV) for _ in range(2)]
    rems = [torch.zeros(rows_pad, rw, device=DEV) for _ in range(2)]
    Z = torch.full((N, ld), 7.0, device=DEV)
    parts = [torch.zeros(max(g.rows, 1), max(fs, 4), device=DEV) for g in graphs]
    launches = [g.source_block_layout()["launches"] for g in graphs]
    for g in graphs:
        ppnp_amd.split_copy(g, Hb[g.row_lo:g.row_hi, :f], mains[0] if fs else None, rems[0])
    for k in range(K):
        cur, nxt = k & 1, (k & 1) ^ 1
        last = k == K - 1
        for g, part in zip(graphs, parts):
            Hr = Hb[g.row_lo:g.row_hi, :f]
            out = dict(out_main=None if last else (mains[nxt] if fs else None),
                       out_rem=None if last else rems[nxt],
                       Z=Z[g.row_lo:g.row_hi, :f] if last else None)
            zin = (mains[cur] if fs else None, rems[cur])
            if overlap and fs:
                ppnp_amd.step_split(g, _lib.PART_LOCAL, zin[0], zin[1], None, f, k, alpha,
                                    partial=part[:, :fs], p_drop=p_drop, seed=seed)
                ppnp_amd.step_split(g, _lib.PART_REMOTE, zin[0], zin[1], Hr, f, k, alpha,
                                    partial=part[:, :fs], p_drop=p_drop, seed=seed, **out)
            else:
                ppnp_amd.step_split(g, _lib.PART_ALL, zin[0], zin[1], Hr, f, k, alpha,
                                    p_drop=p_drop, seed=seed, **out)
    torch.cuda.synchronize()
    ran = [g.source_block_layout()["launches"] - b for g, b in zip(graphs, launches)]
    assert ran == [K] * P  # one remainder pass per iteration on every rank
    assert bool((Z[:, f:] == 7.0).all())  # padding columns of Z untouched
    ref = O.appnp_propagate(O.calc_a_hat(a, mode), H.numpy(), K, alpha, p_drop=p_drop, seed=seed)
    return Z[:, :f].double().cpu().numpy(), ref, (fs, rw)


def _close(Z, ref):
    err = np.abs(Z - ref).max()
    tol = 1e-5 * np.abs(ref).max() + 1e-6
    assert err <= tol, f"max err {err:.3e} > tol {tol:.3e}"


@pytest.mark.parametrize("f,layout", [(100, (96, 4)), (40, (32, 8)), (13, (0, 16)),
                                      (36, (32, 4))])
@pytest.mark.parametrize("P,overlap", [(2, False), (3, True)])
def test_split_rows_match_oracle(adj, f, layout, P, overlap):
    if overlap and layout[0] == 0:
        overlap = False  # narrow rows have no main part to split into local / remote
    Z, ref, got = _run(adj, f, P, 3, overlap)
    assert got == layout
    _close(Z, ref)


@pytest.mark.parametrize("overlap", [False, True])
def test_split_rows_dropout(adj, overlap):
    """The mask is keyed on the global row and column: the same edges drop as on one GPU."""
    Z, ref, _ = _run(adj, 100, 3, 3, overlap, p_drop=0.3)
    _close(Z, ref)


@pytest.mark.parametrize("mode", ["sym", "rw"])
def test_split_rows_weighted_and_rw(weighted, mode):
    """Values in the regrouped copy (a weighted graph is not a unit graph) and 'rw'."""
    Z, ref, _ = _run(weighted, 100, 2, 3, True, p_drop=0.2, mode=mode, alpha=0.15)
    _close(Z, ref)


def test_split_rows_rejects_what_does_not_split(adj):
    """appnp_step_split refuses a width that does not split on the graph (ENOTSUP -> the caller
    uses appnp_step) and unaligned operands (EINVAL)."""
    import ppnp_amd
    from ppnp_amd import _lib

    g = ppnp_amd.Graph.from_csr(adj.indptr, adj.indices, None, N, device=DEV, row_lo=0,
                                row_hi=N // 2, features=100)
    assert g.split_layout(100) == (96, 4) and g.split_layout(64) is None
    main = torch.zeros(N, 96, device=DEV)
    rem = torch.zeros(N, 4, device=DEV)
    H = torch.zeros(N // 2, 100, device=DEV)
    with pytest.raises(RuntimeError, match="not supported"):
        ppnp_amd.step_split(g, _lib.PART_ALL, main[:, :64], rem, H[:, :64], 64, 0, 0.1,
                            out_main=main, out_rem=rem)
    Hodd = torch.zeros(N // 2, 101, device=DEV)[:, :100]  # ld 101: no 16-B rows
    with pytest.raises(RuntimeError, match="invalid argument"):
        ppnp_amd.step_split(g, _lib.PART_ALL, main, rem, Hodd, 100, 0, 0.1, out_main=main,
                            out_rem=rem)
    with pytest.raises(RuntimeError, match="invalid argument"):  # LOCAL needs split_local
        ppnp_amd.step_split(g, _lib.PART_LOCAL, main, rem, None, 100, 0, 0.1,
                            partial=torch.zeros(N // 2, 96, device=DEV))
