"""GPU parity of the split-row path (appnp_blocks.hip): fp32 rows of F = 32q + r features,
1 <= r <= 4, gather q cache lines and take the r remainder columns from the L2-resident pass
over A_hat blocked by source rows (APPNP_GRAPH_SOURCE_BLOCKS); with APPNP_GRAPH_SB_W8 / _W16
the pass takes up to 8 / 16 columns, and narrow rows (F <= 8 / 16) run wholly in it.

The graph has more than 2^17 nodes (three source blocks), a hub row (> 512 entries, dispatched
first by the wide kernel) and isolated nodes.  Tolerance: the fp32 bar of test_gpu_parity.py,
max|Z - Z_ref| <= 1e-5 max|Z_ref| + 1e-6, against the float64 oracle.
"""

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import ppnp_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
N = 300_000  # > 2^17 * 2: three source blocks, above the latency regime (2^16 rows)


def close_fp32(Z, ref):
    Z = np.asarray(Z, dtype=np.float64)
    err = np.abs(Z - ref).max()
    tol = 1e-5 * np.abs(ref).max() + 1e-6
    assert err <= tol, f"max err {err:.3e} > tol {tol:.3e}"


@pytest.fixture(scope="module")
def adj():
    a = O.synth_graph(N, 600_000, seed=5).tolil()
    rng = np.random.default_rng(6)
    hub = rng.choice(np.arange(1, N), size=3000, replace=False)
    a[0, hub] = 1.0  # a hub row (and its 3000 mirrored entries)
    a[hub, 0] = 1.0
    a = sp.csr_matrix(a, dtype=np.float32)
    a.sort_indices()
    return a


@pytest.fixture(scope="module")
def ahat(adj):
    return O.calc_a_hat(adj, "sym")


@pytest.fixture(scope="module")
def graphs(adj):
    import ppnp_amd

    split = ppnp_amd.Graph.from_scipy(adj, device=DEV, source_blocks=True)
    plain = ppnp_amd.Graph.from_scipy(adj, device=DEV, source_blocks=False)
    return split, plain


def _h(f, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(N, f, generator=g)


@pytest.mark.parametrize("f", [100, 97, 36, 68, 132])
@pytest.mark.parametrize("K", [2, 3])
def test_split_matches_oracle(graphs, ahat, f, K):
    import ppnp_amd

    H = _h(f, f + K)
    Z = ppnp_amd.propagate_forward(graphs[0], H.to(DEV), K, 0.1)
    close_fp32(Z.double().cpu().numpy(), O.appnp_propagate(ahat, H.numpy(), K, 0.1))


@pytest.mark.parametrize("f", [100, 33])
def test_split_dropout_matches_oracle(graphs, ahat, f):
    import ppnp_amd

    H = _h(f, 11)
    Z = ppnp_amd.propagate_forward(graphs[0], H.to(DEV), 3, 0.1, p_drop=0.3, seed=21)
    ref = O.appnp_propagate(ahat, H.numpy(), 3, 0.1, p_drop=0.3, seed=21)
    close_fp32(Z.double().cpu().numpy(), ref)


@pytest.mark.parametrize("f", [100, 128, 101, 64])
def test_split_agrees_with_plain_path(graphs, f):
    """The split path against the whole-row path on the same graph (F = 128, 101, 64 do not
    split: both graphs must then give bitwise the same result)."""
    import ppnp_amd

    H = _h(f, 3).to(DEV)
    a = ppnp_amd.propagate_forward(graphs[0], H, 10, 0.1)
    b = ppnp_amd.propagate_forward(graphs[1], H, 10, 0.1)
    if f % 32 in (1, 2, 3, 4):
        ref = b.double().cpu().numpy()
        close_fp32(a.double().cpu().numpy(), ref)
    else:
        assert torch.equal(a, b)


def test_split_padded_views_and_determinism(graphs, ahat):
    """H and Z as column views of wider buffers (ld 104 / 112); run-to-run bitwise equal."""
    import ppnp_amd

    f = 100
    H = _h(f, 8)
    Hb = torch.zeros(N, 104, device=DEV)
    Hb[:, :f] = H.to(DEV)
    Zb = torch.full((N, 112), 7.0, device=DEV)
    Z = ppnp_amd.propagate_forward(graphs[0], Hb[:, :f], 4, 0.2, out=Zb[:, :f])
    close_fp32(Z.double().cpu().numpy(), O.appnp_propagate(ahat, H.numpy(), 4, 0.2))
    assert bool((Zb[:, f:] == 7.0).all())  # padding columns untouched
    Z2 = ppnp_amd.propagate_forward(graphs[0], Hb[:, :f], 4, 0.2)
    assert torch.equal(Z, Z2)


def test_split_backward_and_training_path(graphs, ahat):
    """The autograd op composes the split forward and the split adjoint."""
    import ppnp_amd

    f = 100
    H = _h(f, 9).to(DEV).requires_grad_(True)
    Z = ppnp_amd.propagate(graphs[0], H, 3, 0.1)
    W = torch.randn_like(Z)
    (Z * W).sum().backward()
    dref = O.appnp_backward(ahat, W.double().cpu().numpy(), 3, 0.1)
    close_fp32(H.grad.double().cpu().numpy(), dref)


def test_split_plan_replay(graphs):
    """The split path captured into a hipGraph (appnp_plan_*): bitwise the eager result."""
    import ppnp_amd
    from ppnp_amd.ops import PropagatePlan

    H = _h(100, 12).to(DEV)
    plan = PropagatePlan(graphs[0], H, K=4, alpha=0.1)
    try:
        assert torch.equal(plan().clone(), ppnp_amd.propagate_forward(graphs[0], H, 4, 0.1))
        H.mul_(-0.5)  # refill in place and replay
        assert torch.equal(plan().clone(), ppnp_amd.propagate_forward(graphs[0], H, 4, 0.1))
    finally:
        plan.close()


def test_split_point_follows_gather_locality(graphs):
    """Split rows only where gathers miss L2: a uniform graph splits F = 100 at 96; a graph whose
    edges stay within communities of consecutive nodes keeps whole rows (its last line is
    mostly an L2 hit); bf16 and F = 128 never split."""
    import ppnp_amd
    from ppnp_amd import synth

    assert graphs[0].split_point(100) == 96
    assert graphs[0].split_point(97) == 96 and graphs[0].split_point(36) == 32
    assert graphs[0].split_point(128) == 0 and graphs[0].split_point(101) == 0
    assert graphs[0].split_point(100, torch.bfloat16) == 0
    assert graphs[1].split_point(100) == 0  # built without source blocks
    ip, ix = synth.community_graph(N, 1_500_000, 7, device=DEV)
    local = ppnp_amd.Graph.from_csr(ip, ix, None, N, device=DEV, source_blocks=True)
    assert local.split_point(100) == 0


@pytest.mark.parametrize("mode", ["sym", "rw"])
def test_split_weighted_and_rw(adj, mode):
    """Edge weights travel with the source-blocked copy (bval), and 'rw' (not symmetric) uses
    the same path."""
    import ppnp_amd

    w = adj.copy()
    rng = np.random.default_rng(13)
    w.data = rng.uniform(0.5, 2.0, size=w.nnz).astype(np.float32)
    w = ((w + w.T) * 0.5).tocsr()
    w.sort_indices()
    G = ppnp_amd.Graph.from_scipy(w, mode=mode, device=DEV, features=100)
    assert G.split_point(100) == 96
    H = _h(100, 14)
    Z = ppnp_amd.propagate_forward(G, H.to(DEV), 3, 0.15, p_drop=0.2, seed=5)
    ref = O.appnp_propagate(O.calc_a_hat(w, mode), H.numpy(), 3, 0.15, p_drop=0.2, seed=5)
    close_fp32(Z.double().cpu().numpy(), ref)


@pytest.mark.parametrize("case", ["unit-rw", "self-loops"])
def test_split_value_free_layout(adj, case):
    """A unit graph (every entry of A+I is 1) stores no values in the source-blocked copy: the
    remainder buffers carry dr o Z and the epilogue scales by dl (sym: dinv both sides, rw:
    dinv and 1).  'rw' exercises dr = 1; self loops in an unweighted A make the diagonal of
    A+I equal 2, so that graph must keep its values -- same parity either way."""
    import ppnp_amd

    mode = "rw" if case == "unit-rw" else "sym"
    a = adj
    if case == "self-loops":
        a = (adj + sp.diags(np.r_[np.ones(1000), np.zeros(N - 1000)].astype(np.float32))).tocsr()
        a.eliminate_zeros()
        a.sort_indices()
    G = ppnp_amd.Graph.from_scipy(a, mode=mode, device=DEV, features=100)
    assert G.split_point(100) == 96
    w = adj.copy()
    w.data = np.full(w.nnz, 2.0, dtype=np.float32)  # weighted twin: same pattern, with values
    Gw = ppnp_amd.Graph.from_scipy(w, mode=mode, device=DEV, features=100)
    if case == "unit-rw":
        assert G.source_block_bytes() < Gw.source_block_bytes()  # no value stream
    else:
        assert G.source_block_bytes() >= Gw.source_block_bytes()  # values kept
    H = _h(100, 15)
    Z = ppnp_amd.propagate_forward(G, H.to(DEV), 3, 0.15, p_drop=0.2, seed=9)
    ref = O.appnp_propagate(O.calc_a_hat(a, mode), H.numpy(), 3, 0.15, p_drop=0.2, seed=9)
    close_fp32(Z.double().cpu().numpy(), ref)
    Z = ppnp_amd.propagate_forward(G, H.to(DEV), 4, 0.1)
    close_fp32(Z.double().cpu().numpy(), O.appnp_propagate(O.calc_a_hat(a, mode), H.numpy(), 4, 0.1))


def test_split_exact_size_last_row(graphs, ahat):
    """H and Z whose storage ends exactly at the last valid column (ld 100, F = 97): the split
    copy and the remainder epilogue read and write only the valid columns of that row."""
    import ppnp_amd

    f, ld = 97, 100
    H = _h(f, 15)
    hs = torch.zeros((N - 1) * ld + f, device=DEV)
    Hv = hs.as_strided((N, f), (ld, 1))
    Hv.copy_(H.to(DEV))
    zs = torch.full(((N - 1) * ld + f,), 3.0, device=DEV)
    Zv = zs.as_strided((N, f), (ld, 1))
    ppnp_amd.propagate_forward(graphs[0], Hv, 3, 0.1, out=Zv)
    close_fp32(Zv.double().cpu().numpy(), O.appnp_propagate(ahat, H.numpy(), 3, 0.1))
    pad = zs[: (N - 1) * ld].view(N - 1, ld)[:, f:]
    assert bool((pad == 3.0).all())  # the gaps between rows are untouched


@pytest.mark.parametrize("f,K,p", [(100, 2, 0.0), (97, 3, 0.0), (36, 3, 0.25), (100, 4, 0.3)])
def test_split_adjoint_matches_oracle(graphs, ahat, f, K, p):
    """appnp_propagate_bwd in the split layout (self-adjoint A_hat), against the float64
    adjoint of the oracle, with the transposed dropout keys."""
    import ppnp_amd

    dZ = _h(f, 20 + f + K)
    dH = ppnp_amd.propagate_backward(graphs[0], dZ.to(DEV), K, 0.1, p_drop=p, seed=9)
    ref = O.appnp_backward(ahat, dZ.numpy(), K, 0.1, p_drop=p, seed=9)
    close_fp32(dH.double().cpu().numpy(), ref)
    plain = ppnp_amd.propagate_backward(graphs[1], dZ.to(DEV), K, 0.1, p_drop=p, seed=9)
    close_fp32(dH.double().cpu().numpy(), plain.double().cpu().numpy())
    again = ppnp_amd.propagate_backward(graphs[0], dZ.to(DEV), K, 0.1, p_drop=p, seed=9)
    assert torch.equal(dH, again)


def test_split_multi_pass_graph():
    """More rows than one persistent launch holds in LDS (CUs x 16 waves x 640 rows: 2.6 M on
    MI355X): the remainder pass sweeps the source blocks once per pass of row groups.  A
    3 M-node graph, F = 36 (32 + 4), K = 2, against the float64 oracle; run-to-run bitwise."""
    import ppnp_amd

    n = 3_000_000
    a = O.synth_graph(n, 3_000_000, seed=17)
    G = ppnp_amd.Graph.from_scipy(a, device=DEV, features=36)
    assert G.split_point(36) == 32 and G.source_block_bytes() > 0
    H = torch.randn(n, 36, generator=torch.Generator().manual_seed(18))
    Z = ppnp_amd.propagate_forward(G, H.to(DEV), 2, 0.1)
    close_fp32(Z.double().cpu().numpy(), O.appnp_propagate(O.calc_a_hat(a, "sym"), H.numpy(), 2,
                                                           0.1))
    assert torch.equal(Z, ppnp_amd.propagate_forward(G, H.to(DEV), 2, 0.1))


def test_source_blocks_only_when_requested():
    """the regrouped copy costs ~8 B per nonzero, so it is built only for a feature
    width that takes the split path (or on explicit request)."""
    import ppnp_amd

    a = O.synth_graph(70_000, 140_000, seed=19)
    assert ppnp_amd.Graph.from_scipy(a, device=DEV).source_block_bytes() == 0
    # whole lines already (64 = 2 x 32) or one line that is too wide for the pass (17-32)
    assert ppnp_amd.Graph.from_scipy(a, device=DEV, features=64).source_block_bytes() == 0
    assert ppnp_amd.Graph.from_scipy(a, device=DEV, features=20).source_block_bytes() == 0
    assert ppnp_amd.Graph.from_scipy(a, device=DEV, features=100).source_block_bytes() > 0
    assert ppnp_amd.Graph.from_scipy(a, device=DEV, features=7).source_block_bytes() > 0  # W8


def _hook_child(case, ahat, H, K, tmp_path):
    """Run tests/hook_worker.py on the test library (libppnp_amd_test.so, the product library
    has no fault hooks) and return its Z."""
    import os
    import subprocess
    import sys

    from ppnp_amd import _lib

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    data, out = tmp_path / "in.npz", tmp_path / "out.npz"
    np.savez(data, indptr=ahat.indptr.astype(np.int32), indices=ahat.indices.astype(np.int32),
             n=np.int64(N), H=H.numpy())
    env = dict(os.environ, PPNP_AMD_LIB=_lib.TEST_LIB_PATH, PYTHONPATH=root)
    proc = subprocess.run([sys.executable, os.path.join(root, "tests", "hook_worker.py"),
                           "--case", case, "--data", str(data), "--out", str(out),
                           "--K", str(K)],
                          env=env, cwd=root, capture_output=True, text=True, timeout=110)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    return np.load(out)["Z"]


def test_source_blocks_best_effort_fallback(ahat, tmp_path):
    """a graph whose regrouped copy cannot be built (here: more source blocks than
    the limit, lowered for the test through the test library's APPNP_SB_MAX_BLOCKS) is still
    created, warns, and gathers whole rows -- with the same results."""
    H = _h(100, 31)
    Z = _hook_child("max-blocks", ahat, H, 2, tmp_path)
    # ahat's pattern is A + I; an unweighted graph of that pattern (self loops merged) has the
    # same A_hat up to the diagonal weight 2 -- compare against the oracle of that graph
    a = sp.csr_matrix((np.ones(ahat.nnz, dtype=np.float32), ahat.indices, ahat.indptr),
                      shape=ahat.shape)
    close_fp32(Z, O.appnp_propagate(O.calc_a_hat(a, "sym"), H.numpy(), 2, 0.1))


# ---- wider remainders: APPNP_GRAPH_SB_W8 / APPNP_GRAPH_SB_W16 (2 / 4 lanes per entry) --------


@pytest.fixture(scope="module")
def wide(adj):
    """Graphs whose source-blocked copy is laid out for 8 and 16 remainder columns (chosen by
    Graph from the named width: 40 = 32 + 8, narrow rows of 13)."""
    import ppnp_amd

    g8 = ppnp_amd.Graph.from_scipy(adj, device=DEV, features=40)
    g16 = ppnp_amd.Graph.from_scipy(adj, device=DEV, features=13)
    assert g8.source_block_bytes() > 0 and g16.source_block_bytes() > 0
    return {8: g8, 16: g16}


@pytest.mark.parametrize("w,f", [(8, 40), (8, 37), (8, 8), (8, 5), (8, 3), (8, 100),
                                 (16, 47), (16, 44), (16, 48), (16, 13), (16, 16), (16, 9),
                                 (16, 100)])
@pytest.mark.parametrize("K", [2, 3])
def test_wide_remainder_matches_oracle(wide, ahat, w, f, K):
    """Remainders of 5-8 columns and narrow rows against the float64 oracle (F = 100 on the W8
    graph: r = 4 runs the wide pass too; 47, 44, 48 = 32 + 9..16 keep whole rows, and so does
    every F > 32 on the W16 graph, whose 4-lane pass costs more than the extra line:
    profiles/r3_wide_copy_f100.txt)."""
    import ppnp_amd

    G = wide[w]
    r = f % 32 if f > 32 else f
    if f > 32 and (r > 8 or w == 16):
        r = 0
    assert G.remainder_cols(f) == r and G.split_point(f) == (f - r if r else 0)
    H = _h(f, 40 + f + K)
    # leading dimensions that are multiples of 4 (16-B vectors: the split path's condition)
    ld = (f + 3) // 4 * 4
    Hb = torch.zeros(N, ld, device=DEV)
    Hb[:, :f] = H.to(DEV)
    Zb = torch.empty(N, ld, device=DEV)
    before = G.source_block_layout()["launches"]
    Z = ppnp_amd.propagate_forward(G, Hb[:, :f], K, 0.1, out=Zb[:, :f])
    # the path taken, not just the one reported: K remainder launches iff the split applies
    assert G.source_block_layout()["launches"] - before == (K if r else 0)
    close_fp32(Z.double().cpu().numpy(), O.appnp_propagate(ahat, H.numpy(), K, 0.1))
    Z2 = ppnp_amd.propagate_forward(G, Hb[:, :f], K, 0.1, out=torch.empty_like(Zb)[:, :f])
    assert torch.equal(Z, Z2)  # deterministic


def test_wide_remainder_limits(wide, graphs):
    """What each layout takes: 17-32 columns and remainders wider than the layout stay whole."""
    assert wide[8].remainder_cols(41) == 0 and wide[8].remainder_cols(12) == 0
    assert wide[16].remainder_cols(20) == 0 and wide[16].remainder_cols(49) == 0
    assert wide[16].remainder_cols(47) == 0 and wide[16].remainder_cols(40) == 0
    assert wide[16].remainder_cols(100) == 0 and wide[8].remainder_cols(100) == 4
    assert wide[16].remainder_cols(64) == 0 and wide[8].remainder_cols(64) == 0
    assert graphs[0].remainder_cols(3) == 3 and graphs[0].remainder_cols(5) == 0  # W4: narrow <= 4
    assert graphs[1].remainder_cols(3) == 0  # no copy


@pytest.mark.parametrize("w,f,K,p", [(16, 12, 3, 0.3), (8, 40, 3, 0.25), (16, 16, 2, 0.0),
                                     (8, 8, 4, 0.0)])
def test_wide_remainder_dropout_and_adjoint(wide, ahat, w, f, K, p):
    """Edge dropout (counter-hash mask) and the adjoint (transposed keys, adjoint epilogue into
    dH's valid columns) through the wide pass, against the float64 oracle."""
    import ppnp_amd

    G = wide[w]
    H = _h(f, 60 + f)
    Z = ppnp_amd.propagate_forward(G, H.to(DEV), K, 0.1, p_drop=p, seed=23)
    close_fp32(Z.double().cpu().numpy(),
               O.appnp_propagate(ahat, H.numpy(), K, 0.1, p_drop=p, seed=23))
    dH = ppnp_amd.propagate_backward(G, H.to(DEV), K, 0.1, p_drop=p, seed=23)
    close_fp32(dH.double().cpu().numpy(),
               O.appnp_backward(ahat, H.numpy(), K, 0.1, p_drop=p, seed=23))


def test_wide_remainder_padded_views(wide, ahat):
    """Narrow rows as column views of wider buffers (F = 13 in ld 16 / 20): the padding columns
    of Z stay untouched and H's padding is never read into the result."""
    import ppnp_amd

    f = 13
    H = _h(f, 71)
    Hb = torch.full((N, 16), float("nan"), device=DEV)
    Hb[:, :f] = H.to(DEV)
    Zb = torch.full((N, 20), 5.0, device=DEV)
    Z = ppnp_amd.propagate_forward(wide[16], Hb[:, :f], 3, 0.1, out=Zb[:, :f])
    close_fp32(Z.double().cpu().numpy(), O.appnp_propagate(ahat, H.numpy(), 3, 0.1))
    assert bool((Zb[:, f:] == 5.0).all())


@pytest.mark.parametrize("mode", ["sym", "rw"])
def test_wide_remainder_weighted_and_rw(adj, mode):
    """Values in the wide copy (weighted graph) and 'rw' normalisation."""
    import ppnp_amd

    wgt = adj.copy()
    rng = np.random.default_rng(29)
    wgt.data = rng.uniform(0.5, 2.0, size=wgt.nnz).astype(np.float32)
    wgt = ((wgt + wgt.T) * 0.5).tocsr()
    wgt.sort_indices()
    G = ppnp_amd.Graph.from_scipy(wgt, mode=mode, device=DEV, features=40)
    assert G.remainder_cols(40) == 8
    H = _h(40, 33)
    Z = ppnp_amd.propagate_forward(G, H.to(DEV), 3, 0.15, p_drop=0.2, seed=7)
    ref = O.appnp_propagate(O.calc_a_hat(wgt, mode), H.numpy(), 3, 0.15, p_drop=0.2, seed=7)
    close_fp32(Z.double().cpu().numpy(), ref)


@pytest.mark.parametrize("f", [3, 4])
def test_narrow_rows_on_the_four_column_layout(graphs, ahat, f):
    """F <= 4 on the shipped 4-column copy: no main part (fs = 0), every column in the pass
    (LPE = 1), forward and adjoint against the float64 oracle."""
    import ppnp_amd

    G = graphs[0]
    assert G.remainder_cols(f) == f and G.split_point(f) == 0
    H = _h(f, 80 + f)
    Hb = torch.zeros(N, 4, device=DEV)
    Hb[:, :f] = H.to(DEV)
    Zb = torch.full((N, 4), 9.0, device=DEV)
    before = G.source_block_layout()["launches"]
    Z = ppnp_amd.propagate_forward(G, Hb[:, :f], 3, 0.1, out=Zb[:, :f])
    assert G.source_block_layout()["launches"] - before == 3  # ran in the pass
    close_fp32(Z.double().cpu().numpy(), O.appnp_propagate(ahat, H.numpy(), 3, 0.1))
    assert bool((Zb[:, f:] == 9.0).all())
    # a packed [N, f] H of f < 4 columns has no 16-B rows: whole rows, reported as such
    Hp = H.to(DEV).contiguous()
    before = G.source_block_layout()["launches"]
    Zp = ppnp_amd.propagate_forward(G, Hp, 3, 0.1)
    assert G.source_block_layout()["launches"] - before == (3 if f == 4 else 0)
    close_fp32(Zp.double().cpu().numpy(), O.appnp_propagate(ahat, H.numpy(), 3, 0.1))
    if f == 4:  # the adjoint makes dZ contiguous: ld 4 keeps the 16-B vectors
        dH = ppnp_amd.propagate_backward(G, H.to(DEV), 3, 0.1)
        close_fp32(dH.double().cpu().numpy(), O.appnp_backward(ahat, H.numpy(), 3, 0.1))


def test_source_blocks_enomem_leaves_no_stale_error(ahat, tmp_path):
    """a regrouped copy whose allocation really fails (the test library's
    APPNP_SB_TEST_OOM asks for 2^60 bytes) is tolerated -- the graph is created without it,
    warns, and the failed hipMalloc's error is cleared, so the first propagation and an
    unrelated torch kernel both succeed (checked in the child), with the oracle's result."""
    H = _h(100, 37)
    Z = _hook_child("oom", ahat, H, 3, tmp_path)
    a = sp.csr_matrix((np.ones(ahat.nnz, dtype=np.float32), ahat.indices, ahat.indptr),
                      shape=ahat.shape)
    close_fp32(Z, O.appnp_propagate(O.calc_a_hat(a, "sym"), H.numpy(), 3, 0.1))


def test_workspace_covers_the_wide_split_layout(wide):
    """appnp_workspace_bytes counts the split buffers of a W8 / W16 copy ([n, fs] +
    [n, 4 LPE] each), which are wider than a packed narrow row, so the split path runs from a
    workspace of exactly that size instead of silently falling back to whole rows."""
    import ctypes as C

    from ppnp_amd import _lib

    lib = _lib.load()
    for w, f in ((16, 8), (16, 4), (8, 4), (16, 13)):
        G = wide[w]
        ws = int(lib.appnp_workspace_bytes(G.handle, f, f, _lib.F32))
        buf = ((N * 16 * (w // 4) + 255) // 256) * 256  # fs = 0: the remainder part only
        assert ws >= 2 * buf, (w, f, ws, buf)
        H = torch.zeros(N, 4 * ((f + 3) // 4), device=DEV)[:, :f]
        Z = torch.empty(N, 4 * ((f + 3) // 4), device=DEV)[:, :f]
        wsb = torch.empty(ws, dtype=torch.uint8, device=DEV)
        before = G.source_block_layout()["launches"]
        rc = lib.appnp_propagate(G.handle, C.c_void_p(H.data_ptr()), H.stride(0),
                                 C.c_void_p(Z.data_ptr()), Z.stride(0), f, _lib.F32, 2, 0.1,
                                 0.0, 0, C.c_void_p(wsb.data_ptr()), ws,
                                 C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0
        assert G.source_block_layout()["launches"] - before == 2, (w, f)


@pytest.mark.parametrize("f,ld", [(100, 128), (36, 64), (132, 160), (100, 104)])
@pytest.mark.parametrize("p", [0.0, 0.25])
def test_split_from_line_aligned_h(graphs, ahat, f, ld, p):
    """H in a wider buffer whose padding holds NaN (ld a multiple of 32 floats, whole-line rows,
    or 104: 16-B but not line aligned), forward and adjoint on the split path against the
    float64 oracle and bitwise against a packed H: the split copy reads the remainder's last
    16-B piece across the row end and must zero what lies past column F."""
    import ppnp_amd

    G = graphs[0]
    H = _h(f, 90 + f)
    Hb = torch.full((N, ld), float("nan"), device=DEV)
    Hb[:, :f] = H.to(DEV)
    assert Hb.data_ptr() % 128 == 0
    before = G.source_block_layout()["launches"]
    Z = ppnp_amd.propagate_forward(G, Hb[:, :f], 3, 0.1, p_drop=p, seed=5)
    assert G.source_block_layout()["launches"] - before == 3  # the split path
    close_fp32(Z.double().cpu().numpy(),
               O.appnp_propagate(ahat, H.numpy(), 3, 0.1, p_drop=p, seed=5))
    Zp = ppnp_amd.propagate_forward(G, H.to(DEV).contiguous(), 3, 0.1, p_drop=p, seed=5)
    assert torch.equal(Z, Zp)  # same sums, whichever buffer the first step gathered from
    dH = ppnp_amd.propagate_backward(G, Hb[:, :f], 3, 0.1, p_drop=p, seed=5)
    close_fp32(dH.double().cpu().numpy(),
               O.appnp_backward(ahat, H.numpy(), 3, 0.1, p_drop=p, seed=5))
