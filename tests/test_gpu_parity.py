"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference fixtures.

Tolerances (north_star: "within a stated fp32 tolerance"):
  fp32 storage : max|Z - Z_ref| <= 1e-5 * max|Z_ref| + 1e-6   
  bf16 storage : max|Z - Z_ref| <= 2e-2 * max|Z_ref|, argmax agreement >= 0.98 (section 7 step 5)
  A_hat build  : bit-exact (int32 structure, fp32 values == float32(reference fp64))
"""

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import ppnp_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _lib():
    import ppnp_amd

    return ppnp_amd


def adj_of(g, prefix="adj"):
    n = int(g["n"])
    return sp.csr_matrix((g[f"{prefix}_data"], g[f"{prefix}_indices"], g[f"{prefix}_indptr"]),
                         shape=(n, n))


def close_fp32(Z, ref):
    Z = np.asarray(Z, dtype=np.float64)
    err = np.abs(Z - ref).max()
    tol = 1e-5 * np.abs(ref).max() + 1e-6
    assert err <= tol, f"max err {err:.3e} > tol {tol:.3e}"


def to_np(t):
    return t.float().cpu().numpy().astype(np.float64)


# ---------------------------------------------------------------------------------------
# A_hat construction (helpers.py:58-66) -- bit-exact
# ---------------------------------------------------------------------------------------


@pytest.mark.parametrize("ds", ["cora", "citeseer"])
@pytest.mark.parametrize("mode", ["sym", "rw"])
def test_graph_build_bit_exact(ds, mode, request):
    g = request.getfixturevalue(ds)
    pa = _lib()
    G = pa.Graph.from_scipy(adj_of(g), mode=mode, device=DEV)
    rp, col, val, _ = G.csr()
    assert np.array_equal(rp.cpu().numpy(), g[f"ahat_{mode}_indptr"])
    assert np.array_equal(col.cpu().numpy(), g[f"ahat_{mode}_indices"])
    ref = g[f"ahat_{mode}_data"].astype(np.float32)
    assert np.array_equal(val.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    assert G.symmetric


@pytest.mark.parametrize("name", ["complete5", "complete2", "path3", "isolated3", "weighted4",
                                  "selfloop3"])
@pytest.mark.parametrize("mode", ["sym", "rw"])
def test_graph_build_kat(kat, name, mode):
    pa = _lib()
    n = len(kat[f"{name}_indptr"]) - 1
    G = pa.Graph.from_csr(kat[f"{name}_indptr"], kat[f"{name}_indices"], kat[f"{name}_data"], n,
                          mode=mode, device=DEV)
    rp, col, val, _ = G.csr()
    dense = sp.csr_matrix((val.cpu().numpy(), col.cpu().numpy(), rp.cpu().numpy()),
                          shape=(n, n)).toarray()
    ref = kat[f"{name}_ahat_{mode}_dense"].astype(np.float32)
    assert np.array_equal(dense.astype(np.float32), ref)


def test_graph_rejects_unsorted():
    pa = _lib()
    indptr = np.array([0, 2, 3, 4], dtype=np.int32)
    indices = np.array([2, 1, 0, 0], dtype=np.int32)  # row 0 unsorted
    with pytest.raises(pa._lib.AppnpError) as e:
        pa.Graph.from_csr(indptr, indices, None, 3, device=DEV)
    assert e.value.code == pa._lib.APPNP_EINVAL


# ---------------------------------------------------------------------------------------
# propagation vs the reference fixtures
# ---------------------------------------------------------------------------------------


@pytest.mark.parametrize("ds", ["cora", "citeseer"])
@pytest.mark.parametrize("mode,K,alpha,key", [("sym", 10, 0.1, "Z_sym_K10_a0.1"),
                                              ("sym", 20, 0.2, "Z_sym_K20_a0.2"),
                                              ("rw", 10, 0.1, "Z_rw_K10_a0.1")])
def test_propagate_fixture(ds, mode, K, alpha, key, request):
    g = request.getfixturevalue(ds)
    pa = _lib()
    G = pa.Graph.from_scipy(adj_of(g), mode=mode, device=DEV)
    H = torch.from_numpy(g["H"]).to(DEV)
    Z = pa.propagate_forward(G, H, K, alpha)
    close_fp32(to_np(Z), g[key])


def test_propagate_converges_to_ppr(cora):
    """K -> infinity limit equals compute_ppr(adj, a) @ H (helpers.py:68-71)."""
    pa = _lib()
    G = pa.Graph.from_scipy(adj_of(cora), device=DEV)
    H = torch.from_numpy(cora["H"]).to(DEV)
    Z = to_np(pa.propagate_forward(G, H, 200, 0.1))
    ref = cora["pprH_a0.1"]
    assert np.abs(Z - ref).max() <= 1e-5 * np.abs(ref).max()


# ---------------------------------------------------------------------------------------
# shapes, widths, dtypes, edge cases vs the oracle on seeded synthetic graphs
# ---------------------------------------------------------------------------------------


def synth(n, m, seed):
    return O.synth_graph(n, m, seed)


@pytest.mark.parametrize("F", [1, 2, 3, 4, 6, 7, 8, 15, 16, 33, 64, 100, 128, 256, 300, 520])
def test_propagate_widths(F):
    pa = _lib()
    adj = synth(3000, 15000, seed=F)
    G = pa.Graph.from_scipy(adj, device=DEV)
    ah = O.calc_a_hat(adj, "sym")
    H = torch.randn(3000, F, generator=torch.Generator().manual_seed(F))
    Z = pa.propagate_forward(G, H.to(DEV), 10, 0.1)
    close_fp32(to_np(Z), O.appnp_propagate(ah, H.numpy(), 10, 0.1))


@pytest.mark.parametrize("K", [0, 1, 2, 3])
def test_propagate_small_K(K):
    pa = _lib()
    adj = synth(500, 2000, seed=7)
    G = pa.Graph.from_scipy(adj, device=DEV)
    H = torch.randn(500, 12, generator=torch.Generator().manual_seed(1))
    Z = pa.propagate_forward(G, H.to(DEV), K, 0.15)
    close_fp32(to_np(Z), O.appnp_propagate(O.calc_a_hat(adj, "sym"), H.numpy(), K, 0.15))


def test_propagate_padded_ld():
    """H/Z with a leading dimension > F (row slices of a wider buffer)."""
    pa = _lib()
    adj = synth(800, 4000, seed=3)
    G = pa.Graph.from_scipy(adj, device=DEV)
    base = torch.randn(800, 40, generator=torch.Generator().manual_seed(2)).to(DEV)
    H = base[:, :30]
    Zbuf = torch.zeros(800, 36, device=DEV)
    pa.propagate_forward(G, H, 5, 0.1, out=Zbuf[:, :30])
    ref = O.appnp_propagate(O.calc_a_hat(adj, "sym"), H.cpu().numpy(), 5, 0.1)
    close_fp32(to_np(Zbuf[:, :30]), ref)
    assert torch.all(Zbuf[:, 30:] == 0)


def test_propagate_isolated_and_weighted(kat):
    pa = _lib()
    for name in ("isolated3", "weighted4", "selfloop3"):
        n = len(kat[f"{name}_indptr"]) - 1
        for mode in ("sym", "rw"):
            G = pa.Graph.from_csr(kat[f"{name}_indptr"], kat[f"{name}_indices"],
                                  kat[f"{name}_data"], n, mode=mode, device=DEV)
            H = torch.randn(n, 5, generator=torch.Generator().manual_seed(0))
            Z = to_np(pa.propagate_forward(G, H.to(DEV), 300, 0.1))
            ref = kat[f"{name}_ppr_{mode}_a0.1"] @ H.numpy().astype(np.float64)
            assert np.abs(Z - ref).max() <= 1e-5 * np.abs(ref).max() + 1e-6


def test_complete_graph_closed_form(kat):
    """K_n: Z_K = a H + (1-a) mean_rows(H) for every K >= 1."""
    pa = _lib()
    n = 5
    G = pa.Graph.from_csr(kat["complete5_indptr"], kat["complete5_indices"],
                          kat["complete5_data"], n, device=DEV)
    H = torch.randn(n, 9, generator=torch.Generator().manual_seed(5)).double()
    ref = 0.1 * H + 0.9 * H.mean(0, keepdim=True)
    for K in (1, 4, 10):
        Z = to_np(pa.propagate_forward(G, H.float().to(DEV), K, 0.1))
        assert np.abs(Z - ref.numpy()).max() < 1e-6


def test_empty_and_edgeless():
    pa = _lib()
    # graph with nodes but no edges: A_hat = I -> Z = H
    indptr = np.zeros(6, dtype=np.int32)
    G = pa.Graph.from_csr(indptr, np.zeros(0, dtype=np.int32), None, 5, device=DEV)
    H = torch.randn(5, 3).to(DEV)
    assert torch.allclose(pa.propagate_forward(G, H, 10, 0.1), H, atol=1e-6)
    # zero feature columns
    Z = pa.propagate_forward(G, torch.zeros(5, 0, device=DEV), 10, 0.1)
    assert Z.shape == (5, 0)


def test_bf16_storage():
    pa = _lib()
    adj = synth(18333, 81894, seed=3)  # MS-Academic-sized (config 3)
    G = pa.Graph.from_scipy(adj, device=DEV)
    H = torch.randn(18333, 15, generator=torch.Generator().manual_seed(0))
    Zb = to_np(pa.propagate_forward(G, H.bfloat16().to(DEV), 20, 0.2))
    ref = O.appnp_propagate(O.calc_a_hat(adj, "sym"), H.bfloat16().float().numpy(), 20, 0.2)
    assert np.abs(Zb - ref).max() <= 2e-2 * np.abs(ref).max()
    assert (Zb.argmax(1) == ref.argmax(1)).mean() >= 0.98


def test_deterministic():
    pa = _lib()
    adj = synth(5000, 40000, seed=11)
    G = pa.Graph.from_scipy(adj, device=DEV)
    H = torch.randn(5000, 100, generator=torch.Generator().manual_seed(3)).to(DEV)
    a = pa.propagate_forward(G, H, 10, 0.1)
    b = pa.propagate_forward(G, H, 10, 0.1)
    assert torch.equal(a, b)


# ---------------------------------------------------------------------------------------
# edge dropout (bit-exact mask vs the oracle's counter hash) and backward
# ---------------------------------------------------------------------------------------


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_edge_dropout_matches_oracle(p):
    pa = _lib()
    adj = synth(2000, 10000, seed=5)
    G = pa.Graph.from_scipy(adj, device=DEV)
    H = torch.randn(2000, 16, generator=torch.Generator().manual_seed(9))
    Z = to_np(pa.propagate_forward(G, H.to(DEV), 6, 0.1, p_drop=p, seed=1234))
    ref = O.appnp_propagate(O.calc_a_hat(adj, "sym"), H.numpy(), 6, 0.1, p_drop=p, seed=1234)
    close_fp32(Z, ref)
    Z2 = to_np(pa.propagate_forward(G, H.to(DEV), 6, 0.1, p_drop=p, seed=1235))
    assert np.abs(Z2 - Z).max() > 1e-3  # a different seed gives a different mask


@pytest.mark.parametrize("p", [0.0, 0.3])
@pytest.mark.parametrize("K", [1, 2, 5])
def test_backward_matches_oracle(p, K):
    pa = _lib()
    adj = synth(1500, 6000, seed=2)
    G = pa.Graph.from_scipy(adj, device=DEV)
    dZ = torch.randn(1500, 8, generator=torch.Generator().manual_seed(4))
    dH = to_np(pa.propagate_backward(G, dZ.to(DEV), K, 0.1, p_drop=p, seed=77))
    ref = O.appnp_backward(O.calc_a_hat(adj, "sym"), dZ.numpy(), K, 0.1, p_drop=p, seed=77)
    close_fp32(dH, ref)


def test_autograd_gradcheck_small():
    pa = _lib()
    adj = synth(60, 200, seed=1)
    G = pa.Graph.from_scipy(adj, device=DEV)
    H = torch.randn(60, 4, device=DEV, requires_grad=True)
    Z = pa.propagate(G, H, 4, 0.2, p_drop=0.2, seed=3)
    W = torch.randn_like(Z)
    (Z * W).sum().backward()
    # <J H, W> == <H, J^T W> on the same mask (linearity in H)
    Hd = H.detach()
    lhs = (pa.propagate_forward(G, Hd, 4, 0.2, 0.2, 3) * W).sum().item()
    rhs = (Hd * H.grad).sum().item()
    assert abs(lhs - rhs) <= 1e-4 * max(1.0, abs(lhs))


def test_backward_unsupported_without_transpose():
    pa = _lib()
    adj = synth(100, 300, seed=1)
    G = pa.Graph.from_scipy(adj, mode="rw", device=DEV)
    with pytest.raises(pa._lib.AppnpError) as e:
        pa.propagate_backward(G, torch.randn(100, 3, device=DEV), 3, 0.1)
    assert e.value.code == pa._lib.APPNP_ENOTSUP


@pytest.mark.parametrize("mode", ["rw", "sym"])
@pytest.mark.parametrize("directed", [False, True])
@pytest.mark.parametrize("p", [0.0, 0.25])
def test_backward_with_transpose(mode, directed, p):
    """rw and directed graphs: the adjoint runs over A_hat^T built at creation."""
    pa = _lib()
    adj = synth(1200, 5000, seed=3)
    if directed:
        adj = sp.triu(adj, format="csr").astype(np.float32)
        adj.sort_indices()
    G = pa.Graph.from_scipy(adj, mode=mode, device=DEV, transpose=True)
    dZ = torch.randn(1200, 6, generator=torch.Generator().manual_seed(2))
    dH = to_np(pa.propagate_backward(G, dZ.to(DEV), 5, 0.1, p_drop=p, seed=8))
    ref = O.appnp_backward(O.calc_a_hat(adj, mode), dZ.numpy(), 5, 0.1, p_drop=p, seed=8)
    close_fp32(dH, ref)


# ---------------------------------------------------------------------------------------
# model surface (model.py:41-67)
# ---------------------------------------------------------------------------------------


@pytest.mark.parametrize("ds", ["cora", "citeseer"])
def test_ppnp_and_appnp_logits(ds, request):
    g = request.getfixturevalue(ds)
    pa = _lib()
    n, C = int(g["n"]), int(g["n_classes"])
    X = torch.from_numpy(g["ppnp_X"])
    idx = torch.from_numpy(g["ppnp_idx"])
    ref = g["ppnp_logits"]
    # unchanged PPNP surface with the reference's dense ppr
    ppr = torch.from_numpy(O.compute_ppr(adj_of(g), 0.1)).float()
    net = pa.PPNP(n_features=X.shape[1], n_classes=C, ppr=ppr)
    net.encoder[1].weight.data.copy_(torch.from_numpy(g["ppnp_W1"]))
    net.encoder[4].weight.data.copy_(torch.from_numpy(g["ppnp_W2"]))
    net = net.to(DEV).eval()
    with torch.no_grad():
        out = net(X.to(DEV), idx.to(DEV)).cpu().numpy()
    assert np.abs(out - ref).max() <= 1e-4 * np.abs(ref).max()
    # APPNP drop-in: same weights, HIP propagation with large K converges to the PPNP logits
    ap = pa.APPNP(n_features=X.shape[1], n_classes=C, adj=adj_of(g), alpha=0.1, K=200)
    ap.encoder.load_state_dict(net.encoder.state_dict())
    ap = ap.to(DEV).eval()
    with torch.no_grad():
        out2 = ap(X.to(DEV), idx.to(DEV)).cpu().numpy()
    assert np.abs(out2 - ref).max() <= 1e-4 * np.abs(ref).max()
    with pytest.raises(Exception):
        ap(X.to(DEV))
    # batch mode (model.py:65)
    sub = ppr[idx[:16]].to(DEV)
    with torch.no_grad():
        out3 = ap(X.to(DEV), idx=None, ppr=sub).cpu().numpy()
    ref3 = g["ppnp_logits_ppr_mode"]
    assert np.abs(out3 - ref3).max() <= 1e-4 * np.abs(ref3).max()


def test_appnp_eval_memo(cora):
    """Eval-mode, no-grad forwards of the same X and weights share one propagation (main.py
    evaluates stopping and validation sets back to back); any change recomputes."""
    pa = _lib()
    g = cora
    X = torch.from_numpy(g["ppnp_X"]).to(DEV)
    idx = torch.from_numpy(g["ppnp_idx"]).to(DEV)
    ap = pa.APPNP(n_features=X.shape[1], n_classes=int(g["n_classes"]), adj=adj_of(g)).to(DEV)
    ap.eval()
    with torch.no_grad():
        a = ap(X, idx)
        b = ap(X, idx[:7])
        assert ap.memo_hits == 1 and torch.equal(a[:7], b)
    opt = torch.optim.SGD(ap.parameters(), lr=0.1)
    ap.train()
    loss = ap(X, idx).square().sum()  # train mode: no memo, dropout active
    opt.zero_grad()
    loss.backward()
    opt.step()  # weights change in place
    ap.eval()
    with torch.no_grad():
        c = ap(X, idx)
        assert ap.memo_hits == 1 and not torch.equal(a, c)
        X.mul_(2.0)  # an in-place edit of X is seen too
        d = ap(X, idx)
        assert ap.memo_hits == 1 and not torch.equal(c, d)
    e = ap(X, idx)  # grad enabled: never memoised
    assert ap.memo_hits == 1 and torch.allclose(d, e)


# ---------------------------------------------------------------------------------------
# row-partitioned step (multi-GPU building block): held rows, local/remote split
# ---------------------------------------------------------------------------------------


@pytest.mark.parametrize("lo,hi", [(0, 700), (700, 1400), (1400, 2000), (0, 2000)])
def test_step_rows_and_split(lo, hi):
    pa = _lib()
    from ppnp_amd import _lib as L

    n, F = 2000, 24
    adj = synth(n, 9000, seed=21)
    ah = O.calc_a_hat(adj, "sym")
    Zin = torch.randn(n, F, generator=torch.Generator().manual_seed(1))
    H = torch.randn(hi - lo, F, generator=torch.Generator().manual_seed(2))
    ref = 0.8 * (ah[lo:hi] @ Zin.double().numpy()) + 0.2 * H.double().numpy()
    G = pa.Graph.from_scipy(adj, device=DEV, row_lo=lo, row_hi=hi, split_local=True)
    assert G.rows == hi - lo and G.n == n
    out = torch.empty(hi - lo, F, device=DEV)
    pa.step(G, Zin.to(DEV), H.to(DEV), out, 0, 0.2)
    close_fp32(to_np(out), ref)
    part = torch.empty(hi - lo, F, device=DEV)
    out2 = torch.empty(hi - lo, F, device=DEV)
    pa.step(G, Zin.to(DEV), None, part, 0, 0.2, part=L.PART_LOCAL)
    pa.step(G, Zin.to(DEV), H.to(DEV), out2, 0, 0.2, part=L.PART_REMOTE, partial=part)
    close_fp32(to_np(out2), ref)


def test_step_dropout_uses_global_row_keys():
    """A row shard applies the same mask as the full graph (key = global (row, col))."""
    pa = _lib()
    n, F, lo, hi = 1500, 8, 600, 1100
    adj = synth(n, 6000, seed=4)
    Zin = torch.randn(n, F, generator=torch.Generator().manual_seed(3)).to(DEV)
    H = torch.randn(n, F, generator=torch.Generator().manual_seed(4)).to(DEV)
    Gfull = pa.Graph.from_scipy(adj, device=DEV)
    Gpart = pa.Graph.from_scipy(adj, device=DEV, row_lo=lo, row_hi=hi)
    full = torch.empty(n, F, device=DEV)
    part = torch.empty(hi - lo, F, device=DEV)
    pa.step(Gfull, Zin, H, full, 3, 0.1, p_drop=0.4, seed=99)
    pa.step(Gpart, Zin, H[lo:hi], part, 3, 0.1, p_drop=0.4, seed=99)
    assert torch.equal(full[lo:hi], part)


# ---------------------------------------------------------------------------------------
# vector tails: F not a multiple of the 16-B vector, padded rows; padding never read/written
# ---------------------------------------------------------------------------------------


@pytest.mark.parametrize("dtype,F,ld", [(torch.float32, 30, 32), (torch.float32, 7, 8),
                                        (torch.float32, 101, 128), (torch.bfloat16, 100, 128),
                                        (torch.bfloat16, 15, 16), (torch.bfloat16, 3, 8),
                                        (torch.bfloat16, 13, 16), (torch.bfloat16, 70, 72)])
def test_tail_fragments(dtype, F, ld):
    pa = _lib()
    n = 2500
    adj = synth(n, 12000, seed=F)
    G = pa.Graph.from_scipy(adj, device=DEV)
    Hc = torch.randn(n, F, generator=torch.Generator().manual_seed(F)).to(dtype)
    Hbuf = torch.full((n, ld), float("nan"), dtype=dtype, device=DEV)
    Hbuf[:, :F] = Hc.to(DEV)
    Zbuf = torch.full((n, ld), float("nan"), dtype=dtype, device=DEV)
    pa.propagate_forward(G, Hbuf[:, :F], 7, 0.1, out=Zbuf[:, :F])
    assert torch.isnan(Zbuf[:, F:]).all()          # padding not written
    Z = to_np(Zbuf[:, :F])
    assert np.isfinite(Z).all()                   # padding (NaN) never read into results
    ref = O.appnp_propagate(O.calc_a_hat(adj, "sym"), Hc.float().numpy(), 7, 0.1)
    if dtype == torch.float32:
        close_fp32(Z, ref)
    else:
        assert np.abs(Z - ref).max() <= 2e-2 * np.abs(ref).max()


def test_bf16_backward():
    pa = _lib()
    adj = synth(3000, 12000, seed=8)
    G = pa.Graph.from_scipy(adj, device=DEV)
    dZ = torch.randn(3000, 20, generator=torch.Generator().manual_seed(1)).bfloat16()
    dH = to_np(pa.propagate_backward(G, dZ.to(DEV), 6, 0.1))
    ref = O.appnp_backward(O.calc_a_hat(adj, "sym"), dZ.float().numpy(), 6, 0.1)
    assert np.abs(dH - ref).max() <= 2e-2 * np.abs(ref).max()


# ---------------------------------------------------------------------------------------
# device SparseGraph.standardize (sparsegraph.py:191-222) vs the oracle / reference fixtures
# ---------------------------------------------------------------------------------------


def _std_check(adj, select_lcc=True):
    from ppnp_amd.data import standardize_device

    a = sp.csr_matrix(adj, dtype=np.float32)
    a.sort_indices()
    ip, ix, nm = standardize_device(a.indptr, a.indices, a.data, a.shape[0],
                                    select_lcc=select_lcc, device=DEV)
    ref, keep = O.standardize(a, select_lcc=select_lcc)
    assert np.array_equal(nm.cpu().numpy(), keep)
    assert np.array_equal(ip.cpu().numpy(), ref.indptr)
    assert np.array_equal(ix.cpu().numpy(), ref.indices)


@pytest.mark.parametrize("ds", ["cora", "citeseer"])
def test_standardize_reference_datasets(ds, request):
    g = request.getfixturevalue(ds)
    n = int(g["adj_raw_n"])
    raw = sp.csr_matrix((g["adj_raw_data"], g["adj_raw_indices"], g["adj_raw_indptr"]),
                        shape=(n, n))
    _std_check(raw)
    # and it lands exactly on the reference's standardized adjacency
    from ppnp_amd.data import standardize_device

    ip, ix, _ = standardize_device(raw.indptr, raw.indices, raw.data, n, device=DEV)
    assert np.array_equal(ip.cpu().numpy(), g["adj_indptr"])
    assert np.array_equal(ix.cpu().numpy(), g["adj_indices"])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_standardize_messy_graphs(seed):
    rng = np.random.default_rng(seed)
    n = 3000
    # directed, weighted, self loops, many small components + duplicates
    src = rng.integers(0, n, 4000)
    dst = np.where(rng.random(4000) < 0.7, (src + rng.integers(1, 30, 4000)) % n,
                   rng.integers(0, n, 4000))
    w = rng.choice([1.0, 2.0, 0.5], 4000).astype(np.float32)
    a = sp.coo_matrix((w, (src, dst)), shape=(n, n)).tocsr()
    a.setdiag(np.where(rng.random(n) < 0.1, 3.0, 0.0))
    a.eliminate_zeros()
    _std_check(a, select_lcc=True)
    _std_check(a, select_lcc=False)


def test_standardize_tie_and_isolated():
    """Two largest components of equal size.  The reference's pick is
    np.argsort(sizes)[::-1][:1], and numpy's argsort is not stable (its tie order depends on
    the numpy build / CPU SIMD sort), so the reference itself is platform-defined here; the
    device rule is documented and deterministic: the tied component whose smallest node is
    largest."""
    from ppnp_amd.data import standardize_device

    rows = [0, 1, 5, 6, 9]
    cols = [1, 2, 6, 7, 9]
    a = sp.csr_matrix((np.ones(5, np.float32), (rows, cols)), shape=(10, 10))
    _, _, nm = standardize_device(a.indptr, a.indices, a.data, 10, device=DEV)
    assert nm.cpu().tolist() == [5, 6, 7]
    _, _, nm = standardize_device(np.zeros(11, np.int32), np.zeros(0, np.int32), None, 10,
                                  device=DEV)
    assert nm.cpu().tolist() == [9]  # all isolated: ten singletons tie


# ---------------------------------------------------------------------------------------
# batch-main.py's PPR rows (batch-main.py:111-117, 140-146) without the dense inverse
# ---------------------------------------------------------------------------------------


@pytest.mark.parametrize("mode", ["sym", "rw"])
def test_ppr_rows_match_compute_ppr(cora, mode):
    from ppnp_amd.ppr import ppr_rows

    pa = _lib()
    adj = adj_of(cora)
    G = pa.Graph.from_scipy(adj, mode=mode, device=DEV)
    idx = torch.tensor([0, 5, 17, 2809, 1400, 77])
    rows = ppr_rows(G, idx, K=200, alpha=0.1).cpu().numpy()
    ref = O.compute_ppr(adj, 0.1, mode)[idx.numpy()]
    assert np.abs(rows - ref).max() <= 1e-5 * np.abs(ref).max()
    top = ppr_rows(G, idx, K=200, alpha=0.1, topk=64).cpu().numpy()
    assert ((top > 0).sum(1) >= 64).all() and ((top > 0).sum(1) <= 66).all()
    for r in range(len(idx)):
        ref_top = set(np.argsort(-ref[r])[:60])
        assert ref_top <= set(np.nonzero(top[r])[0])


def test_batch_topk_quirk_matches_batch_main(cora):
    """batch-main.py:115-116 verbatim on the reference PPR vs the APPNP-built one."""
    from ppnp_amd.ppr import batch_topk_quirk

    pa = _lib()
    adj = adj_of(cora)
    G = pa.Graph.from_scipy(adj, device=DEV)
    P = batch_topk_quirk(G, 128, K=200, alpha=0.1).cpu()
    full = torch.FloatTensor(O.compute_ppr(adj, alpha=0.1))
    ref = full.clone()
    thresh, _ = ref.topk(128, axis=-1)
    ref[ref < thresh[:, -1]] = 0
    kept, kept_ref = P > 0, ref > 0
    # the fp64 PPR has exact ties at many k-th values; fp32 iteration breaks them by rounding,
    # so entries may flip only where they sit within rounding distance of their threshold
    flip = kept != kept_ref
    gap = (full - thresh[:, -1][None, :]).abs()
    assert (gap[flip] <= 1e-5 * full.abs().max()).all()
    assert flip.float().mean() < 1e-3
    both = kept & kept_ref
    assert (P[both] - ref[both]).abs().max() <= 1e-5 * ref.abs().max()


def test_minibatch_forward_like_batch_main(cora):
    """The batch-main.py:140-146 call pattern with sparse PPR rows from APPNP."""
    from ppnp_amd.ppr import ppr_rows

    pa = _lib()
    adj = adj_of(cora)
    n, C = int(cora["n"]), int(cora["n_classes"])
    X = torch.from_numpy(cora["ppnp_X"]).to(DEV)
    model = pa.APPNP(n_features=X.shape[1], n_classes=C, adj=adj, K=200).to(DEV).eval()
    model.encoder[1].weight.data.copy_(torch.from_numpy(cora["ppnp_W1"]))
    model.encoder[4].weight.data.copy_(torch.from_numpy(cora["ppnp_W2"]))
    idx_batch = torch.from_numpy(cora["ppnp_idx"][:32]).to(DEV)
    ppr_sub = ppr_rows(model.graph(), idx_batch, K=200, alpha=0.1)
    sel = (ppr_sub > 0).any(dim=0)
    with torch.no_grad():
        out = model(X[sel], idx=None, ppr=ppr_sub[:, sel]).cpu().numpy()
    ref = cora["ppnp_logits"][:32]
    assert np.abs(out - ref).max() <= 1e-4 * np.abs(ref).max()


def test_batch_main_loop_runs_unchanged_on_appnp(cora):
    """batch-main.py:140-146 verbatim against an APPNP model: ``model.ppr[idx_batch]`` is the
    lazy dense PPR (K chosen to converge), the minibatch logits equal the reference's
    PPNP.forward fixture, and ``ppr_topk`` reproduces the sparsified buffer of
    batch-main.py:115-116."""
    pa = _lib()
    adj = adj_of(cora)
    C = int(cora["n_classes"])
    X = torch.from_numpy(cora["ppnp_X"]).to(DEV)
    model = pa.APPNP(n_features=X.shape[1], n_classes=C, adj=adj).to(DEV).eval()
    model.encoder[1].weight.data.copy_(torch.from_numpy(cora["ppnp_W1"]))
    model.encoder[4].weight.data.copy_(torch.from_numpy(cora["ppnp_W2"]))
    idx_batch = torch.from_numpy(cora["ppnp_idx"][:32]).to(DEV)
    # --- batch-main.py:140-146, unchanged ---
    ppr_sub = model.ppr[idx_batch]
    sel = (ppr_sub > 0).any(dim=0)
    ppr_sub = ppr_sub[:, sel]
    X_batch = X[sel].cuda()
    with torch.no_grad():
        logits = model(X_batch, idx=None, ppr=ppr_sub)
    # ---
    ref = cora["ppnp_logits"][:32]
    assert np.abs(logits.cpu().numpy() - ref).max() <= 1e-4 * np.abs(ref).max()
    full = torch.FloatTensor(O.compute_ppr(adj, alpha=0.1))
    assert (model.ppr.cpu() - full).abs().max() <= 1e-5 * full.abs().max()
    model.ppr_topk = 64
    thresh, _ = full.topk(64, axis=-1)
    kept, kept_ref = model.ppr.cpu() > 0, full >= thresh[:, -1]
    assert (kept != kept_ref).float().mean() < 1e-3


def test_compiled_training_step_matches_eager(cora):
    """torch.compile(fullgraph=True) of the main.py:121-127 training step (forward, loss with
    the L2 term, backward) through the ``ppnp_amd::propagate`` op: no graph break (fullgraph
    raises on one), and loss and gradients bit-identical to eager.  Dropout off so both runs
    draw no random numbers."""
    import torch.nn.functional as Fn

    pa = _lib()
    C = int(cora["n_classes"])
    X = torch.from_numpy(cora["ppnp_X"]).to(DEV)
    n = X.shape[0]
    idx = torch.from_numpy(cora["ppnp_idx"]).to(DEV)
    y = torch.randint(0, C, (idx.numel(),), generator=torch.Generator().manual_seed(3)).to(DEV)
    torch.manual_seed(0)
    eager = pa.APPNP(n_features=X.shape[1], n_classes=C, adj=adj_of(cora), drop_prob=0.0).to(DEV)
    comp = pa.APPNP(n_features=X.shape[1], n_classes=C, adj=adj_of(cora), drop_prob=0.0).to(DEV)
    comp.load_state_dict(eager.state_dict())
    eager.graph(), comp.graph()  # A_hat built eagerly (setup, not traced)

    def loss_fn(model, X, idx, y):
        logits = model(X, idx)
        return Fn.cross_entropy(logits, y) + 5e-3 / 2 * model.get_norm()

    compiled = torch.compile(loss_fn, backend="aot_eager", fullgraph=True)
    for model, fn in ((eager, loss_fn), (comp, compiled)):
        model.train()
        model.zero_grad()
        fn(model, X, idx, y).backward()
    le = loss_fn(eager, X, idx, y)
    lc = compiled(comp, X, idx, y)
    assert torch.equal(le, lc)
    for (name, pe), pc in zip(eager.named_parameters(), comp.parameters()):
        assert torch.equal(pe.grad, pc.grad), name
    assert n == int(cora["n"])


def test_appnp_memo_new_tensor_same_address(cora):
    """Two fresh X tensors in a row under no_grad: the second may land at the address the
    first just freed, with the same shape and version 0 -- it must still be propagated
    (the memo keys on the tensor objects, not on their addresses)."""
    pa = _lib()
    n = int(cora["n"])
    F = int(cora["ppnp_X"].shape[1])
    ap = pa.APPNP(n_features=F, n_classes=int(cora["n_classes"]), adj=adj_of(cora)).to(DEV)
    ap.eval()
    idx = torch.arange(n, device=DEV)
    outs = []
    with torch.no_grad():
        for s in range(3):
            g = torch.Generator(device=DEV).manual_seed(100 + s)
            outs.append(ap(torch.randn(n, F, device=DEV, generator=g), idx).clone())
    assert ap.memo_hits == 0
    assert not torch.equal(outs[0], outs[1]) and not torch.equal(outs[1], outs[2])


# ---------------------------------------------------------------------------------------
# sparse encoder input (model.py:36-38, 47 on a CSR X): appnp_spmm / appnp_csr_transpose
# ---------------------------------------------------------------------------------------


def _rand_csr(rows, cols, density, seed):
    a = sp.random(rows, cols, density=density, format="csr", dtype=np.float32,
                  random_state=np.random.RandomState(seed))
    a.sort_indices()
    return a


@pytest.mark.parametrize("F", [1, 7, 64, 130])
def test_spmm_matches_dense(F):
    from ppnp_amd.sparse import spmm

    A = _rand_csr(900, 700, 0.02, F)
    B = torch.randn(700, F, generator=torch.Generator().manual_seed(F))
    dev = lambda x: torch.from_numpy(x).to(DEV)  # noqa: E731
    Cm = spmm(dev(A.indptr), dev(A.indices), dev(A.data), 900, 700, B.to(DEV))
    close_fp32(to_np(Cm), A.astype(np.float64) @ B.double().numpy())


def test_spmm_dropout_mask_and_transpose():
    from ppnp_amd.sparse import SparseFeatures, spmm

    A = _rand_csr(500, 300, 0.05, 1)
    X = SparseFeatures.from_scipy(A, device=DEV)
    ip, ix, dv = X.transpose()
    At = A.T.tocsr()
    At.sort_indices()
    assert np.array_equal(ip.cpu().numpy(), At.indptr)
    assert np.array_equal(ix.cpu().numpy(), At.indices)
    assert np.array_equal(dv.cpu().numpy(), At.data)
    # mask: oracle counter hash at k = 0, kept entries scaled by 1/(1-p)
    B = torch.randn(300, 16, generator=torch.Generator().manual_seed(2))
    Cm = spmm(X.indptr, X.indices, X.data, 500, 300, B.to(DEV), p_drop=0.5, seed=11)
    M = O.masked_operator(A.astype(np.float64), 0, 0.5, 11)
    close_fp32(to_np(Cm), M @ B.double().numpy())
    # transposed product with the transposed key replays the same mask: (M o A)^T
    G = torch.randn(500, 16, generator=torch.Generator().manual_seed(3))
    D = spmm(ip, ix, dv, 300, 500, G.to(DEV), p_drop=0.5, seed=11, transposed_key=True)
    close_fp32(to_np(D), M.T @ G.double().numpy())


def test_sparse_linear_grad():
    from ppnp_amd.sparse import SparseFeatures, sparse_linear

    A = _rand_csr(400, 250, 0.04, 5)
    X = SparseFeatures.from_scipy(A, device=DEV)
    W = torch.randn(250, 32, device=DEV, requires_grad=True)
    Y = sparse_linear(X, W, p_drop=0.3, seed=7)
    G = torch.randn_like(Y)
    (Y * G).sum().backward()
    M = torch.from_numpy(O.masked_operator(A.astype(np.float64), 0, 0.3, 7).toarray()).float()
    Wd = W.detach().cpu().requires_grad_(True)
    Yd = M @ Wd
    (Yd * G.cpu()).sum().backward()
    assert torch.allclose(Y.cpu(), Yd, atol=1e-5, rtol=1e-5)
    assert torch.allclose(W.grad.cpu(), Wd.grad, atol=1e-4, rtol=1e-5)


def test_model_sparse_input_matches_dense(cora):
    from ppnp_amd.sparse import SparseFeatures

    pa = _lib()
    adj = adj_of(cora)
    Xd = torch.from_numpy(cora["ppnp_X"])
    Xd[Xd < 0.9] = 0  # make it sparse
    Xs = SparseFeatures.from_scipy(sp.csr_matrix(Xd.numpy()), device=DEV)
    C = int(cora["n_classes"])
    model = pa.APPNP(n_features=Xd.shape[1], n_classes=C, adj=adj, K=10).to(DEV).eval()
    idx = torch.arange(0, 2810, 7, device=DEV)
    with torch.no_grad():
        a = model(Xd.to(DEV), idx)
        b = model(Xs, idx)
    assert torch.allclose(a, b, atol=1e-5, rtol=1e-4)


# ---------------------------------------------------------------------------------------
# power-law rows: hubs handled by whole wavefronts inside the narrow launch
# ---------------------------------------------------------------------------------------


def _hub_graph(n=4000, seed=0):
    rng = np.random.default_rng(seed)
    hubs = [0, 17, 999, n - 1]
    src = np.concatenate([np.repeat(hubs, [3000, 500, 120, 33]),
                          rng.integers(0, n, 6000)])
    dst = np.concatenate([rng.integers(0, n, 3653), rng.integers(0, n, 6000)])
    a = sp.coo_matrix((np.ones(len(src), np.float32), (src, dst)), shape=(n, n)).tocsr()
    a = ((a + a.T) > 0).astype(np.float32).tocsr()
    a.setdiag(0)
    a.eliminate_zeros()
    a.sort_indices()
    return a


@pytest.mark.parametrize("F", [3, 7, 16, 100])
@pytest.mark.parametrize("p", [0.0, 0.3])
def test_hub_rows_forward_backward(F, p):
    pa = _lib()
    adj = _hub_graph()
    assert np.diff(adj.indptr).max() > 1000
    G = pa.Graph.from_scipy(adj, device=DEV)
    ah = O.calc_a_hat(adj, "sym")
    H = torch.randn(adj.shape[0], F, generator=torch.Generator().manual_seed(F))
    Z = to_np(pa.propagate_forward(G, H.to(DEV), 6, 0.1, p_drop=p, seed=4))
    close_fp32(Z, O.appnp_propagate(ah, H.numpy(), 6, 0.1, p_drop=p, seed=4))
    dH = to_np(pa.propagate_backward(G, H.to(DEV), 6, 0.1, p_drop=p, seed=4))
    close_fp32(dH, O.appnp_backward(ah, H.numpy(), 6, 0.1, p_drop=p, seed=4))


def test_plan_replay_matches_propagate():
    """appnp_plan_*: the captured K-launch graph gives bitwise the eager result, and replays
    pick up in-place refills of H."""
    from ppnp_amd.ops import PropagatePlan

    pa = _lib()
    adj = synth(6000, 30000, seed=12)
    G = pa.Graph.from_scipy(adj, device=DEV)
    H = torch.randn(6000, 12, generator=torch.Generator().manual_seed(1)).to(DEV)
    plan = PropagatePlan(G, H, K=10, alpha=0.1)
    assert torch.equal(plan().clone(), pa.propagate_forward(G, H, 10, 0.1))
    H.mul_(-2.0)
    torch.cuda.synchronize()
    assert torch.equal(plan().clone(), pa.propagate_forward(G, H, 10, 0.1))
    plan.close()


@pytest.mark.parametrize("deg", [4, 14])
@pytest.mark.parametrize("F", [3, 13, 25, 100])
def test_bandwidth_regime_row_shapes(deg, F):
    """Graphs above the latency regime (> 64k rows): mean row length < kWideAvgRow takes the
    G-lane row kernel for narrow F, >= kWideAvgRow a wavefront per row (launch_step)."""
    pa = _lib()
    n = 70_000
    adj = synth(n, deg * n, seed=deg + F)
    G = pa.Graph.from_scipy(adj, device=DEV)
    assert (G.nnz_hat >= 24 * n) == (deg == 14)
    ah = O.calc_a_hat(adj, "sym")
    H = torch.randn(n, F, generator=torch.Generator().manual_seed(F))
    p = 0.3 if F == 13 else 0.0
    Z = to_np(pa.propagate_forward(G, H.to(DEV), 4, 0.1, p_drop=p, seed=9))
    close_fp32(Z, O.appnp_propagate(ah, H.numpy(), 4, 0.1, p_drop=p, seed=9))
