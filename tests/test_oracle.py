"""CPU: pin the oracle (oracle/ppnp_oracle.py) to the reference's golden vectors.

The fixtures in tests/golden/ were produced by tests/golden/make_golden.py from the
reference's own helpers.calc_A_hat / compute_ppr / model.PPNP / SparseGraph.standardize.
"""

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import ppnp_oracle as O


def adj_of(g, prefix="adj"):
    n = int(g["n"]) if prefix == "adj" else int(g["adj_raw_n"])
    return sp.csr_matrix((g[f"{prefix}_data"], g[f"{prefix}_indices"], g[f"{prefix}_indptr"]),
                         shape=(n, n))


@pytest.mark.parametrize("ds", ["cora", "citeseer"])
def test_standardize_matches_reference(ds, request):
    g = request.getfixturevalue(ds)
    a, keep = O.standardize(adj_of(g, "adj_raw"), select_lcc=True)
    ref = adj_of(g)
    assert a.shape == ref.shape
    assert np.array_equal(a.indptr, ref.indptr)
    assert np.array_equal(a.indices, ref.indices)
    assert np.all(a.data == 1)


@pytest.mark.parametrize("ds", ["cora", "citeseer"])
@pytest.mark.parametrize("mode", ["sym", "rw"])
def test_calc_a_hat_bit_exact(ds, mode, request):
    g = request.getfixturevalue(ds)
    ah = O.calc_a_hat(adj_of(g), mode)
    assert np.array_equal(ah.indptr, g[f"ahat_{mode}_indptr"])
    assert np.array_equal(ah.indices, g[f"ahat_{mode}_indices"])
    assert np.array_equal(ah.data, g[f"ahat_{mode}_data"])  # fp64, bit for bit


@pytest.mark.parametrize("name", ["complete5", "complete2", "path3", "isolated3", "weighted4",
                                  "selfloop3"])
@pytest.mark.parametrize("mode", ["sym", "rw"])
def test_kat_operator_and_ppr(kat, name, mode):
    n = len(kat[f"{name}_indptr"]) - 1
    a = sp.csr_matrix((kat[f"{name}_data"], kat[f"{name}_indices"], kat[f"{name}_indptr"]),
                      shape=(n, n))
    assert np.array_equal(O.calc_a_hat(a, mode).toarray(), kat[f"{name}_ahat_{mode}_dense"])
    np.testing.assert_allclose(O.compute_ppr(a, 0.1, mode), kat[f"{name}_ppr_{mode}_a0.1"],
                               rtol=1e-12, atol=1e-14)


def test_path3_values(kat):
    """P3 sym values 0.5 / 0.40825 / 0.3333."""
    d = kat["path3_ahat_sym_dense"]
    assert d[0, 0] == pytest.approx(0.5)
    assert d[0, 1] == pytest.approx(1 / np.sqrt(6))
    assert d[1, 1] == pytest.approx(1 / 3)


@pytest.mark.parametrize("ds", ["cora", "citeseer"])
@pytest.mark.parametrize("mode,K,alpha,key", [("sym", 10, 0.1, "Z_sym_K10_a0.1"),
                                              ("sym", 20, 0.2, "Z_sym_K20_a0.2"),
                                              ("rw", 10, 0.1, "Z_rw_K10_a0.1")])
def test_propagate_matches_fixture(ds, mode, K, alpha, key, request):
    g = request.getfixturevalue(ds)
    Z = O.appnp_propagate(O.calc_a_hat(adj_of(g), mode), g["H"], K, alpha)
    np.testing.assert_allclose(Z, g[key], rtol=0, atol=1e-12)


def test_closed_form_identity(cora):
    ah = O.calc_a_hat(adj_of(cora), "sym")
    H = cora["H"]
    for K in (0, 1, 5, 10):
        np.testing.assert_allclose(O.appnp_closed_form(ah, H, K, 0.1),
                                   O.appnp_propagate(ah, H, K, 0.1), atol=1e-12)


@pytest.mark.parametrize("mode,key", [("sym", "pprH_a0.1"), ("rw", "pprH_rw_a0.1")])
def test_limit_is_compute_ppr(cora, mode, key):
    """lim_K Z_K = compute_ppr(adj, a) @ H (helpers.py:68-71)."""
    Z = O.appnp_propagate(O.calc_a_hat(adj_of(cora), mode), cora["H"], 300, 0.1)
    np.testing.assert_allclose(Z, cora[key], atol=1e-9)


def test_ppnp_forward_matches_reference(cora):
    """model.py:61-67 propagation with the fixture's encoder output."""
    X = torch.from_numpy(cora["ppnp_X"])
    W1 = torch.from_numpy(cora["ppnp_W1"])
    W2 = torch.from_numpy(cora["ppnp_W2"])
    H = (torch.relu(X @ W1) @ W2.T).double().numpy()
    ppr = O.compute_ppr(adj_of(cora), 0.1)
    out = O.ppnp_forward(ppr, H, idx=cora["ppnp_idx"])
    ref = cora["ppnp_logits"]
    assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()
    with pytest.raises(Exception):
        O.ppnp_forward(ppr, H)


def test_edge_mask_statistics_and_determinism():
    rows = np.repeat(np.arange(2000), 50)
    cols = np.tile(np.arange(50), 2000)
    for p in (0.1, 0.5, 0.9):
        keep = O.edge_keep_mask(rows, cols, 3, p, seed=42)
        assert abs(keep.mean() - (1 - p)) < 0.01
        assert np.array_equal(keep, O.edge_keep_mask(rows, cols, 3, p, seed=42))
    k0 = O.edge_keep_mask(rows, cols, 0, 0.5, seed=1)
    k1 = O.edge_keep_mask(rows, cols, 1, 0.5, seed=1)
    assert (k0 != k1).mean() > 0.4  # a fresh mask every iteration
    assert O.edge_keep_mask(rows, cols, 0, 0.0, seed=1).all()


def test_splitmix_scalar_vector_agree():
    xs = [0, 1, 2**63 + 5, 2**64 - 1, 123456789]
    v = O._splitmix64(np.array(xs, dtype=np.uint64))
    assert [int(a) for a in v] == [O._splitmix64(x) for x in xs]


@pytest.mark.parametrize("p", [0.0, 0.4])
def test_backward_is_adjoint(p):
    """<J H, G> == <H, J^T G> for the (masked) APPNP map."""
    adj = O.synth_graph(300, 1200, seed=3)
    ah = O.calc_a_hat(adj, "sym")
    rng = np.random.default_rng(0)
    H, G = rng.standard_normal((300, 5)), rng.standard_normal((300, 5))
    for K in (1, 3, 6):
        lhs = np.sum(O.appnp_propagate(ah, H, K, 0.1, p, 9) * G)
        rhs = np.sum(H * O.appnp_backward(ah, G, K, 0.1, p, 9))
        assert lhs == pytest.approx(rhs, rel=1e-10)


def test_torch_cpu_baseline_matches(cora):
    ah = O.calc_a_hat(adj_of(cora), "sym")
    A = O.torch_sparse_operator(ah)
    Z = O.appnp_propagate_torch_cpu(A, torch.from_numpy(cora["H"]), 10, 0.1)
    ref = cora["Z_sym_K10_a0.1"]
    assert np.abs(Z.double().numpy() - ref).max() <= 1e-5 * np.abs(ref).max()


def test_synth_graph_properties():
    a = O.synth_graph(1000, 5000, seed=1)
    assert (a != a.T).nnz == 0
    assert a.diagonal().sum() == 0
    assert np.all(a.data == 1)
    assert a.has_sorted_indices


def test_drop_threshold_follows_the_float_abi():
    """p crosses the C ABI as a float: the oracle's threshold is float32(p) * 2^24 (0.3 ->
    5033165, one more than the double 0.3 gives), matching set_drop in appnp_capi.hip."""
    assert O.drop_threshold(0.3) == 5033165
    assert O.drop_threshold(0.5) == 1 << 23
    assert O.drop_threshold(0.0) == 0
