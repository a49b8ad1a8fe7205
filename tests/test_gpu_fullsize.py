"""GPU parity at BASELINE.json's full size (products-synth: 2,449,029 nodes, 126M nnz of A_hat,
F = 100, K = 10) through size-independent properties -- the oracle cannot run the whole
graph in seconds, so each check is one it can verify exactly or on a sample:

* fixed points: sym A_hat D^1/2 1 = D^1/2 1, so H = sqrt(D) x c is returned unchanged by every
  iteration; rw A_hat 1 = 1, so constant columns are;
* linearity: P(a H1 + b H2) = a P(H1) + b P(H2);
* one step on sampled rows against a float64 CPU evaluation of the same rows of A_hat;
* the device A_hat's row sums (rw) are 1 and its structure is A + I;
* bitwise determinism of the full K=10 propagation.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def products():
    from ppnp_amd import synth

    n, m, F, K, alpha, _ = synth.CONFIGS["products-synth"]
    indptr, indices = synth.graph_for("products-synth", device=DEV)  # the session's copy
    return dict(n=n, F=F, K=K, alpha=alpha, indptr=indptr, indices=indices)


@pytest.fixture(scope="module")
def graph_sym(products):
    import ppnp_amd

    return ppnp_amd.Graph.from_csr(products["indptr"], products["indices"], None, products["n"],
                                   device=DEV, features=products["F"])


def _deg(graph):
    _, _, _, dinv = graph.csr()
    return dinv


def test_structure_is_a_plus_i(products, graph_sym):
    rp, col, _, _ = graph_sym.csr()
    n = products["n"]
    a_len = (products["indptr"][1:] - products["indptr"][:-1]).long()
    assert torch.equal((rp[1:] - rp[:-1]).long(), a_len + 1)  # one merged diagonal per row
    assert graph_sym.nnz_hat == int(products["indices"].numel()) + n
    assert graph_sym.symmetric


def test_sym_fixed_point(products, graph_sym):
    import ppnp_amd

    dinv = _deg(graph_sym)  # 1/sqrt(D), fp64
    sqrt_d = (1.0 / dinv).float()
    c = torch.linspace(-1.0, 2.0, products["F"], device=DEV)
    H = sqrt_d[:, None] * c[None, :]
    Z = ppnp_amd.propagate_forward(graph_sym, H, products["K"], products["alpha"])
    rel = ((Z - H).abs() / (H.abs() + 1e-6)).max().item()
    assert rel <= 1e-5, rel


def test_rw_constants_fixed_point(products):
    import ppnp_amd

    G = ppnp_amd.Graph.from_csr(products["indptr"], products["indices"], None, products["n"],
                                mode="rw", device=DEV)
    rp, _, val, _ = G.csr()
    seg = torch.repeat_interleave(torch.arange(G.n, device=DEV), (rp[1:] - rp[:-1]).long())
    rowsum = torch.zeros(G.n, dtype=torch.float64, device=DEV).index_add_(0, seg, val.double())
    assert (rowsum - 1).abs().max().item() <= 1e-6
    H = torch.ones(G.n, products["F"], device=DEV) * torch.arange(products["F"], device=DEV)
    Z = ppnp_amd.propagate_forward(G, H, products["K"], products["alpha"])
    assert ((Z - H).abs() <= 1e-5 * (H.abs() + 1)).all()


def test_linearity(products, graph_sym):
    import ppnp_amd

    g = torch.Generator(device=DEV).manual_seed(1)
    n, F = products["n"], products["F"]
    H1 = torch.randn(n, F, device=DEV, generator=g)
    H2 = torch.randn(n, F, device=DEV, generator=g)
    K, al = products["K"], products["alpha"]
    lhs = ppnp_amd.propagate_forward(graph_sym, 2.0 * H1 - 0.5 * H2, K, al)
    rhs = 2.0 * ppnp_amd.propagate_forward(graph_sym, H1, K, al) - 0.5 * ppnp_amd.propagate_forward(
        graph_sym, H2, K, al)
    err = (lhs - rhs).abs().max().item()
    assert err <= 1e-4 * rhs.abs().max().item(), err


def test_one_step_sampled_rows(products, graph_sym):
    """Z_1 on 2,000 random rows vs a float64 CPU evaluation of those rows."""
    import ppnp_amd

    g = torch.Generator(device=DEV).manual_seed(2)
    n, F, al = products["n"], products["F"], products["alpha"]
    H = torch.randn(n, F, device=DEV, generator=g)
    Z1 = ppnp_amd.propagate_forward(graph_sym, H, 1, al)
    rp, col, val, _ = graph_sym.csr()
    rows = torch.randint(0, n, (2000,), device=DEV, generator=g)
    rp_c, col_c, val_c = rp.cpu().numpy(), col.cpu().numpy(), val.cpu().numpy()
    Hc = H.double().cpu().numpy()
    ref = np.empty((2000, F))
    for k, r in enumerate(rows.cpu().numpy()):
        b, e = rp_c[r], rp_c[r + 1]
        ref[k] = (1 - al) * (val_c[b:e].astype(np.float64) @ Hc[col_c[b:e]]) + al * Hc[r]
    got = Z1[rows].double().cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def test_full_propagation_deterministic(products, graph_sym):
    import ppnp_amd

    g = torch.Generator(device=DEV).manual_seed(3)
    H = torch.randn(products["n"], products["F"], device=DEV, generator=g)
    a = ppnp_amd.propagate_forward(graph_sym, H, products["K"], products["alpha"])
    b = ppnp_amd.propagate_forward(graph_sym, H, products["K"], products["alpha"])
    assert torch.equal(a, b)
