"""CPU: the benchmark's synthetic graph generators (ppnp_amd/synth.py) produce what the C ABI
expects of A -- int32 CSR, columns strictly increasing in each row, symmetric pattern, no self
loops -- and the structure each workload claims."""

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from ppnp_amd import synth

N, M = 20_000, 120_000


def _check_csr(indptr, indices, n):
    ip = indptr.numpy().astype(np.int64)
    ix = indices.numpy().astype(np.int64)
    assert indptr.dtype == torch.int32 and indices.dtype == torch.int32
    assert ip[0] == 0 and ip[-1] == len(ix) and np.all(np.diff(ip) >= 0)
    rows = np.repeat(np.arange(n), np.diff(ip))
    assert np.all((ix >= 0) & (ix < n))
    assert not np.any(ix == rows)  # no self loops
    same_row = rows[1:] == rows[:-1]
    assert np.all(ix[1:][same_row] > ix[:-1][same_row])  # sorted, no duplicates
    a = sp.csr_matrix((np.ones(len(ix)), ix, ip), shape=(n, n))
    assert (a - a.T).nnz == 0  # symmetric pattern
    return rows, ix


@pytest.mark.parametrize("gen", ["uniform", "chung_lu", "community"])
def test_generator_csr_contract(gen):
    fn = {"uniform": synth.uniform_graph, "chung_lu": synth.chung_lu_graph,
          "community": synth.community_graph}[gen]
    indptr, indices = fn(N, M, 3, device="cpu")
    rows, cols = _check_csr(indptr, indices, N)
    assert 1.7 * M < len(cols) <= 2 * M  # symmetrised, few duplicates at this density


def test_community_locality_and_uniform_spread():
    _, ix = synth.community_graph(N, M, 4, block=1024, device="cpu")
    ip, _ = synth.community_graph(N, M, 4, block=1024, device="cpu")
    rows = np.repeat(np.arange(N), np.diff(ip.numpy()))
    inside = np.mean(ix.numpy() // 1024 == rows // 1024)
    assert 0.85 < inside < 0.95  # 90 % of the pairs drawn inside, both directions kept
    ip_u, ix_u = synth.uniform_graph(N, M, 4, device="cpu")
    rows_u = np.repeat(np.arange(N), np.diff(ip_u.numpy()))
    assert np.mean(ix_u.numpy() // 1024 == rows_u // 1024) < 0.1


def test_chung_lu_is_skewed():
    ip, _ = synth.chung_lu_graph(N, M, 5, device="cpu")
    deg = np.diff(ip.numpy())
    assert deg.max() > 20 * deg.mean()  # hubs


def test_workload_table():
    for name, (n, m, f, k, alpha, dtype) in synth.CONFIGS.items():
        assert n > 0 and m > 0 and f > 0 and k > 0 and 0 < alpha < 1
        assert name in synth.DESCRIPTIONS
    assert synth.CONFIGS["products-synth"][:5] == (2449029, 61859140, 100, 10, 0.1)


@pytest.mark.parametrize("name", ["pubmed-synth", "ms-academic-synth", "arxiv-synth"])
def test_uniform_graph_is_the_survey_instance(name):
    """The benchmark's graph is SURVEY.md 8(d)'s numpy default_rng instance: bit-identical CSR
    to oracle.synth_graph (the same recipe restated with scipy) for the config's n, m, seed.
    products-synth uses the same function at its own n, m and seed 4 (too slow for scipy here)."""
    from oracle import ppnp_oracle as O

    n, m = synth.CONFIGS[name][:2]
    seed = synth.SEEDS[name]
    ip, ix = synth.uniform_graph(n, m, seed, device="cpu")
    ref = O.synth_graph(n, m, seed)
    assert np.array_equal(ip.numpy().astype(np.int64), ref.indptr.astype(np.int64))
    assert np.array_equal(ix.numpy().astype(np.int64), ref.indices.astype(np.int64))


def test_features_are_cpu_generator_draws():
    """H ~ N(0,1) from a CPU torch.Generator seeded 0, whatever the device."""
    H = synth.features(100, 7, device="cpu")
    g = torch.Generator().manual_seed(0)
    assert torch.equal(H, torch.randn(100, 7, generator=g))


def test_graph_cache_returns_the_generator_arrays(tmp_path, monkeypatch):
    """PPNP_SYNTH_CACHE (set by tests/conftest.py for the GPU session and its child ranks): the
    first call writes the workload's CSR, later calls read it back, and both equal the
    generator's own arrays."""
    from ppnp_amd import synth

    monkeypatch.delenv("PPNP_SYNTH_CACHE", raising=False)
    ip0, ix0 = synth.graph_for("pubmed-synth", device="cpu")
    monkeypatch.setenv("PPNP_SYNTH_CACHE", str(tmp_path))
    ip1, ix1 = synth.graph_for("pubmed-synth", device="cpu")
    assert (tmp_path / "pubmed-synth.npz").exists()
    ip2, ix2 = synth.graph_for("pubmed-synth", device="cpu")
    for a, b, c in ((ip0, ip1, ip2), (ix0, ix1, ix2)):
        assert torch.equal(a, b) and torch.equal(a, c) and a.dtype == c.dtype == torch.int32
