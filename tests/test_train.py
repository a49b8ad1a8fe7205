"""Training harness (ppnp_amd/train.py): host bookkeeping pinned to the reference (CPU) and
end-to-end accuracy on the GPU against run.sh:19-23's published targets."""

import numpy as np
import pytest
import scipy.sparse as sp

from ppnp_amd import train as T


@pytest.mark.parametrize("ds", ["cora", "citeseer"])
@pytest.mark.parametrize("tag", ["a", "b"])
def test_gen_splits_match_reference(ds, tag, request):
    g = request.getfixturevalue(ds)
    args = {"ntrain_per_class": 20, "nstopping": 500, "nknown": 1500,
            "seed": int(g[f"split_{tag}_seed"])}
    tr, st, va = T.gen_splits(g["labels"], args, test=False)
    assert np.array_equal(tr, g[f"split_{tag}_train"])
    assert np.array_equal(st, g[f"split_{tag}_stop"])
    assert np.array_equal(va, g[f"split_{tag}_valid"])
    _, _, te = T.gen_splits(g["labels"], args, test=True)
    assert np.array_equal(te, g[f"split_{tag}_test"])


@pytest.mark.parametrize("ds", ["cora", "citeseer"])
def test_normalize_attributes(ds, request):
    g = request.getfixturevalue(ds)
    attr = sp.csr_matrix((g["attr_data"], g["attr_indices"], g["attr_indptr"]),
                         shape=tuple(g["attr_shape"]))
    xn = T.normalize_attributes(attr)
    rs = np.asarray(abs(xn).sum(axis=1)).ravel()
    np.testing.assert_allclose(rs, g["attr_l1_rowsum"], rtol=1e-6)


def test_early_stopping_semantics():
    es = T.SimpleEarlyStopping(model=None, patience=3)
    assert es.record == (None,)  # reference quirk preserved
    assert not es.should_stop(0.5, 1.0, 0, record={"e": 0})
    assert not es.should_stop(0.6, 0.9, 1, record={"e": 1})
    assert es.record == {"e": 1}
    # worse in both acc and loss: patience counts down
    assert not es.should_stop(0.4, 2.0, 2)
    assert not es.should_stop(0.4, 2.0, 3)
    assert es.should_stop(0.4, 2.0, 4)
    assert es.best_epoch == 1


@pytest.mark.gpu
def test_cora_accuracy_matches_run_sh():
    """APPNP (K=10) trained with the main.py protocol, 12 runs: the mean sits in the band of the
    reference's published Cora-ML accuracy (run.sh:19-20: 0.856 +- 0.009 over 32 runs of PPNP;
    the reference's own main.py re-run gives 0.830 +- 0.014), and within 0.015 of
    the dense-PPR PPNP trained on the same 12 seeds and splits -- a paired check that catches a
    regression of a point or two, where a run-to-run std of ~0.02 hides it in a 4-run band."""
    s = T.main(["--dataset", "cora_ml", "--n-runs", "12", "--seed", "123"])
    p = T.main(["--dataset", "cora_ml", "--n-runs", "12", "--seed", "123", "--model", "ppnp"])
    assert 0.82 <= s["valid_acc_mean"] <= 0.87, s
    assert s["valid_acc_std"] <= 0.035, s
    assert abs(s["valid_acc_mean"] - p["valid_acc_mean"]) <= 0.015, (s, p)


@pytest.mark.gpu
def test_citeseer_accuracy_matches_run_sh():
    """run.sh:22-23 publishes Citeseer 0.760 +- 0.012 (PyTorch 1.2); the reference's main.py
    re-run today gives 0.733 +- 0.014 (profiles/r1_train_accuracy.md).  12 runs."""
    s = T.main(["--dataset", "citeseer", "--n-runs", "12", "--seed", "123"])
    assert 0.71 <= s["valid_acc_mean"] <= 0.77, s
    assert s["valid_acc_std"] <= 0.04, s


@pytest.mark.gpu
def test_cora_accuracy_sparse_input():
    """Same protocol with X kept as a CSR on the GPU (sparse encoder input)."""
    s = T.main(["--dataset", "cora_ml", "--n-runs", "3", "--seed", "123", "--sparse-x"])
    assert 0.81 <= s["valid_acc_mean"] <= 0.89, s
