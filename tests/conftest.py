import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    # one on-disk copy of each synthetic graph for the whole session, child processes included
    # (ppnp_amd.synth.graph_for): the products-scale tests draw the 124 M-key graph once
    if not os.environ.get("PPNP_SYNTH_CACHE"):
        import tempfile

        os.environ["PPNP_SYNTH_CACHE"] = tempfile.mkdtemp(prefix="ppnp_synth_")
        config._ppnp_synth_cache = os.environ["PPNP_SYNTH_CACHE"]


def pytest_unconfigure(config):
    d = getattr(config, "_ppnp_synth_cache", None)
    if d:
        import shutil

        shutil.rmtree(d, ignore_errors=True)


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def cora():
    return load_golden("cora_ml")


@pytest.fixture(scope="session")
def citeseer():
    return load_golden("citeseer")


@pytest.fixture(scope="session")
def kat():
    return load_golden("kat")
