"""GPU: the in-library random-line probe behind bench.py's roofline.box_line_rate
(appnp_line_rate_probe, ppnp_amd/csrc/appnp_probe.hip) and the bench line's build provenance.

The probe only reads its table, so it must leave it untouched; it must handle tables of any
size (a whole number of lines is gathered from a 128-B aligned start inside the storage) and
report a rate in the range the gather probe measured (tools/gather_probe.hip: 53-60 G lines/s
for 64 MB-1 GB tables on an idle MI355X)."""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.mark.parametrize("nbytes", [128, 4096 + 44, 1 << 20, 1 << 28])
def test_probe_reads_only_and_reports_a_rate(nbytes):
    from ppnp_amd.ops import line_rate_probe

    t = torch.arange(nbytes // 4, dtype=torch.float32, device=DEV)
    before = t.clone()
    res = line_rate_probe(t, 1 << 22)
    torch.cuda.synchronize()
    assert torch.equal(t, before)
    assert res["lines"] == 1 << 22 and res["ms"] > 0 and res["G_lines_s"] > 0
    assert res["table_MB"] * 2**20 <= t.untyped_storage().nbytes()


def test_probe_rate_on_a_bench_sized_table():
    """A 1 GB table (the bench's H): the rate lands in the band the standalone probe measured,
    with room for box-to-box spread."""
    from ppnp_amd.ops import line_rate_probe

    t = torch.zeros(1 << 28, dtype=torch.float32, device=DEV)
    res = line_rate_probe(t, 1 << 30)
    assert 30.0 < res["G_lines_s"] < 120.0, res


def test_bench_build_info_matches_the_tree():
    """The library this process loaded was compiled from the sources in this tree."""
    import bench

    info = bench.build_info()
    assert info["match"], info
