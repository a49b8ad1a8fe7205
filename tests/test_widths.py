"""CPU: which source-blocked copy ``Graph.from_csr(features=F)`` asks for (graph.remainder_width),
the host half of appnp_capi.hip's ``remainder_cols`` rule:

* fp32 rows of F = 32q + r features, 1 <= r <= 8, beside whole lines: the narrowest copy that
  holds r (W4 for r <= 4, W8 for 5-8); wider remainders keep whole rows;
* narrow rows F <= 16 run wholly in the pass (W4 / W8 / W16); 17-32 columns are one line already;
* never a W16 copy beside whole lines (measured slower than the extra line:
  profiles/r3_wide_copy_f100.txt);
* nothing for bf16, for graphs in the latency regime (n <= 2^16) or for F outside [1, 256]."""

import pytest
import torch

from ppnp_amd.graph import remainder_width, splits_rows

BIG = 2_449_029


@pytest.mark.parametrize("f,w", [(100, 4), (36, 4), (33, 4), (40, 8), (37, 8), (47, 0), (48, 0),
                                 (64, 0), (96, 0), (128, 0), (132, 4), (200, 8), (256, 0),
                                 (1, 4), (3, 4), (4, 4), (5, 8), (8, 8), (9, 16), (13, 16),
                                 (16, 16), (17, 0), (25, 0), (32, 0)])
def test_width_for_each_shape(f, w):
    assert remainder_width(BIG, f) == w
    assert splits_rows(BIG, f) == (w > 0)


def test_no_w16_beside_whole_lines():
    assert all(remainder_width(BIG, f) in (0, 4, 8) for f in range(33, 257))


@pytest.mark.parametrize("n,f,dtype", [(BIG, 100, torch.bfloat16), (1 << 16, 100, torch.float32),
                                       (BIG, 0, torch.float32), (BIG, 257, torch.float32),
                                       (BIG, 300, torch.float32)])
def test_no_copy(n, f, dtype):
    assert remainder_width(n, f, dtype) == 0 and not splits_rows(n, f, dtype)


def test_source_block_flags():
    """The ``mode`` bits Graph.from_csr(features=F) and the native row engine ask for."""
    from ppnp_amd import _lib
    from ppnp_amd.graph import source_block_flags

    assert source_block_flags(BIG, 13) == _lib.GRAPH_SB_W16
    assert source_block_flags(BIG, 40) == _lib.GRAPH_SB_W8
    assert source_block_flags(BIG, 7) == _lib.GRAPH_SB_W8
    assert source_block_flags(BIG, 100) == _lib.GRAPH_SOURCE_BLOCKS
    assert source_block_flags(BIG, 3) == _lib.GRAPH_SOURCE_BLOCKS
    assert source_block_flags(BIG, 64) == 0 and source_block_flags(1000, 100) == 0
