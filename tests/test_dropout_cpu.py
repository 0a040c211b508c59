"""Dropout mask function (no GPU): the oracle's numpy restatement and the C ABI's
vitmi_dropout_hash (the function every device kernel evaluates) agree bit for bit, and the
keep rate matches the requested rate.  Reference: layers.Dropout at models/CvT(Par).py:189,
255, 257 (rate 0.1 in training)."""
import numpy as np
import pytest

from oracle import vit_ref
from vitmi import _lib


@pytest.mark.parametrize("seed,site", [(0, 0), (12345, 7), (2**31 - 1, 35), (0xDEADBEEF, 2)])
def test_hash_matches_library(seed, site):
    lib = _lib.lib()
    rows = np.array([0, 1, 2, 196, 197, 50431, 123457, 2**31 + 5], dtype=np.uint64)
    cols = np.array([0, 1, 3, 767, 768, 3071, 2303], dtype=np.uint64)
    ref = vit_ref.dropout_hash(seed, site, rows, cols)
    for i, r in enumerate(rows):
        for j, c in enumerate(cols):
            assert lib.vitmi_dropout_hash(seed & 0xFFFFFFFF, site, int(r) & 0xFFFFFFFF, int(c)) == int(ref[i, j])


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_keep_rate(p):
    thresh, scale = vit_ref.dropout_params(p)
    h = vit_ref.dropout_hash(7, 3, np.arange(512), np.arange(768))
    keep = (h >= thresh).mean()
    assert abs(keep - (1 - p)) < 0.005
    assert scale == pytest.approx(1 / (1 - p))
    # different sites / seeds give (nearly) independent masks
    h2 = vit_ref.dropout_hash(7, 4, np.arange(512), np.arange(768))
    agree = ((h >= thresh) == (h2 >= thresh)).mean()
    assert abs(agree - ((1 - p) ** 2 + p ** 2)) < 0.01
