"""Pin oracle/cvt_ref.py (the CvT restatement) against golden vectors of the
reference's own PyTorch module old_codes/MS_CvT.py (tests/golden/mscvt_cvt_dwbn.npz, made by
tests/golden/gen_golden.py): dw_bn q/k/v projections (depthwise 3x3 + training-mode
BatchNorm), strided overlapping conv embeddings, a cls token in the last stage.  No GPU."""
import os

import numpy as np
import pytest
import torch

from oracle import cvt_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden", "mscvt_cvt_dwbn.npz")


def mscvt_cfg():
    """MS_CvT semantics (old_codes/MS_CvT.py): symmetric padding, embed LayerNorm, scale
    1/sqrt(D), no q/k/v bias, BatchNorm2d eps 1e-5, separate norm1/norm2, LN eps 1e-5."""
    return cvt_ref.CvTConfig(
        img_size=32, in_chans=1, num_classes=2,
        stages=[cvt_ref.CvTStage(64, 7, 4, 1, padding=2),
                cvt_ref.CvTStage(128, 3, 2, 2, with_cls_token=True, padding=1)],
        attn_scale="dim", ln_eps=1e-5, bn_eps=1e-5, qkv_bias=False, tie_norms=False, embed_norm=True,
        dtype="fp32")


def load():
    z = np.load(GOLD)
    params = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p::")}
    grads = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("g::")}
    return (torch.from_numpy(z["input"]), torch.from_numpy(z["target"]), params,
            torch.from_numpy(z["logits"]), float(z["loss"]), grads)


def test_param_names_match_fixture():
    _, _, params, _, _, _ = load()
    shapes = cvt_ref.param_shapes(mscvt_cfg())
    assert set(shapes) == set(params)
    for k, s in shapes.items():
        assert tuple(params[k].shape) == tuple(s), k


def test_cvt_oracle_matches_mscvt_golden():
    img, tgt, params, logits_ref, loss_ref, grads_ref = load()
    logits, loss, grads = cvt_ref.forward_backward(img, tgt, params, mscvt_cfg())
    assert (logits - logits_ref).abs().max().item() < 1e-5
    assert abs(loss.item() - loss_ref) < 1e-5
    # floor: the norm1 gradients of a stage are ~1e-7 (BatchNorm right after norm1 cancels its
    # scale in q/k/v), where float noise is the whole relative difference
    for k, g in grads_ref.items():
        den = max(g.norm().item(), 1e-4)
        assert (grads[k] - g).norm().item() / den < 1e-4, k


def test_same_padding_geometry():
    # TF 'same' (models/CvT(Par).py:203-207): asymmetric, the extra pad goes after
    assert cvt_ref.conv_geometry(128, 7, 4, None) == (32, 1, 2)
    assert cvt_ref.conv_geometry(32, 3, 2, None) == (16, 0, 1)
    assert cvt_ref.conv_geometry(16, 3, 2, None) == (8, 0, 1)
    assert cvt_ref.conv_geometry(32, 7, 4, 2) == (8, 2, 2)


def test_keras_spec_shapes():
    cfg = cvt_ref.CvTConfig(img_size=64)
    p = cvt_ref.init_params(cfg, 0)
    img, tgt = cvt_ref.synthetic_batch(cfg, 2)
    out = cvt_ref.forward(img, p, cfg)
    assert out.shape == (2, 1)
