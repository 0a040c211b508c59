"""Pin oracle/cvt_ref.py (the CvT restatement) against golden vectors of the
reference's own PyTorch module old_codes/MS_CvT.py (tests/golden/mscvt_cvt_dwbn.npz, made by
tests/golden/gen_golden.py): dw_bn q/k/v projections (depthwise 3x3 + training-mode
BatchNorm), strided overlapping conv embeddings, a cls token in the last stage.  No GPU."""
import os

import dataclasses

import numpy as np
import pytest
import torch

from oracle import cvt_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden", "mscvt_cvt_dwbn.npz")
GOLD_AVG = os.path.join(os.path.dirname(__file__), "golden", "mscvt_cvt_avg.npz")


def mscvt_cfg():
    """MS_CvT semantics (old_codes/MS_CvT.py): symmetric padding, embed LayerNorm, scale
    1/sqrt(D), no q/k/v bias, BatchNorm2d eps 1e-5, separate norm1/norm2, LN eps 1e-5."""
    return cvt_ref.CvTConfig(
        img_size=32, in_chans=1, num_classes=2,
        stages=[cvt_ref.CvTStage(64, 7, 4, 1, padding=2),
                cvt_ref.CvTStage(128, 3, 2, 2, with_cls_token=True, padding=1)],
        attn_scale="dim", ln_eps=1e-5, bn_eps=1e-5, qkv_bias=False, tie_norms=False, embed_norm=True,
        dtype="fp32")


def mscvt_avg_cfg():
    """mscvt_cfg with the 'avg' q/k/v projection in both stages (torch AvgPool2d counts the
    padding: avg_count_pad)."""
    c = mscvt_cfg()
    return c.replace(stages=[dataclasses.replace(s, qkv_method="avg") for s in c.stages], avg_count_pad=True)


def load(path=GOLD):
    z = np.load(path)
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


def test_cvt_oracle_matches_mscvt_avg_golden():
    img, tgt, params, logits_ref, loss_ref, grads_ref = load(GOLD_AVG)
    cfg = mscvt_avg_cfg()
    assert set(cvt_ref.param_shapes(cfg)) == set(params)
    logits, loss, grads = cvt_ref.forward_backward(img, tgt, params, cfg)
    assert (logits - logits_ref).abs().max().item() < 1e-5
    assert abs(loss.item() - loss_ref) < 1e-5
    for k, g in grads_ref.items():
        den = max(g.norm().item(), 1e-4)
        assert (grads[k] - g).norm().item() / den < 1e-4, k


def test_avg_projection_same_padding_divisor():
    # TF AveragePooling2D 'same' divides by the in-bounds count: a constant image stays constant
    cfg = cvt_ref.CvTConfig(img_size=32, stages=[cvt_ref.CvTStage(64, 7, 4, 1, qkv_method="avg")])
    x = torch.ones(1, 4, 5, 5)
    y = torch.nn.functional.avg_pool2d(x, 3, 1, 1, count_include_pad=cfg.avg_count_pad)
    assert torch.allclose(y, x)
    assert cvt_ref.qkv_methods(cfg.stages[0]) == ("linear", "avg", "avg")


def test_proc_head_is_concat_then_dense():
    """models/CvT(Par).py:343-350: Dense(256, relu) x 2 on the process parameters, concatenated
    AFTER the image features, then Final_Dense; restated with explicit matrices."""
    cfg = cvt_ref.CvTConfig(img_size=32, proc_dim=5)
    p = cvt_ref.init_params(cfg, 1)
    img, _ = cvt_ref.synthetic_batch(cfg, 3)
    proc = cvt_ref.synthetic_proc(cfg, 3)
    f = cvt_ref.forward_features(img, p, cfg)
    h = torch.clamp(proc @ p["proc.fc1.weight"].t() + p["proc.fc1.bias"], min=0)
    h = torch.clamp(h @ p["proc.fc2.weight"].t() + p["proc.fc2.bias"], min=0)
    W = p["head.weight"]
    ref = f @ W[:, :f.shape[1]].t() + h @ W[:, f.shape[1]:].t() + p["head.bias"]
    assert torch.allclose(cvt_ref.forward(img, p, cfg, proc), ref, atol=1e-5)


def test_keras_dense_factors_compose_to_the_held_map():
    """keras_dense: the oracle applies each Dense pair as two layers (models/CvT(Par).py:
    132-137,180-188); with the pair composed into one map (W2 W1, W2 b1 + b2) the default oracle
    gives the same logits -- the forward equivalence the composed build relies on."""
    cfg = cvt_ref.CvTConfig(img_size=32, num_classes=2, keras_dense=True,
                            stages=[cvt_ref.CvTStage(16, 7, 4, 1), cvt_ref.CvTStage(32, 3, 2, 2, with_cls_token=True)])
    p = cvt_ref.init_params(cfg, seed=2)
    comp = {k: v for k, v in p.items() if ".mha_" not in k}
    for i in range(len(cfg.stages)):
        a = f"stage{i}.blocks.0.attn."
        for c in "qkv":
            comp[a + f"proj_{c}.weight"] = p[a + f"mha_{c}.weight"] @ p[a + f"proj_{c}.weight"]
            comp[a + f"proj_{c}.bias"] = p[a + f"mha_{c}.weight"] @ p[a + f"proj_{c}.bias"] + p[a + f"mha_{c}.bias"]
        comp[a + "proj.weight"] = p[a + "proj.weight"] @ p[a + "mha_o.weight"]
        comp[a + "proj.bias"] = p[a + "proj.weight"] @ p[a + "mha_o.bias"] + p[a + "proj.bias"]
    img, _ = cvt_ref.synthetic_batch(cfg, 3, seed=3)
    with torch.no_grad():
        y_fact = cvt_ref.forward(img, p, cfg)
        y_comp = cvt_ref.forward(img, comp, cfg.replace(keras_dense=False))
    assert set(p) - set(comp) == {k for k in p if ".mha_" in k}
    assert torch.allclose(y_fact, y_comp, rtol=1e-4, atol=1e-5)
