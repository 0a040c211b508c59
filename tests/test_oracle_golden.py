"""Pin the CPU oracle (oracle/vit_ref.py) against golden vectors made from
(i) the reference's own PyTorch module old_codes/MS_CvT.py and (ii) an offline
transformers ViT (tests/golden/gen_golden.py).  No GPU, no reference at run time."""
import os

import numpy as np
import pytest
import torch

from oracle import vit_ref
from vitmi.config import ViTConfig

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    z = np.load(os.path.join(GOLD, name))
    params = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p::")}
    grads = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("g::")}
    return z, params, grads


CASES = {
    # MS_CvT semantics: scale D**-0.5 (MS_CvT.py:100), no qkv bias (:82), LN in
    # ConvEmbed (:358), eps 1e-5, no pos-embed.
    "mscvt_vit_stage.npz": ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=2, num_heads=2,
                                     num_classes=2, attn_scale="dim", ln_eps=1e-5, qkv_bias=False,
                                     embed_norm=True, pos_embed=False),
    # standard ViT semantics (Keras knobs: head-dim scale, bias, eps 1e-6) + pos-embed
    "hf_vit.npz": ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=2, num_heads=2,
                            num_classes=2, attn_scale="head", ln_eps=1e-6, qkv_bias=True,
                            embed_norm=False, pos_embed=True),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_golden(name):
    cfg = CASES[name]
    z, params, grads = _load(name)
    assert set(params) == set(vit_ref.param_shapes(cfg)), "parameter set mismatch"
    for k, shp in vit_ref.param_shapes(cfg).items():
        assert tuple(params[k].shape) == tuple(shp), k
    img = torch.from_numpy(z["input"])
    tgt = torch.from_numpy(z["target"])
    logits, loss, g = vit_ref.forward_backward(img, tgt, params, cfg)
    np.testing.assert_allclose(logits.numpy(), z["logits"], atol=1e-5, rtol=1e-5)
    assert abs(loss.item() - float(z["loss"])) < 1e-5
    for k, ref in grads.items():
        assert vit_ref.rel_err(g[k], ref) < 1e-4, k


def test_flop_model_matches_baseline():
    from vitmi.config import config_c1, config_c2, config_c3, config_c5
    assert abs(config_c1().flops_per_image_fwd() / 1e9 - 0.188) < 2e-3
    assert abs(config_c2().flops_per_image_fwd() / 1e9 - 9.197) < 2e-3
    assert abs(config_c3().flops_per_image_fwd() / 1e9 - 35.126) < 2e-3
    assert abs(config_c5().flops_per_image_fwd() / 1e9 - 382.13) < 2e-2
