"""Generate the golden fixtures that pin ``oracle/vit_ref.py``.

Run in the survey/build container (needs ``/root/reference``; never on the GPU
box):  ``python tests/golden/gen_golden.py``.  Outputs small ``.npz`` files next
to this script; only those DATA files are committed, nothing of the reference's
source.

Fixtures
--------
``mscvt_vit_stage.npz``
    The reference's own PyTorch module ``old_codes/MS_CvT.py``
    (``ConvolutionalVisionTransformer``, ``:491-623``) configured as a one-stage
    ViT: ``QKV_PROJ_METHOD='avg'`` with ``KERNEL_QKV=1, PADDING_KV=0`` makes the
    K/V projections an identity AvgPool2d(1) and Q 'linear' (``:103-114,145-155``)
    — the all-'linear' method crashes at ``:191-198``.  MS_CvT semantics:
    attention scale ``D**-0.5`` (``:100``), no qkv bias (``:82``), LayerNorm in
    ConvEmbed (``:358``), LN eps 1e-5, exact GELU (``nn.GELU``), no pos-embed.
    Imported with three in-memory stubs for its absent imports
    (``torch._six.container_abcs``, ``timm.models.layers``, ``.registry``).
``hf_vit.npz``
    ``transformers.ViTForImageClassification`` built OFFLINE from a config
    (never ``from_pretrained``): standard ViT semantics (learned pos-embed, head-dim
    scale, qkv bias, LN eps 1e-6 to match the Keras reference).

Each file holds ``input``, ``target``, ``p::<name>`` parameters (oracle
naming), ``logits``, ``loss`` and ``g::<name>`` gradients of the CE loss.
"""
from __future__ import annotations

import collections.abc
import importlib.util
import os
import sys
import types
from functools import partial

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/old_codes/MS_CvT.py"


def _trunc_normal_(t, mean=0.0, std=1.0, a=-2.0, b=2.0):
    with torch.no_grad():
        return nn.init.trunc_normal_(t, mean=mean, std=std, a=a, b=b)


def load_mscvt():
    """Import MS_CvT.py from the reference with stubs for its missing deps."""
    six = types.ModuleType("torch._six")
    six.container_abcs = collections.abc
    sys.modules["torch._six"] = six
    timm = types.ModuleType("timm")
    timm_models = types.ModuleType("timm.models")
    timm_layers = types.ModuleType("timm.models.layers")

    class DropPath(nn.Identity):  # only ever built with drop_path=0 here
        def __init__(self, *a, **k):
            super().__init__()

    timm_layers.DropPath = DropPath
    timm_layers.trunc_normal_ = _trunc_normal_
    sys.modules["timm"] = timm
    sys.modules["timm.models"] = timm_models
    sys.modules["timm.models.layers"] = timm_layers
    pkg = types.ModuleType("mscvt_pkg")
    pkg.__path__ = []
    reg = types.ModuleType("mscvt_pkg.registry")
    reg.register_model = lambda f: f
    sys.modules["mscvt_pkg"] = pkg
    sys.modules["mscvt_pkg.registry"] = reg
    spec = importlib.util.spec_from_file_location("mscvt_pkg.MS_CvT", REF)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["mscvt_pkg.MS_CvT"] = mod
    spec.loader.exec_module(mod)
    return mod


def randomize_(model, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if p.dim() == 1 and ("norm" in name or "layernorm" in name):
                if name.endswith("weight"):
                    p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=g))
                else:
                    p.copy_(0.1 * torch.randn(p.shape, generator=g))
            elif name.endswith("bias"):
                p.copy_(0.05 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(0.05 * torch.randn(p.shape, generator=g))


def save(path, img, tgt, params, logits, loss, grads):
    d = {"input": img.numpy(), "target": tgt.numpy(), "logits": logits.detach().numpy(),
         "loss": np.array(loss.item(), dtype=np.float32)}
    for k, v in params.items():
        d["p::" + k] = v.detach().float().numpy()
    for k, v in grads.items():
        d["g::" + k] = v.detach().float().numpy()
    np.savez_compressed(path, **d)
    print("wrote", path, sum(v.size for v in d.values()) * 4 / 1e6, "MB raw")


def gen_mscvt():
    ms = load_mscvt()
    D, H, depth, P, img_size = 128, 2, 2, 8, 32
    spec = {
        "NUM_STAGES": 1, "PATCH_SIZE": [P], "PATCH_STRIDE": [P], "PATCH_PADDING": [0],
        "DIM_EMBED": [D], "DEPTH": [depth], "NUM_HEADS": [H], "MLP_RATIO": [4.0],
        "QKV_BIAS": [False], "DROP_RATE": [0.0], "ATTN_DROP_RATE": [0.0], "DROP_PATH_RATE": [0.0],
        "CLS_TOKEN": [True], "QKV_PROJ_METHOD": ["avg"], "KERNEL_QKV": [1], "PADDING_Q": [0],
        "PADDING_KV": [0], "STRIDE_KV": [1], "STRIDE_Q": [1],
    }
    torch.manual_seed(0)
    model = ms.ConvolutionalVisionTransformer(in_chans=3, num_classes=2, act_layer=nn.GELU,
                                              norm_layer=partial(nn.LayerNorm, eps=1e-5), spec=spec)
    randomize_(model, 1)
    g = torch.Generator().manual_seed(2)
    img = torch.rand(4, 3, img_size, img_size, generator=g)
    tgt = torch.randint(0, 2, (4,), generator=g)
    logits = model(img)
    loss = nn.functional.cross_entropy(logits, tgt)
    loss.backward()
    sd = dict(model.named_parameters())

    def rn(name):
        return name.replace("stage0.", "")

    params, grads = {}, {}
    for name, p in sd.items():
        if ".attn.proj_q." in name or ".attn.proj_k." in name or ".attn.proj_v." in name:
            continue
        params[rn(name)] = p
        grads[rn(name)] = p.grad
    for i in range(depth):
        pre = f"stage0.blocks.{i}.attn."
        w = [sd[pre + f"proj_{c}.weight"] for c in "qkv"]
        params[f"blocks.{i}.attn.qkv.weight"] = torch.cat([x.detach() for x in w], 0)
        grads[f"blocks.{i}.attn.qkv.weight"] = torch.cat([x.grad for x in w], 0)
    save(os.path.join(HERE, "mscvt_vit_stage.npz"), img, tgt, params, logits, loss, grads)


def gen_mscvt_cvt():
    """``mscvt_cvt_dwbn.npz``: MS_CvT's ConvolutionalVisionTransformer with the dw_bn q/k/v
    projection (``old_codes/MS_CvT.py:124-144``: depthwise 3x3 + BatchNorm2d, training mode)
    in two stages shaped like the reference's Keras spec (``models/CvT(Par).py:66-72``):
    ConvEmbed k7 s4 (D 64, 1 head) and k3 s2 (D 128, 2 heads, cls token), 1-channel 32x32
    input.  Pins ``oracle/cvt_ref.py`` in its MS_CvT knob setting."""
    ms = load_mscvt()
    spec = {
        "NUM_STAGES": 2, "PATCH_SIZE": [7, 3], "PATCH_STRIDE": [4, 2], "PATCH_PADDING": [2, 1],
        "DIM_EMBED": [64, 128], "DEPTH": [1, 1], "NUM_HEADS": [1, 2], "MLP_RATIO": [4.0, 4.0],
        "QKV_BIAS": [False, False], "DROP_RATE": [0.0, 0.0], "ATTN_DROP_RATE": [0.0, 0.0],
        "DROP_PATH_RATE": [0.0, 0.0], "CLS_TOKEN": [False, True], "QKV_PROJ_METHOD": ["dw_bn", "dw_bn"],
        "KERNEL_QKV": [3, 3], "PADDING_Q": [1, 1], "PADDING_KV": [1, 1], "STRIDE_KV": [1, 1], "STRIDE_Q": [1, 1],
    }
    torch.manual_seed(0)
    model = ms.ConvolutionalVisionTransformer(in_chans=1, num_classes=2, act_layer=nn.GELU,
                                              norm_layer=partial(nn.LayerNorm, eps=1e-5), spec=spec)
    randomize_(model, 5)
    model.train()
    g = torch.Generator().manual_seed(6)
    img = torch.rand(4, 1, 32, 32, generator=g)
    tgt = torch.randint(0, 2, (4,), generator=g)
    logits = model(img)
    loss = nn.functional.cross_entropy(logits, tgt)
    loss.backward()
    params, grads = {}, {}
    for name, p in model.named_parameters():
        n = (name.replace(".patch_embed.proj.", ".embed.").replace(".patch_embed.norm.", ".embed.norm.")
             .replace(".conv.weight", ".weight"))
        params[n] = p
        grads[n] = p.grad
    save(os.path.join(HERE, "mscvt_cvt_dwbn.npz"), img, tgt, params, logits, loss, grads)


def gen_mscvt_cvt_avg():
    """``mscvt_cvt_avg.npz``: as ``gen_mscvt_cvt`` with the other two q/k/v projection methods
    (``old_codes/MS_CvT.py:145-157``): 'avg' in both stages (AvgPool2d(3, 1, 1) on k and v, q
    'linear' = identity), the cls token in stage 2.  (An all-'linear' stage cannot run in
    MS_CvT: ``Attention.forward`` reads q before assignment when no conv_proj exists, ``:190-198``.)"""
    ms = load_mscvt()
    spec = {
        "NUM_STAGES": 2, "PATCH_SIZE": [7, 3], "PATCH_STRIDE": [4, 2], "PATCH_PADDING": [2, 1],
        "DIM_EMBED": [64, 128], "DEPTH": [1, 1], "NUM_HEADS": [1, 2], "MLP_RATIO": [4.0, 4.0],
        "QKV_BIAS": [False, False], "DROP_RATE": [0.0, 0.0], "ATTN_DROP_RATE": [0.0, 0.0],
        "DROP_PATH_RATE": [0.0, 0.0], "CLS_TOKEN": [False, True], "QKV_PROJ_METHOD": ["avg", "avg"],
        "KERNEL_QKV": [3, 3], "PADDING_Q": [1, 1], "PADDING_KV": [1, 1], "STRIDE_KV": [1, 1], "STRIDE_Q": [1, 1],
    }
    torch.manual_seed(0)
    model = ms.ConvolutionalVisionTransformer(in_chans=1, num_classes=2, act_layer=nn.GELU,
                                              norm_layer=partial(nn.LayerNorm, eps=1e-5), spec=spec)
    randomize_(model, 7)
    model.train()
    g = torch.Generator().manual_seed(8)
    img = torch.rand(4, 1, 32, 32, generator=g)
    tgt = torch.randint(0, 2, (4,), generator=g)
    logits = model(img)
    loss = nn.functional.cross_entropy(logits, tgt)
    loss.backward()
    params, grads = {}, {}
    for name, p in model.named_parameters():
        n = name.replace(".patch_embed.proj.", ".embed.").replace(".patch_embed.norm.", ".embed.norm.")
        params[n] = p
        grads[n] = p.grad
    save(os.path.join(HERE, "mscvt_cvt_avg.npz"), img, tgt, params, logits, loss, grads)


def gen_hf():
    from transformers import ViTConfig as HFConfig, ViTForImageClassification
    D, H, depth, P, img_size = 128, 2, 2, 8, 32
    cfg = HFConfig(image_size=img_size, patch_size=P, num_channels=3, hidden_size=D,
                   num_hidden_layers=depth, num_attention_heads=H, intermediate_size=4 * D,
                   hidden_act="gelu", layer_norm_eps=1e-6, qkv_bias=True, num_labels=2,
                   hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    cfg._attn_implementation = "eager"
    torch.manual_seed(0)
    model = ViTForImageClassification(cfg).eval()
    randomize_(model, 3)
    g = torch.Generator().manual_seed(4)
    img = torch.rand(4, 3, img_size, img_size, generator=g)
    tgt = torch.randint(0, 2, (4,), generator=g)
    logits = model(pixel_values=img).logits
    loss = nn.functional.cross_entropy(logits, tgt)
    loss.backward()
    sd = dict(model.named_parameters())
    m = {
        "vit.embeddings.cls_token": "cls_token",
        "vit.embeddings.position_embeddings": "pos_embed",
        "vit.embeddings.patch_embeddings.projection.weight": "patch_embed.proj.weight",
        "vit.embeddings.patch_embeddings.projection.bias": "patch_embed.proj.bias",
        "vit.layernorm.weight": "norm.weight", "vit.layernorm.bias": "norm.bias",
        "classifier.weight": "head.weight", "classifier.bias": "head.bias",
    }
    params, grads = {}, {}
    for k, v in m.items():
        params[v] = sd[k]
        grads[v] = sd[k].grad
    for i in range(depth):
        L = f"vit.layers.{i}."   # transformers 5.x naming
        B = f"blocks.{i}."
        for src, dst in [("layernorm_before", "norm1"), ("layernorm_after", "norm2"),
                         ("attention.o_proj", "attn.proj"), ("mlp.fc1", "mlp.fc1"),
                         ("mlp.fc2", "mlp.fc2")]:
            for leaf in ("weight", "bias"):
                params[B + dst + "." + leaf] = sd[L + src + "." + leaf]
                grads[B + dst + "." + leaf] = sd[L + src + "." + leaf].grad
        for leaf in ("weight", "bias"):
            ps = [sd[L + f"attention.{c}_proj.{leaf}"] for c in "qkv"]
            params[B + "attn.qkv." + leaf] = torch.cat([x.detach() for x in ps], 0)
            grads[B + "attn.qkv." + leaf] = torch.cat([x.grad for x in ps], 0)
    save(os.path.join(HERE, "hf_vit.npz"), img, tgt, params, logits, loss, grads)


if __name__ == "__main__":
    torch.set_num_threads(4)
    if "--cvt-only" not in sys.argv:
        gen_hf()  # before the MS_CvT stubs: a stub 'timm' module confuses transformers' import probe
    if os.path.exists(REF):
        if "--cvt-only" not in sys.argv:
            gen_mscvt()
        gen_mscvt_cvt()
        gen_mscvt_cvt_avg()
    else:
        print("reference absent; MS_CvT fixture not regenerated")
