"""Where does the bf16 gradient error at N = 290 come from?  (verdict r04 item 1)

For a few ViT-Ti configurations, runs the GPU fwd+bwd and the CPU oracle on the same inputs and
prints the worst per-parameter relative errors and, for block 0's qkv bias, the q / k / v thirds
separately (reference norm and error norm of each).  Variants switch the attention kernels
(whole-sequence vs streamed) and the fused bias-gradient sums, so a number can be pinned on the
kernel that makes it.
usage: python tools/diag_grad_precision.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from oracle import vit_ref  # noqa: E402
from vitmi import ops  # noqa: E402
from vitmi.config import config_c1  # noqa: E402
from vitmi.modules import VisionTransformer, cross_entropy  # noqa: E402


def gpu_grads(cfg, params, img, tgt):
    model = VisionTransformer(cfg).cuda()
    model.load_param_dict(params)
    loss = cross_entropy(model(img.cuda()), tgt.cuda())
    loss.backward()
    return {k: p.grad.detach().cpu() for k, p in model.named_parameters()}


def chain_biases(cfg, g, params):
    """The bias gradients formed from the fp32 column sums upstream of them through the linear
    maps (what the fix computes): qkv v-third = colsum(dO) = proj.bias grad @ Wo; k-third = 0
    (softmax shift invariance); norm1.bias = qkv.bias grad @ Wqkv; norm2.bias = fc1.bias grad @ W1."""
    g = dict(g)
    D = cfg.embed_dim
    for b in range(cfg.depth):
        p = f"blocks.{b}."
        qb = g[p + "attn.qkv.bias"].double().clone()
        qb[2 * D:] = g[p + "attn.proj.bias"].double() @ params[p + "attn.proj.weight"].double()
        qb[D:2 * D] = 0
        g[p + "attn.qkv.bias"] = qb.float()
        g[p + "norm1.bias"] = (qb @ params[p + "attn.qkv.weight"].double()).float()
        g[p + "norm2.bias"] = (g[p + "mlp.fc1.bias"].double() @ params[p + "mlp.fc1.weight"].double()).float()
    return g


def report(tag, cfg, g, g_ref, full=False):
    errs = sorted(((vit_ref.rel_err(g[k], g_ref[k]), k) for k in g_ref), reverse=True)
    print(f"== {tag}: N={cfg.seq_len} D={cfg.embed_dim} depth={cfg.depth} dtype={cfg.dtype}")
    for e, k in errs[:(40 if full else 6)]:
        print(f"   {k:32s} rel {e:.3e}  |ref| {g_ref[k].norm():.3e}")
    D = cfg.embed_dim
    for b in (0, cfg.depth - 1):
        k = f"blocks.{b}.attn.qkv.bias"
        r, x = g_ref[k].double(), g[k].double()
        parts = []
        for i, nm in enumerate("qkv"):
            rr, xx = r[i * D:(i + 1) * D], x[i * D:(i + 1) * D]
            parts.append(f"{nm}: |ref| {rr.norm():.2e} |err| {(xx - rr).norm():.2e}")
        print(f"   {k}: " + "; ".join(parts))
    sys.stdout.flush()


def main():
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    for img_size in (272, 224, 64):
        cfg = config_c1(dtype="bf16", img_size=img_size, depth=4)
        params = vit_ref.init_params(cfg, seed=8)
        img, tgt = vit_ref.synthetic_batch(cfg, 2)
        _, _, g_ref = vit_ref.forward_backward(img, tgt, params, cfg)
        report("fp32", cfg.replace(dtype="fp32"), gpu_grads(cfg.replace(dtype="fp32"), params, img, tgt), g_ref)
        g16 = gpu_grads(cfg, params, img, tgt)
        report("bf16 default", cfg, g16, g_ref, full=True)
        report("bf16 + bias chain (emulated)", cfg, chain_biases(cfg, g16, params), g_ref, full=True)
        report("fp32 oracle + bias chain (identity check)", cfg, chain_biases(cfg, g_ref, params), g_ref)
        prev = ops.attention_set_policy(1)
        report("bf16 streamed attention", cfg, gpu_grads(cfg, params, img, tgt), g_ref)
        ops.attention_set_policy(prev)
        d = ops.attention_bwd.__defaults__
        ops.attention_bwd.__defaults__ = (None, False)
        report("bf16 unfused qkv-bias sums", cfg, gpu_grads(cfg, params, img, tgt), g_ref)
        ops.attention_bwd.__defaults__ = d


if __name__ == "__main__":
    main()
