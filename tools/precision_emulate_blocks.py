"""Per-block precision mixes of the ViT-B forward (round 5): some blocks fully bf16, the others with
the bf16x3 knob's split operands, against the fp32 oracle.  Shows whether the 1e-3 logits bound
could be met with the knob on a few blocks only (it cannot: any two bf16 blocks exceed it).
usage: python tools/precision_emulate_blocks.py"""
import sys, os, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, 'transformer-stm_amd'), os.path.join(ROOT, 'tools')):
    sys.path.insert(0, _p)
import precision_emulate as pe
from oracle import vit_ref
from vitmi.config import preset
import torch.nn.functional as F
torch.set_num_threads(8)
ALL=set(pe.ALL)
KNOB={"QKV","PR"}
def forward(img,p,cfg,bf16_blocks,patch_split=True):
    # per block: bf16 (all roundings) or the knob (split operands)
    R=lambda on,x: pe.r(x,on)
    D,H=cfg.embed_dim,cfg.num_heads; dh=D//H; Pz=cfg.patch_size; B=img.shape[0]
    patches=F.unfold(img,Pz,stride=Pz).transpose(1,2)
    wp=p["patch_embed.proj.weight"].reshape(D,-1)
    if not patch_split: patches, wp = pe.r(patches,True), pe.r(wp,True)
    x=patches@wp.t()+p["patch_embed.proj.bias"]
    x=torch.cat([p["cls_token"].expand(B,1,D),x],1)+p["pos_embed"]
    N=x.shape[1]; scale=dh**-0.5
    for i in range(cfg.depth):
        pre=f"blocks.{i}."; b16= i in bf16_blocks
        rs = ALL if b16 else KNOB
        W=lambda k: pe.r(p[pre+k], b16)
        h=pe.r(vit_ref.layer_norm(x,p[pre+"norm1.weight"],p[pre+"norm1.bias"],cfg.ln_eps),"LN" in rs)
        qkv=pe.r(h@W("attn.qkv.weight").t()+p[pre+"attn.qkv.bias"],True)
        q,k,v=(t.reshape(B,N,H,dh).transpose(1,2) for t in qkv.split(D,-1))
        a=torch.softmax((q@k.transpose(-1,-2))*scale,-1)
        o=pe.r((pe.r(a,True)@v).transpose(1,2).reshape(B,N,D),"O" in rs)
        x=x+o@W("attn.proj.weight").t()+p[pre+"attn.proj.bias"]
        h2=pe.r(vit_ref.layer_norm(x,p[pre+"norm2.weight"],p[pre+"norm2.bias"],cfg.ln_eps),"LN" in rs)
        act=pe.r(F.gelu(h2@W("mlp.fc1.weight").t()+p[pre+"mlp.fc1.bias"]),"ACT" in rs)
        x=x+act@W("mlp.fc2.weight").t()+p[pre+"mlp.fc2.bias"]
    c=vit_ref.layer_norm(x[:,0],p["norm.weight"],p["norm.bias"],cfg.ln_eps)
    return c@p["head.weight"].t()+p["head.bias"]
for init in ("random","default"):
    cfg=preset("vit_base_16",img_size=224,num_classes=2,dtype="fp32",depth=12)
    params=vit_ref.init_params(cfg,seed=0,randomize_all=init=="random")
    img,_=vit_ref.synthetic_batch(cfg,2)
    with torch.no_grad():
        ref=vit_ref.forward(img,params,cfg)
        print(init, "knob everywhere", (forward(img,params,cfg,set())-ref).abs().max().item())
        print(init, "bf16 everywhere", (forward(img,params,cfg,set(range(12)),False)-ref).abs().max().item())
        for lo,hi in ((0,4),(0,6),(0,8),(4,12),(6,12),(8,12),(2,12),(0,2),(10,12)):
            e=(forward(img,params,cfg,set(range(lo,hi)))-ref).abs().max().item()
            print(init, f"bf16 blocks {lo}-{hi-1}, split elsewhere + patch: {e:.2e}", flush=True)
