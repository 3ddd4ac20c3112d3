"""Stage-by-stage comparison of one fused ViT block on the GPU against the CPU oracle (teacher-forced:
the oracle's residual stream enters the block). Prints, per quantizer, the fraction of differing codes
and, per fp32 stage, the relative error — to locate which stage carries a block's parity error.

    python tools/diag_block.py [--model vit_base_patch16_224] [--block 1] [--batch 2] [--img-seed 5]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import quant_oracle as O  # noqa: E402
from quantized_vit_amd import _lib, vit_model  # noqa: E402
from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def codes_cmp(name, got, want):
    got, want = got.cpu().to(torch.int32), want.cpu().to(torch.int32)
    d = (got - want).abs()
    print(f"  {name:28s} codes differ {100 * (d > 0).float().mean().item():8.4f}%  max|diff| {d.max().item()}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_base_patch16_224")
    ap.add_argument("--block", type=int, default=1)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--img-seed", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    model = build_quantized_vit(a.model, seed=0).to(dev)
    cfg = O.ViTConfig(embed_dim=model.embed_dim, depth=len(model.blocks), num_heads=model.blocks[0].attn.num_heads)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    img = synthetic_images(a.batch, 224, seed=a.img_seed)
    trace = []
    with torch.no_grad():
        O.vit_forward(sd, cfg, img, trace=trace)
    i = a.block
    x = trace[i]
    blk = model.blocks[i]
    pre = f"blocks.{i}"
    B, N, C = x.shape
    M = B * N

    def lq(name):
        return O.LayerQ.from_state(sd, f"{pre}.{name}.", cfg.quant_type, cfg.quant_mode)

    def oracle_codes(v, name):
        q = lq(name)
        return O.quant_codes(v, q.quant_type, q.d_act, q.q_m_act, q.t_act)

    with torch.no_grad():
        # oracle stages
        h1 = O._layer_norm(x, sd, pre + ".norm1")
        qkv = O._qlin(h1, sd, pre + ".attn.qkv", cfg)
        qh, kh, vh = qkv.reshape(B, N, 3, -1, 64).permute(2, 0, 3, 1, 4)
        att = ((qh @ kh.transpose(-2, -1)) * 0.125).softmax(-1)
        ao = (att @ vh).transpose(1, 2).reshape(B, N, -1)
        x1 = x + O._qlin(ao, sd, pre + ".attn.proj", cfg)
        h2 = O._layer_norm(x1, sd, pre + ".norm2")
        f1 = O._qlin(h2, sd, pre + ".mlp.fc1", cfg)
        g1 = F.gelu(f1)
        x2 = x1 + O._qlin(g1, sd, pre + ".mlp.fc2", cfg)

        # GPU stages, each fed the oracle's input
        xg = x.to(dev).reshape(M, C).contiguous()
        p = blk.attn.qkv.quant_plan()
        c1 = torch.empty((M, p.kpad), dtype=torch.int8, device=dev)
        _lib.layernorm_quant_i8(xg, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, p.qtype, p.d_act, p.qm_act,
                                p.t_act, 0, c1, p.kpad)
        codes_cmp("norm1 -> qkv act codes", c1[:, :C], oracle_codes(h1.reshape(M, C), "attn.qkv"))
        c1o = oracle_codes(h1.reshape(M, C), "attn.qkv").to(torch.int8).to(dev)
        qg = blk.attn.qkv.gemm_codes(c1o.contiguous(), p, _lib.EPI_F32)[:, :p.n]
        print(f"  qkv (oracle codes in)        rel {rel(qg, qkv.reshape(M, -1)):.3e}")
        pp = blk.attn.proj.quant_plan()
        ca = torch.empty((M, pp.kpad), dtype=torch.int8, device=dev)
        blk.attn.core_hip(qkv.reshape(M, -1).to(dev).contiguous(), B, N, ca, _lib.ATT_I8, 1.0, pp)
        codes_cmp("attention -> proj act codes", ca[:, :C], oracle_codes(ao.reshape(M, C), "attn.proj"))
        af = torch.empty((M, C), device=dev)
        blk.attn.core_hip(qkv.reshape(M, -1).to(dev).contiguous(), B, N, af)
        print(f"  attention fp32               rel {rel(af, ao.reshape(M, C)):.3e}")
        cao = oracle_codes(ao.reshape(M, C), "attn.proj").to(torch.int8).to(dev)
        xr = x.to(dev).reshape(M, C).contiguous().clone()
        blk.attn.proj.gemm_codes(cao.contiguous(), pp, _lib.EPI_F32_RESID, out=xr)
        print(f"  x + proj (oracle codes in)   rel {rel(xr, x1.reshape(M, C)):.3e}")
        p1 = blk.mlp.fc1.quant_plan()
        c2 = torch.empty((M, p1.kpad), dtype=torch.int8, device=dev)
        x1g = x1.to(dev).reshape(M, C).contiguous()
        _lib.layernorm_quant_i8(x1g, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps, p1.qtype, p1.d_act, p1.qm_act,
                                p1.t_act, 0, c2, p1.kpad)
        codes_cmp("norm2 -> fc1 act codes", c2[:, :C], oracle_codes(h2.reshape(M, C), "mlp.fc1"))
        c2o = oracle_codes(h2.reshape(M, C), "mlp.fc1").to(torch.int8).to(dev).contiguous()
        p2 = blk.mlp.fc2.quant_plan()
        hid = torch.zeros((M, p2.kpad), dtype=torch.int8, device=dev)
        blk.mlp.fc1.gemm_codes(c2o, p1, _lib.EPI_I8_GELU, out=hid, next_layer=blk.mlp.fc2)
        codes_cmp("fc1+gelu -> fc2 act codes", hid[:, :p1.n], oracle_codes(g1.reshape(M, -1), "mlp.fc2"))
        f1g = blk.mlp.fc1.gemm_codes(c2o, p1, _lib.EPI_F32)[:, :p1.n]
        print(f"  fc1 fp32 (oracle codes in)   rel {rel(f1g, f1.reshape(M, -1)):.3e}")
        cg = oracle_codes(g1.reshape(M, -1), "mlp.fc2")
        hid2 = torch.zeros((M, p2.kpad), dtype=torch.int8, device=dev)
        hid2[:, :p1.n] = cg.to(torch.int8).to(dev)
        xr2 = x1.to(dev).reshape(M, C).contiguous().clone()
        blk.mlp.fc2.gemm_codes(hid2, p2, _lib.EPI_F32_RESID, out=xr2)
        print(f"  x1 + fc2 (oracle codes in)   rel {rel(xr2, x2.reshape(M, C)):.3e}")
        # quantizer parameters of this block
        for nm in ("attn.qkv", "attn.proj", "mlp.fc1", "mlp.fc2"):
            q = lq(nm)
            print(f"  {nm:10s} act d {q.d_act:.4e} qm {q.q_m_act:.4e} t {q.t_act}  wt d {q.d_wt:.4e} qm {q.q_m_wt:.4e}")
        out = blk.forward_fused_(x.to(dev).contiguous().clone())
        print(f"  whole block                  rel {rel(out, x2):.3e}")


if __name__ == "__main__":
    main()
