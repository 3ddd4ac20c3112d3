"""GPU parity of the module surface and the ViT caller against the CPU oracle's fake-quant forward.

North-star bar: logits match the reference fake-quant CPU forward on identical int4 weights within
1e-3 relative (norm-wise). Module-level outputs (single layer) are held to 1e-5 relative.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import quant_oracle as O
from quantized_vit_amd import _lib, vit_model
from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images
from quantized_vit_amd.quant_layers import (QuantizationMode, QuantizationType, QuantizeConv2d, QuantizeLinear,
                                            epilogue_table, initialize_quant_layer)

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm()).item()


def _layer_q(m):
    sd = m.state_dict()
    qt = m.quant_type.value
    return O.LayerQ.from_state(sd, "", qt, m.quant_mode.value)


def _calibrated_linear(dev, k, n, qt, bits=4, t_act=1.0, seed=0):
    torch.manual_seed(seed)
    lin = nn.Linear(k, n)
    q = QuantizeLinear.from_module(lin, quant_type=qt, quant_mode=QuantizationMode.WEIGHT_AND_ACTIVATION,
                                   num_bits=bits).to(dev).eval()
    with torch.no_grad():
        q.q_m_act.fill_(2.0)
        q.d_quant_act.fill_(np.exp(t_act * np.log(2.0)) / 127)
        if hasattr(q, "t_quant_act"):
            q.t_quant_act.fill_(t_act)
    q.invalidate()
    return q


@pytest.mark.parametrize("qt", [QuantizationType.SYMMETRIC_LINEAR, QuantizationType.SYMMETRIC_NONLINEAR,
                                QuantizationType.DGE])
@pytest.mark.parametrize("k,n,bits", [(768, 3072, 4), (3072, 768, 4), (200, 77, 4), (768, 768, 6)])
def test_quantize_linear_vs_oracle(dev, qt, k, n, bits):
    q = _calibrated_linear(dev, k, n, qt, bits)
    plan = q.quant_plan()
    assert plan.int_path and plan.wfmt == (_lib.W4 if bits <= 4 else _lib.W8)
    x = torch.randn(3, 70, k) * 0.7
    with torch.no_grad():
        y = q(x.to(dev))
    ref = O.quantize_linear(x, q.weight.detach().cpu(), q.bias.detach().cpu(), _layer_q(q))
    assert y.shape == ref.shape
    assert rel(y, ref) < 1e-5


def test_quantize_linear_reference_identity_limit_on_gpu(dev):
    """OTO/tests/quantization/test_quant_layers.py:10-35 run on the GPU module (fp32 fake-quant path:
    d = 1e-4, q_m = 10 gives 10^5 levels, beyond int8)."""
    torch.manual_seed(0)
    q = QuantizeLinear(256, 128, bias=True, d_quant_init=1e-4, t_quant_init=1.0, q_m_init=10.0).to(dev).eval()
    lin = nn.Linear(256, 128).to(dev).eval()
    with torch.no_grad():
        lin.weight.copy_(torch.rand(128, 256))
        q.weight.copy_(lin.weight)
        q.bias.copy_(lin.bias)
    x = torch.rand(1, 256, device=dev)
    with torch.no_grad():
        a, b = q(x), lin(x)
    assert not q.quant_plan().int_path
    assert torch.allclose(a, b, rtol=1e-4, atol=1e-8) or (a - b).abs().max().item() <= 1e-4


def test_quantize_conv2d_reference_identity_limit_on_gpu(dev):
    """test_quant_layers.py:38-78 on the GPU module."""
    torch.manual_seed(0)
    q = QuantizeConv2d(3, 64, 3, stride=1, padding=1, bias=True, d_quant_init=1e-4, q_m_init=10.0).to(dev).eval()
    conv = nn.Conv2d(3, 64, 3, stride=1, padding=1, bias=True).to(dev).eval()
    with torch.no_grad():
        conv.weight.copy_(torch.rand(64, 3, 3, 3))
        q.weight.copy_(conv.weight)
        q.bias.copy_(conv.bias)
        x = torch.rand(1, 3, 32, 32, device=dev)
        a, b = q(x), conv(x)
    assert torch.allclose(a, b, rtol=1e-4, atol=1e-8) or (a - b).abs().max().item() <= 1e-4


@pytest.mark.parametrize("cfg", [dict(cin=3, cout=768, k=16, s=16, p=0, H=224),
                                 dict(cin=16, cout=32, k=3, s=1, p=1, H=24), dict(cin=8, cout=20, k=3, s=2, p=1, H=15)])
def test_quantize_conv2d_int_path_vs_oracle(dev, cfg):
    torch.manual_seed(1)
    conv = nn.Conv2d(cfg["cin"], cfg["cout"], cfg["k"], stride=cfg["s"], padding=cfg["p"], bias=True)
    q = QuantizeConv2d.from_module(conv, quant_type=QuantizationType.SYMMETRIC_NONLINEAR,
                                   quant_mode=QuantizationMode.WEIGHT_AND_ACTIVATION, num_bits=4).to(dev).eval()
    with torch.no_grad():
        q.q_m_act.fill_(1.0)
        q.d_quant_act.fill_(1.0 / 127)
    q.invalidate()
    assert q.quant_plan().int_path
    x = torch.rand(2, cfg["cin"], cfg["H"], cfg["H"]) * 2 - 1
    with torch.no_grad():
        y = q(x.to(dev))
    ref = O.quantize_conv2d(x, q.weight.detach().cpu(), q.bias.detach().cpu(), _layer_q(q), stride=cfg["s"],
                            padding=cfg["p"])
    assert y.shape == ref.shape and y.is_contiguous()
    assert rel(y, ref) < 1e-5


def test_weight_only_mode_runs_wonly_kernel(dev):
    """The default WEIGHT_ONLY mode: fp32 activations against the packed codes (qvit_gemm_wonly)."""
    torch.manual_seed(2)
    q = QuantizeLinear.from_module(nn.Linear(64, 32), quant_type=QuantizationType.SYMMETRIC_NONLINEAR,
                                   num_bits=4).to(dev).eval()
    x = torch.randn(5, 64)
    with torch.no_grad():
        y = q(x.to(dev))
    assert not q.quant_plan().int_path and q.quant_plan().extra.get("wonly")
    ref = O.quantize_linear(x, q.weight.detach().cpu(), q.bias.detach().cpu(), _layer_q(q))
    assert rel(y, ref) < 1e-5


@pytest.mark.parametrize("bits", [16, 32])
@pytest.mark.parametrize("qt", [QuantizationType.SYMMETRIC_NONLINEAR, QuantizationType.SYMMETRIC_LINEAR])
def test_weight_and_activation_wide_bits_fp_path(dev, bits, qt):
    """WEIGHT_AND_ACTIVATION at the reference's own initial widths (model_to_quantize_model's num_bits=16,
    train_geta_test.py:277-280's 32): levels beyond int8 take the fake-quant fp32 path for both operands
    (this crashed on a missing fake-quant weight)."""
    torch.manual_seed(bits)
    lin = QuantizeLinear.from_module(nn.Linear(96, 40), quant_type=qt,
                                     quant_mode=QuantizationMode.WEIGHT_AND_ACTIVATION, num_bits=bits).to(dev).eval()
    conv = QuantizeConv2d.from_module(nn.Conv2d(3, 24, 4, stride=4, padding=0, bias=True), quant_type=qt,
                                      quant_mode=QuantizationMode.WEIGHT_AND_ACTIVATION, num_bits=bits).to(dev).eval()
    x = torch.randn(5, 96) * 0.05
    img = (torch.rand(2, 3, 32, 32) * 2 - 1) * 0.05
    with torch.no_grad():
        y, yc = lin(x.to(dev)), conv(img.to(dev))
    assert not lin.quant_plan().int_path and not conv.quant_plan().int_path
    # 16 bits: the linear layer runs qvit_gemm_wonly on wide codes (fake-quant fp32 activations); 32 bits: F.linear
    assert bool(lin.quant_plan().extra.get("wonly")) == (bits == 16)
    assert bits != 16 or lin.quant_plan().wfmt in (_lib.W16, _lib.W24)
    ref = O.quantize_linear(x, lin.weight.detach().cpu(), lin.bias.detach().cpu(), _layer_q(lin))
    refc = O.quantize_conv2d(img, conv.weight.detach().cpu(), conv.bias.detach().cpu(), _layer_q(conv), stride=4,
                             padding=0)
    assert rel(y, ref) < 1e-5 and rel(yc, refc) < 1e-5


def test_bound_codes_reach_grouped_conv_library_path(dev):
    """a conv whose plan is on the int path but whose forward takes the library conv
    (groups > 1) must run exactly the weight codes bound by load_weight_codes, not re-derived ones."""
    torch.manual_seed(11)
    conv = nn.Conv2d(8, 16, 3, stride=1, padding=1, groups=2, bias=True)
    q = QuantizeConv2d.from_module(conv, quant_type=QuantizationType.SYMMETRIC_NONLINEAR,
                                   quant_mode=QuantizationMode.WEIGHT_AND_ACTIVATION, num_bits=4).to(dev).eval()
    with torch.no_grad():
        q.q_m_act.fill_(1.0)
        q.d_quant_act.fill_(1.0 / 127)
    codes = torch.randint(-7, 8, tuple(q.weight.shape), generator=torch.Generator().manual_seed(3))
    q.load_weight_codes(codes)
    assert q.quant_plan().int_path and not q._int_conv_ok()
    x = (torch.rand(2, 8, 12, 12) * 2 - 1).to(dev)
    with torch.no_grad():
        y = q(x)
        ref = F.conv2d(q.quantize_act(x), q.d_quant_wt * codes.float().to(dev), q.bias, 1, 1, 1, 2)
    assert torch.equal(q.weight_codes().cpu(), codes.reshape(16, -1).float())
    assert rel(y, ref) < 1e-6


def test_plan_cache_tracks_parameter_versions(dev):
    q = _calibrated_linear(dev, 128, 64, QuantizationType.SYMMETRIC_NONLINEAR)
    p1 = q.quant_plan()
    assert q.quant_plan() is p1
    with torch.no_grad():
        q.weight.mul_(0.5)          # bumps the version counter
    p2 = q.quant_plan()
    assert p2 is not p1
    x = torch.randn(4, 128)
    with torch.no_grad():
        y = q(x.to(dev))
    assert rel(y, O.quantize_linear(x, q.weight.detach().cpu(), q.bias.detach().cpu(), _layer_q(q))) < 1e-5


def _oracle_logits(model, cfg, img):
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        return O.vit_forward(sd, cfg, img)


def check_vit_parity(model, cfg, img, dev, block_tol=1e-3, floor_factor=2.5):
    """Parity of the GPU ViT against the CPU oracle, on identical int4 weights (the reference's own
    weight codes are bound to every layer first).

    1. Teacher-forced: the patch embedding, every block and the head are run on the GPU on the
       ORACLE's input to that stage; each output must match the oracle's within block_tol
       (north-star tolerance, applied per stage), or, for a block, within floor_factor x that
       block's own fp64-vs-fp32 distance on the same input (a block whose quantizers sit on many
       near-ties differs from itself by more than 1e-3 between fp32 and fp64).
    2. End-to-end, tie-resolved (parity_tools): every quantizer boundary of the full GPU forward is
       compared with the oracle's; each differing code must be a proven rounding tie (<= 1e-4 of the
       codes), and with the ties resolved alike the logits agree within TIE_E2E."""
    from parity_tools import load_oracle_weight_codes, tie_resolved_vit_check
    load_oracle_weight_codes(model, cfg)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    trace = []
    with torch.no_grad():
        ref32 = O.vit_forward(sd, cfg, img, trace=trace)
        sd64 = {k: v.double() for k, v in sd.items()}
        x = model.patch_embed(img.to(dev))
        x = torch.cat((model.cls_token.expand(x.shape[0], -1, -1), x), dim=1) + model.pos_embed
        errs = {"embed": rel(x, trace[0])}
        tols = {}
        for i, blk in enumerate(model.blocks):
            assert blk.fused_ok(x)
            out = blk.forward_fused_(trace[i].to(dev).contiguous().clone())
            errs[f"block{i}"] = rel(out, trace[i + 1])
            stage_floor = rel(O.vit_block(trace[i].double(), sd64, cfg, i), trace[i + 1])
            tols[f"block{i}"] = max(block_tol, floor_factor * stage_floor)
        head = model.head(model.norm(trace[-1].to(dev))[:, 0])
        errs["head"] = rel(head, ref32)
    worst = max(errs.values())
    r = tie_resolved_vit_check(model, cfg, img, dev)
    print(f"teacher-forced worst stage {worst:.2e} ({max(errs, key=errs.get)}); end-to-end tie-resolved "
          f"{r['rel']:.3e} ({r['flips']} tie flips of {r['codes']} codes)")
    bad = {k: (e, tols.get(k, block_tol)) for k, e in errs.items() if e >= tols.get(k, block_tol)}
    assert not bad, bad
    assert not r["missing"] and not r["bad"], (r["missing"], r["bad"])
    assert r["rel"] <= TIE_E2E, r["rel"]
    return errs, r


def test_vit_tiny_golden_logits(dev):
    z = np.load(os.path.join(GOLDEN, "vit_tiny_b2_logits.npz"))
    model = build_quantized_vit("vit_tiny_patch16_224", num_classes=int(z["num_classes"]), seed=int(z["seed"]),
                                depth=int(z["depth"])).to(dev)
    img = synthetic_images(int(z["batch"]), 224, seed=int(z["img_seed"]))
    with torch.no_grad():
        y = model(img.to(dev))
    assert rel(y, torch.from_numpy(z["logits"])) < 1e-3


@pytest.mark.parametrize("t_act", [1.0, 0.9])
def test_vit_tiny_b8_vs_oracle(dev, t_act):
    model = build_quantized_vit("vit_tiny_patch16_224", seed=3, t_act=t_act).to(dev)
    cfg = O.ViTConfig(embed_dim=192, depth=12, num_heads=3)
    check_vit_parity(model, cfg, synthetic_images(8, 224, seed=0), dev)


@pytest.mark.parametrize("qt", [QuantizationType.SYMMETRIC_NONLINEAR, QuantizationType.SYMMETRIC_LINEAR])
def test_vit_shipping_weight_codes_end_to_end(dev, qt):
    """The shipped configuration end to end: the device derives its own weight codes (no
    load_weight_codes), and the logits must sit within 2.5x the reference's own fp32-vs-fp64 distance
    (+1e-4) of the oracle's fp32 forward on the same images."""
    model = build_quantized_vit("vit_tiny_patch16_224", seed=8, quant_type=qt).to(dev)
    cfg = O.ViTConfig(embed_dim=192, depth=12, num_heads=3,
                      quant_type=O.LINEAR if qt == QuantizationType.SYMMETRIC_LINEAR else O.NONLINEAR)
    assert all(getattr(m, "_weight_codes", None) is None for m in model.modules())
    img = synthetic_images(4, 224, seed=3)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        y = model(img.to(dev))
        ref32 = O.vit_forward(sd, cfg, img)
        ref64 = O.vit_forward({k: v.double() for k, v in sd.items()}, cfg, img.double())
    floor = rel(ref32, ref64)
    err = rel(y, ref32)
    print(f"shipping path: rel {err:.3e}, reference fp32-vs-fp64 floor {floor:.3e}")
    assert err <= 2.5 * floor + 1e-4, (err, floor)


@pytest.mark.parametrize("name,depth,batch", [("vit_tiny_patch16_224", 4, 3), ("vit_base_patch16_224", 2, 5)])
def test_vit_resid_ln_fusion_bit_identical(dev, name, depth, batch):
    """The LayerNorms carried by the residual GEMMs (qvit_gemm_resid_ln: proj -> norm2, fc2 -> next norm1)
    give the very same logits as the separate LayerNorm launches."""
    model = build_quantized_vit(name, seed=6, depth=depth).to(dev)
    img = synthetic_images(batch, 224, seed=2).to(dev)
    outs = []
    saved = vit_model.FUSE_RESID_LN
    for fuse in (True, False):
        vit_model.FUSE_RESID_LN = fuse
        try:
            with torch.no_grad():
                outs.append(model(img).cpu())
        finally:
            vit_model.FUSE_RESID_LN = saved
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("batch", [1, 5])
def test_vit_fc1_weight_stationary_bit_identical(dev, batch):
    """fc1 on the weight-stationary schedule (norm2 -> QVIT_ACT_T32 codes -> qvit_gemm_a32, the opt-in
    FC1_WEIGHT_STATIONARY route) gives the very same logits as the tile schedule."""
    model = build_quantized_vit("vit_base_patch16_224", seed=7, depth=2).to(dev)
    img = synthetic_images(batch, 224, seed=3).to(dev)
    assert model.blocks[0].mlp.fc1.a32_fits(model.blocks[0].mlp.fc1.quant_plan(), _lib.EPI_I8_GELU)
    outs = []
    saved = vit_model.FC1_WEIGHT_STATIONARY
    for ws in (True, False):
        vit_model.FC1_WEIGHT_STATIONARY = ws
        try:
            with torch.no_grad():
                outs.append(model(img).cpu())
        finally:
            vit_model.FC1_WEIGHT_STATIONARY = saved
    assert torch.equal(outs[0], outs[1])


def test_vit_linear_quantizer_vs_oracle(dev):
    model = build_quantized_vit("vit_tiny_patch16_224", seed=5, quant_type=QuantizationType.SYMMETRIC_LINEAR).to(dev)
    cfg = O.ViTConfig(embed_dim=192, depth=12, num_heads=3, quant_type=O.LINEAR)
    check_vit_parity(model, cfg, synthetic_images(4, 224, seed=1), dev)


def test_vit_fused_equals_modulewise(dev):
    """The fused block pipeline vs running each module on its own (both on the GPU)."""
    model = build_quantized_vit("vit_tiny_patch16_224", seed=4, depth=4).to(dev)
    img = synthetic_images(4, 224, seed=2).to(dev)
    with torch.no_grad():
        fused = model(img)
        x = model.patch_embed(img)
        x = torch.cat((model.cls_token.expand(x.shape[0], -1, -1), x), dim=1) + model.pos_embed
        for blk in model.blocks:
            x = x + blk.attn(blk.norm1(x))
            x = x + blk.mlp(blk.norm2(x))
        ref = model.head(model.norm(x)[:, 0])
    assert rel(fused, ref) < 1e-4


def stage_forced_block(model, cfg, sd, x, i, dev):
    """Block i with the ORACLE's values entering every kernel (quantizer-boundary forcing): each stage
    of the fused block is compared in isolation, so one tie flip cannot cascade through attention.
    Returns {stage: (kind, metric...)}: codes -> ("codes", flip fraction, non-tie count) where every
    flipped code must be a proven rounding tie (parity_tools.tie_check); fp32 -> ("fp32", rel).
    The production kernels are the ones checked: the fused qkv projection + attention kernel when the
    block takes it (N <= 208), else the qkv GEMM and the attention kernel separately."""
    from parity_tools import tie_check
    blk = model.blocks[i]
    pre = f"blocks.{i}"
    B, N, C = x.shape
    M = B * N
    res = {}

    def lq(name):
        return O.LayerQ.from_state(sd, f"{pre}.{name}.", cfg.quant_type, cfg.quant_mode)

    def ocodes(v, name):
        q = lq(name)
        return O.quant_codes(v.reshape(M, -1), q.quant_type, q.d_act, q.q_m_act, q.t_act)

    def cmp_codes(stage, got, v, name):
        """GPU codes of the values v (oracle's) quantized by layer `name`'s activation quantizer."""
        q = lq(name)
        st = tie_check(v.reshape(M, -1), got.cpu(), ocodes(v, name), q.quant_type, q.d_act, q.q_m_act, q.t_act)
        res[stage] = ("codes", st["flips"] / st["total"], st["non_ties"])

    def gemm_ref(name, layer, a_codes):
        """fp64 d_a d_w (A . W^T) + b on the weight codes the device packed (the reference's own codes
        when they were loaded with load_weight_codes); their agreement with the reference's
        quantize_weight is a stage of its own ("weight codes": ties only, none when loaded)."""
        q = lq(name)
        w = layer.weight.detach().cpu()
        wg = layer.weight_codes().cpu().double()
        ref_codes = O.quant_codes(w, q.quant_type, q.d_wt, q.q_m_wt, q.t_wt)
        st = tie_check(w, wg, ref_codes.double(), q.quant_type, q.d_wt, q.q_m_wt, q.t_wt)
        res[name + " weight codes"] = ("codes", st["flips"] / st["total"], st["non_ties"])
        out = q.d_act * q.d_wt * (a_codes.double() @ wg.t())
        return out + layer.bias.detach().cpu().double() if layer.bias is not None else out

    h1 = O._layer_norm(x, sd, pre + ".norm1")
    qkv = O._qlin(h1, sd, pre + ".attn.qkv", cfg)
    q_, k_, v_ = qkv.reshape(B, N, 3, -1, cfg.hd()).permute(2, 0, 3, 1, 4)
    ao = (((q_ @ k_.transpose(-2, -1)) * cfg.hd() ** -0.5).softmax(-1) @ v_).transpose(1, 2).reshape(B, N, -1)
    x1 = x + O._qlin(ao, sd, pre + ".attn.proj", cfg)
    h2 = O._layer_norm(x1, sd, pre + ".norm2")
    g1 = F.gelu(O._qlin(h2, sd, pre + ".mlp.fc1", cfg))
    x2 = x1 + O._qlin(g1, sd, pre + ".mlp.fc2", cfg)

    pq, pp, p1, p2 = (blk.attn.qkv.quant_plan(), blk.attn.proj.quant_plan(), blk.mlp.fc1.quant_plan(),
                      blk.mlp.fc2.quant_plan())
    c = torch.empty((M, pq.kpad), dtype=torch.int8, device=dev)
    _lib.layernorm_quant_i8(x.to(dev).reshape(M, C).contiguous(), blk.norm1.weight, blk.norm1.bias, blk.norm1.eps,
                            pq.qtype, pq.d_act, pq.qm_act, pq.t_act, 0, c, pq.kpad,
                            code_table=epilogue_table(pq, _lib.EPI_I8))
    cmp_codes("norm1 codes", c[:, :C], h1, "attn.qkv")
    want_c = ocodes(h1, "attn.qkv").to(torch.int8)
    c = torch.zeros((M, pq.kpad), dtype=torch.int8, device=dev)
    c[:, :C] = want_c.to(dev)
    g_qkv = blk.attn.qkv.gemm_codes(c, pq, _lib.EPI_F32)[:, :pq.n]
    res["qkv"] = ("fp32", rel(g_qkv, gemm_ref("attn.qkv", blk.attn.qkv, want_c)))
    a = blk.attn
    fused = (N <= _lib.QKV_ATT_MAX_N and pq.wfmt == _lib.W4 and pq.kpad % 256 == 0
             and a.num_heads * 64 <= _lib.QKV_ATT_MAX_C and a.split_ok(pq))
    if fused:
        # the production kernel: qkv projection + attention + proj's quantizer on the oracle's LN codes
        ca = torch.zeros((M, pp.kpad), dtype=torch.int8, device=dev)
        _lib.qkv_attention(c, B, N, pq.kpad, pq.packed_codes(), pq.npad, pq.d_act, pq.d_wt, pq.bias_pad, a.num_heads,
                           a.scale, ca, _lib.ATT_I8, vit_model.attention_in_scale(pq), pp.qtype, pp.d_act, pp.qm_act,
                           pp.t_act, epi_table=epilogue_table(pp, _lib.EPI_I8))
        cmp_codes("fused qkv+attention codes", ca[:, :C], ao, "attn.proj")
    elif a.split_ok(pq):
        # the production path beyond 208 tokens: qkv GEMM -> fp16 hi/lo head planes -> streaming attention
        s_in = vit_model.attention_in_scale(pq)
        hi = torch.empty(M * pq.n, dtype=torch.float16, device=dev)
        lo = torch.empty_like(hi)
        _lib.gemm_qkv_split(c, M, pq.kpad, pq.packed_codes(), pq.wfmt, pq.n, pq.npad, pq.d_act, pq.d_wt, pq.bias_pad, N,
                            s_in, hi, lo)
        ca = torch.zeros((M, pp.kpad), dtype=torch.int8, device=dev)
        _lib.attention_split(hi, lo, B, N, a.num_heads, 64, a.scale, ca, _lib.ATT_I8, s_in, pp.qtype, pp.d_act,
                             pp.qm_act, pp.t_act, epi_table=epilogue_table(pp, _lib.EPI_I8))
        cmp_codes("split qkv -> attention codes", ca[:, :C], ao, "attn.proj")
    ca = torch.zeros((M, pp.kpad), dtype=torch.int8, device=dev)
    blk.attn.core_hip(qkv.reshape(M, -1).to(dev).contiguous(), B, N, ca, _lib.ATT_I8, 1.0, pp)
    cmp_codes("attention codes", ca[:, :C], ao, "attn.proj")
    ca = torch.zeros((M, pp.kpad), dtype=torch.int8, device=dev)
    want_a = ocodes(ao, "attn.proj").to(torch.int8)
    ca[:, :C] = want_a.to(dev)
    xr = x.to(dev).reshape(M, C).contiguous().clone()
    blk.attn.proj.gemm_codes(ca, pp, _lib.EPI_F32_RESID, out=xr)
    res["x + proj"] = ("fp32", rel(xr, x.reshape(M, C).double() + gemm_ref("attn.proj", blk.attn.proj, want_a)))
    c2 = torch.empty((M, p1.kpad), dtype=torch.int8, device=dev)
    _lib.layernorm_quant_i8(x1.to(dev).reshape(M, C).contiguous(), blk.norm2.weight, blk.norm2.bias,
                            blk.norm2.eps, p1.qtype, p1.d_act, p1.qm_act, p1.t_act, 0, c2, p1.kpad,
                            code_table=epilogue_table(p1, _lib.EPI_I8))
    cmp_codes("norm2 codes", c2[:, :C], h2, "mlp.fc1")
    c2 = torch.zeros((M, p1.kpad), dtype=torch.int8, device=dev)
    c2[:, :C] = ocodes(h2, "mlp.fc1").to(torch.int8).to(dev)
    hid = torch.zeros((M, p2.kpad), dtype=torch.int8, device=dev)
    blk.mlp.fc1.gemm_codes(c2, p1, _lib.EPI_I8_GELU, out=hid, next_layer=blk.mlp.fc2)
    cmp_codes("fc1+gelu codes", hid[:, :p1.n], g1, "mlp.fc2")
    hid = torch.zeros((M, p2.kpad), dtype=torch.int8, device=dev)
    want_g = ocodes(g1, "mlp.fc2").to(torch.int8)
    hid[:, :p1.n] = want_g.to(dev)
    xr2 = x1.to(dev).reshape(M, C).contiguous().clone()
    blk.mlp.fc2.gemm_codes(hid, p2, _lib.EPI_F32_RESID, out=xr2)
    res["x1 + fc2"] = ("fp32", rel(xr2, x1.reshape(M, C).double() + gemm_ref("mlp.fc2", blk.mlp.fc2, want_g)))
    gemm_ref("mlp.fc1", blk.mlp.fc1, c2[:, :C].cpu())   # records fc1's weight-code stage
    return res


def assert_stages(res, i, weights_loaded, act_budget=1e-4, w_budget=1e-5):
    for name, r in res.items():
        if r[0] == "fp32":
            assert r[1] <= 1e-6, (i, name, r)
        else:
            assert r[2] == 0, (i, name, "non-tie code differences", r)       # every flip is a proven tie
            if "weight" in name:
                assert r[1] == 0 if weights_loaded else r[1] <= w_budget, (i, name, r)
            else:
                assert r[1] <= act_budget, (i, name, r)


def test_vit_base_b2_vs_oracle(dev):
    """ViT-B on identical int4 weights (the reference's own quantize_weight codes, bound with
    load_weight_codes). Stage forcing: every kernel of every block on the oracle's input — fp32 stages
    within 1e-6 of an fp64 product of the same codes, activation codes identical except proven rounding
    ties (<= 1e-4 of them). End to end: the full GPU forward's quantizer boundaries are laid beside the
    oracle's, every differing code must be a proven tie, and with the ties resolved alike the logits
    agree within TIE_E2E (north star: 1e-3)."""
    from parity_tools import load_oracle_weight_codes, tie_resolved_vit_check
    model = build_quantized_vit("vit_base_patch16_224", seed=0).to(dev)
    cfg = O.ViTConfig()
    assert load_oracle_weight_codes(model, cfg) == 4 * cfg.depth + 2
    img = synthetic_images(2, 224, seed=5)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    trace = []
    with torch.no_grad():
        O.vit_forward(sd, cfg, img, trace=trace)
        for i in range(cfg.depth):
            assert_stages(stage_forced_block(model, cfg, sd, trace[i], i, dev), i, weights_loaded=True)
    r = tie_resolved_vit_check(model, cfg, img, dev)
    print(f"ViT-B b2 tie-resolved: rel {r['rel']:.2e}, {r['flips']} tie flips of {r['codes']} codes")
    assert not r["missing"] and not r["bad"], (r["missing"], r["bad"])
    assert r["rel"] <= TIE_E2E, r["rel"]


# logits agreement once ties are resolved alike: fp32 rounding only (measured ~1e-6 on ViT-B)
TIE_E2E = 2e-5


@pytest.mark.parametrize("name,cfg_kw,batch,qt,t_act", [
    ("vit_tiny_patch16_224", dict(embed_dim=192, depth=12, num_heads=3), 8, QuantizationType.SYMMETRIC_NONLINEAR, 0.9),
    ("vit_tiny_patch16_224", dict(embed_dim=192, depth=12, num_heads=3), 4, QuantizationType.SYMMETRIC_LINEAR, 1.0),
    ("vit_base_patch16_224", dict(), 4, QuantizationType.SYMMETRIC_NONLINEAR, 1.0),
])
def test_vit_tie_resolved_end_to_end(dev, name, cfg_kw, batch, qt, t_act):
    """End-to-end logits on identical int4 weights, ties resolved alike (see parity_tools)."""
    from parity_tools import load_oracle_weight_codes, tie_resolved_vit_check
    model = build_quantized_vit(name, seed=11, quant_type=qt, t_act=t_act).to(dev)
    cfg = O.ViTConfig(quant_type=qt.value, **cfg_kw)
    load_oracle_weight_codes(model, cfg)
    r = tie_resolved_vit_check(model, cfg, synthetic_images(batch, 224, seed=3), dev)
    print(f"{name} b{batch} {qt.value} t_act={t_act}: rel {r['rel']:.2e}, {r['flips']} tie flips of {r['codes']}")
    assert not r["missing"] and not r["bad"], (r["missing"], r["bad"])
    assert r["rel"] <= TIE_E2E, r["rel"]


def test_device_weight_codes_vs_reference(dev):
    """The device's own weight quantizer (no codes loaded) against the reference's quantize_weight on every
    ViT-B layer: identical except proven rounding ties of exp(t log|w|) (torch's CPU exp/log are MKL VML
    results, not correctly rounded; the device rounds correctly), <= 1e-5 of the codes."""
    from parity_tools import oracle_weight_codes, tie_check
    model = build_quantized_vit("vit_base_patch16_224", seed=0).to(dev)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    flips = total = 0
    for name, m in model.named_modules():
        if isinstance(m, (QuantizeLinear, QuantizeConv2d)):
            q = O.LayerQ.from_state(sd, name + ".", m.quant_type.value, m.quant_mode.value)
            w = sd[name + ".weight"]
            st = tie_check(w, m.weight_codes().cpu().reshape(w.shape), oracle_weight_codes(
                sd, name, m.quant_type.value, m.quant_mode.value).float(), q.quant_type, q.d_wt, q.q_m_wt, q.t_wt)
            assert st["non_ties"] == 0, (name, st)
            flips += st["flips"]
            total += st["total"]
    print(f"device weight codes: {flips} tie flips of {total}")
    assert flips <= 1e-5 * total


def test_pruned_shapes_vs_oracle(dev):
    """Compressed checkpoints prune whole heads (qkv N = 3*h'*64) and arbitrary MLP neurons
    (operator.py:1208-1246, pruning_compression.py:64-131,217-291)."""
    torch.manual_seed(9)
    m = vit_model.VisionTransformer(embed_dim=192, depth=2, num_heads=3, num_classes=37)
    for blk in m.blocks:   # prune to 2 heads and 500 hidden neurons
        a = blk.attn
        a.qkv = nn.Linear(192, 3 * 2 * 64)
        a.num_heads = 2
        a.proj = nn.Linear(128, 192)
        blk.mlp.fc1 = nn.Linear(192, 500)
        blk.mlp.fc2 = nn.Linear(500, 192)
    from quantized_vit_amd.calibrate import collect_input_absmax, set_activation_quant
    from quantized_vit_amd.quant_model import model_to_quantize_model
    m.eval()
    img = synthetic_images(2, 224, seed=1)
    absmax = collect_input_absmax(m, img)
    m = model_to_quantize_model(m, num_bits=4, quant_mode="weight_and_activation")
    set_activation_quant(m, absmax)
    m = m.to(dev)
    with torch.no_grad():
        y = m(img.to(dev))
    cfg = O.ViTConfig(embed_dim=192, depth=2, num_heads=3, num_classes=37)
    check_vit_parity(m, cfg, img, dev)


def test_vit_large_384_stage_forced(dev):
    """BASELINE config 4 (ViT-L/16 @384: 577 tokens, embed 1024, 16 heads): the sequence is longer than
    the fused qkv+attention kernel holds, so the blocks take the split-operand path (qkv GEMM to fp16
    hi/lo head planes + the streaming attention kernel). Two blocks on identical int4 weights, stage by
    stage against the oracle (bars as for ViT-B), then the tie-resolved end-to-end logits."""
    from parity_tools import load_oracle_weight_codes, tie_resolved_vit_check
    model = build_quantized_vit("vit_large_patch16_384", seed=0, depth=2).to(dev)
    cfg = O.ViTConfig(img_size=384, embed_dim=1024, depth=2, num_heads=16)
    load_oracle_weight_codes(model, cfg)
    img = synthetic_images(1, 384, seed=5)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    trace = []
    with torch.no_grad():
        O.vit_forward(sd, cfg, img, trace=trace)
        assert trace[0].shape[1] == 577
        for i in range(cfg.depth):
            res = stage_forced_block(model, cfg, sd, trace[i], i, dev)
            assert "split qkv -> attention codes" in res
            assert_stages(res, i, weights_loaded=True)
    r = tie_resolved_vit_check(model, cfg, img, dev)
    assert not r["missing"] and not r["bad"], (r["missing"], r["bad"])
    assert r["rel"] <= TIE_E2E, r["rel"]
