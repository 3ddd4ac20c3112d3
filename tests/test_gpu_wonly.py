"""Weight-only QuantizeLinear (the reference's default quant_mode, quant_model.py:23) on the hand-written
qvit_gemm_wonly: fp32 activations against the packed int4 / int8 weight codes.

Reference: quant_layers.py:495-499 — quantize_act is the identity outside WEIGHT_AND_ACTIVATION (:356-358), so
forward = F.linear(x, quantize_weight(W), b) with W's fake-quant values d_w k.

Bar: the kernel is an fp32 GEMM of x and the integer codes (x split into three exact bf16 terms, exact products,
fp32 accumulation), so every output must lie within a normal fp32-GEMM error of the fp64 value:
|y - y64| <= 1e-5 (|x| |d_w k|^T + |b|) elementwise — 1e-5 relative to the sum of the terms' magnitudes, about
40x the typical fp32 accumulation error at K = 3072.
"""
import pytest
import torch
import torch.nn as nn

from oracle import quant_oracle as O
from quantized_vit_amd import _lib
from quantized_vit_amd.quant_layers import QuantizationMode, QuantizationType, QuantizeLinear
from test_gpu_kernels import _p, pack_codes

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _check_close(y, x, codes, d_w, bias):
    """y (device fp32) against the fp64 value, elementwise within TOL of the terms' magnitudes."""
    xd, wd = x.double(), (d_w * codes.double())
    ref = xd @ wd.t() + (bias.double() if bias is not None else 0.0)
    mag = xd.abs() @ wd.abs().t() + (bias.double().abs() if bias is not None else 0.0)
    err = (y.double() - ref).abs()
    bad = err > TOL * mag + 1e-30
    assert not bad.any(), (f"{int(bad.sum())} outputs off, worst rel {float((err / (mag + 1e-30)).max()):.3g} "
                           f"at {bad.nonzero()[0].tolist()}")
    return float((err / (mag + 1e-30)).max())


def _run(dev, x, codes, wfmt, d_w, bias):
    M, K = x.shape
    N = codes.shape[0]
    packed, npad, kpad = pack_codes(codes, wfmt, dev)
    xp = torch.zeros((M, kpad), dtype=torch.float32, device=dev)
    xp[:, :K] = x
    ldy = (N + 3) // 4 * 4
    y = torch.full((M, ldy), float("nan"), device=dev)
    bias_pad = _lib.pad_bias(bias, N, npad, dev) if bias is not None else None
    _lib.gemm_wonly(xp, M, kpad, packed, wfmt, N, npad, _p(d_w, dev), bias_pad, y)
    torch.cuda.synchronize()
    return y[:, :N]


@pytest.mark.parametrize("wfmt", [_lib.W4, _lib.W8])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (5, 32, 64), (64, 256, 128), (77, 300, 768), (300, 768, 3072),
                                   (129, 2304, 768), (1000, 100, 1000)])
def test_gemm_wonly_vs_fp64(dev, wfmt, M, N, K):
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K + wfmt)
    lim = 8 if wfmt == _lib.W4 else 128
    codes = torch.randint(-lim, lim, (N, K), generator=g)
    if wfmt == _lib.W8:
        codes = codes.clamp(-127, 127)
    x = (torch.randn(M, K, generator=g) * 3).to(dev)
    bias = (torch.randn(N, generator=g) * 0.1).to(dev)
    y = _run(dev, x, codes.to(dev), wfmt, 0.0123, bias)
    assert torch.isfinite(y).all()
    _check_close(y, x, codes.to(dev), 0.0123, bias)


@pytest.mark.parametrize("scale", [1e-30, 1e-6, 1e6, 1e30])
def test_gemm_wonly_exponent_range(dev, scale):
    """fp32 operands far from 1: the bf16 split keeps fp32's exponent range (no fp16-style underflow)."""
    g = torch.Generator().manual_seed(11)
    M, N, K = 96, 256, 256
    codes = torch.randint(-8, 8, (N, K), generator=g)
    x = (torch.randn(M, K, generator=g) * scale).to(dev)
    y = _run(dev, x, codes.to(dev), _lib.W4, 0.5, None)
    _check_close(y, x, codes.to(dev), 0.5, None)


@pytest.mark.parametrize("wfmt", [_lib.W4, _lib.W8])
@pytest.mark.parametrize("M,N,K", [(1, 768, 3072), (197, 768, 3072), (197, 2304, 768), (50, 300, 1000)])
def test_gemm_wonly_split_k(dev, wfmt, M, N, K):
    """Small M (one image, one token): the K range split over several workgroups per tile, the partials summed
    in a fixed order — within the bar, deterministic, and close to the unsplit launch."""
    g = torch.Generator().manual_seed(M * N + K)
    lim = 8 if wfmt == _lib.W4 else 127
    codes = torch.randint(-lim, lim, (N, K), generator=g).to(dev)
    x = torch.randn(M, K, generator=g).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    packed, npad, kpad = pack_codes(codes.cpu(), wfmt, dev)
    xp = torch.zeros((M, kpad), device=dev)
    xp[:, :K] = x
    bias_pad = _lib.pad_bias(bias, N, npad, dev)
    outs = []
    for split in (True, True, False):
        y = torch.full((M, (N + 3) // 4 * 4), float("nan"), device=dev)
        _lib.gemm_wonly(xp, M, kpad, packed, wfmt, N, npad, _p(0.02, dev), bias_pad, y, split=split)
        torch.cuda.synchronize()
        outs.append(y[:, :N].clone())
    assert torch.equal(outs[0], outs[1]), "split-K result must be deterministic"
    for y in outs:
        _check_close(y, x, codes, 0.02, bias)


@pytest.mark.parametrize("lim", [32639, 32768, 5000000])
@pytest.mark.parametrize("M,N,K", [(1, 40, 96), (77, 300, 768), (197, 768, 3072), (700, 512, 256)])
def test_gemm_wonly_wide_vs_fp64(dev, M, N, K, lim):
    """Codes beyond int8 as balanced base-256 digits: W16 (|k| <= 32639) and W24 (the 16-bit saturation code
    32768 and wider), including the extreme codes and the digit boundaries."""
    g = torch.Generator().manual_seed(M + N + K + lim)
    codes = torch.randint(-lim, lim + 1, (N, K), generator=g).float()
    codes.view(-1)[:8] = torch.tensor([lim, -lim, 127., 128., -128., -129., 255., -1.])
    codes = codes.to(dev)
    x = torch.randn(M, K, generator=g).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    npad, kpad = (N + 255) // 256 * 256, (K + 127) // 128 * 128
    packed, wfmt = _lib.pack_weight_wide(codes, npad, kpad)
    assert wfmt == (_lib.W16 if lim <= 32639 else _lib.W24)
    xp = torch.zeros((M, kpad), device=dev)
    xp[:, :K] = x
    for split in (True, False):
        y = torch.full((M, (N + 3) // 4 * 4), float("nan"), device=dev)
        _lib.gemm_wonly(xp, M, kpad, packed, wfmt, N, npad, _p(3e-5, dev), _lib.pad_bias(bias, N, npad, dev), y,
                        split=split)
        torch.cuda.synchronize()
        _check_close(y[:, :N], x, codes, 3e-5, bias)


@pytest.mark.parametrize("mode", [QuantizationMode.WEIGHT_ONLY, QuantizationMode.WEIGHT_AND_ACTIVATION])
@pytest.mark.parametrize("qt", [QuantizationType.SYMMETRIC_NONLINEAR, QuantizationType.SYMMETRIC_LINEAR])
def test_default_16bit_linear_vs_oracle(dev, qt, mode):
    """model_to_quantize_model's defaults (num_bits = 16, quant_model.py:21-23): 32767 levels per side run
    qvit_gemm_wonly on W16 codes (W+A: the activations fake-quantized to fp32 first) and match the oracle's fp32
    fake-quant F.linear."""
    torch.manual_seed(16)
    q = QuantizeLinear.from_module(nn.Linear(768, 200), quant_type=qt, quant_mode=mode, num_bits=16).to(dev).eval()
    plan = q.quant_plan()
    assert plan.extra.get("wonly") and plan.wfmt in (_lib.W16, _lib.W24) and not plan.int_path
    x = torch.randn(2, 30, 768)
    with torch.no_grad():
        y = q(x.to(dev))
    sd = {k: v.detach().cpu() for k, v in q.state_dict().items()}
    lq = O.LayerQ.from_state(sd, "", q.quant_type.value, q.quant_mode.value)
    ref = O.quantize_linear(x, sd["weight"], sd["bias"], lq)
    xq = O.qact(x, lq) if mode == QuantizationMode.WEIGHT_AND_ACTIVATION else x
    mag = xq.reshape(-1, 768).abs().double() @ O.qweight(sd["weight"], lq).abs().double().t() + sd["bias"].abs().double()
    err = (y.cpu().reshape(-1, 200).double() - ref.reshape(-1, 200).double()).abs()
    assert (err <= 2 * TOL * mag).all(), float((err / mag).max())


def test_gemm_wonly_production_size(dev):
    """The ViT-B/16 b256 fc1 shape (M = 50 432) in weight-only mode: many tiles per XCD range, the fp64
    reference on the device."""
    g = torch.Generator().manual_seed(5)
    M, N, K = 256 * 197, 3072, 768
    codes = torch.randint(-8, 8, (N, K), generator=g).to(dev)
    x = torch.randn(M, K, generator=g).to(dev)
    bias = (torch.randn(N, generator=g) * 0.1).to(dev)
    y = _run(dev, x, codes, _lib.W4, 0.01, bias)
    _check_close(y, x, codes, 0.01, bias)


def test_gemm_wonly_argument_validation(dev):
    x = torch.zeros((4, 128), device=dev)
    codes = torch.zeros((8, 128), dtype=torch.int64)
    packed, npad, kpad = pack_codes(codes, _lib.W4, dev)
    y = torch.zeros((4, 8), device=dev)
    with pytest.raises(_lib.QvitError):  # K not a multiple of QVIT_TILE_K
        _lib.gemm_wonly(x, 4, 64, packed, _lib.W4, 8, npad, _p(1.0, dev), None, y)
    with pytest.raises(_lib.QvitError):  # bad weight format
        _lib.gemm_wonly(x, 4, 128, packed, 5, 8, npad, _p(1.0, dev), None, y)
    with pytest.raises(_lib.QvitError):  # misaligned output
        _lib.gemm_wonly(x, 4, 128, packed, _lib.W4, 8, npad, _p(1.0, dev), None, torch.zeros(40, device=dev)[1:33].view(4, 8))


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("qt", [QuantizationType.SYMMETRIC_NONLINEAR, QuantizationType.SYMMETRIC_LINEAR])
def test_weight_only_linear_vs_oracle(dev, bits, qt):
    """QuantizeLinear.from_module in the default WEIGHT_ONLY mode takes qvit_gemm_wonly (4-bit -> int4
    codes, 8-bit -> int8) and matches the oracle's fp32 fake-quant forward (quant_layers.py:495-499)."""
    torch.manual_seed(bits)
    lin = nn.Linear(768, 300)
    q = QuantizeLinear.from_module(lin, quant_type=qt, quant_mode=QuantizationMode.WEIGHT_ONLY,
                                   num_bits=bits).to(dev).eval()
    plan = q.quant_plan()
    assert plan.extra.get("wonly") and not plan.int_path
    assert plan.wfmt == (_lib.W4 if bits == 4 else _lib.W8)
    x = torch.randn(3, 50, 768)
    with torch.no_grad():
        y = q(x.to(dev))
    assert y.shape == (3, 50, 300)
    sd = {k: v.detach().cpu() for k, v in q.state_dict().items()}
    lq = O.LayerQ.from_state(sd, "", q.quant_type.value, q.quant_mode.value)
    # the codes the kernel runs are the oracle's quantize_weight codes (nonlinear: ulp-level exp/log ties aside,
    # each off by one)
    codes = q.weight_codes()
    own = O.quant_codes(sd["weight"], lq.quant_type, lq.d_wt, lq.q_m_wt, lq.t_wt)
    dc = (codes.cpu() - own).abs()
    assert dc.max().item() <= 1 and (dc > 0).float().mean().item() <= 1e-4
    # and the layer is F.linear(x, d_w k, b) to fp32-GEMM accuracy
    d_w = float(q.d_quant_wt.detach().reshape(-1)[0])
    _check_close(y.reshape(-1, 300), x.reshape(-1, 768).to(dev), codes, d_w, q.bias.detach())
    # against the oracle's own forward (fp32 F.linear on its fake-quant weight) where the codes agree
    if not (dc > 0).any():
        ref = O.quantize_linear(x, sd["weight"], sd["bias"], lq)
        xd, wd = x.reshape(-1, 768).double(), (d_w * own).double()
        mag = xd.abs() @ wd.abs().t() + sd["bias"].double().abs()
        err = (y.cpu().reshape(-1, 300).double() - ref.reshape(-1, 300).double()).abs()
        assert (err <= 2 * TOL * mag).all(), float((err / mag).max())


def test_weight_only_bound_codes(dev):
    """Codes bound with load_weight_codes are the ones the weight-only kernel runs."""
    torch.manual_seed(4)
    q = QuantizeLinear.from_module(nn.Linear(256, 130), quant_type=QuantizationType.SYMMETRIC_NONLINEAR,
                                   quant_mode=QuantizationMode.WEIGHT_ONLY, num_bits=4).to(dev).eval()
    codes = torch.randint(-7, 8, (130, 256))
    q.load_weight_codes(codes)
    x = torch.randn(17, 256, device=dev)
    with torch.no_grad():
        y = q(x)
    assert q.quant_plan().extra.get("wonly")
    d_w = float(q.d_quant_wt.detach().reshape(-1)[0])
    _check_close(y, x, codes.to(dev), d_w, q.bias.detach())


@pytest.mark.parametrize("bits", [4, 16])
@pytest.mark.parametrize("cfg", [dict(cin=3, cout=768, k=16, s=16, p=0, H=224), dict(cin=16, cout=40, k=3, s=2, p=1, H=15)])
def test_weight_only_conv2d_vs_oracle(dev, cfg, bits):
    """QuantizeConv2d in WEIGHT_ONLY mode (the patch embedding and a padded strided conv): the input patches as
    fp32 rows against the packed codes on qvit_gemm_wonly, vs the oracle's fp32 F.conv2d on the fake-quant weight
    (quant_layers.py:575-587)."""
    import torch.nn.functional as F
    from quantized_vit_amd.quant_layers import QuantizeConv2d
    torch.manual_seed(bits + cfg["k"])
    conv = nn.Conv2d(cfg["cin"], cfg["cout"], cfg["k"], stride=cfg["s"], padding=cfg["p"], bias=True)
    q = QuantizeConv2d.from_module(conv, quant_type=QuantizationType.SYMMETRIC_NONLINEAR,
                                   quant_mode=QuantizationMode.WEIGHT_ONLY, num_bits=bits).to(dev).eval()
    assert q.quant_plan().extra.get("wonly")
    x = torch.randn(2, cfg["cin"], cfg["H"], cfg["H"])
    with torch.no_grad():
        y = q(x.to(dev))
    sd = {k: v.detach().cpu() for k, v in q.state_dict().items()}
    lq = O.LayerQ.from_state(sd, "", q.quant_type.value, q.quant_mode.value)
    ref = O.quantize_conv2d(x, sd["weight"], sd["bias"], lq, stride=cfg["s"], padding=cfg["p"])
    assert y.shape == ref.shape and y.is_contiguous()
    mag = F.conv2d(x.abs().double(), O.qweight(sd["weight"], lq).abs().double(), sd["bias"].abs().double(),
                   stride=cfg["s"], padding=cfg["p"])
    err = (y.cpu().double() - ref.double()).abs()
    assert (err <= 2 * TOL * mag).all(), float((err / mag).max())
