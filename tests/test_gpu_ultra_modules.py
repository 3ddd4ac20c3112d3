"""The weight-only convolution (qvit_conv_wonly) and UltraNet's module surface on it: Conv2d_Q.forward
(reference `4-bit quantization/quant_ultra.py:85-89`) and Linear_Q.forward (:210-222), plus the weight-only
QuantizeConv2d.forward (quant_layers.py:575-587) that shares the kernel.

Bars: the kernel against F.conv2d in fp64 on the same fp32 operands, elementwise within
4 K 2^-24 (|x| * |w|) (fp32 accumulation of K terms, the reference's own fp32 conv has the same
error order); the modules against the oracle's fp32 CPU conv on the oracle's fake-quant weight within the same
elementwise bound plus one weight quantum where the GPU's tanh rounds a weight code to the other side of a
tie (<= 1e-4 of codes, checked separately in test_gpu_ultranet.py); at 416 x 416 for the UltraNet shapes.
"""
import pytest
import torch
import torch.nn.functional as F

from oracle import ultranet_oracle as U
from quantized_vit_amd import _lib
from quantized_vit_amd.quant_ultra import conv2d_Q_fn, linear_Q_fn, weight_quantize_fn

pytestmark = pytest.mark.gpu


def _pack(codes: torch.Tensor, wfmt: int, dev):
    n, k = codes.shape
    npad, kpad = (n + 255) // 256 * 256, (k + 127) // 128 * 128
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    packed = _lib.pack_weight(codes.float().contiguous().to(dev), _lib.QT_LINEAR, torch.ones(1, device=dev),
                              torch.full((1,), 1024.0, device=dev), None, wfmt, npad, kpad, ovf)
    assert int(ovf.item()) == 0
    return packed, npad, kpad


def _assert_conv_close(got, x, w, bias, stride, padding, dilation, slack_w=None):
    """got vs fp64 F.conv2d(x, w) elementwise within 4 K 2^-24 (|x| conv |w|) (+ slack_w (|x| conv 1) when
    weight codes may differ by one quantum)."""
    x64, w64 = x.double().cpu(), w.double().cpu()
    b64 = None if bias is None else bias.double().cpu()
    ref = F.conv2d(x64, w64, b64, stride, padding, dilation)
    mag = F.conv2d(x64.abs(), w64.abs(), None if b64 is None else b64.abs(), stride, padding, dilation)
    K = w.shape[1] * w.shape[2] * w.shape[3]
    tol = 4 * K * 2.0 ** -24 * mag + 1e-30
    if slack_w is not None:
        tol = tol + slack_w * F.conv2d(x64.abs(), torch.ones_like(w64), None, stride, padding, dilation)
    g = got.double().cpu()
    assert g.shape == ref.shape, (g.shape, ref.shape)
    err = (g - ref).abs()
    worst = (err / tol).max().item()
    assert worst <= 1.0, worst
    return ref, tol


# (B, C, H, W, N, kh, kw, stride, padding, dilation, wfmt)
GEOMETRIES = [
    (2, 3, 37, 29, 16, 3, 3, (1, 1), (1, 1), (1, 1), _lib.W4),      # UltraNet conv0 shape, odd sizes
    (2, 16, 30, 26, 32, 3, 3, (2, 2), (1, 1), (1, 1), _lib.W4),     # stride 2
    (1, 8, 21, 23, 36, 3, 5, (1, 2), (1, 2), (2, 1), _lib.W8),      # kh != kw, dilation, asymmetric padding
    (3, 64, 13, 13, 36, 1, 1, (1, 1), (0, 0), (1, 1), _lib.W4),     # the head's 1 x 1 (36 outputs)
    (2, 3, 64, 64, 300, 16, 16, (16, 16), (0, 0), (1, 1), _lib.W4),  # patch embedding, N > 256
    (1, 5, 7, 7, 9, 3, 3, (1, 1), (3, 3), (1, 1), _lib.W8),         # padding > kernel reach, split-K path
    (4, 64, 52, 52, 64, 3, 3, (1, 1), (1, 1), (1, 1), _lib.W4),     # UltraNet block 3 shape, no split
    (1, 5, 7, 7, 80, 3, 3, (1, 1), (2, 2), (1, 1), _lib.W8),        # N > 64: the wide schedule's split-K path
    (2, 64, 20, 18, 64, 3, 3, (1, 1), (1, 1), (1, 1), _lib.W8),     # int8 panel past 24 KiB: the wide schedule
]


@pytest.mark.parametrize("geo", GEOMETRIES, ids=lambda g: "x".join(map(str, g[:7])))
def test_conv_wonly_geometries(dev, geo):
    B, C, H, W, N, kh, kw, stride, padding, dilation, wfmt = geo
    g = torch.Generator().manual_seed(B * 1000 + C * 10 + N)
    lvl = 7 if wfmt == _lib.W4 else 127
    codes = torch.randint(-lvl, lvl + 1, (N, C * kh * kw), generator=g)
    x = torch.randn(B, C, H, W, generator=g)
    bias = torch.randn(N, generator=g) if N % 2 == 0 else None
    d = torch.tensor([0.0371], dtype=torch.float32)
    packed, npad, kpad = _pack(codes, wfmt, dev)
    bias_pad = _lib.pad_bias(None if bias is None else bias.to(dev), N, npad, dev)
    y = _lib.conv_wonly(x.to(dev), (kh, kw), stride, padding, dilation, packed, wfmt, N, npad, kpad, d.to(dev),
                        bias_pad)
    w = (codes.double() * d.double()).view(N, C, kh, kw)
    _assert_conv_close(y, x, w, bias, stride, padding, dilation)


NARROW = [g for g in GEOMETRIES if g[4] <= 64] + [
    (3, 40, 19, 17, 1, 3, 3, (1, 1), (1, 1), (1, 1), _lib.W4),      # one output channel, 6 stages
    (2, 7, 25, 25, 48, 5, 5, (2, 1), (2, 2), (1, 1), _lib.W4),      # 3 feature tiles, ragged last stage
]


@pytest.mark.parametrize("geo", NARROW, ids=lambda g: "x".join(map(str, g[:7])) + f"w{g[10]}")
def test_conv_wonly_narrow_equals_wide(dev, geo):
    """The narrow schedule (N <= 64: LDS-resident weights, lane-per-pixel gather) gives the wide schedule's values
    bit for bit: the same MFMAs on the same operands in the same order per accumulator (the wide schedule without
    its split-K path, whose partial sums are added in another order)."""
    B, C, H, W, N, kh, kw, stride, padding, dilation, wfmt = geo
    g = torch.Generator().manual_seed(B * 7 + C * 3 + N)
    lvl = 7 if wfmt == _lib.W4 else 127
    codes = torch.randint(-lvl, lvl + 1, (N, C * kh * kw), generator=g)
    x = torch.randn(B, C, H, W, generator=g).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    d = torch.tensor([0.0213], device=dev)
    packed, npad, kpad = _pack(codes, wfmt, dev)
    bias_pad = _lib.pad_bias(bias, N, npad, dev)
    fits = _lib.narrow_conv_fits(wfmt, N, C * kh * kw)
    outs = []
    prev = _lib.conv_wonly_narrow(1)
    try:
        for on in (1, 0):
            _lib.conv_wonly_narrow(on)
            outs.append(_lib.conv_wonly(x, (kh, kw), stride, padding, dilation, packed, wfmt, N, npad, kpad, d,
                                        bias_pad, split=False).cpu())
    finally:
        _lib.conv_wonly_narrow(prev)
    panel = (C * kh * kw + 63) // 64 * 16 * ((N + 15) // 16) * (32 if wfmt == _lib.W4 else 64)
    assert fits == (panel <= 24 * 1024 and (C * kh * kw + 63) // 64 * 64 <= 1024)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("geo", [NARROW[0], NARROW[1], NARROW[-1], GEOMETRIES[6]], ids=lambda g: "x".join(map(str, g[:7])))
@pytest.mark.parametrize("a_bit", [4, 2, 7])
def test_conv_wonly_bn_act_equals_composed(dev, geo, a_bit):
    """qvit_conv_wonly_bn_act = the conv, then fma(y, alpha, shift) with the ultra_bn_fold coefficients, then the
    activation quantizer's values (qvit_fake_quant_f32). The composed reference takes z = y alpha + shift from
    fp64 (exact) rounded once to fp32, i.e. the FMA's value except when the fp64 rounding itself lands on an fp32 tie
    (never in practice); the codes must agree exactly."""
    B, C, H, W, N, kh, kw, stride, padding, dilation, wfmt = geo
    g = torch.Generator().manual_seed(N + a_bit)
    lvl = 7 if wfmt == _lib.W4 else 127
    codes = torch.randint(-lvl, lvl + 1, (N, C * kh * kw), generator=g)
    x = (torch.rand(B, C, H, W, generator=g)).to(dev)
    d = torch.tensor([1.0 / 7], device=dev)
    packed, npad, kpad = _pack(codes, wfmt, dev)
    bn = torch.nn.BatchNorm2d(N).eval()
    with torch.no_grad():
        bn.running_mean.copy_(torch.randn(N, generator=g) * 2)
        bn.running_var.copy_(torch.rand(N, generator=g) * 20 + 0.5)
        bn.weight.copy_(torch.rand(N, generator=g) * 0.3 + 0.1)
        bn.bias.copy_(torch.rand(N, generator=g) * 0.4 + 0.3)
    bn = bn.to(dev)
    alpha, shift = _lib.ultra_bn_fold(bn, dev)
    n = 2 ** a_bit - 1
    got = _lib.conv_wonly_bn_act(x, (kh, kw), stride, padding, dilation, packed, wfmt, N, npad, kpad, d, None, alpha,
                                 shift, n)
    assert got is not None
    y = _lib.conv_wonly(x, (kh, kw), stride, padding, dilation, packed, wfmt, N, npad, kpad, d, None)
    z = (y.double() * alpha.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1)).float()
    want = _lib.fake_quant_f32(z.contiguous(), _lib.QT_ULTRA_ACT, None, None, None, n).reshape(z.shape)
    assert torch.equal(got, want)
    assert len(torch.unique(got)) > min(n, 3)


def test_conv2d_q_forward_bn_act_fallbacks(dev):
    """forward_bn_act fuses only eval-mode BN on running statistics and 1..7-bit quantizers, else returns None."""
    from quantized_vit_amd.quant_ultra import activation_quantize_fn
    conv = conv2d_Q_fn(4)(8, 16, kernel_size=3, padding=1, bias=False).to(dev)
    bn = torch.nn.BatchNorm2d(16).to(dev).eval()
    x = torch.rand(1, 8, 12, 12, device=dev)
    with torch.no_grad():
        assert conv.forward_bn_act(x, bn, activation_quantize_fn(4)) is not None
        assert conv.forward_bn_act(x, bn, activation_quantize_fn(8)) is None
        assert conv.forward_bn_act(x, bn.train(), activation_quantize_fn(4)) is None
        wide = conv2d_Q_fn(4)(8, 80, kernel_size=3, padding=1, bias=False).to(dev)
        assert wide.forward_bn_act(x, torch.nn.BatchNorm2d(80).to(dev).eval(), activation_quantize_fn(4)) is None


def test_conv_wonly_non_contiguous_and_rejects(dev):
    g = torch.Generator().manual_seed(5)
    codes = torch.randint(-7, 8, (16, 27), generator=g)
    packed, npad, kpad = _pack(codes, _lib.W4, dev)
    d = torch.tensor([0.05], device=dev)
    xs = torch.randn(2, 20, 20, 3, generator=g).to(dev).permute(0, 3, 1, 2)   # channels-last view
    y = _lib.conv_wonly(xs, (3, 3), (1, 1), (1, 1), (1, 1), packed, _lib.W4, 16, npad, kpad, d, None)
    _assert_conv_close(y, xs.cpu(), codes.double().view(16, 3, 3, 3) * 0.05, None, 1, 1, 1)
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    x = torch.zeros(1, 3, 8, 8, device=dev)
    out = torch.empty(1, 16, 8, 8, device=dev)
    args = lambda **kw: dict(dict(X=x.data_ptr(), B=1, C=3, H=8, W=8, kh=3, kw=3, sh=1, sw=1, ph=1, pw=1, dh=1, dw=1,
                                  Wp=packed.data_ptr(), wfmt=_lib.W4, N=16, npad=npad, K=kpad, d=d.data_ptr(),
                                  bias=0, Y=out.data_ptr(), ws=0, wsb=0, st=s), **kw)
    call = lambda a: lib.qvit_conv_wonly(*a.values())
    assert call(args()) == 0
    assert call(args(K=64)) != 0            # K not a multiple of the K tile
    assert call(args(C=20)) != 0            # K < C kh kw
    assert call(args(H=1, ph=0)) != 0       # kernel larger than the padded input
    assert call(args(npad=100)) != 0        # npad not a multiple of the weight tile
    assert call(args(wfmt=5)) != 0
    assert call(args(Wp=0)) != 0
    torch.cuda.synchronize()


def _oracle_conv_q(x, w, b, stride, padding):
    return U.conv_q(x, w, b, stride, padding)


@pytest.mark.parametrize("shape", [
    # (B, cin, cout, H, ks, pad, bias, input kind) at the UltraNet resolutions
    (2, 3, 16, 416, 3, 1, False, "image"),   # layers.0 on k/255 images, 416 x 416
    (2, 16, 32, 208, 3, 1, False, "codes"),  # layers.4
    (2, 64, 64, 26, 3, 1, False, "codes"),   # layers.16 (after four pools)
    (2, 64, 36, 26, 1, 0, True, "codes"),    # layers.28 (head, with bias)
])
def test_conv2d_q_module_vs_oracle(dev, shape):
    B, cin, cout, H, ks, pad, has_bias, kind = shape
    g = torch.Generator().manual_seed(cin * 100 + cout)
    conv = conv2d_Q_fn(4)(cin, cout, kernel_size=ks, stride=1, padding=pad, bias=has_bias)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.1)
        if has_bias:
            conv.bias.copy_(torch.randn(cout, generator=g) * 0.1)
    conv = conv.to(dev)
    if kind == "image":
        x = torch.randint(0, 256, (B, cin, H, H), generator=g).float() / 255.0
    else:
        x = torch.randint(0, 16, (B, cin, H, H), generator=g).float() / 15.0
    with torch.no_grad():
        y = conv(x.to(dev))
    wq_dev = weight_quantize_fn(4)(conv.weight.detach()).cpu()
    wq_ref = U.weight_quantize(conv.weight.detach().cpu())
    assert ((wq_dev - wq_ref).abs() > 0).float().mean().item() <= 1e-4
    b = conv.bias.detach().cpu() if has_bias else None
    # the kernel's arithmetic against fp64 on the device's fake-quant weight ...
    _assert_conv_close(y, x, wq_dev, b, 1, pad, 1)
    # ... and against the oracle's fp32 conv (the reference's op sequence), one quantum of slack where codes differ
    want = _oracle_conv_q(x, conv.weight.detach().cpu(), b, 1, pad)
    slack = 1.0 / 7 if bool((wq_dev != wq_ref).any()) else None
    _, tol = _assert_conv_close(y, x, wq_ref, b, 1, pad, 1, slack_w=slack)
    # the oracle's own fp32 conv carries the same order of rounding: twice the bound
    assert ((y.double().cpu() - want.double()).abs() <= 2 * tol).all()


def test_conv2d_q_repacks_on_weight_update(dev):
    conv = conv2d_Q_fn(4)(8, 16, kernel_size=3, padding=1, bias=False).to(dev)
    x = torch.rand(1, 8, 12, 12, device=dev)
    with torch.no_grad():
        y0 = conv(x).clone()
        conv.weight.mul_(-1.0)          # in place: the packed codes must follow
        y1 = conv(x)
    assert torch.allclose(y1, -y0, rtol=0, atol=1e-6)


@pytest.mark.parametrize("w_bit", [2, 4, 6, 8])
def test_conv2d_q_bit_widths(dev, w_bit):
    g = torch.Generator().manual_seed(w_bit)
    conv = conv2d_Q_fn(w_bit)(16, 24, kernel_size=3, padding=1, bias=True)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(24, generator=g))
    conv = conv.to(dev)
    x = torch.rand(2, 16, 33, 31, generator=g)
    with torch.no_grad():
        y = conv(x.to(dev))
    wq = weight_quantize_fn(w_bit)(conv.weight.detach()).cpu()
    _assert_conv_close(y, x, wq, conv.bias.detach().cpu(), 1, 1, 1)


@pytest.mark.parametrize("dims", [(7, 64, 36), (300, 200, 513), (1, 1024, 10)])
def test_linear_q_vs_oracle(dev, dims):
    M, fin, fout = dims
    g = torch.Generator().manual_seed(M + fin)
    lin = linear_Q_fn(4)(fin, fout, bias=True)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(fout, fin, generator=g) * 0.1)
        lin.bias.copy_(torch.randn(fout, generator=g) * 0.1)
    lin = lin.to(dev)
    x = torch.randn(M, fin, generator=g)
    with torch.no_grad():
        y = lin(x.to(dev)).cpu().double()
    wq = weight_quantize_fn(4)(lin.weight.detach()).cpu().double()
    ref = x.double() @ wq.T + lin.bias.detach().cpu().double()
    mag = x.double().abs() @ wq.abs().T + lin.bias.detach().cpu().double().abs()
    assert ((y - ref).abs() / (4 * fin * 2.0 ** -24 * mag + 1e-30)).max().item() <= 1.0
    want = F.linear(x, U.weight_quantize(lin.weight.detach().cpu()), lin.bias.detach().cpu())   # oracle op
    assert ((y - want.double()).abs() / (4 * fin * 2.0 ** -24 * mag + 1e-30)).max().item() <= 2.0


def test_ultranet_module_level_forward_vs_oracle(dev):
    """UltraNetQua.forward off the fused path (image side not a multiple of 16): the per-module chain
    Conv2d_Q (qvit_conv_wonly) -> BatchNorm2d -> activation_quantize_fn (HIP) -> MaxPool2d, at 408 x 408,
    against the oracle's forward. Tie flips of the 4-bit activations move downstream codes, so end to end the bar
    is 1e-3 or 2.5 x the reference's own fp64-vs-fp32 distance, as for the fused network."""
    from quantized_vit_amd.ultranet import random_ultranet, synthetic_images_u8
    model = random_ultranet(seed=2, device=dev, calib_batch=2, img_size=408)
    img = synthetic_images_u8(2, 408, seed=9)
    assert not model.fused_ok(img.to(dev))
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        gio, gp = model(img.to(dev))
        io, p = U.ultranet_forward(sd, img)
        io64, p64 = U.ultranet_forward({k: v.double() for k, v in sd.items()}, img.double())

    def rel(a, b):
        a, b = a.double().cpu(), b.double().cpu()
        return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
    for got, want, want64 in ((gio, io, io64), (gp[0], p, p64)):
        assert rel(got, want) <= max(1e-3, 2.5 * rel(want64, want)), (rel(got, want), rel(want64, want))


def test_prepare_packs_before_the_first_forward(dev):
    """prepare() packs the codes up front; the forward then reuses them and gives the same result."""
    from quantized_vit_amd.quant_layers import QuantizationMode, QuantizationType, QuantizeLinear
    g = torch.Generator().manual_seed(21)
    lin = torch.nn.Linear(96, 40)
    q = QuantizeLinear.from_module(lin, quant_type=QuantizationType.SYMMETRIC_NONLINEAR,
                                   quant_mode=QuantizationMode.WEIGHT_ONLY, num_bits=4).to(dev).eval()
    x = torch.randn(5, 96, generator=g).to(dev)
    assert q.prepare() is q and q._qplan is not None
    plan = q._qplan
    with torch.no_grad():
        y = q(x)
    assert q._qplan is plan
    q.invalidate()
    with torch.no_grad():
        assert torch.equal(q(x), y)
    conv = conv2d_Q_fn(4)(8, 16, kernel_size=3, padding=1, bias=False).to(dev)
    assert conv.prepare() is conv and conv._codes.key is not None
    key = conv._codes.key
    with torch.no_grad():
        conv(torch.rand(1, 8, 10, 10, device=dev))
    assert conv._codes.key == key


def test_conv2d_q_invalidate_and_grad(dev):
    """a .data edit is picked up after invalidate() (the packed codes key on the version counter, which
    .data bypasses), and under autograd the module takes the reference's F.conv2d so the input gradient flows."""
    g = torch.Generator().manual_seed(3)
    conv = conv2d_Q_fn(4)(16, 32, kernel_size=3, stride=1, padding=1, bias=False).to(dev)
    x = (torch.randint(0, 16, (1, 16, 20, 20), generator=g).float() / 15.0).to(dev)
    with torch.no_grad():
        y0 = conv(x)
        conv.weight.data.mul_(-1.0)      # bypasses the version counter: the cached codes are now stale ...
        stale = conv(x)
        conv.invalidate()                # ... until invalidated
        y1 = conv(x)
    assert torch.equal(stale, y0)
    torch.testing.assert_close(y1, -y0, rtol=0, atol=1e-5)
    xg = x.clone().requires_grad_(True)
    conv(xg).sum().backward()             # grad mode: F.conv2d on quantize_fn(weight)
    assert xg.grad is not None and xg.grad.abs().sum().item() > 0


def test_forward_modules_keeps_hooks(dev):
    """A forward hook on a BatchNorm2d (hook-based calibration / feature capture) is called: with hooks present the
    conv -> BN -> quantizer triple runs module by module instead of as the fused launch, and the hook
    sees the BN output the unfused path computes."""
    from quantized_vit_amd.ultranet import random_ultranet, synthetic_images_u8
    model = random_ultranet(seed=2, device=dev, calib_batch=1, img_size=408)
    img = synthetic_images_u8(1, 408, seed=9).to(dev)
    bn = model.layers[1]
    assert isinstance(bn, torch.nn.BatchNorm2d)
    seen = []
    h = bn.register_forward_hook(lambda mod, inp, out: seen.append(out.shape))
    try:
        with torch.no_grad():
            model(img)
    finally:
        h.remove()
    assert len(seen) == 1 and seen[0][1] == bn.num_features
