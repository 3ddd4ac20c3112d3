"""GPU parity of qvit_attention (Attention.forward's core, reference vit_model.py:133-149).

Reference: the same softmax(q k^T * scale) v evaluated in fp64 on the CPU from the same fp32 qkv.
Bars: fp32 output within 2e-6 of max|out| for ordinary logits; 1e-5 for near one-hot rows with logits of
std ~36 (the fp16 hi/lo split carries each operand to 22 bits, so a logit's absolute error grows with
sum |q_i k_i|, and a softmax row turns it into the same relative error on the output); int8-code output
equal to the oracle's quantizer applied to the fp64 result except at rounding ties (<= 1e-3 of codes,
each off by one).
"""
import math

import pytest
import torch

from oracle import quant_oracle as O
from quantized_vit_amd import _lib

pytestmark = pytest.mark.gpu


def _p(v, dev):
    return torch.tensor([float(v)], dtype=torch.float32, device=dev)


def ref_attention(qkv: torch.Tensor, B: int, N: int, H: int, hd: int, scale: float) -> torch.Tensor:
    """vit_model.py:133-149 in fp64."""
    x = qkv[:, :3 * H * hd].double().reshape(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    q, k, v = x[0], x[1], x[2]
    a = ((q @ k.transpose(-2, -1)) * scale).softmax(dim=-1)
    return (a @ v).transpose(1, 2).reshape(B * N, H * hd)


def run(dev, B, N, H, qkv, scale, mode=_lib.ATT_F32, in_scale=1.0, **qkw):
    if mode == _lib.ATT_F32:
        out = torch.full((B * N, H * 64), float("nan"), device=dev)
    else:
        out = torch.zeros((B * N, H * 64), dtype=torch.int8, device=dev)
    _lib.attention(qkv.to(dev), B, N, H, 64, scale, out, mode, in_scale, **qkw)
    torch.cuda.synchronize()
    return out.cpu()


@pytest.mark.parametrize("B,N,H", [(2, 197, 12), (1, 1, 1), (3, 33, 2), (1, 64, 3), (2, 577, 2), (1, 300, 1)])
def test_attention_fp32_vs_fp64(dev, B, N, H):
    g = torch.Generator().manual_seed(N * 7 + H)
    qkv = torch.randn(B * N, 3 * H * 64, generator=g) * 1.5
    scale = 64 ** -0.5
    ref = ref_attention(qkv, B, N, H, 64, scale)
    out = run(dev, B, N, H, qkv, scale)
    assert torch.isfinite(out).all()
    err = (out.double() - ref).abs().max().item()
    assert err <= 2e-6 * ref.abs().max().item(), err


def test_attention_row_stride_and_peaked_softmax(dev):
    """ldq wider than 3*H*hd (qkv sliced from a padded GEMM output) and near one-hot softmax rows."""
    B, N, H = 2, 197, 4
    g = torch.Generator().manual_seed(5)
    full = torch.randn(B * N, 3 * H * 64 + 64, generator=g) * 6.0
    qkv = full[:, :3 * H * 64]
    ref = ref_attention(qkv, B, N, H, 64, 0.125)
    out = torch.empty((B * N, H * 64), device=dev)
    _lib.attention(full.to(dev)[:, :3 * H * 64], B, N, H, 64, 0.125, out)
    torch.cuda.synchronize()
    err = (out.cpu().double() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item(), err


@pytest.mark.parametrize("slope", [0.04, 0.08, 0.15])
def test_attention_running_max_rescale_branch(dev, slope):
    """Logits that rise with the key index (slope per key, natural units) plus one late spike: the
    online softmax's running max grows by less than the deferral threshold in some key blocks (kept) and
    by more in others (rescale of o and l), at block positions fixed by the data. Full-tensor fp64 check."""
    B, N, H = 2, 197, 2
    g = torch.Generator().manual_seed(int(slope * 1000))
    qkv = torch.randn(B * N, 3 * H * 64, generator=g) * 0.2
    x = qkv.view(B, N, 3, H, 64)
    u = torch.randn(64, generator=g)
    u /= u.norm()
    j = torch.arange(N, dtype=torch.float32)
    x[:, :, 0] += 4.0 * u                                        # q . u = 4 for every query
    x[:, :, 1] += (slope * j / (4.0 * 0.125))[None, :, None, None] * u   # logit of key j ~ slope * j
    x[0, 170, 1, 0] += (12.0 / (4.0 * 0.125)) * u                # +12 at key 170 (block 5), image 0 head 0
    x[1, 40, 1, 1] += (12.0 / (4.0 * 0.125)) * u                 # +12 at key 40 (block 1), image 1 head 1
    ref = ref_attention(qkv, B, N, H, 64, 0.125)
    out = run(dev, B, N, H, qkv, 0.125)
    assert torch.isfinite(out).all()
    err = (out.double() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item(), err


def test_attention_in_scale_large_inputs(dev):
    """|q|, |k|, |v| beyond the fp16 range: a power-of-two in_scale keeps the split exact."""
    B, N, H = 1, 100, 2
    g = torch.Generator().manual_seed(9)
    qkv = torch.randn(B * N, 3 * H * 64, generator=g)
    qkv[:, 2 * H * 64:] *= 2.0e5           # v beyond 65504
    qkv[:, :2 * H * 64] *= 1.5             # ordinary logits: this test isolates the scaling
    ref = ref_attention(qkv, B, N, H, 64, 0.125)
    out = run(dev, B, N, H, qkv, 0.125, in_scale=2.0 ** -5)   # |v| <= ~1e6 -> < 65504 after scaling
    err = (out.double() - ref).abs().max().item()
    assert err <= 2e-6 * ref.abs().max().item(), err


@pytest.mark.parametrize("qt,t", [(O.LINEAR, 1.0), (O.NONLINEAR, 1.0), (O.NONLINEAR, 0.8)])
def test_attention_int8_codes_vs_oracle(dev, qt, t):
    B, N, H = 2, 197, 12
    g = torch.Generator().manual_seed(11)
    qkv = torch.randn(B * N, 3 * H * 64, generator=g)
    ref = ref_attention(qkv, B, N, H, 64, 0.125)
    d, qm = 1.2 / 127, 1.2
    if qt == O.NONLINEAR:
        d = qm ** t / 127
    want = O.quant_codes(ref.float(), qt, d, qm, t if qt == O.NONLINEAR else None).to(torch.int32)
    qtc = _lib.QT_LINEAR if qt == O.LINEAR else _lib.QT_NONLINEAR
    got = run(dev, B, N, H, qkv, 0.125, mode=_lib.ATT_I8, out_qtype=qtc, out_d=_p(d, dev), out_qm=_p(qm, dev),
              out_t=_p(t, dev) if qt == O.NONLINEAR else None).to(torch.int32)
    diff = (got - want).abs()
    assert diff.max().item() <= 1
    assert (diff > 0).float().mean().item() <= 1e-3


def test_attention_argument_validation(dev):
    qkv = torch.zeros(10, 3 * 64, device=dev)
    out = torch.zeros(10, 64, device=dev)
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    assert lib.qvit_attention(qkv.data_ptr(), 1, 10, 1, 32, 192, 0.125, 1.0, 0, out.data_ptr(), 64, 0, None, None,
                              None, 0, s) == -1            # head_dim != 64
    assert lib.qvit_attention(qkv.data_ptr(), 1, 10, 1, 64, 100, 0.125, 1.0, 0, out.data_ptr(), 64, 0, None, None,
                              None, 0, s) == -1            # ldq < 3 H hd
    assert lib.qvit_attention(qkv.data_ptr(), 1, 10, 1, 64, 192, 0.125, 1.0, 1, out.data_ptr(), 64, 1, None, None,
                              None, 0, s) == -1            # int8 mode without quantizer params
    assert lib.qvit_attention(qkv.data_ptr(), 1, 10, 1, 64, 192, 0.125, 0.0, 0, out.data_ptr(), 64, 0, None, None,
                              None, 0, s) == -1            # in_scale must be > 0


# ---- split-operand path (qvit_gemm_qkv_split -> qvit_attention_split; the fused block) ----------------
def split_planes(qkv: torch.Tensor, B: int, N: int, H: int, in_scale: float):
    """fp16 hi/lo planes [B][3H][N][64] of in_scale * qkv, rounded exactly as the kernels split."""
    x = qkv[:, :3 * H * 64].float() * in_scale
    hi = x.half()
    lo = (x - hi.float()).half()
    f = lambda t: t.reshape(B, N, 3 * H, 64).permute(0, 2, 1, 3).contiguous().reshape(-1)
    return f(hi), f(lo)


def run_split(dev, B, N, H, qkv, scale, mode=_lib.ATT_F32, in_scale=1.0, **qkw):
    hi, lo = split_planes(qkv, B, N, H, in_scale)
    if mode == _lib.ATT_F32:
        out = torch.full((B * N, H * 64), float("nan"), device=dev)
    else:
        out = torch.zeros((B * N, H * 64), dtype=torch.int8, device=dev)
    _lib.attention_split(hi.to(dev), lo.to(dev), B, N, H, 64, scale, out, mode, in_scale, **qkw)
    torch.cuda.synchronize()
    return out.cpu()


@pytest.mark.parametrize("B,N,H", [(2, 197, 12), (1, 1, 1), (3, 33, 2), (1, 64, 3), (2, 577, 2), (1, 300, 1),
                                   (4, 197, 3)])
def test_attention_split_bitwise_equals_fp32_input_kernel(dev, B, N, H):
    """Same arithmetic in the same order: the split-input kernel reproduces qvit_attention bit for bit."""
    g = torch.Generator().manual_seed(N * 5 + H)
    qkv = torch.randn(B * N, 3 * H * 64, generator=g) * 1.5
    a = run(dev, B, N, H, qkv, 0.125)
    b = run_split(dev, B, N, H, qkv, 0.125)
    assert torch.isfinite(b).all()
    assert torch.equal(a, b)


def test_attention_split_int8_and_in_scale(dev):
    B, N, H = 2, 197, 12
    g = torch.Generator().manual_seed(13)
    qkv = torch.randn(B * N, 3 * H * 64, generator=g)
    qkv[:, 2 * H * 64:] *= 3.0e4
    kw = dict(out_qtype=_lib.QT_NONLINEAR, out_d=_p(4e4 ** 0.9 / 127, dev), out_qm=_p(4e4, dev),
              out_t=_p(0.9, dev))
    a = run(dev, B, N, H, qkv, 0.125, mode=_lib.ATT_I8, in_scale=2.0 ** -2, **kw)
    b = run_split(dev, B, N, H, qkv, 0.125, mode=_lib.ATT_I8, in_scale=2.0 ** -2, **kw)
    assert torch.equal(a, b)
    assert len(torch.unique(b)) > 50


@pytest.mark.parametrize("wfmt", [_lib.W4, _lib.W8])
@pytest.mark.parametrize("seq,B", [(197, 3), (50, 7), (1, 130)])
def test_gemm_qkv_split_equals_f32_epilogue(dev, wfmt, seq, B):
    """hi/lo planes are the exact split of in_scale times the QVIT_EPI_F32 output, head-major."""
    from test_gpu_kernels import act_buffer, pack_codes
    H = 4
    M, N, K = B * seq, 3 * H * 64, 384
    g = torch.Generator().manual_seed(seq + B + wfmt)
    a = torch.randint(-127, 128, (M, K), generator=g)
    lim = 7 if wfmt == _lib.W4 else 127
    w = torch.randint(-lim, lim + 1, (N, K), generator=g)
    bias = torch.randn(N, generator=g)
    packed, npad, kpad = pack_codes(w, wfmt, dev)
    bias_pad = _lib.pad_bias(bias.to(dev), N, npad, dev)
    A = act_buffer(a, kpad, dev)
    da, dw = _p(0.01, dev), _p(0.003, dev)
    ref = torch.empty((M, N), device=dev)
    _lib.gemm(A, M, kpad, packed, wfmt, N, npad, da, dw, bias_pad, _lib.EPI_F32, ref)
    s = 2.0 ** -3
    hi = torch.full((M * N,), float("nan"), dtype=torch.float16, device=dev)
    lo = torch.full((M * N,), float("nan"), dtype=torch.float16, device=dev)
    _lib.gemm_qkv_split(A, M, kpad, packed, wfmt, N, npad, da, dw, bias_pad, seq, s, hi, lo)
    torch.cuda.synchronize()
    whi, wlo = split_planes(ref.cpu(), B, seq, H, s)
    assert torch.equal(hi.cpu(), whi) and torch.equal(lo.cpu(), wlo)


def test_split_argument_validation(dev):
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(4096, dtype=torch.float16, device=dev)
    out = torch.zeros(10, 64, device=dev)
    p = buf.data_ptr()
    assert lib.qvit_attention_split(p, p, 1, 10, 1, 32, 0.125, 1.0, 0, out.data_ptr(), 64, 0, None, None, None, 0,
                                    None, s) == -1    # head_dim
    assert lib.qvit_attention_split(p, None, 1, 10, 1, 64, 0.125, 1.0, 0, out.data_ptr(), 64, 0, None, None, None,
                                    0, None, s) == -3  # NULL lo plane
    assert lib.qvit_attention_split(p + 2, p, 1, 10, 1, 64, 0.125, 1.0, 0, out.data_ptr(), 64, 0, None, None, None,
                                    0, None, s) == -2  # misaligned
    assert lib.qvit_attention_split(p, p, 1, 10, 1, 64, 0.125, 1.0, 0, out.data_ptr(), 64, 0, None, None, None,
                                    0, p + 4, s) == -2  # misaligned code table
    one = _p(1.0, dev).data_ptr()
    # N % 64, M % seq, in_scale
    assert lib.qvit_gemm_qkv_split(p, 10, 128, 128, p, 4, 96, 256, one, one, None, 10, 1.0, p, p, s) == -1
    assert lib.qvit_gemm_qkv_split(p, 10, 128, 128, p, 4, 192, 256, one, one, None, 3, 1.0, p, p, s) == -1
    assert lib.qvit_gemm_qkv_split(p, 10, 128, 128, p, 4, 192, 256, one, one, None, 10, 0.0, p, p, s) == -1
    # qvit_gemm does not accept the split epilogue
    assert lib.qvit_gemm(p, 10, 128, 128, p, 4, 192, 256, one, one, None, 5, p, 192, 0, None, None, None, 0, None,
                         s) == -1


@pytest.mark.parametrize("qt,t", [(O.LINEAR, 1.0), (O.NONLINEAR, 1.0), (O.NONLINEAR, 0.8)])
@pytest.mark.parametrize("ldo", [12 * 64, 12 * 64 + 4])
def test_attention_split_code_table_equals_direct(dev, qt, t, ldo):
    """The int8 epilogue through the quantizer's code table (and the 16-B transposed stores, ldo % 16 == 0)
    writes exactly the codes of the per-element quantizer (and of the fp32-input kernel)."""
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    B, N, H = 3, 197, 12
    g = torch.Generator().manual_seed(17 + ldo)
    qkv = torch.randn(B * N, 3 * H * 64, generator=g)
    d, qm = 0.9 / 127, 0.9
    if qt == O.NONLINEAR:
        d = qm ** t / 127
    qtc = _lib.QT_LINEAR if qt == O.LINEAR else _lib.QT_NONLINEAR
    kw = dict(out_qtype=qtc, out_d=_p(d, dev), out_qm=_p(qm, dev), out_t=_p(t, dev) if qt == O.NONLINEAR else None)
    geo = epilogue_table_geometry(qtc, d, qm, t, saturation_level(qtc, d, qm, t), False)
    table = _lib.epi_table_build(_lib.EPI_I8, qtc, kw["out_d"], kw["out_qm"], kw["out_t"], 0, *geo, dev)
    assert int(table[12:16].view(torch.int32).item()) == 1
    hi, lo = split_planes(qkv, B, N, H, 1.0)
    outs = []
    for tab in (None, table):
        out = torch.zeros((B * N, ldo), dtype=torch.int8, device=dev)
        _lib.attention_split(hi.to(dev), lo.to(dev), B, N, H, 64, 0.125, out, _lib.ATT_I8, 1.0, epi_table=tab, **kw)
        torch.cuda.synchronize()
        outs.append(out.cpu())
    ref = run(dev, B, N, H, qkv, 0.125, mode=_lib.ATT_I8, **kw)
    assert torch.equal(outs[0][:, :H * 64], ref) and torch.equal(outs[1][:, :H * 64], ref)
    assert (outs[1][:, H * 64:] == 0).all()
    assert len(torch.unique(ref)) > 100


# ---- fused qkv projection + attention (qvit_qkv_attention) -------------------------------------------
def _fused_case(dev, B, N, H, seed, K=768):
    from test_gpu_kernels import act_buffer, pack_codes
    g = torch.Generator().manual_seed(seed)
    C = 64 * H
    a = torch.randint(-60, 61, (B * N, K), generator=g)
    w = torch.randint(-7, 8, (3 * C, K), generator=g)
    bias = torch.randn(3 * C, generator=g) * 0.3
    packed, npad, kpad = pack_codes(w, _lib.W4, dev)
    bias_pad = _lib.pad_bias(bias.to(dev), 3 * C, npad, dev)
    return act_buffer(a, kpad, dev), packed, npad, kpad, bias_pad, _p(0.004, dev), _p(0.003, dev)


def _split_path(dev, B, N, H, A, packed, npad, kpad, bias_pad, da, dw, s, out, mode, **kw):
    C = 64 * H
    hi = torch.empty(B * N * 3 * C, dtype=torch.float16, device=dev)
    lo = torch.empty_like(hi)
    _lib.gemm_qkv_split(A, B * N, kpad, packed, _lib.W4, 3 * C, npad, da, dw, bias_pad, N, s, hi, lo)
    _lib.attention_split(hi, lo, B, N, H, 64, 0.125, out, mode, s, **kw)
    torch.cuda.synchronize()
    return out.cpu()


# K != 768 runs the runtime-K projection loop (NKC = 0), K = 768 the unrolled one. N covers the key-block
# paths of the 32x32 attention: 7 blocks straight-line (193 .. 208; 193 leaves one valid key in the last
# block), the two-blocks-per-iteration loop with an even / odd block count, a last block masked with its
# second 16 keys all past N (N % 32 in 1 .. 16: 1, 100, 130, 193, 208) or not (17, 50), and unmasked (N a
# multiple of 32: 64, 96, 160)
@pytest.mark.parametrize("B,N,H,K", [(3, 197, 12, 768), (2, 50, 4, 768), (1, 208, 2, 768), (5, 1, 3, 768),
                                     (2, 17, 12, 768), (9, 100, 1, 768), (3, 197, 8, 512), (2, 197, 12, 1024),
                                     (40, 197, 3, 256), (2, 64, 3, 768), (1, 96, 5, 768), (2, 160, 2, 768),
                                     (2, 130, 3, 768), (2, 193, 4, 768)])
def test_qkv_attention_fused_f32_vs_split_path(dev, B, N, H, K):
    A, packed, npad, kpad, bias_pad, da, dw = _fused_case(dev, B, N, H, seed=B * 1000 + N + H, K=K)
    ref = _split_path(dev, B, N, H, A, packed, npad, kpad, bias_pad, da, dw, 2.0 ** -2,
                      torch.full((B * N, 64 * H), float("nan"), device=dev), _lib.ATT_F32)
    out = torch.full((B * N, 64 * H), float("nan"), device=dev)
    _lib.qkv_attention(A, B, N, kpad, packed, npad, da, dw, bias_pad, H, 0.125, out, _lib.ATT_F32, 2.0 ** -2)
    torch.cuda.synchronize()
    got = out.cpu()
    assert torch.isfinite(got).all()
    err = (got.double() - ref.double()).abs().max().item()
    assert err <= 2e-6 * ref.abs().max().item(), err


@pytest.mark.parametrize("B,N,H", [(4, 197, 12), (3, 64, 6), (2, 208, 4), (3, 17, 5)])
def test_qkv_attention_fused_int8_codes(dev, B, N, H):
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    A, packed, npad, kpad, bias_pad, da, dw = _fused_case(dev, B, N, H, seed=7 + N)
    qm, t = 0.5, 0.9
    d = qm ** t / 127
    kw = dict(out_qtype=_lib.QT_NONLINEAR, out_d=_p(d, dev), out_qm=_p(qm, dev), out_t=_p(t, dev))
    geo = epilogue_table_geometry(_lib.QT_NONLINEAR, d, qm, t, saturation_level(_lib.QT_NONLINEAR, d, qm, t), False)
    table = _lib.epi_table_build(_lib.EPI_I8, _lib.QT_NONLINEAR, kw["out_d"], kw["out_qm"], kw["out_t"], 0, *geo,
                                 dev)
    ref = _split_path(dev, B, N, H, A, packed, npad, kpad, bias_pad, da, dw, 1.0,
                      torch.zeros((B * N, 64 * H), dtype=torch.int8, device=dev), _lib.ATT_I8, epi_table=table, **kw)
    out = torch.full((B * N, 64 * H), 99, dtype=torch.int8, device=dev)
    _lib.qkv_attention(A, B, N, kpad, packed, npad, da, dw, bias_pad, H, 0.125, out, _lib.ATT_I8, 1.0,
                       epi_table=table, **kw)
    torch.cuda.synchronize()
    diff = (out.cpu().to(torch.int32) - ref.to(torch.int32)).abs()
    assert diff.max().item() <= 1
    assert (diff > 0).float().mean().item() <= 1e-3
    assert len(torch.unique(ref)) > 60


# known answer: zero weights, q bias -30, k bias +30, so every score of a row is the same large negative
# number (-1.04e4 in log2 units after scaling) and the softmax is uniform: out = v's bias on every row (the f32
# output undoes in_scale), exact up to the fp16 hi/lo operand split
def test_qkv_attention_fused_uniform_rows(dev):
    from test_gpu_kernels import pack_codes
    B, N, H, K = 2, 197, 2, 768
    C = 64 * H
    A, _, _, kpad, _, da, dw = _fused_case(dev, B, N, H, seed=5)
    packed, npad, kpad2 = pack_codes(torch.zeros(3 * C, K, dtype=torch.int64), _lib.W4, dev)
    assert kpad2 == kpad
    g = torch.Generator().manual_seed(9)
    vb = torch.randn(C, generator=g)
    bias = torch.cat([torch.full((C,), -30.0), torch.full((C,), 30.0), vb])
    bias_pad = _lib.pad_bias(bias.to(dev), 3 * C, npad, dev)
    out = torch.full((B * N, C), float("nan"), device=dev)
    _lib.qkv_attention(A, B, N, kpad, packed, npad, da, dw, bias_pad, H, 0.125, out, _lib.ATT_F32, 2.0 ** -2)
    torch.cuda.synchronize()
    got = out.cpu()
    assert torch.isfinite(got).all()
    ref = vb.expand(B * N, C)
    assert (got - ref).abs().max().item() <= 4e-6 * ref.abs().max().item()


# the output epilogue's other paths: the per-element quantizer (no code table) and rows whose stride is not a
# multiple of 16 B (4-B stores instead of the permlane32-paired 16-B ones); the output is a column view of a
# wider buffer, whose pad columns must stay untouched
@pytest.mark.parametrize("use_table,pad", [(False, 0), (True, 4), (False, 4)])
def test_qkv_attention_fused_int8_store_paths(dev, use_table, pad):
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    B, N, H = 3, 197, 4
    C = 64 * H
    A, packed, npad, kpad, bias_pad, da, dw = _fused_case(dev, B, N, H, seed=11 + pad)
    qm, t = 0.5, 0.9
    d = qm ** t / 127
    kw = dict(out_qtype=_lib.QT_NONLINEAR, out_d=_p(d, dev), out_qm=_p(qm, dev), out_t=_p(t, dev))
    table = None
    if use_table:
        geo = epilogue_table_geometry(_lib.QT_NONLINEAR, d, qm, t, saturation_level(_lib.QT_NONLINEAR, d, qm, t),
                                      False)
        table = _lib.epi_table_build(_lib.EPI_I8, _lib.QT_NONLINEAR, kw["out_d"], kw["out_qm"], kw["out_t"], 0, *geo,
                                     dev)
    ref = _split_path(dev, B, N, H, A, packed, npad, kpad, bias_pad, da, dw, 1.0,
                      torch.zeros((B * N, C), dtype=torch.int8, device=dev), _lib.ATT_I8, epi_table=table, **kw)
    big = torch.full((B * N, C + pad), 99, dtype=torch.int8, device=dev)
    out = big[:, :C]
    _lib.qkv_attention(A, B, N, kpad, packed, npad, da, dw, bias_pad, H, 0.125, out, _lib.ATT_I8, 1.0,
                       epi_table=table, **kw)
    torch.cuda.synchronize()
    diff = (out.cpu().to(torch.int32) - ref.to(torch.int32)).abs()
    assert diff.max().item() <= 1
    assert (diff > 0).float().mean().item() <= 1e-3
    assert len(torch.unique(ref)) > 60
    if pad:
        assert (big[:, C:].cpu() == 99).all()


def test_qkv_attention_argument_validation(dev):
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(1 << 16, dtype=torch.int8, device=dev)
    p = buf.data_ptr()
    one = _p(1.0, dev).data_ptr()
    args = lambda **o: [o.get("A", p), o.get("B", 1), o.get("N", 10), o.get("K", 256), o.get("lda", 256), p,
                        o.get("wfmt", 4), o.get("npad", 256), one, one, None, o.get("H", 1), o.get("hd", 64), 0.125,
                        1.0, 0, p, 64, 0, None, None, None, 0, None, s]
    assert lib.qvit_qkv_attention(*args()) == 0
    assert lib.qvit_qkv_attention(*args(N=209)) == -1        # N > 208
    assert lib.qvit_qkv_attention(*args(wfmt=8)) == -1       # int4 weights only
    assert lib.qvit_qkv_attention(*args(B=1 << 17, N=200, lda=1 << 8)) == -1   # A past 32-bit offsets
    assert lib.qvit_qkv_attention(*args(K=128, lda=256)) == -1   # K % 256
    assert lib.qvit_qkv_attention(*args(hd=32)) == -1
    assert lib.qvit_qkv_attention(*args(A=None)) == -3
    assert lib.qvit_qkv_attention(*args(A=p + 4)) == -2
    torch.cuda.synchronize()
