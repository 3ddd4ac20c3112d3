"""Parity at the production schedule: the sizes the headline bench runs (ViT-B/16, batch 256,
M = 256 * 197 = 50 432 token rows), where every persistent kernel walks many work items per workgroup —
GEMM tiles with the next tile's operand stream issued in the previous tile's tail, (image, head) units of
the fused qkv + attention kernel with next-unit prefetch and the weight-ring slot carried across units,
LayerNorm rows per wave. Every case asserts that it actually reaches that regime (work items per resident
workgroup > 2), then checks the results against the CPU oracle (integer work bit-exact; codes identical
except proven rounding ties; fp32 within 1e-6 of fp64).

Reference call sites: QuantizeLinear.forward quant_layers.py:495-499 (qkv/proj/fc1/fc2 at
vit_model.py:133,151,172,175), Attention vit_model.py:125-153, Block vit_model.py:202-208.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import quant_oracle as O
from parity_tools import tie_check
from quantized_vit_amd import _lib
from test_gpu_kernels import _p, act_buffer, pack_codes

pytestmark = pytest.mark.gpu

B256 = 256
TOKENS = 197
M256 = B256 * TOKENS          # 50 432
BM, BN, BLOCKS_PER_CU = 128, 256, 2


def _cus(dev):
    return torch.cuda.get_device_properties(dev).multi_processor_count


def _tiles(M, N):
    return math.ceil(M / BM) * math.ceil(N / BN)


def _gemm_case(dev, M, N, K, seed, wlim=8):
    g = torch.Generator().manual_seed(seed)
    a = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int16)
    w = torch.randint(-wlim, wlim, (N, K), generator=g, dtype=torch.int16)
    packed, npad, kpad = pack_codes(w, _lib.W4, dev)
    return a, w, act_buffer(a, kpad, dev), packed, npad, kpad


def _exact_accumulators(a, w):
    """sum_k a w on the CPU: every partial sum is an integer below 2^24 (|a| <= 127, |w| <= 8,
    K <= 3072 -> < 3.2e6), so fp32 GEMM is exact in any summation order."""
    return a.float() @ w.float().t()


@pytest.mark.parametrize("N,K,layer", [(3072, 768, "fc1"), (768, 3072, "fc2"), (2304, 768, "qkv"),
                                       (768, 768, "proj")])
def test_gemm_b256_int32_exact(dev, N, K, layer):
    tiles = _tiles(M256, N)
    assert tiles > 2 * BLOCKS_PER_CU * _cus(dev), "must run several tiles per persistent block"
    a, w, A, packed, npad, kpad = _gemm_case(dev, M256, N, K, seed=N + K)
    C = torch.full((M256, N), -7, dtype=torch.int32, device=dev)
    _lib.gemm(A, M256, kpad, packed, _lib.W4, N, npad, None, None, None, _lib.EPI_I32, C)
    got = C.cpu()
    ref = _exact_accumulators(a, w)
    bad = (got.float() != ref)
    assert not bad.any(), f"{layer}: {int(bad.sum())} wrong accumulators, first at {bad.nonzero()[0].tolist()}"


@pytest.mark.parametrize("N,K,layer", [(768, 3072, "fc2"), (768, 768, "proj")])
def test_gemm_b256_residual_epilogue(dev, N, K, layer):
    """x += d_a d_w acc + b in place (the proj / fc2 epilogue, residual rows prefetched per tile)."""
    assert _tiles(M256, N) > 2 * BLOCKS_PER_CU * _cus(dev)
    a, w, A, packed, npad, kpad = _gemm_case(dev, M256, N, K, seed=3 * N + K)
    g = torch.Generator().manual_seed(99)
    bias = torch.randn(N, generator=g)
    base = torch.randn(M256, N, generator=g)
    d_a, d_w = 0.0123, 0.00457
    C = base.to(dev)
    _lib.gemm(A, M256, kpad, packed, _lib.W4, N, npad, _p(d_a, dev), _p(d_w, dev),
              _lib.pad_bias(bias.to(dev), N, npad, dev), _lib.EPI_F32_RESID, C)
    alpha = float(torch.tensor(d_a, dtype=torch.float32) * torch.tensor(d_w, dtype=torch.float32))
    ref = alpha * _exact_accumulators(a, w).double() + bias.double() + base.double()
    err = ((C.cpu().double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-6, err


def _resid_ln_case(dev, M, N, K, seed, qt=O.NONLINEAR, t=1.0, table=True):
    """qvit_gemm_resid_ln against its two-launch form (qvit_gemm EPI_F32_RESID, then qvit_layernorm_quant_i8 on
    the updated rows) on the same inputs: the residual rows and the LayerNorm codes must be bit-identical (the
    LayerNorm behind the tiles runs the standalone kernel's row routine, ln_common.h)."""
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    a, w, A, packed, npad, kpad = _gemm_case(dev, M, N, K, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    bias = torch.randn(N, generator=g) * 0.2
    base = torch.randn(M, N, generator=g)
    gamma = (torch.rand(N, generator=g) + 0.5).to(dev)
    beta = (torch.randn(N, generator=g) * 0.1).to(dev)
    d_a, d_w = 0.0123, 0.00457
    qtc = _lib.QT_LINEAR if qt == O.LINEAR else _lib.QT_NONLINEAR
    qmn, dn = 3.0, 3.0 ** t / 127
    q = dict(out_d=_p(dn, dev), out_qm=_p(qmn, dev), out_t=_p(t, dev) if qt == O.NONLINEAR else None)
    tab = None
    if table:
        geo = epilogue_table_geometry(qtc, dn, qmn, t, saturation_level(qtc, dn, qmn, t), False)
        tab = _lib.epi_table_build(_lib.EPI_I8, qtc, q["out_d"], q["out_qm"], q["out_t"], 0, *geo, dev)
    bias_pad = _lib.pad_bias(bias.to(dev), N, npad, dev)
    kpad_c = (N + 127) // 128 * 128
    # two-launch reference
    x_ref = base.to(dev)
    _lib.gemm(A, M, kpad, packed, _lib.W4, N, npad, _p(d_a, dev), _p(d_w, dev), bias_pad, _lib.EPI_F32_RESID, x_ref)
    c_ref = torch.full((M, kpad_c), 77, dtype=torch.int8, device=dev)
    _lib.layernorm_quant_i8(x_ref, gamma, beta, 1e-6, qtc, q["out_d"], q["out_qm"], q["out_t"], 0, c_ref, kpad_c,
                            code_table=tab)
    # fused, twice on the same arrival counters (they are never reset: each launch adds npad / 256 per row block)
    for rep in range(2):
        x = base.to(dev)
        c = torch.full((M, kpad_c), 55, dtype=torch.int8, device=dev)
        _lib.gemm_resid_ln(A, M, kpad, packed, _lib.W4, N, npad, _p(d_a, dev), _p(d_w, dev), bias_pad, x, gamma, beta,
                           1e-6, qtc, q["out_d"], q["out_qm"], q["out_t"], 0, tab, c, kpad_c)
        torch.cuda.synchronize()
        assert torch.equal(x.cpu(), x_ref.cpu()), f"rep {rep}: residual rows differ"
        dc = (c.cpu() != c_ref.cpu())
        assert not dc.any(), f"rep {rep}: {int(dc.sum())} codes differ, first at {dc.nonzero()[0].tolist()}"
    assert len(torch.unique(c_ref)) > 50
    return c_ref


@pytest.mark.parametrize("N,K,layer", [(768, 3072, "fc2"), (768, 768, "proj")])
def test_gemm_resid_ln_b256(dev, N, K, layer):
    """proj / fc2 with the next LayerNorm behind the tiles at the production size (1 182 tiles, 394 row
    blocks, the LayerNorm of each by whichever of its 3 tile workgroups arrives last)."""
    assert _tiles(M256, N) > 2 * BLOCKS_PER_CU * _cus(dev)
    _resid_ln_case(dev, M256, N, K, seed=N + 5 * K)


@pytest.mark.parametrize("M,N,K,qt,table", [(1000, 768, 768, O.LINEAR, True), (333, 192, 768, O.NONLINEAR, True),
                                            (257, 1024, 1024, O.NONLINEAR, True), (300, 768, 768, O.NONLINEAR, False)])
def test_gemm_resid_ln_shapes(dev, M, N, K, qt, table):
    """Ragged row counts (a partial last row block), one tile per row block (N 192, ViT-Tiny), four (N 1024,
    ViT-L), the linear quantizer, and the per-element quantizer without a code table."""
    _resid_ln_case(dev, M, N, K, seed=M + N, qt=qt, table=table)


def _gemm_fc1(A, M, kpad, packed, npad, N, d_a, d_w, bias_pad, out, path, **kw):
    if path == "a32":  # the weight-stationary schedule on T32 codes (the fused block's fc1)
        _lib.gemm_a32(_lib.rows_to_t32(A, kpad), M, kpad, packed, _lib.W4, N, npad, d_a, d_w, bias_pad,
                      _lib.EPI_I8_GELU, out, **kw)
    else:
        _lib.gemm(A, M, kpad, packed, _lib.W4, N, npad, d_a, d_w, bias_pad, _lib.EPI_I8_GELU, out, **kw)


@pytest.mark.parametrize("path", ["tiles", "a32"])
@pytest.mark.parametrize("qt,t", [(O.NONLINEAR, 1.0), (O.LINEAR, 1.0)])
def test_gemm_b256_gelu_code_epilogue(dev, qt, t, path):
    """fc1: d_a d_w acc + b -> GELU -> fc2's quantizer via the code table, int8 out (4 728 tiles of the persistent
    schedule, or 788 wave tiles of the weight-stationary one on T32 codes: path a32)."""
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    N, K = 3072, 768
    assert _tiles(M256, N) > 2 * BLOCKS_PER_CU * _cus(dev)
    a, w, A, packed, npad, kpad = _gemm_case(dev, M256, N, K, seed=17)
    g = torch.Generator().manual_seed(5)
    bias = torch.randn(N, generator=g) * 0.3
    d_a, d_w = 0.0025, 0.0011
    qtc = _lib.QT_LINEAR if qt == O.LINEAR else _lib.QT_NONLINEAR
    qmn = 2.5
    dn = qmn ** t / 127
    kw = dict(out_qtype=qtc, out_d=_p(dn, dev), out_qm=_p(qmn, dev), out_t=_p(t, dev) if qt == O.NONLINEAR else None)
    geo = epilogue_table_geometry(qtc, dn, qmn, t, saturation_level(qtc, dn, qmn, t), True)
    table = _lib.epi_table_build(_lib.EPI_I8_GELU, qtc, kw["out_d"], kw["out_qm"], kw["out_t"], 0, *geo, dev)
    bias_pad = _lib.pad_bias(bias.to(dev), N, npad, dev)
    outs = []
    for tab in (table, None):
        out = torch.full((M256, N), 99, dtype=torch.int8, device=dev)
        _gemm_fc1(A, M256, kpad, packed, npad, N, _p(d_a, dev), _p(d_w, dev), bias_pad, out, path, epi_table=tab, **kw)
        outs.append(out.cpu())
    assert int(table[12:16].view(torch.int32).item()) == 1
    # the table re-expresses the per-element evaluation (same kernel, same cross-tile schedule)
    dd = (outs[0].to(torch.int32) - outs[1].to(torch.int32)).abs()
    assert dd.max() <= 1 and (dd > 0).float().mean() <= 1e-5
    # against the oracle's quantizer of the exact value GELU(alpha acc + b), evaluated in fp64
    alpha = float(torch.tensor(d_a, dtype=torch.float32) * torch.tensor(d_w, dtype=torch.float32))
    v = F.gelu(alpha * _exact_accumulators(a, w).double() + bias.double())
    own = O.quant_codes(v.float(), qt, dn, qmn, t)
    st = tie_check(v, outs[0].float(), own, qt, dn, qmn, t)
    assert st["non_ties"] == 0, st
    assert st["flips"] <= 2e-4 * st["total"], st
    assert len(torch.unique(outs[0])) > 50


def test_qkv_split_b256(dev):
    """The ViT-L path's qkv GEMM (fp16 hi/lo head planes) at ViT-B b256 size vs the fp32 epilogue."""
    N, K = 2304, 768
    a, w, A, packed, npad, kpad = _gemm_case(dev, M256, N, K, seed=23)
    d_a, d_w = _p(0.004, dev), _p(0.003, dev)
    bias_pad = _lib.pad_bias(torch.randn(N).to(dev) * 0.3, N, npad, dev)
    hi = torch.empty(M256 * N, dtype=torch.float16, device=dev)
    lo = torch.empty_like(hi)
    _lib.gemm_qkv_split(A, M256, kpad, packed, _lib.W4, N, npad, d_a, d_w, bias_pad, TOKENS, 1.0, hi, lo)
    f32 = torch.empty((M256, N), device=dev)
    _lib.gemm(A, M256, kpad, packed, _lib.W4, N, npad, d_a, d_w, bias_pad, _lib.EPI_F32, f32)
    # planes [B][3H][N][64]  ->  [B*N, 3*H*64]
    H = N // 192
    planes = (hi.float() + lo.float()).view(B256, 3 * H, TOKENS, 64).permute(0, 2, 1, 3).reshape(M256, N)
    err = ((planes - f32).abs().max() / f32.abs().max()).item()
    assert err <= 2.0 ** -21, err


# ---- fused qkv projection + attention at B = 256 ---------------------------------------------------
def _attention_fp64(A, w, bias, d_a, d_w, images, N, H):
    """fp64 reference of qkv = d_a d_w (A W^T) + b -> softmax(q k^T / 8) v for the given images."""
    C = 64 * H
    out = {}
    for b in images:
        a = A[b * N:(b + 1) * N].double()
        qkv = d_a * d_w * (a @ w.double().t()) + bias.double()
        x = qkv.reshape(N, 3, H, 64).permute(1, 2, 0, 3)
        att = ((x[0] @ x[1].transpose(-2, -1)) * 0.125).softmax(-1) @ x[2]
        out[b] = att.permute(1, 0, 2).reshape(N, C)
    return out


def test_qkv_attention_fused_b256(dev):
    """3 072 (image, head) units over one persistent workgroup per CU: fused output vs the split path
    (every unit) and vs fp64 on the images at both ends of every XCD's unit range."""
    from test_gpu_attention import _split_path
    B, N, H, K = B256, TOKENS, 12, 768
    C = 64 * H
    assert B * H > 2 * _cus(dev), "must run several units per workgroup"
    g = torch.Generator().manual_seed(2024)
    a = torch.randint(-60, 61, (B * N, K), generator=g, dtype=torch.int16)
    w = torch.randint(-7, 8, (3 * C, K), generator=g, dtype=torch.int16)
    bias = torch.randn(3 * C, generator=g) * 0.3
    packed, npad, kpad = pack_codes(w, _lib.W4, dev)
    A = act_buffer(a, kpad, dev)
    bias_pad = _lib.pad_bias(bias.to(dev), 3 * C, npad, dev)
    d_a, d_w = 0.004, 0.003
    da, dw = _p(d_a, dev), _p(d_w, dev)
    out = torch.full((B * N, C), float("nan"), device=dev)
    _lib.qkv_attention(A, B, N, kpad, packed, npad, da, dw, bias_pad, H, 0.125, out, _lib.ATT_F32, 0.25)
    torch.cuda.synchronize()
    got = out.cpu()
    assert torch.isfinite(got).all()
    ref_split = _split_path(dev, B, N, H, A, packed, npad, kpad, bias_pad, da, dw, 0.25,
                            torch.full((B * N, C), float("nan"), device=dev), _lib.ATT_F32)
    scale = ref_split.abs().max().item()
    assert (got - ref_split).abs().max().item() <= 2e-6 * scale
    # images at the start and the end of each XCD's contiguous unit range (B*H/8 = 384 units = 32 images)
    per_xcd = B // 8
    images = sorted({x * per_xcd + o for x in range(8) for o in (0, 1, per_xcd - 2, per_xcd - 1)})
    alpha = float(torch.tensor(d_a, dtype=torch.float32) * torch.tensor(d_w, dtype=torch.float32))
    ref = _attention_fp64(a, w, bias, alpha, 1.0, images, N, H)
    for b in images:
        err = (got[b * N:(b + 1) * N].double() - ref[b]).abs().max().item()
        assert err <= 2e-6 * scale, (b, err)


def test_qkv_attention_fused_b256_int8(dev):
    """The production mode: proj's quantizer via the code table, int8 codes out, at B = 256, against the
    split path's codes and against the oracle's quantizer of the fp64 attention (proven ties only)."""
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    from test_gpu_attention import _split_path
    B, N, H, K = B256, TOKENS, 12, 768
    C = 64 * H
    g = torch.Generator().manual_seed(77)
    a = torch.randint(-60, 61, (B * N, K), generator=g, dtype=torch.int16)
    w = torch.randint(-7, 8, (3 * C, K), generator=g, dtype=torch.int16)
    bias = torch.randn(3 * C, generator=g) * 0.3
    packed, npad, kpad = pack_codes(w, _lib.W4, dev)
    A = act_buffer(a, kpad, dev)
    bias_pad = _lib.pad_bias(bias.to(dev), 3 * C, npad, dev)
    d_a, d_w = 0.004, 0.003
    da, dw = _p(d_a, dev), _p(d_w, dev)
    qm, t = 0.5, 0.9
    d = qm ** t / 127
    kw = dict(out_qtype=_lib.QT_NONLINEAR, out_d=_p(d, dev), out_qm=_p(qm, dev), out_t=_p(t, dev))
    geo = epilogue_table_geometry(_lib.QT_NONLINEAR, d, qm, t, saturation_level(_lib.QT_NONLINEAR, d, qm, t), False)
    table = _lib.epi_table_build(_lib.EPI_I8, _lib.QT_NONLINEAR, kw["out_d"], kw["out_qm"], kw["out_t"], 0, *geo, dev)
    out = torch.full((B * N, C), 99, dtype=torch.int8, device=dev)
    _lib.qkv_attention(A, B, N, kpad, packed, npad, da, dw, bias_pad, H, 0.125, out, _lib.ATT_I8, 1.0,
                       epi_table=table, **kw)
    torch.cuda.synchronize()
    got = out.cpu()
    ref = _split_path(dev, B, N, H, A, packed, npad, kpad, bias_pad, da, dw, 1.0,
                      torch.zeros((B * N, C), dtype=torch.int8, device=dev), _lib.ATT_I8, epi_table=table, **kw)
    diff = (got.to(torch.int32) - ref.to(torch.int32)).abs()
    assert diff.max().item() <= 1 and (diff > 0).float().mean().item() <= 1e-3
    # every code where the fused and split paths differ must be a proven rounding tie of the exact attention:
    # the fp64 reference (on the device) of every image holding such a code, plus both ends of every XCD's range
    per_xcd = B // 8
    diff_images = sorted(set((diff.amax(1).nonzero().flatten() // N).tolist()))
    images = sorted({x * per_xcd + o for x in range(8) for o in (0, per_xcd - 1)} | set(diff_images))
    alpha = float(torch.tensor(d_a, dtype=torch.float32) * torch.tensor(d_w, dtype=torch.float32))
    ref64 = _attention_fp64(a.to(dev), w.to(dev), bias.to(dev), alpha, 1.0, images, N, H)
    flips = 0
    for b in images:
        v = ref64[b].cpu()
        own = O.quant_codes(v.float(), O.NONLINEAR, d, qm, t)
        for codes in (got, ref):
            st = tie_check(v, codes[b * N:(b + 1) * N].float(), own, O.NONLINEAR, d, qm, t)
            assert st["non_ties"] == 0 and st["flips"] <= 1e-3 * st["total"], (b, st)
        flips += int((diff[b * N:(b + 1) * N] > 0).sum())
    assert flips == int((diff > 0).sum()), "every fused / split difference was tie-checked"


@pytest.mark.parametrize("K", [512, 1024])
def test_qkv_attention_fused_runtime_k(dev, K):
    """K != 768 takes the kernel's runtime k-loop (NKC = 0) instead of the unrolled one."""
    from test_gpu_attention import _fused_case, _split_path
    B, N, H = 40, 197, 12
    A, packed, npad, kpad, bias_pad, da, dw = _fused_case(dev, B, N, H, seed=K, K=K)
    assert kpad == K
    ref = _split_path(dev, B, N, H, A, packed, npad, kpad, bias_pad, da, dw, 2.0 ** -2,
                      torch.full((B * N, 64 * H), float("nan"), device=dev), _lib.ATT_F32)
    out = torch.full((B * N, 64 * H), float("nan"), device=dev)
    _lib.qkv_attention(A, B, N, kpad, packed, npad, da, dw, bias_pad, H, 0.125, out, _lib.ATT_F32, 2.0 ** -2)
    torch.cuda.synchronize()
    got = out.cpu()
    assert torch.isfinite(got).all()
    assert (got.double() - ref.double()).abs().max().item() <= 2e-6 * ref.abs().max().item()


# ---- persistent LayerNorm + quantizer at M = 50 432 -------------------------------------------------
def test_layernorm_quant_b256(dev):
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    rows, cols = M256, 768
    g = torch.Generator().manual_seed(31)
    x = torch.randn(rows, cols, generator=g) * 2 + 0.3
    gamma = torch.rand(cols, generator=g) + 0.5
    beta = torch.randn(cols, generator=g) * 0.1
    qm, t = 3.0, 1.0
    d = qm / 127
    geo = epilogue_table_geometry(_lib.QT_NONLINEAR, d, qm, t, saturation_level(_lib.QT_NONLINEAR, d, qm, t), False)
    table = _lib.epi_table_build(_lib.EPI_I8, _lib.QT_NONLINEAR, _p(d, dev), _p(qm, dev), _p(t, dev), 0, *geo, dev)
    outs = []
    xd = x.to(dev)
    for tab in (table, None):
        out = torch.full((rows, cols), 77, dtype=torch.int8, device=dev)
        _lib.layernorm_quant_i8(xd, gamma.to(dev), beta.to(dev), 1e-6, _lib.QT_NONLINEAR, _p(d, dev), _p(qm, dev),
                                _p(t, dev), 0, out, cols, code_table=tab)
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])
    v = F.layer_norm(x.double(), (cols,), gamma.double(), beta.double(), 1e-6)
    st = tie_check(v, outs[0].float(), O.quant_codes(v.float(), O.NONLINEAR, d, qm, t), O.NONLINEAR, d, qm, t)
    assert st["non_ties"] == 0 and st["flips"] <= 1e-4 * st["total"], st


# ---- the production block and forward ---------------------------------------------------------------
def test_vit_base_block_b256_stage_forced(dev):
    """One ViT-B block at batch 256 (the bench's per-GPU batch), every kernel on the oracle's input, on
    identical int4 weights: the fused qkv + attention kernel, the residual GEMMs and fc1's GELU-code
    epilogue all on their multi-tile / multi-unit schedules."""
    from parity_tools import load_oracle_weight_codes
    from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images
    from test_gpu_model import assert_stages, stage_forced_block
    model = build_quantized_vit("vit_base_patch16_224", seed=0, depth=1).to(dev)
    cfg = O.ViTConfig(depth=1)
    load_oracle_weight_codes(model, cfg)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    trace = []
    with torch.no_grad():
        O.vit_forward(sd, cfg, synthetic_images(B256, 224, seed=21), trace=trace)
        res = stage_forced_block(model, cfg, sd, trace[0], 0, dev)
    assert "fused qkv+attention codes" in res
    assert_stages(res, 0, weights_loaded=True)


def test_vit_base_b64_tie_resolved_end_to_end(dev):
    """The full production forward at batch 64 (fc1: 1 188 tiles over 512 resident GEMM blocks; 768
    attention units over 256 workgroups), every quantizer boundary against the oracle's, ties resolved."""
    from parity_tools import load_oracle_weight_codes, tie_resolved_vit_check
    from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images
    from test_gpu_model import TIE_E2E
    assert _tiles(64 * TOKENS, 3072) > 2 * BLOCKS_PER_CU * _cus(dev) and 64 * 12 > 2 * _cus(dev)
    model = build_quantized_vit("vit_base_patch16_224", seed=0).to(dev)
    cfg = O.ViTConfig()
    load_oracle_weight_codes(model, cfg)
    r = tie_resolved_vit_check(model, cfg, synthetic_images(64, 224, seed=8), dev)
    print(f"ViT-B b64 tie-resolved: rel {r['rel']:.2e}, {r['flips']} tie flips of {r['codes']} codes")
    assert not r["missing"] and not r["bad"], (r["missing"], r["bad"])
    assert r["rel"] <= TIE_E2E, r["rel"]


# ---- configs[3]: ViT-L/16 @ 384, batch 128 (M = 128 * 577 = 73 856 token rows) ----------------------------------
B128, TOK_L = 128, 577
M128 = B128 * TOK_L           # 73 856


@pytest.mark.parametrize("N,K,layer", [(4096, 1024, "fc1"), (1024, 4096, "fc2")])
def test_gemm_vitl_b128_int32_exact(dev, N, K, layer):
    """The ViT-L/16 @ 384 MLP GEMMs at the configs[3] bench size, int32-exact."""
    assert _tiles(M128, N) > 2 * BLOCKS_PER_CU * _cus(dev), "must run several tiles per persistent block"
    a, w, A, packed, npad, kpad = _gemm_case(dev, M128, N, K, seed=N + 2 * K)
    C = torch.full((M128, N), -7, dtype=torch.int32, device=dev)
    _lib.gemm(A, M128, kpad, packed, _lib.W4, N, npad, None, None, None, _lib.EPI_I32, C)
    got = C.cpu()
    del C, A
    ref = _exact_accumulators(a, w)
    bad = (got.float() != ref)
    assert not bad.any(), f"{layer}: {int(bad.sum())} wrong accumulators, first at {bad.nonzero()[0].tolist()}"


def test_qkv_split_attention_vitl_b128(dev):
    """configs[3]'s attention at its bench size: the qkv GEMM into fp16 hi/lo head planes (qvit_gemm_qkv_split,
    M = 73 856, N = 3 072, K = 1 024), then the streaming split attention (qvit_attention_split: B 128, H 16,
    N 577, 128 x 16 x 10 (image, head, 64-query group) units over the persistent grid), against fp64 attention of
    the planes' exact values on the images at both ends of every XCD's unit range (images 16 x and 16 x + 15)."""
    B, N, H, K = B128, TOK_L, 16, 1024
    C = 64 * H
    ngroups = (N + 63) // 64
    assert B * H * ngroups > 2 * 2 * _cus(dev), "each attention workgroup must walk several units"
    g = torch.Generator().manual_seed(31)
    a = torch.randint(-60, 61, (B * N, K), generator=g, dtype=torch.int16)
    w = torch.randint(-7, 8, (3 * C, K), generator=g, dtype=torch.int16)
    bias = torch.randn(3 * C, generator=g) * 0.3
    packed, npad, kpad = pack_codes(w, _lib.W4, dev)
    A = act_buffer(a, kpad, dev)
    del a
    hi = torch.empty(B * N * 3 * C, dtype=torch.float16, device=dev)
    lo = torch.empty_like(hi)
    _lib.gemm_qkv_split(A, B * N, kpad, packed, _lib.W4, 3 * C, npad, _p(0.004, dev), _p(0.003, dev),
                        _lib.pad_bias(bias.to(dev), 3 * C, npad, dev), N, 1.0, hi, lo)
    out = torch.full((B * N, C), float("nan"), device=dev)
    _lib.attention_split(hi, lo, B, N, H, 64, 0.125, out, _lib.ATT_F32, 1.0)
    torch.cuda.synchronize()
    sel = [16 * x + e for x in range(8) for e in (0, 15)]
    planes = (hi.view(B, 3 * H, N, 64)[sel].double() + lo.view(B, 3 * H, N, 64)[sel].double()).cpu()
    q, k, v = planes[:, :H], planes[:, H:2 * H], planes[:, 2 * H:]
    ref = (((q @ k.transpose(-2, -1)) * 0.125).softmax(dim=-1) @ v).transpose(1, 2).reshape(len(sel), N, C)
    got = out.view(B, N, C)[sel].cpu().double()
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item()
    assert err <= 2e-6 * ref.abs().max().item(), err
