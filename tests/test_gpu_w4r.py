"""The register-weight GEMM paths (QVIT_W4R: qvit_pack_weight_w4r image; QVIT_W8R: qvit_pack_weight_w8r image, the
codes as 16x-scaled int8 operands; each wave's weight rows loaded into registers) against the LDS-staged QVIT_W4
path on the same codes: byte-identical outputs for every epilogue,
including the tile schedules the two paths sequence differently (K = 128: no steady step; K = 256: the peeled
steps of the fp32 epilogues; row and column tails; several tiles per workgroup), and for the qkv split GEMM.
The W4 path itself is pinned to the oracle by test_gpu_kernels.py."""
import pytest
import torch

from quantized_vit_amd import _lib
from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
from test_gpu_kernels import _p, _round_up, act_buffer, pack_codes

pytestmark = pytest.mark.gpu

SHAPES = [(1, 1, 1), (300, 200, 200), (257, 2304, 768), (1576, 768, 192), (33, 3072, 768), (129, 768, 3072),
          (64, 100, 1000), (515, 384, 384), (5000, 1024, 768)]
EPIS = [_lib.EPI_I32, _lib.EPI_F32, _lib.EPI_F32_RESID, _lib.EPI_I8, _lib.EPI_I8_GELU]


def _run(dev, wimg, wfmt, A, M, kpad, N, npad, bias_pad, epi, base, table, q):
    if epi == _lib.EPI_I32:
        C = torch.full((M, _round_up(N, 4)), -7, dtype=torch.int32, device=dev)
    elif epi in (_lib.EPI_I8, _lib.EPI_I8_GELU):
        C = torch.full((M, _round_up(N, 16)), 99, dtype=torch.int8, device=dev)
    else:
        C = base.clone()
    _lib.gemm(A, M, kpad, wimg, wfmt, N, npad, _p(0.0031, dev), _p(0.0017, dev), bias_pad, epi, C,
              **(dict(epi_table=table, **q) if epi in (_lib.EPI_I8, _lib.EPI_I8_GELU) else {}))
    torch.cuda.synchronize()
    return C


def _reg_image(packed, npad, kpad, wfmt):
    if wfmt == _lib.W4R:
        img = _lib.pack_weight_w4r(packed, npad, kpad)
        assert img.numel() == packed.numel()
    else:
        img = _lib.pack_weight_w8r(packed, npad, kpad)
        assert img.numel() == 2 * packed.numel()
    return img


@pytest.mark.parametrize("wreg", [_lib.W4R, _lib.W8R])
@pytest.mark.parametrize("epi", EPIS)
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_w4r_equals_w4(dev, epi, M, N, K, wreg):
    g = torch.Generator().manual_seed(M * 3 + N * 5 + K * 7 + epi)
    a = torch.randint(-127, 128, (M, K), generator=g)
    w = torch.randint(-8, 8, (N, K), generator=g)
    packed, npad, kpad = pack_codes(w, _lib.W4, dev)
    w4r = _reg_image(packed, npad, kpad, wreg)
    A = act_buffer(a, kpad, dev)
    bias_pad = _lib.pad_bias((torch.randn(N, generator=g) * 0.3).to(dev), N, npad, dev)
    base = torch.randn(M, _round_up(N, 4), generator=g).to(dev)
    qt, dn, qmn, t = _lib.QT_NONLINEAR, 1.2 / 127, 1.2, 1.0
    q = dict(out_qtype=qt, out_d=_p(dn, dev), out_qm=_p(qmn, dev), out_t=_p(t, dev))
    table = None
    if epi in (_lib.EPI_I8, _lib.EPI_I8_GELU):
        geo = epilogue_table_geometry(qt, dn, qmn, t, saturation_level(qt, dn, qmn, t), epi == _lib.EPI_I8_GELU)
        table = _lib.epi_table_build(epi, qt, q["out_d"], q["out_qm"], q["out_t"], 0, *geo, dev)
    ref = _run(dev, packed, _lib.W4, A, M, kpad, N, npad, bias_pad, epi, base, table, q)
    got = _run(dev, w4r, wreg, A, M, kpad, N, npad, bias_pad, epi, base, table, q)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("wreg", [_lib.W4R, _lib.W8R])
@pytest.mark.parametrize("B,seq,H,K", [(3, 197, 12, 768), (2, 50, 4, 768), (1, 577, 16, 1024)])
def test_gemm_qkv_split_w4r_equals_w4(dev, B, seq, H, K, wreg):
    g = torch.Generator().manual_seed(B + seq + H)
    M, N = B * seq, 3 * H * 64
    a = torch.randint(-127, 128, (M, K), generator=g)
    w = torch.randint(-8, 8, (N, K), generator=g)
    packed, npad, kpad = pack_codes(w, _lib.W4, dev)
    w4r = _reg_image(packed, npad, kpad, wreg)
    A = act_buffer(a, kpad, dev)
    bias_pad = _lib.pad_bias(torch.randn(N, generator=g).to(dev), N, npad, dev)
    outs = []
    for img, wf in ((packed, _lib.W4), (w4r, wreg)):
        hi = torch.empty(M * N, dtype=torch.float16, device=dev)
        lo = torch.empty(M * N, dtype=torch.float16, device=dev)
        _lib.gemm_qkv_split(A, M, kpad, img, wf, N, npad, _p(0.004, dev), _p(0.0011, dev), bias_pad, seq, 0.5,
                            hi, lo)
        torch.cuda.synchronize()
        outs.append((hi.view(torch.int16), lo.view(torch.int16)))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_quant_linear_plan_holds_w4r(dev):
    """The module path runs its int GEMMs on the register image (quant_layers.GEMM_WREG), built on first use with the
    packed codes then released (one int4 copy per layer), and matches the W4 form re-packed on demand."""
    from quantized_vit_amd import quant_layers as QL
    if not QL.GEMM_W4R:
        pytest.skip("QVIT_GEMM_WREG=w4")
    torch.manual_seed(0)
    lin = QL.QuantizeLinear.from_module(torch.nn.Linear(768, 3072).to(dev), num_bits=4,
                                        quant_mode=QL.QuantizationMode.WEIGHT_AND_ACTIVATION).eval()
    with torch.no_grad():
        x = torch.randn(300, 768, device=dev)
        y = lin(x)
        plan = lin.quant_plan()
        assert plan.int_path and plan.wfmt == _lib.W4 and plan.extra.get("wreg") is not None
        assert plan.extra["wreg"][1] == {"w4r": _lib.W4R, "w8r": _lib.W8R}[QL.GEMM_WREG]
        assert plan.packed is None
        w4r, mode = plan.extra.pop("wreg"), QL.GEMM_WREG
        QL.GEMM_WREG = "w4"
        try:
            y4 = lin(x)   # the LDS-staged W4 GEMM on the re-packed codes
        finally:
            QL.GEMM_WREG = mode
            plan.extra["wreg"] = w4r
        assert plan.packed is not None
    assert torch.equal(y, y4)
