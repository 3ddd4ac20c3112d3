"""The weight-stationary schedule of the int8-code GEMM (csrc/gemm_ws.hip, the fc1 shape class of
QViT_with_GETA/vit_model.py:172 -> quant_layers.py:495-499) against the persistent-tile schedule (gemm_kernel).

qvit_gemm takes the weight-stationary kernel when N = npad = 32 panels of 96 rows and K is 768 or 1024; the same
weights packed with one extra 256-row tile of padding (npad = N + 256) do not fit it, so the same call runs
gemm_kernel. Both evaluate v = fma(d_a d_w / 16, float(16 acc), b) and the same code table (or per-element
quantizer), so the codes must agree BYTE FOR BYTE, on every row count (ragged last wave-tile, fewer wave-tiles than
waves, the b256 production size) and with or without a valid code table. The oracle comparison of the same shape
at b256 is tests/test_gpu_production.py::test_gemm_b256_gelu_code_epilogue (it runs this schedule now).
"""
import pytest
import torch

from oracle import quant_oracle as O
from quantized_vit_amd import _lib
from test_gpu_kernels import _p, act_buffer

pytestmark = pytest.mark.gpu


def _pack(w, npad, dev):
    n, k = w.shape
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    packed = _lib.pack_weight(w.float().to(dev).contiguous(), _lib.QT_LINEAR, _p(1.0, dev), _p(1000.0, dev), None,
                              _lib.W4, npad, k, ovf)
    torch.cuda.synchronize()
    assert ovf.item() == 0
    return packed


def _run(dev, M, N, K, gelu, use_table, qt=O.NONLINEAR, t=1.0, seed=3):
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    g = torch.Generator().manual_seed(seed + M)
    a = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int16)
    w = torch.randint(-8, 8, (N, K), generator=g, dtype=torch.int16)
    bias = torch.randn(N, generator=g) * 0.4
    A = act_buffer(a, K, dev)
    qtc = _lib.QT_LINEAR if qt == O.LINEAR else _lib.QT_NONLINEAR
    qmn = 2.0
    dn = qmn ** t / 127
    kw = dict(out_qtype=qtc, out_d=_p(dn, dev), out_qm=_p(qmn, dev), out_t=_p(t, dev) if qt == O.NONLINEAR else None)
    epi = _lib.EPI_I8_GELU if gelu else _lib.EPI_I8
    if use_table:
        geo = epilogue_table_geometry(qtc, dn, qmn, t, saturation_level(qtc, dn, qmn, t), gelu)
        kw["epi_table"] = _lib.epi_table_build(epi, qtc, kw["out_d"], kw["out_qm"], kw["out_t"], 0, *geo, dev)
    outs = []
    for npad in (N, N + 256):  # weight-stationary / persistent-tile schedule
        packed = _pack(w, npad, dev)
        bias_pad = _lib.pad_bias(bias.to(dev), N, npad, dev)
        out = torch.full((M, N), 77, dtype=torch.int8, device=dev)
        _lib.gemm(A, M, K, packed, _lib.W4, N, npad, _p(0.003, dev), _p(0.0012, dev), bias_pad, epi, out, **kw)
        torch.cuda.synchronize()
        outs.append(out.cpu())
    if use_table:
        assert int(kw["epi_table"][12:16].view(torch.int32).item()) == 1
    return outs


@pytest.mark.parametrize("M", [1, 63, 64, 65, 300, 511, 6304 + 40])
@pytest.mark.parametrize("gelu", [True, False])
def test_ws_bit_identical_to_tile_schedule(dev, M, gelu):
    ws, tiles = _run(dev, M, 3072, 768, gelu, use_table=True)
    assert torch.equal(ws, tiles)
    assert len(torch.unique(ws)) > (20 if gelu else 50)


@pytest.mark.parametrize("M,K", [(300, 768), (1000, 1024)])
@pytest.mark.parametrize("qt,t", [(O.NONLINEAR, 1.0), (O.NONLINEAR, 0.85), (O.LINEAR, 1.0)])
def test_ws_per_element_quantizer_bit_identical(dev, M, K, qt, t):
    """No code table: both schedules run the per-element (GELU +) quantizer, K = 1024 included."""
    ws, tiles = _run(dev, M, 3072, K, True, use_table=False, qt=qt, t=t)
    assert torch.equal(ws, tiles)


def test_ws_b256_bit_identical(dev):
    """The production size (M = 256 x 197 = 50 432: 788 wave-tiles, 98-99 per XCD, 12-13 per wave)."""
    ws, tiles = _run(dev, 256 * 197, 3072, 768, True, use_table=True, seed=11)
    assert torch.equal(ws, tiles)
