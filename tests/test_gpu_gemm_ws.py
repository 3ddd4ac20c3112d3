"""The weight-stationary int8-code GEMM on QVIT_ACT_T32 activations (qvit_gemm_a32, csrc/gemm_ws.hip: the fc1 shape
class of QViT_with_GETA/vit_model.py:172 -> quant_layers.py:495-499) and its producer, the LayerNorm + quantizer
writing that layout (qvit_layernorm_quant_i8_t32, vit_model.py:206-207 norm2 + quant_layers.py:356-381).

Both re-express existing kernels on another data layout / schedule with the same arithmetic:
  * qvit_layernorm_quant_i8_t32 must write exactly the codes of qvit_layernorm_quant_i8, permuted (byte for byte);
  * qvit_gemm_a32 on the T32 form of codes must give exactly the int8 codes of qvit_gemm (gemm_kernel) on the
    row-major codes: both evaluate v = fma(d_a d_w / 16, float(16 acc), b) and the same code table or per-element
    quantizer. Checked on every row count class (ragged 64-row wave tile, fewer wave tiles than waves, the b256
    production size), with and without a code table, K = 768 and 1024.
The oracle comparison of the fc1 shape at b256 (tie-checked codes) is
tests/test_gpu_production.py::test_gemm_b256_gelu_code_epilogue_t32.
"""
import pytest
import torch

from oracle import quant_oracle as O
from quantized_vit_amd import _lib
from test_gpu_kernels import _p, act_buffer, pack_codes

pytestmark = pytest.mark.gpu


def test_t32_layout_round_trip():
    g = torch.Generator().manual_seed(1)
    for M, K in ((1, 64), (65, 768), (300, 1024)):
        c = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int8)
        t = _lib.rows_to_t32(c, K)
        assert t.numel() == _lib.t32_rows(M) * K
        assert torch.equal(_lib.t32_to_rows(t, M, K), c)
        # the documented offset of column c of row r
        r, col = M - 1, K - 5
        off = (r // 32 * (K // 32) + col // 32) * 1024 + ((r % 32) + 32 * ((col // 16) % 2)) * 16 + col % 16
        assert t[off] == c[r, col]


def _run(dev, M, N, K, gelu, use_table, qt=O.NONLINEAR, t=1.0, seed=3):
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    g = torch.Generator().manual_seed(seed + M)
    a = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int16)
    w = torch.randint(-8, 8, (N, K), generator=g, dtype=torch.int16)
    bias = torch.randn(N, generator=g) * 0.4
    packed, npad, kpad = pack_codes(w, _lib.W4, dev)
    assert npad == N and kpad == K
    A = act_buffer(a, kpad, dev)
    qtc = _lib.QT_LINEAR if qt == O.LINEAR else _lib.QT_NONLINEAR
    qmn = 2.0
    dn = qmn ** t / 127
    kw = dict(out_qtype=qtc, out_d=_p(dn, dev), out_qm=_p(qmn, dev), out_t=_p(t, dev) if qt == O.NONLINEAR else None)
    epi = _lib.EPI_I8_GELU if gelu else _lib.EPI_I8
    assert _lib.gemm_a32_fits(K, _lib.W4, N, npad, epi)
    if use_table:
        geo = epilogue_table_geometry(qtc, dn, qmn, t, saturation_level(qtc, dn, qmn, t), gelu)
        kw["epi_table"] = _lib.epi_table_build(epi, qtc, kw["out_d"], kw["out_qm"], kw["out_t"], 0, *geo, dev)
    bias_pad = _lib.pad_bias(bias.to(dev), N, npad, dev)
    d_a, d_w = _p(0.003, dev), _p(0.0012, dev)
    tiles = torch.full((M, N), 77, dtype=torch.int8, device=dev)
    _lib.gemm(A, M, K, packed, _lib.W4, N, npad, d_a, d_w, bias_pad, epi, tiles, **kw)
    ws = torch.full((M, N), 55, dtype=torch.int8, device=dev)
    _lib.gemm_a32(_lib.rows_to_t32(A, K), M, K, packed, _lib.W4, N, npad, d_a, d_w, bias_pad, epi, ws, **kw)
    torch.cuda.synchronize()
    if use_table:
        assert int(kw["epi_table"][12:16].view(torch.int32).item()) == 1
    return ws.cpu(), tiles.cpu()


@pytest.mark.parametrize("M", [1, 63, 64, 65, 300, 511, 6304 + 40])
@pytest.mark.parametrize("gelu", [True, False])
def test_a32_bit_identical_to_tile_schedule(dev, M, gelu):
    ws, tiles = _run(dev, M, 3072, 768, gelu, use_table=True)
    assert torch.equal(ws, tiles)
    assert len(torch.unique(ws)) > (20 if gelu else 50)


@pytest.mark.parametrize("M,K", [(300, 768), (1000, 1024)])
@pytest.mark.parametrize("qt,t", [(O.NONLINEAR, 1.0), (O.NONLINEAR, 0.85), (O.LINEAR, 1.0)])
def test_a32_per_element_quantizer_bit_identical(dev, M, K, qt, t):
    """No code table: both schedules run the per-element (GELU +) quantizer, K = 1024 included."""
    ws, tiles = _run(dev, M, 3072, K, True, use_table=False, qt=qt, t=t)
    assert torch.equal(ws, tiles)


def test_a32_b256_bit_identical(dev):
    """The production size (M = 256 x 197 = 50 432: 788 wave tiles, 98-99 per XCD, 12-13 per wave)."""
    ws, tiles = _run(dev, 256 * 197, 3072, 768, True, use_table=True, seed=11)
    assert torch.equal(ws, tiles)


def test_a32_rejects_other_shapes(dev):
    assert not _lib.gemm_a32_fits(768, _lib.W4, 768, 768, _lib.EPI_I8_GELU)
    assert not _lib.gemm_a32_fits(768, _lib.W4, 3072, 3328, _lib.EPI_I8_GELU)
    assert not _lib.gemm_a32_fits(768, _lib.W8, 3072, 3072, _lib.EPI_I8_GELU)
    assert not _lib.gemm_a32_fits(768, _lib.W4, 3072, 3072, _lib.EPI_F32)
    A = torch.zeros(64 * 768, dtype=torch.int8, device=dev)
    C = torch.zeros((64, 768), dtype=torch.int8, device=dev)
    with pytest.raises(_lib.QvitError):
        _lib.gemm_a32(A, 64, 768, A, _lib.W4, 768, 768, _p(1.0, dev), _p(1.0, dev), None, _lib.EPI_I8, C,
                      out_qtype=_lib.QT_LINEAR, out_d=_p(1.0, dev), out_qm=_p(1.0, dev))


@pytest.mark.parametrize("M,cols,kpad", [(1, 768, 768), (197, 768, 768), (300, 1024, 1024), (65, 192, 256),
                                          (256 * 197, 768, 768)])
@pytest.mark.parametrize("table", [True, False])
def test_layernorm_t32_equals_row_major(dev, M, cols, kpad, table):
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    g = torch.Generator().manual_seed(M + cols)
    x = (torch.randn(M, cols, generator=g) * 1.5 + 0.2).to(dev)
    gamma = (torch.rand(cols, generator=g) + 0.5).to(dev)
    beta = (torch.randn(cols, generator=g) * 0.1).to(dev)
    d, qm, t = 2.2 / 127, 2.2, 1.0
    tab = None
    if table:
        geo = epilogue_table_geometry(_lib.QT_NONLINEAR, d, qm, t, saturation_level(_lib.QT_NONLINEAR, d, qm, t), False)
        tab = _lib.epi_table_build(_lib.EPI_I8, _lib.QT_NONLINEAR, _p(d, dev), _p(qm, dev), _p(t, dev), 0, *geo, dev)
    rows = torch.full((M, kpad), 91, dtype=torch.int8, device=dev)
    _lib.layernorm_quant_i8(x, gamma, beta, 1e-6, _lib.QT_NONLINEAR, _p(d, dev), _p(qm, dev), _p(t, dev), 0, rows, kpad,
                            code_table=tab)
    t32 = torch.full((_lib.t32_rows(M) * kpad,), 93, dtype=torch.int8, device=dev)
    _lib.layernorm_quant_i8_t32(x, gamma, beta, 1e-6, _lib.QT_NONLINEAR, _p(d, dev), _p(qm, dev), _p(t, dev), 0, t32,
                                kpad, code_table=tab)
    torch.cuda.synchronize()
    assert torch.equal(_lib.t32_to_rows(t32, M, kpad).cpu(), rows.cpu())
