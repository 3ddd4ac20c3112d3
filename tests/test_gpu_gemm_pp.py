"""The ping-pong int8-code GEMM schedule (gemm_pp_kernel: two 4-wave halves of one workgroup alternate between
matrix and DMA / epilogue intervals) against the two-block schedule (gemm_kernel) it replaces for fc1-class
layers (quant_layers.py:495-499 QuantizeLinear.forward -> fc2's activation quantizer, vit_model.py:173 GELU).

Both run the same integer MFMA contraction and the same per-element epilogue, so the codes must be identical
bit for bit; QVIT_GEMM_PP=0 selects gemm_kernel for the comparison. The shapes cover the model's fc1 (ViT-B b256
and a ViT-L-width slice), ragged M (a partial last row tile, fewer tiles than workgroups, one tile per
workgroup), N below the padded width (dropped columns), K from 12 to 48 stages, W8 weights, no bias, and the
direct quantizer (no code table) as well as the table path. The oracle check of the same kernel is
test_gpu_kernels.py::test_gemm_int8_code_epilogue (K = 768 takes this schedule).
"""
import os

import pytest
import torch

from oracle import quant_oracle as O
from quantized_vit_amd import _lib
from test_gpu_kernels import QT, _p, act_buffer, pack_codes

pytestmark = pytest.mark.gpu


def _run(dev, pp, A, M, kpad, packed, wfmt, N, npad, bias_pad, epi, ldc, kw, table):
    out = torch.full((M, ldc), 99, dtype=torch.int8, device=dev)
    old = os.environ.get("QVIT_GEMM_PP")
    os.environ["QVIT_GEMM_PP"] = "1" if pp else "0"
    try:
        _lib.gemm(A, M, kpad, packed, wfmt, N, npad, _p(0.004, dev), _p(0.0011, dev), bias_pad, epi, out,
                  epi_table=table, **kw)
        torch.cuda.synchronize()
    finally:
        if old is None:
            del os.environ["QVIT_GEMM_PP"]
        else:
            os.environ["QVIT_GEMM_PP"] = old
    return out.cpu()


CASES = [
    # M, N, K, wfmt, gelu, table, bias
    (50432, 3072, 768, _lib.W4, True, True, True),     # ViT-B/16 b256 fc1
    (4099, 4096, 1024, _lib.W4, True, True, True),     # ViT-L fc1 width, ragged M
    (300, 640, 768, _lib.W4, True, True, True),        # N < npad: dropped columns
    (128, 3072, 768, _lib.W4, True, True, True),       # one row tile: <= 1 tile per workgroup
    (1000, 768, 3072, _lib.W4, False, True, True),     # 48 stages per tile, plain quantizer
    (2049, 1024, 768, _lib.W8, True, True, False),     # int8 weights, no bias
    (1500, 1536, 768, _lib.W4, True, False, True),     # direct quantizer (no table)
    (777, 768, 1536, _lib.W4, False, False, True),     # direct, plain
]


@pytest.mark.parametrize("M,N,K,wfmt,gelu,use_table,use_bias", CASES)
def test_pingpong_equals_two_block_schedule(dev, M, N, K, wfmt, gelu, use_table, use_bias):
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randint(-127, 128, (M, K), generator=g)
    lim = 8 if wfmt == _lib.W4 else 21   # W8: a code range that keeps the epilogue values inside the quantizer's
    w = torch.randint(-lim, lim, (N, K), generator=g)
    packed, npad, kpad = pack_codes(w, wfmt, dev)
    bias_pad = _lib.pad_bias((torch.randn(N, generator=g) * 0.5).to(dev), N, npad, dev) if use_bias else None
    qt, t, qmn = O.NONLINEAR, 1.0, 1.4
    dn = qmn ** t / 127
    qtc = QT[qt]
    kw = dict(out_qtype=qtc, out_d=_p(dn, dev), out_qm=_p(qmn, dev), out_t=_p(t, dev))
    epi = _lib.EPI_I8_GELU if gelu else _lib.EPI_I8
    table = None
    if use_table:
        L = saturation_level(qtc, dn, qmn, t)
        geo = epilogue_table_geometry(qtc, dn, qmn, t, L, gelu)
        table = _lib.epi_table_build(epi, qtc, kw["out_d"], kw["out_qm"], kw["out_t"], 0, *geo, dev)
    A = act_buffer(a, kpad, dev)
    ldc = (N + 15) // 16 * 16
    two_block = _run(dev, False, A, M, kpad, packed, wfmt, N, npad, bias_pad, epi, ldc, kw, table)
    pingpong = _run(dev, True, A, M, kpad, packed, wfmt, N, npad, bias_pad, epi, ldc, kw, table)
    assert len(torch.unique(two_block[:, :N])) > 20
    assert torch.equal(pingpong[:, :N], two_block[:, :N])
    assert (pingpong[:, N:] == 99).all()   # nothing written past N
