"""The stream-K tail of the fp32-epilogue GEMM (qvit_gemm_sk, csrc/gemm_w4a8.hip): the residual GEMMs of the fused
block, Attention.proj and Mlp.fc2 (QViT_with_GETA/vit_model.py:151,175) + Block.forward's residual adds (:206-207).

The tail only re-schedules the last partial round of tiles: their K range is split over otherwise idle workgroups and
the int32 partials are summed before the unchanged epilogue. Integer sums, so the outputs must equal qvit_gemm's
bit for bit. Checked on the production shapes (fc2 K = 3072, proj K = 768 at b256), on small M (every tile a tail
tile, split up to nk / 2 ways), on K = 128 / 256 (no split / two-way split), both weight formats, both epilogues, and
over repeated launches on one workspace (the arrival counters must come back to zero). The oracle comparison of
the b256 residual GEMMs is tests/test_gpu_production.py (which now runs through this path).
"""
import pytest
import torch

from quantized_vit_amd import _lib
from test_gpu_kernels import _p, act_buffer, pack_codes

pytestmark = pytest.mark.gpu

SHAPES = [(256 * 197, 768, 3072), (256 * 197, 768, 768), (197, 768, 3072), (1, 768, 768), (300, 256, 256),
          (1000, 768, 128), (4096, 1000, 640), (33, 3072, 768)]


def _case(dev, M, N, K, wfmt, seed):
    g = torch.Generator().manual_seed(seed)
    lvl = 7 if wfmt == _lib.W4 else 127
    a = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int16)
    w = torch.randint(-lvl - 1, lvl + 1, (N, K), generator=g, dtype=torch.int16)
    packed, npad, kpad = pack_codes(w, wfmt, dev)
    A = act_buffer(a, kpad, dev)
    bias = _lib.pad_bias((torch.randn(N, generator=g) * 0.5).to(dev), N, npad, dev)
    resid = (torch.randn(M, N, generator=g) * 2).to(dev)
    return A, packed, npad, kpad, bias, resid


@pytest.mark.parametrize("wfmt", [_lib.W4, _lib.W8])
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("epi", [_lib.EPI_F32_RESID, _lib.EPI_F32])
def test_gemm_sk_bit_identical(dev, wfmt, M, N, K, epi):
    if wfmt == _lib.W8 and M > 10000 and epi == _lib.EPI_F32:
        pytest.skip("covered by the W4 / residual production cases")
    A, packed, npad, kpad, bias, resid = _case(dev, M, N, K, wfmt, M + N + K + wfmt)
    da, dw = _p(0.0021, dev), _p(0.0173, dev)
    want = resid.clone()
    _lib.gemm(A, M, kpad, packed, wfmt, N, npad, da, dw, bias, epi, want)
    ws = torch.zeros(int(_lib.load().qvit_gemm_sk_workspace_bytes(M, kpad, A.stride(0), npad, wfmt)),
                     dtype=torch.uint8, device=dev)
    cb = ((npad // 256) * ((M + 127) // 128) * 4 + 255) // 256 * 256
    for rep in range(2):   # the second launch reuses the counters the first one left
        got = resid.clone()
        _lib.gemm_sk(A, M, kpad, packed, wfmt, N, npad, da, dw, bias, epi, got, ws)
        torch.cuda.synchronize()
        assert torch.equal(got, want), rep
        assert int(ws[:cb].view(torch.int32).abs().sum().item()) == 0   # every arrival counter back at zero


def test_gemm_sk_rejects(dev):
    A, packed, npad, kpad, bias, resid = _case(dev, 64, 256, 256, _lib.W4, 1)
    lib = _lib.load()
    need = int(lib.qvit_gemm_sk_workspace_bytes(64, kpad, A.stride(0), npad, _lib.W4))
    assert need > 0 and lib.qvit_gemm_sk_workspace_bytes(0, kpad, kpad, npad, _lib.W4) == 0
    ws = torch.zeros(need, dtype=torch.uint8, device=dev)
    da, dw = _p(1.0, dev), _p(1.0, dev)
    with pytest.raises(_lib.QvitError):   # short workspace
        _lib.gemm_sk(A, 64, kpad, packed, _lib.W4, 256, npad, da, dw, bias, _lib.EPI_F32, resid, ws[:need - 256])
    with pytest.raises(_lib.QvitError):   # not an fp32 epilogue
        _lib.gemm_sk(A, 64, kpad, packed, _lib.W4, 256, npad, da, dw, bias, _lib.EPI_I32, resid, ws)
    with pytest.raises(_lib.QvitError):   # misaligned workspace
        _lib.gemm_sk(A, 64, kpad, packed, _lib.W4, 256, npad, da, dw, bias, _lib.EPI_F32, resid, ws[16:])
    torch.cuda.synchronize()
