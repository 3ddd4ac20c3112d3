"""The reference-held known-answer vectors pushed through the HIP kernels themselves.

tests/test_oracle.py pins the CPU oracle with the same vectors; here each one goes through the C-ABI
kernel that replaces the reference function, so these kernels are pinned to the reference directly,
not only transitively through the oracle:

* KAT-3 (OTO/tests/quantization/test_quant_layers.py:80-98, DGE forward = d * round(x / d)):
  x = 0.3, d = 0.2, q_m = 1: x / d is exactly 1.5 in fp32, round-half-to-even gives code 2, value 0.4.
  Through qvit_quantize_act_i8 (codes), qvit_fake_quant_f32 (values) and qvit_pack_weight (as a weight,
  read back through an int32 GEMM on identity activation codes).
* KAT-1 / KAT-2 (4-bit quantization/quantization.py:95-100 on the array of :95; weight_quantize_int and
  weight_quantize_float, quant_ultra.py:30-56 weight_quantize_fn's arithmetic) through
  qvit_ultra_weight_codes.
* KAT-4 (quantization.py:68-89 bn_act_quantize_int on the text's parameters) through the integer-deploy
  epilogue of qvit_ultra_conv_int: the product's host folding must give the KAT's (inc_q, bias_q), and the
  kernel's clamp((acc inc + bias + 2^(S-1)) >> S) on those values must equal the oracle's integer restatement
  on every output.
"""
import numpy as np
import pytest
import torch

from oracle import quant_oracle as O
from oracle import quantization_np as Q
from quantized_vit_amd import _lib, ultra_deploy

pytestmark = pytest.mark.gpu

KAT_ARRAY = [-0.6, 0.1, -0.2, 0.5, 0.3, 0.8, -3.9]     # quantization.py:95


def _scalars(dev, *vals):
    return [torch.tensor([v], dtype=torch.float32, device=dev) for v in vals]


# x values around KAT-3: exact fp32 ties (0.3/0.2 = 1.5, 0.1/0.2 = 0.5, 0.5/0.2 = 2.5), saturation at q_m
KAT3_X = [0.3, -0.3, 0.1, -0.1, 0.5, 0.7, 0.0, 1.0, 1.3, -2.0]


def test_kat3_act_codes_and_values(dev):
    d, qm = _scalars(dev, 0.2, 1.0)
    x = torch.tensor(KAT3_X, dtype=torch.float32)
    for careful in (0, _lib.QT_FORCE_CAREFUL):
        codes = torch.zeros((1, 16), dtype=torch.int8, device=dev)
        _lib.quantize_act_i8(x.reshape(1, -1).to(dev), _lib.QT_LINEAR | careful, d, qm, None, 0, codes, 16)
        got = codes[0, :len(KAT3_X)].cpu().to(torch.int32)
        assert got[0].item() == 2 and got[1].item() == -2          # the KAT: 1.5 -> 2 (half-to-even)
        want = O.quant_codes(x, O.LINEAR, 0.2, 1.0).to(torch.int32)
        assert torch.equal(got, want), (got, want)
        assert got.tolist() == [2, -2, 0, 0, 2, 4, 0, 5, 5, -5]
        vals = _lib.fake_quant_f32(x.to(dev), _lib.QT_LINEAR | careful, d, qm, None).cpu()
        # expected = d_quant * torch.round(input / d_quant) (test_quant_layers.py:97), in fp32
        d32 = torch.tensor([0.2], dtype=torch.float32)
        assert vals[0].item() == (d32 * torch.round(torch.tensor([0.3]) / d32)).item()
        assert vals[0].item() == pytest.approx(0.4, abs=1e-7)
        assert torch.equal(vals, O.fake_quant(x, O.LINEAR, 0.2, 1.0))


@pytest.mark.parametrize("wfmt", ["W4", "W8"])
def test_kat3_weight_pack_through_gemm(dev, wfmt):
    """qvit_pack_weight on KAT-3's values, read back exactly: an int32 GEMM of identity activation codes
    gives C[m, n] = k_w[n, m]."""
    N, K = 12, 128
    w = torch.zeros(N, K)
    vals = torch.tensor(KAT3_X, dtype=torch.float32)
    for n in range(N):
        w[n, :len(KAT3_X)] = torch.roll(vals, n) * (1 if n % 2 == 0 else -1)
        w[n, 64 + n] = 0.3
    d, qm = _scalars(dev, 0.2, 1.0)
    wf = getattr(_lib, wfmt)
    overflow = torch.zeros(1, dtype=torch.int32, device=dev)
    npad = _lib.TILE_N
    packed = _lib.pack_weight(w.to(dev), _lib.QT_LINEAR, d, qm, None, wf, npad, K, overflow)
    assert int(overflow.item()) == 0
    eye = torch.eye(K, dtype=torch.int8, device=dev).contiguous()
    C = torch.zeros((K, 16), dtype=torch.int32, device=dev)
    _lib.gemm(eye, K, K, packed, wf, N, npad, None, None, None, _lib.EPI_I32, C)
    got = C[:, :N].t().cpu()
    want = O.quant_codes(w, O.LINEAR, 0.2, 1.0).to(torch.int32)
    assert torch.equal(got, want)
    assert got[0, 0].item() == 2 and got[0, 64].item() == 2       # KAT-3 as a weight code


def test_kat1_kat2_ultra_weight_codes(dev):
    w = torch.tensor(KAT_ARRAY, dtype=torch.float32).reshape(1, 7, 1, 1)   # cout 1, cin 7, 1x1
    codes = _lib.ultra_weight_codes(w.to(dev), 4, 16, 16).cpu()
    assert codes[0, :7].tolist() == [-4, 1, -1, 3, 2, 5, -7]                # KAT-1 (quantization.py:95-100)
    assert codes[0, 7:].abs().sum().item() == 0 and codes[1:].abs().sum().item() == 0
    codes3, vals3 = _lib.ultra_weight_codes(w.to(dev), 3, 16, 16, values=True)
    assert codes3[0, :7].cpu().tolist() == [-2, 0, -1, 1, 1, 2, -3]          # KAT-2 codes
    np.testing.assert_allclose(vals3.cpu().reshape(-1).double().numpy(),
                               np.array([-2, 0, -1, 1, 1, 2, -3]) / 3.0, rtol=0, atol=1e-7)
    # the product's host restatement agrees with the reference arithmetic (quantization.py:24-31)
    assert ultra_deploy.weight_quantize_int(np.array(KAT_ARRAY), 4).tolist() == [-4, 1, -1, 3, 2, 5, -7]


def _float_bits_chunk(c: int, log2n: int = 26) -> torch.Tensor:
    """The 2^log2n fp32 values whose bit patterns are c * 2^log2n ... (c + 1) * 2^log2n - 1."""
    ints = torch.arange(1 << log2n, dtype=torch.int64) + (c << log2n)
    ints = torch.where(ints >= 2 ** 31, ints - 2 ** 32, ints).to(torch.int32)
    return ints.view(torch.float32)


def _same_bits_or_both_nan(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return (a.view(torch.int32) == b.view(torch.int32)) | (torch.isnan(a) & torch.isnan(b))


def test_gelu_bit_exact_all_floats(dev):
    """nn.GELU (vit_model.py:173) on the device (qvit_gelu_f32 = the gelu_ref the fc1 code-table epilogue is built
    from) equals the oracle's GELU (torch's ATen CPU kernel, oracle/quant_oracle.py:gelu) bit for bit on EVERY
    fp32 input: all 2^32 bit patterns (NaNs compared as NaN). VERDICT r03 #1: the fc2 input sits at GELU's flat
    minimum, where ulp differences of two GELU evaluations flipped codes wholesale."""
    bad = 0
    for c in range(64):
        x = _float_bits_chunk(c)
        want = O.gelu(x)
        got = _lib.gelu_f32(x.to(dev)).cpu()
        ok = _same_bits_or_both_nan(got, want)
        if not bool(ok.all()):
            i = int((~ok).nonzero()[0])
            bad += int((~ok).sum())
            print(f"chunk {c}: first mismatch x={x[i].item()!r} got={got[i].item()!r} want={want[i].item()!r}")
    assert bad == 0, f"{bad} fp32 inputs where the device GELU differs from the oracle's"


@pytest.mark.parametrize("pool", [False, True])
def test_kat4_integer_deploy_epilogue(dev, pool):
    inc2, bias2 = ultra_deploy.bn_act_quantize_int(np.array([1, .5]), np.array([0, .1]), np.array([0, .2]),
                                                   np.array([1, 4]), 1e-5, w_bit=4, in_bit=4, out_bit=4, l_shift=8)
    assert inc2.tolist() == [4681, 1170] and bias2.tolist() == [0, 24576]   # KAT-4 (quantization.py:68-89)
    cin, cout, H, W, sbits = 16, 32, 12, 12, 4 - 1 + 4 + 8
    inc = np.tile(inc2, cout // 2).astype(np.int32)
    bias = np.tile(bias2, cout // 2).astype(np.int32)
    rng = np.random.default_rng(7)
    x = rng.integers(0, 16, size=(cin, H, W)).astype(np.int64)
    # sparse weights keep acc = sum x w in the range where the threshold codes are not all saturated
    wv = rng.integers(-7, 8, size=(cout, cin, 3, 3)) * (rng.random((cout, cin, 3, 3)) < 0.04)
    want = Q.int_threshold(Q.conv_int(x, wv, 1), inc, bias, sbits, 4)
    if pool:
        want = Q.maxpool2(want)
    assert len(np.unique(want)) >= 8                                        # a spread of codes, not all 0 / 15
    xd = torch.from_numpy(x.transpose(1, 2, 0)[None].astype(np.int8)).contiguous().to(dev)
    kpad = (9 * cin + 63) // 64 * 64                                        # K order (ky, kx, c), zero padded
    wk = np.zeros((cout, kpad), dtype=np.int8)
    wk[:, :9 * cin] = wv.transpose(0, 2, 3, 1).reshape(cout, -1)
    wd = torch.from_numpy(wk).to(dev)
    got = _lib.ultra_conv_int(xd, 3, wd, cout, torch.from_numpy(inc).to(dev), torch.from_numpy(bias).to(dev),
                              sbits, 4, pool)
    got = got[0].permute(2, 0, 1).cpu().numpy().astype(np.int64)
    assert np.array_equal(got, want)
