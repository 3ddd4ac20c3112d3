"""Checkpoint conversion and on-disk formats (quantized_vit_amd/convert.py) and the
UltraNet integer-deploy parameter generation (quantized_vit_amd/ultra_deploy.py, F4) on the CPU.

Pinned by: the reference's own comment examples (array_to_string, qnn_mem_process.py:10-12), the
oracle's restatement of array_to_string / weight_quantize_int / bn_act_quantize_int, round trips, and
the state_dict keys of this package's mirror (same keys as the reference's)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import quantization_np as Q
from quantized_vit_amd import convert, ultra_deploy, vit_model
from quantized_vit_amd.quant_layers import QuantizationMode, QuantizationType, QuantizeLinear
from quantized_vit_amd.quant_model import model_to_quantize_model
from quantized_vit_amd.ultranet import UltraNetQua


def _pruned_quantized_vit(qtype=QuantizationType.SYMMETRIC_NONLINEAR, mode=QuantizationMode.WEIGHT_AND_ACTIVATION):
    torch.manual_seed(3)
    m = vit_model.VisionTransformer(img_size=64, patch_size=16, embed_dim=192, depth=3, num_heads=3,
                                    num_classes=11)
    prune = [(2, 500), (3, 768), (1, 64)]          # (heads, mlp hidden) per block, as GETA leaves them
    for blk, (h, hid) in zip(m.blocks, prune):
        blk.attn.qkv = nn.Linear(192, 3 * h * 64)
        blk.attn.proj = nn.Linear(h * 64, 192)
        blk.attn.num_heads = h
        blk.mlp.fc1 = nn.Linear(192, hid)
        blk.mlp.fc2 = nn.Linear(hid, 192)
    m = model_to_quantize_model(m, num_bits=4, quant_type=qtype, quant_mode=mode)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "quant" in n or "q_m" in n:
                p.copy_(torch.rand(1) + 0.05)
    return m.eval(), prune


@pytest.mark.parametrize("qtype", [QuantizationType.SYMMETRIC_NONLINEAR, QuantizationType.SYMMETRIC_LINEAR])
def test_vit_from_pruned_state_dict(qtype):
    m, prune = _pruned_quantized_vit(qtype)
    sd = m.state_dict()
    cfg = convert.vit_config_from_state_dict(sd)
    assert (cfg["img_size"], cfg["patch_size"], cfg["embed_dim"], cfg["depth"], cfg["num_classes"]) == (64, 16, 192, 3, 11)
    assert [(b["heads"], b["hidden"]) for b in cfg["blocks"]] == prune
    assert cfg["quant_type"] == qtype and cfg["quant_mode"] == QuantizationMode.WEIGHT_AND_ACTIVATION
    m2 = convert.vit_from_state_dict(sd)
    sd2 = m2.state_dict()
    assert sd.keys() == sd2.keys()
    for k in sd:
        assert torch.equal(sd[k], sd2[k]), k
    for b1, b2 in zip(m.blocks, m2.blocks):
        assert isinstance(b2.attn.qkv, QuantizeLinear) and b2.attn.num_heads == b1.attn.num_heads
        assert b2.attn.scale == b1.attn.scale   # head_dim (and the softmax scale) survive head pruning
        assert b2.mlp.fc1.out_features == b1.mlp.fc1.out_features


def test_vit_weight_only_state_dict():
    m, _ = _pruned_quantized_vit(mode=QuantizationMode.WEIGHT_ONLY)
    m2 = convert.vit_from_state_dict(m.state_dict())
    assert m2.blocks[0].mlp.fc1.quant_mode == QuantizationMode.WEIGHT_ONLY


def test_load_reference_checkpoint(tmp_path):
    m, _ = _pruned_quantized_vit()
    p = tmp_path / "sd.pt"
    torch.save(m.state_dict(), p)
    assert convert.load_reference_checkpoint(str(p)).state_dict().keys() == m.state_dict().keys()
    p2 = tmp_path / "wrapped.pt"
    torch.save({"model": m.state_dict(), "epoch": 3}, p2)
    assert convert.load_reference_checkpoint(str(p2)).state_dict().keys() == m.state_dict().keys()
    p3 = tmp_path / "module.pt"          # a whole pickled module (predict.py:43): refused, never unpickled
    torch.save(m, p3)
    with pytest.raises(ValueError, match="state_dict"):
        convert.load_reference_checkpoint(str(p3))


def test_ultranet_npz_roundtrip():
    torch.manual_seed(0)
    m = UltraNetQua()
    with torch.no_grad():
        for bn in m.modules():
            if isinstance(bn, nn.BatchNorm2d):
                bn.running_mean.uniform_(-0.1, 0.1)
                bn.running_var.uniform_(0.5, 2.0)
    d = convert.ultranet_to_npz(m)
    # torch_export.py:137-140: arr_0 conv0 weight, arr_1 BN0 gamma, ...; 8 x (w + 5 BN) + head (w, bias)
    assert len(d) == 8 * 6 + 2
    assert d["arr_0"].shape == (16, 3, 3, 3) and d["arr_1"].shape == (16,)
    assert float(d["arr_5"]) == 1e-5 and d["arr_48"].shape == (36, 64, 1, 1) and d["arr_49"].shape == (36,)
    m2 = convert.ultranet_from_npz(d)
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        if a.is_floating_point():
            assert torch.equal(a, b), k
    d_extra = dict(d, arr_50=np.zeros(1))
    with pytest.raises(ValueError):
        convert.ultranet_from_npz(d_extra)


def test_simd_word_packing_known_answers():
    assert convert.pack_simd_word([1, 1, 1], 1) == 0b111          # qnn_mem_process.py:10-12 comment
    assert convert.pack_simd_word([-1, 2], 4) == 0x2F
    assert convert.pack_simd_word([7, -8, 0, 1], 4) == 0x1087
    rng = np.random.default_rng(0)
    for bits in (2, 4, 8):
        v = rng.integers(-(2 ** (bits - 1)), 2 ** (bits - 1), size=37)
        assert convert.pack_simd_word(v, bits) == Q.array_to_string(v, bits)
        assert convert.unpack_simd_word(convert.pack_simd_word(v, bits), 37, bits) == list(v)


def test_hls_weight_layout():
    w = np.array([[1, 2, 3, 4], [5, 6, 7, 8]])
    assert convert.hls_pack_weights(w, 4, pe=2, simd=2) == [[0x21, 0x43], [0x65, 0x87]]
    rng = np.random.default_rng(1)
    for (o, k, pe, simd) in [(16, 27, 16, 3), (32, 144, 8, 16), (36, 64, 2, 8), (8, 10, 4, 4)]:
        codes = rng.integers(-7, 8, size=(o, k))
        res = convert.hls_pack_weights(codes, 4, pe, simd)
        assert len(res) == pe and len(res[0]) == (o // pe) * ((k + simd - 1) // simd)
        assert np.array_equal(convert.hls_unpack_weights(res, o, k, 4, pe, simd), codes)
    conv = rng.integers(-7, 8, size=(4, 3, 3, 3))
    m = convert.hls_weight_matrix(conv)
    assert m.shape == (4, 27) and m[1, 5] == conv[1, 2, 0, 1]   # (ky, kx, c) order: k = (0*3+1)*3 + 2
    inc, bias = convert.hls_inc_bias(np.arange(8), np.arange(8) * 10, pe=4)
    assert inc.tolist() == [[0, 4], [1, 5], [2, 6], [3, 7]] and bias[1, 1] == 50


def test_int_deploy_params_match_reference_restatement():
    rng = np.random.default_rng(2)
    w = rng.normal(0, 0.1, size=(64, 32, 3, 3)).astype(np.float32)
    assert np.array_equal(ultra_deploy.weight_quantize_int(w, 4), Q.weight_quantize_int(w, 4))
    g, b = rng.uniform(0.1, 0.4, 64).astype(np.float32), rng.uniform(0.3, 0.7, 64).astype(np.float32)
    mu, var = rng.normal(0, 0.3, 64).astype(np.float32), rng.uniform(0.2, 2, 64).astype(np.float32)
    for ib, ls in ((8, 8), (4, 8), (4, 0)):
        mine = ultra_deploy.bn_act_quantize_int(g, b, mu, var, np.float32(1e-5), 4, ib, 4, ls)
        ref = Q.bn_act_quantize_int(g, b, mu, var, np.float32(1e-5), w_bit=4, in_bit=ib, out_bit=4, l_shift=ls)
        assert np.array_equal(mine[0], ref[0]) and np.array_equal(mine[1], ref[1])


def test_int_threshold_oracle_known_answers():
    # round half up of (acc inc + bias) / 2^S, clamped to [0, 15]
    acc = np.array([[[0, 1, 2, 3, 100, -5]]])
    out = Q.int_threshold(acc, np.array([3]), np.array([1]), 2, 4)
    assert out.tolist() == [[[0, 1, 2, 3, 15, 0]]]   # (1+2)>>2=0, (4+2)>>2=1, (7+2)>>2=2, (10+2)>>2=3
