"""Module surface parity with OTO/quantization/quant_layers.py and quant_model.py (CPU-only:
construction, parameters, state_dict keys, conversion, errors). Forward needs a GPU (tests_gpu)."""
import pytest
import torch
import torch.nn as nn

import quantized_vit_amd as qva
from quantized_vit_amd import _lib, vit_model
from quantized_vit_amd.quant_layers import (QuantizationMode, QuantizationType, QuantizeConv2d, QuantizeLinear,
                                            initialize_quant_layer, saturation_level)
from quantized_vit_amd.quant_model import get_bitwidth_dict, get_quant_param_dict, model_to_quantize_model


@pytest.mark.parametrize("qt", list(QuantizationType))
@pytest.mark.parametrize("mode", list(QuantizationMode))
def test_state_dict_keys_match_reference(qt, mode):
    # quant_layers.py:315-325
    m = QuantizeLinear(8, 4, bias=True, quant_type=qt, quant_mode=mode)
    keys = set(m.state_dict())
    expect = {"weight", "bias", "d_quant_wt", "q_m_wt"}
    if qt == QuantizationType.SYMMETRIC_NONLINEAR:
        expect.add("t_quant_wt")
    if mode == QuantizationMode.WEIGHT_AND_ACTIVATION:
        expect |= {"d_quant_act", "q_m_act"}
        if qt == QuantizationType.SYMMETRIC_NONLINEAR:
            expect.add("t_quant_act")
    assert keys == expect
    assert all(m.state_dict()[k].shape == (1,) for k in keys if k not in ("weight", "bias"))


def test_defaults_match_reference():
    m = QuantizeLinear(8, 4)
    assert m.quant_type == QuantizationType.SYMMETRIC_LINEAR          # :452
    assert m.quant_mode == QuantizationMode.WEIGHT_ONLY               # :453
    assert m.weight_clip_val == (-2.0, 2.0) and m.act_clip_val == (-2.0, 2.0)
    c = QuantizeConv2d(3, 8, 3)
    assert c.padding == (1, 1) and c.bias is None                      # :509, :512
    assert qva.LAYER_TO_QUANTLAYER == {"Linear": QuantizeLinear, "Conv2d": QuantizeConv2d}


def test_from_module_and_init():
    torch.manual_seed(0)
    lin = nn.Linear(64, 32)
    q = QuantizeLinear.from_module(lin, quant_type=QuantizationType.SYMMETRIC_NONLINEAR,
                                   quant_mode=QuantizationMode.WEIGHT_AND_ACTIVATION, num_bits=4)
    assert torch.equal(q.weight, lin.weight) and torch.equal(q.bias, lin.bias)
    qm = lin.weight.abs().max()
    assert torch.allclose(q.q_m_wt, qm.reshape(1))
    assert torch.allclose(q.d_quant_wt, (qm / 7).reshape(1))
    assert torch.allclose(q.q_m_act, qm.reshape(1))                   # :436-438 (from weight stats)
    assert q.t_quant_wt.item() == 1.0 and q.t_quant_act.item() == 1.0
    assert q.weight_bit == 4                                           # KAT-5 through the module
    conv = nn.Conv2d(3, 16, 16, stride=16)
    qc = QuantizeConv2d.from_module(conv, num_bits=8)
    assert qc.stride == (16, 16) and qc.padding == (0, 0) and qc.kernel_size == (16, 16)


def test_model_to_quantize_model_vit_swaps_50_layers():
    m = vit_model.vit_base_patch16_224(num_classes=10)
    m = model_to_quantize_model(m, num_bits=4, quant_type="symmetric+nonlinear", quant_mode="weight_and_activation")
    ql = [n for n, x in m.named_modules() if isinstance(x, (QuantizeLinear, QuantizeConv2d))]
    assert len(ql) == 50   # train.py:321 comment: patch_embed + 12 x 4 + head
    assert not any(type(x) in (nn.Linear, nn.Conv2d) for x in m.modules())
    pd = get_quant_param_dict(m)
    assert set(pd["blocks.0.mlp.fc1"]) == {"d_quant_wt", "q_m_wt", "t_quant_wt", "d_quant_act", "q_m_act",
                                             "t_quant_act"}
    bd = get_bitwidth_dict(pd)
    assert round(bd["blocks.0.mlp.fc1"]["weight"]) == 4


def test_bad_strings_raise_value_error():
    with pytest.raises(ValueError, match="Invalid quantization type"):
        model_to_quantize_model(nn.Linear(2, 2), quant_type="bogus")
    with pytest.raises(ValueError, match="Invalid quantization mode"):
        model_to_quantize_model(nn.Linear(2, 2), quant_mode="bogus")


def test_state_dict_roundtrip_with_reference_keys():
    a = vit_model.vit_tiny_patch16_224(num_classes=5)
    a = model_to_quantize_model(a, num_bits=4, quant_mode="weight_and_activation")
    b = vit_model.vit_tiny_patch16_224(num_classes=5)
    b = model_to_quantize_model(b, num_bits=4, quant_mode="weight_and_activation")
    b.load_state_dict(a.state_dict())
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k])


def test_cpu_forward_fails_loudly():
    q = QuantizeLinear(16, 8, quant_mode=QuantizationMode.WEIGHT_AND_ACTIVATION)
    with pytest.raises(_lib.QvitError):
        q(torch.randn(2, 16))


def test_saturation_level_host_formula():
    assert saturation_level(_lib.QT_LINEAR, 1 / 7, 1.0) == 7
    assert saturation_level(_lib.QT_NONLINEAR, 0.1, 0.7, 1.0) == 7
    assert saturation_level(_lib.QT_LINEAR, 1e-4, 10.0) == 100000


def test_initialize_quant_layer_ignores_other_modules():
    initialize_quant_layer(nn.Linear(2, 2), num_bits=4)   # no-op, as in the reference (:419-420)


def test_ultranet_state_dict_keys_match_reference():
    """UltraNetQua (mymodel.py:62-130): nn.Sequential of Conv2d_Q / BatchNorm2d / activation_quantize_fn /
    MaxPool2d, so a reference checkpoint's keys are layers.{i}.*."""
    from quantized_vit_amd.ultranet import UltraNetQua
    m = UltraNetQua()
    keys = set(m.state_dict().keys())
    conv_idx = [0, 4, 8, 12, 16, 19, 22, 25]
    want = set()
    for i in conv_idx:
        want.add(f"layers.{i}.weight")
        for k in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
            want.add(f"layers.{i + 1}.{k}")
    want |= {"layers.28.weight", "layers.28.bias"}
    assert keys == want
    assert m.layers[28].weight.shape == (36, 64, 1, 1) and m.layers[0].weight.shape == (16, 3, 3, 3)
    assert m.yololayer.na == 6 and m.yololayer.no == 6


def test_ultranet_cpu_forward_fails_loudly():
    from quantized_vit_amd import _lib
    from quantized_vit_amd.ultranet import UltraNetQua
    m = UltraNetQua().eval()
    with pytest.raises(_lib.QvitError):
        m(torch.rand(1, 3, 64, 64))


def test_trunc_normal_artifacts_redrawn():
    """torch's trunc_normal_(std=.01, a=-2, b=2) turns a uniform draw of exactly -1 into -2.0 (inverse CDF at -inf,
    clamped): ViT-L/16 at seed 0 gets twelve +-2.0 weights, which make those layers' int4 codes all zero but one under
    the per-tensor max quantizer. calibrate.redraw_init_artifacts re-draws exactly those elements; ViT-B/16 at seed 0
    has none and is left bit-identical."""
    import torch
    from quantized_vit_amd import vit_model
    from quantized_vit_amd.calibrate import VIT_CONFIGS, redraw_init_artifacts
    torch.manual_seed(0)
    vl = vit_model.VisionTransformer(num_classes=1000, representation_size=None, **VIT_CONFIGS["vit_large_patch16_384"])
    assert float(vl.head.weight.abs().max()) == 2.0
    assert redraw_init_artifacts(vl) >= 12
    assert max(float(p.abs().max()) for n, p in vl.named_parameters() if p.dim() == 2) < 0.1
    torch.manual_seed(0)
    vb = vit_model.VisionTransformer(num_classes=1000, representation_size=None, **VIT_CONFIGS["vit_base_patch16_224"])
    before = {k: v.clone() for k, v in vb.state_dict().items()}
    assert redraw_init_artifacts(vb) == 0
    assert all(torch.equal(before[k], v) for k, v in vb.state_dict().items())
