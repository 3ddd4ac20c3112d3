"""Synthetic-model setup: activation-range calibration and quantized ViT construction.

The reference initialises a layer's activation quantizer from the WEIGHT statistics
(quant_layers.py:436-438), which saturates almost every activation; trained GETA checkpoints carry
learned values instead. For synthetic benchmarks and parity tests we set them the way GETA's
projection does (optimizer/geta.py:788-804, d = exp(t log|q_m|) / (2^(b-1) - 1)) from q_m = max|x|
of each layer's input on a calibration batch of the un-quantized model.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn as nn

from .quant_layers import QuantizationMode, QuantizationType, QuantizeConv2d, QuantizeLinear
from .quant_model import model_to_quantize_model
from . import vit_model


@torch.no_grad()
def collect_input_absmax(model: nn.Module, x: torch.Tensor) -> Dict[str, float]:
    """max|input| of every nn.Linear / nn.Conv2d (by module name) over one forward of `x`."""
    stats: Dict[str, float] = {}
    hooks = []
    for name, mod in model.named_modules():
        if isinstance(mod, (nn.Linear, nn.Conv2d)):
            def hook(m, inp, out, name=name):
                v = float(inp[0].detach().abs().max())
                stats[name] = max(stats.get(name, 0.0), v)
            hooks.append(mod.register_forward_hook(hook))
    try:
        model(x)
    finally:
        for h in hooks:
            h.remove()
    return stats


def d_quant_for_bits(bits: int, q_m: float, t: float = 1.0) -> float:
    """GETA._d_quant_helper, optimizer/geta.py:788-804."""
    return math.exp(t * math.log(abs(q_m))) / (2 ** (bits - 1) - 1)


@torch.no_grad()
def set_activation_quant(model: nn.Module, absmax: Dict[str, float], bits: int = 8, t: float = 1.0) -> None:
    for name, mod in model.named_modules():
        if isinstance(mod, (QuantizeLinear, QuantizeConv2d)) and \
                mod.quant_mode == QuantizationMode.WEIGHT_AND_ACTIVATION and name in absmax:
            qm = max(absmax[name], 1e-8)
            mod.q_m_act.fill_(qm)
            mod.d_quant_act.fill_(d_quant_for_bits(bits, qm, t))
            if hasattr(mod, "t_quant_act"):
                mod.t_quant_act.fill_(t)
            mod.invalidate()


@torch.no_grad()
def set_weight_quant_t(model: nn.Module, t: float, bits: int = 4) -> None:
    """Re-derives the weight quantizer for a given t (d = max|W|^t / (2^(b-1) - 1))."""
    for mod in model.modules():
        if isinstance(mod, (QuantizeLinear, QuantizeConv2d)) and hasattr(mod, "t_quant_wt"):
            qm = float(mod.q_m_wt)
            mod.t_quant_wt.fill_(t)
            mod.d_quant_wt.fill_(d_quant_for_bits(bits, qm, t))
            mod.invalidate()


@torch.no_grad()
def redraw_init_artifacts(model: nn.Module, limit: float = 1.0) -> int:
    """Re-draws the sampling artifacts of torch.nn.init.trunc_normal_ in a freshly initialised ViT.

    _init_vit_weights (vit_model.py:331-346) draws Linear weights from trunc_normal_(std=.01) and the class / position
    embeddings from trunc_normal_(std=.02), truncated at the absolute bounds [-2, 2] (200 / 100 sigma). torch samples it
    by inverse CDF: uniform_(-1, 1) then erfinv_; a uniform draw of exactly -1 (about 2^-24 per element) becomes -inf and
    is clamped to -2.0. So a ViT-L/16 holds a dozen weights of exactly +-2.0 (12 layers at seed 0, the head among
    them), values the intended distribution gives with probability ~0. Under the per-tensor max quantizer
    (initialize_quant_layer: d = max|W| / 7) such a layer's int4 codes are all 0 but one: the head then has one
    nonzero weight, the logits depend on a single activation code per image, and any logits comparison becomes a coin
    toss on that code's rounding. Every element with |w| >= `limit` (50-100 sigma) is re-drawn from the intended
    normal with the global generator (deterministic for a seed; a model without artifacts is left unchanged).
    Returns the number of elements re-drawn."""
    n = 0
    for name, p in model.named_parameters():
        std = 0.02 if name in ("pos_embed", "cls_token", "dist_token") else 0.01
        if not (name.endswith("weight") and p.dim() == 2) and std == 0.01:
            continue
        mask = p.abs() >= limit
        while bool(mask.any()):
            k = int(mask.sum())
            n += k
            p[mask] = torch.randn(k) * std
            mask = p.abs() >= limit
    return n


VIT_CONFIGS = {
    "vit_tiny_patch16_224": dict(img_size=224, patch_size=16, embed_dim=192, depth=12, num_heads=3),
    "vit_base_patch16_224": dict(img_size=224, patch_size=16, embed_dim=768, depth=12, num_heads=12),
    "vit_large_patch16_384": dict(img_size=384, patch_size=16, embed_dim=1024, depth=24, num_heads=16),
}


@torch.no_grad()
def build_quantized_vit(name: str = "vit_base_patch16_224", num_classes: int = 1000, seed: int = 0,
                        w_bits: int = 4, a_bits: int = 8,
                        quant_type: QuantizationType = QuantizationType.SYMMETRIC_NONLINEAR,
                        t_act: float = 1.0, t_wt: float = 1.0, calib_batch: int = 2, calib_seed: int = 1,
                        device: Optional[torch.device] = None, depth: Optional[int] = None) -> nn.Module:
    """Random-init ViT (reference init, vit_model.py:331-346), swapped to W{w_bits}A{a_bits} fake-quant
    layers (model_to_quantize_model with num_bits=w_bits, WEIGHT_AND_ACTIVATION) and calibrated.

    Calibration runs the fp32 model on `calib_batch` uniform[-1,1) images (seed calib_seed) on
    `device` (CPU if None) before the swap. Deterministic for a given seed and device."""
    cfg = dict(VIT_CONFIGS[name])
    if depth is not None:
        cfg["depth"] = depth
    g = torch.manual_seed(seed)
    model = vit_model.VisionTransformer(num_classes=num_classes, representation_size=None, **cfg)
    redraw_init_artifacts(model)
    dev = device or torch.device("cpu")
    model = model.to(dev).eval()
    gen = torch.Generator(device="cpu").manual_seed(calib_seed)
    img = (torch.rand(calib_batch, 3, cfg["img_size"], cfg["img_size"], generator=gen) * 2 - 1).to(dev)
    absmax = collect_input_absmax(model, img)
    model = model_to_quantize_model(model, num_bits=w_bits, quant_type=quant_type,
                                    quant_mode=QuantizationMode.WEIGHT_AND_ACTIVATION)
    if t_wt != 1.0:
        set_weight_quant_t(model, t_wt, w_bits)
    set_activation_quant(model, absmax, bits=a_bits, t=t_act)
    del g
    return model.eval()


def synthetic_images(batch: int, img_size: int, seed: int = 0, device=None) -> torch.Tensor:
    """uniform[-1,1) NCHW images (predict.py:15-19 normalisation range), seeded on the CPU."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.rand(batch, 3, img_size, img_size, generator=gen) * 2 - 1
    return x.to(device) if device is not None else x
