"""Module swap and parameter introspection — mirrors OTO/quantization/quant_model.py:15-136."""
from __future__ import annotations

import logging
import math
from typing import Dict, Union

import torch.nn as nn

from .quant_layers import LAYER_TO_QUANTLAYER, QuantizationMode, QuantizationType


def model_to_quantize_model(
    model: nn.Module,
    d_quant_init: float = 1e-4,
    t_quant_init: float = 1.0,
    q_m_init: float = 1.0,
    quant_init_by_module: bool = True,
    num_bits: int = 16,
    quant_type: Union[QuantizationType, str] = QuantizationType.SYMMETRIC_NONLINEAR,
    quant_mode: Union[QuantizationMode, str] = QuantizationMode.WEIGHT_ONLY,
) -> nn.Module:
    """Replaces every module whose class name is Linear / Conv2d by its quantized twin
    (quant_model.py:15-82; same defaults, same ValueError messages for bad strings)."""
    logger = logging.getLogger(__name__)
    if isinstance(quant_type, str):
        try:
            quant_type = QuantizationType(quant_type)
        except ValueError:
            raise ValueError(
                f"Invalid quantization type: {quant_type}. Must be one of {[t.value for t in QuantizationType]}")
    if isinstance(quant_mode, str):
        try:
            quant_mode = QuantizationMode(quant_mode)
        except ValueError:
            raise ValueError(
                f"Invalid quantization mode: {quant_mode}. Must be one of {[m.value for m in QuantizationMode]}")

    targets = [(name, module) for name, module in model.named_modules()
               if type(module).__name__ in LAYER_TO_QUANTLAYER]
    for name, module in targets:
        parent = model.get_submodule(".".join(name.split(".")[:-1]))
        target_name = name.split(".")[-1]
        quant_module = LAYER_TO_QUANTLAYER[type(module).__name__].from_module(
            module=module, d_quant_init=d_quant_init, t_quant_init=t_quant_init, q_m_init=q_m_init,
            quant_type=quant_type, quant_mode=quant_mode, quant_init_by_module=quant_init_by_module,
            num_bits=num_bits)
        setattr(parent, target_name, quant_module)
    logger.info(f"Converted {len(targets)} layers to quantized versions")
    return model


def get_quant_param_dict(model: nn.Module) -> Dict[str, Dict[str, float]]:
    """quant_model.py:85-101."""
    param_dict: Dict[str, Dict[str, float]] = {}
    for name, param in model.named_parameters():
        if any(q in name for q in ["d_quant", "t_quant", "q_m"]):
            layer_name = ".".join(name.split(".")[:-1])
            param_name = name.split(".")[-1]
            param_dict.setdefault(layer_name, {})[param_name] = param.item()
    return param_dict


def get_bitwidth_dict(param_dict: Dict[str, Dict[str, float]]) -> Dict[str, Dict[str, float]]:
    """quant_model.py:104-136."""
    bit_dict: Dict[str, Dict[str, float]] = {}

    def _calculate_bitwidth(d_quant: float, q_m: float, t_quant: float = 1.0) -> float:
        return math.log2(math.exp(t_quant * math.log(abs(q_m))) / abs(d_quant) + 1) + 1

    for key, params in param_dict.items():
        bit_dict[key] = {}
        bit_dict[key]["weight"] = _calculate_bitwidth(params["d_quant_wt"], abs(params["q_m_wt"]),
                                                      params.get("t_quant_wt", 1.0))
        if "d_quant_act" in params:
            bit_dict[key]["activation"] = _calculate_bitwidth(params["d_quant_act"], abs(params["q_m_act"]),
                                                              params.get("t_quant_act", 1.0))
    return bit_dict
