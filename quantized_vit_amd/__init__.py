"""quantized_vit_amd — MI355X-native 4-bit QuantizeLinear / QuantizeConv2d forward path.

Drop-in for LongAoTianxia/Quantized_ViT's quantized layers (OTO/quantization/quant_layers.py,
quant_model.py) and its ViT caller (QViT_with_GETA/vit_model.py), computed by hand-written
gfx950 HIP kernels in libqvit_hip.so (C-ABI: include/qvit_hip.h).
"""
from . import _lib
from .quant_layers import (
    LAYER_TO_QUANTLAYER,
    NanInGradientError,
    QuantizationMode,
    QuantizationType,
    QuantizeConv2d,
    QuantizeLinear,
    QuantizeMixin,
    initialize_quant_layer,
)
from .quant_model import get_bitwidth_dict, get_quant_param_dict, model_to_quantize_model

__all__ = [
    "LAYER_TO_QUANTLAYER", "NanInGradientError", "QuantizationMode", "QuantizationType", "QuantizeConv2d",
    "QuantizeLinear", "QuantizeMixin", "initialize_quant_layer", "get_bitwidth_dict", "get_quant_param_dict",
    "model_to_quantize_model",
]
