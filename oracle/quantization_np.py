"""ORACLE — test infrastructure only. NumPy restatement of `4-bit quantization/quantization.py`
(the reference's integer deploy semantics for the UltraNet 4-bit path) and of the DoReFa
quantizers in `4-bit quantization/quant_ultra.py`. Pinned by the known-answer values SURVEY.md §4
derives from the reference text (KAT-1, KAT-2, KAT-4).
"""
from __future__ import annotations

import numpy as np


def uniform_quantize(x: np.ndarray, bit: int = 2) -> np.ndarray:
    """quantization.py:5-9 — round(x * (2^bit - 1)) / (2^bit - 1) (np.round = half-to-even)."""
    n = float(2 ** bit - 1)
    return np.round(x * n) / n


def weight_quantize_float(x: np.ndarray, bit: int = 2) -> np.ndarray:
    """quantization.py:13-19 — tanh, max-abs normalisation, (bit-1)-bit uniform quantizer."""
    w = np.tanh(x)
    w = w / np.max(np.abs(w))
    return uniform_quantize(w, bit=bit - 1)


def weight_quantize_int(x: np.ndarray, bit: int = 2) -> np.ndarray:
    """quantization.py:24-31 — integer weight codes in [-(2^(bit-1)-1), 2^(bit-1)-1]."""
    w = np.tanh(x)
    w = w / np.max(np.abs(w))
    q = w * (2 ** (bit - 1) - 1)
    return np.round(q).astype(np.int32)


def bn_act_w_bias_float(gamma, beta, mean, var, eps):
    """quantization.py:34-46 — BN folding with sqrt(var) + eps (NOT sqrt(var + eps))."""
    w = gamma / (np.sqrt(var) + eps)
    b = beta - (mean / (np.sqrt(var) + eps) * gamma)
    return w, b


def bn_act_quantize_int(gamma, beta, mean, var, eps, w_bit=2, in_bit=4, out_bit=4, l_shift=4):
    """quantization.py:68-89 — integer BN+activation threshold parameters (inc_q, bias_q)."""
    w, b = bn_act_w_bias_float(gamma, beta, mean, var, eps)
    n = 2 ** (w_bit - 1 + in_bit + l_shift) / ((2 ** (w_bit - 1) - 1) * (2 ** in_bit - 1))
    inc_q = np.round((2 ** out_bit - 1) * n * w).astype(np.int32)
    bias_q = (2 ** (w_bit - 1) - 1) * (2 ** in_bit - 1) * (2 ** out_bit - 1) * n * b
    bias_q = np.round(bias_q).astype(np.int32)
    return inc_q, bias_q


def array_to_string(array, elem_bit: int) -> int:
    """qnn_mem_process.py:11-24 — packs element i into bits [elem_bit*i, elem_bit*(i+1)),
    negatives in two's complement. This is the reference's only packed-int4 word format."""
    val = 0
    for i, v in enumerate(array):
        v = int(v)
        if v < 0:
            v = 2 ** elem_bit + v
        val += v * 2 ** (elem_bit * i)
    return val
