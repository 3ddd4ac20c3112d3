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


# ---- integer deploy forward of UltraNet (the FPGA flow's arithmetic) ------------------------------------
# Per-layer bit widths of ultranet_param_gen.py:14-22 (conv 0..8) and the block structure of
# mymodel.py:71-124 (MaxPool after conv 0..3; conv 8 is the 1x1 head with bias, float out).
UN_W_BIT = [4] * 9
UN_IN_BIT = [8, 4, 4, 4, 4, 4, 4, 4, 4]
UN_OUT_BIT = [4, 4, 4, 4, 4, 4, 4, 4, 32]
UN_POOL = [True, True, True, True, False, False, False, False]


def int_threshold(acc: np.ndarray, inc: np.ndarray, bias: np.ndarray, sbits: int, out_bit: int) -> np.ndarray:
    """Integer conv+BN+activation stage: clamp(round((acc inc_q + bias_q) / 2^S), 0, 2^out_bit - 1) per
    channel (axis 0), S = w_bit - 1 + in_bit + l_shift, with the float path's round() taken half up.
    The accelerator's HLS source is not in the reference: parity of this rounding is unpinned."""
    v = acc.astype(np.int64) * inc.astype(np.int64)[:, None, None] + bias.astype(np.int64)[:, None, None]
    v = (v + (1 << (sbits - 1))) >> sbits
    return np.clip(v, 0, 2 ** out_bit - 1)


def conv_int(x: np.ndarray, w: np.ndarray, pad: int) -> np.ndarray:
    """Integer conv, stride 1: x [C][H][W], w [O][C][k][k] -> int64 [O][H][W] (zero padding)."""
    C, H, W = x.shape
    k = w.shape[2]
    xp = np.zeros((C, H + 2 * pad, W + 2 * pad), dtype=np.int64)
    xp[:, pad:pad + H, pad:pad + W] = x
    acc = np.zeros((w.shape[0], H, W), dtype=np.int64)
    for ky in range(k):
        for kx in range(k):
            acc += np.einsum("oc,chw->ohw", w[:, :, ky, kx].astype(np.int64), xp[:, ky:ky + H, kx:kx + W])
    return acc


def maxpool2(x: np.ndarray) -> np.ndarray:
    C, H, W = x.shape
    return x.reshape(C, H // 2, 2, W // 2, 2).max(axis=(2, 4))


def ultranet_int_forward(arrs, img_u8: np.ndarray, l_shift=8):
    """One uint8 image [3][H][W] through the integer flow built from a generate_params npz (arr_i in
    torch_export.py:94-131 order, read as qnn_param_reader.py does). Returns the per-layer codes
    (conv 0..7, [C][H][W]) and the head's fp32 output acc / ((2^(w_bit-1)-1)(2^in_bit-1)) + bias."""
    cnt = 0

    def take():
        nonlocal cnt
        a = np.array(arrs[f"arr_{cnt}"])
        cnt += 1
        return a

    x = img_u8.astype(np.int64)
    outs = []
    for i in range(8):
        w = weight_quantize_int(take(), UN_W_BIT[i])
        gamma, beta, mean, var, eps = take(), take(), take(), take(), take()
        inc, bias = bn_act_quantize_int(gamma, beta, mean, var, eps, w_bit=UN_W_BIT[i], in_bit=UN_IN_BIT[i],
                                        out_bit=UN_OUT_BIT[i], l_shift=l_shift)
        acc = conv_int(x, w, 1)
        x = int_threshold(acc, inc, bias, UN_W_BIT[i] - 1 + UN_IN_BIT[i] + l_shift, UN_OUT_BIT[i])
        if UN_POOL[i]:
            x = maxpool2(x)
        outs.append(x)
    w8 = weight_quantize_int(take(), UN_W_BIT[8])
    b8 = np.asarray(take(), dtype=np.float32)
    acc = conv_int(x, w8, 0)
    den = np.float32((2 ** (UN_W_BIT[8] - 1) - 1) * (2 ** UN_IN_BIT[8] - 1))
    head = acc.astype(np.float32) / den + b8[:, None, None]
    outs.append(head.astype(np.float32))
    return outs
