"""UltraNet integer deploy path on the GPU.

The reference's FPGA flow (`4-bit quantization/`) turns the trained UltraNet into integer parameters —
weight codes (quantization.py:24-31 weight_quantize_int), per-channel BN+activation thresholds
inc_q / bias_q (quantization.py:68-89 bn_act_quantize_int, BN folded with sqrt(var) + eps), read in the
npz export order (qnn_param_reader.py:8-85 over torch_export.py:94-131's generate_params) with the
per-layer bit widths of ultranet_param_gen.py:14-22 — and runs conv + BN + activation in integers:

    code = clamp(round((acc * inc_q + bias_q) / 2^S), 0, 2^out_bit - 1),   S = w_bit - 1 + in_bit + l_shift

Layer 0 takes the 8-bit image itself (in_bit 8); the 1x1 head (out_bit 32) stays float:
acc / ((2^(w_bit-1)-1)(2^in_bit-1)) + bias, then the YOLO decode (mymodel.py:47-60). Every layer here is a
HIP kernel of libqvit_hip.so (qvit_ultra_conv0_int, qvit_ultra_conv_int, qvit_ultra_conv,
qvit_yolo_decode); the host only prepares the integer parameters once, as the reference's scripts do.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from . import _lib

# ultranet_param_gen.py:14-22 (conv 0..8)
W_BIT = [4] * 9
IN_BIT = [8, 4, 4, 4, 4, 4, 4, 4, 4]
OUT_BIT = [4, 4, 4, 4, 4, 4, 4, 4, 32]
L_SHIFT = [8] * 9
POOL = [True, True, True, True, False, False, False, False]   # mymodel.py:71-124: MaxPool after conv 0..3
CONV_SHAPES = [(3, 16), (16, 32), (32, 64), (64, 64), (64, 64), (64, 64), (64, 64), (64, 64)]


def weight_quantize_int(x: np.ndarray, bit: int) -> np.ndarray:
    """quantization.py:24-31: rne(tanh(w) / max|tanh(w)| * (2^(bit-1) - 1)) as int32."""
    w = np.tanh(x)
    w = w / np.max(np.abs(w))
    return np.round(w * (2 ** (bit - 1) - 1)).astype(np.int32)


def bn_act_quantize_int(gamma, beta, mean, var, eps, w_bit: int, in_bit: int, out_bit: int, l_shift: int):
    """quantization.py:68-89: (inc_q, bias_q) int32 with BN folded as gamma / (sqrt(var) + eps)."""
    w = gamma / (np.sqrt(var) + eps)
    b = beta - (mean / (np.sqrt(var) + eps) * gamma)
    n = 2 ** (w_bit - 1 + in_bit + l_shift) / ((2 ** (w_bit - 1) - 1) * (2 ** in_bit - 1))
    inc_q = np.round((2 ** out_bit - 1) * n * w).astype(np.int32)
    bias_q = np.round((2 ** (w_bit - 1) - 1) * (2 ** in_bit - 1) * (2 ** out_bit - 1) * n * b).astype(np.int32)
    return inc_q, bias_q


def _round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


class UltraNetIntDeploy:
    """Integer-parameter UltraNet on the GPU, built from a generate_params npz (path or dict of arrays)."""

    def __init__(self, npz: Union[str, Dict[str, np.ndarray]], device: torch.device,
                 l_shift: Optional[Sequence[int]] = None):
        arrs = np.load(npz, allow_pickle=False) if isinstance(npz, str) else npz
        self.device = device
        self.l_shift = list(l_shift) if l_shift is not None else list(L_SHIFT)
        cnt = 0

        def take():
            nonlocal cnt
            a = np.array(arrs[f"arr_{cnt}"])
            cnt += 1
            return a

        self.layers: List[dict] = []
        for i, (cin, cout) in enumerate(CONV_SHAPES):
            w = take()
            if w.shape != (cout, cin, 3, 3):
                raise ValueError(f"conv {i}: weight shape {w.shape}, expected {(cout, cin, 3, 3)}")
            gamma, beta, mean, var, eps = take(), take(), take(), take(), take()
            codes = weight_quantize_int(w, W_BIT[i])
            inc, bias = bn_act_quantize_int(gamma, beta, mean, var, eps, W_BIT[i], IN_BIT[i], OUT_BIT[i],
                                            self.l_shift[i])
            L = {"cin": cin, "cout": cout, "codes": codes,
                 "sbits": W_BIT[i] - 1 + IN_BIT[i] + self.l_shift[i], "out_bit": OUT_BIT[i], "pool": POOL[i],
                 "inc": torch.from_numpy(inc).to(device), "bias": torch.from_numpy(bias).to(device)}
            if i == 0:   # reference layout [16][3][3][3]
                L["w"] = torch.from_numpy(codes.astype(np.int8)).contiguous().to(device)
            else:        # kernel layout [round_up(cout, 16)][kpad], K order (ky, kx, c)
                L["w"] = self._k_order(codes, cin, cout, 3)
            self.layers.append(L)
        w8 = take()
        if w8.shape != (36, 64, 1, 1):
            raise ValueError(f"conv 8: weight shape {w8.shape}, expected (36, 64, 1, 1)")
        b8 = take()
        self.head_codes = weight_quantize_int(w8, W_BIT[8])
        self.head_w = self._k_order(self.head_codes, 64, 36, 1)
        self.head_bias = torch.from_numpy(np.asarray(b8, dtype=np.float32)).to(device)
        from .ultranet import YOLOLayer
        self.yolo = YOLOLayer([[20, 20], [20, 20], [20, 20], [20, 20], [20, 20], [20, 20]]).eval()  # mymodel.py:65

    def _k_order(self, codes: np.ndarray, cin: int, cout: int, ks: int) -> torch.Tensor:
        kdim = ks * ks * cin
        kpad = _round_up(kdim, 64)
        out = np.zeros((_round_up(cout, 16), kpad), dtype=np.int8)
        out[:cout, :kdim] = codes.transpose(0, 2, 3, 1).reshape(cout, kdim)   # (ky, kx, c)
        return torch.from_numpy(out).to(self.device)

    @torch.no_grad()
    def features(self, img_u8: torch.Tensor) -> List[torch.Tensor]:
        """Per-layer NHWC codes (layers 0..7) and the head's fp32 NHWC output."""
        if not img_u8.is_cuda or img_u8.dtype != torch.uint8:
            raise _lib.QvitError("UltraNetIntDeploy takes a uint8 image tensor on a ROCm device")
        outs = []
        L0 = self.layers[0]
        x = _lib.ultra_conv0_int(img_u8.contiguous(), L0["w"], L0["inc"], L0["bias"], L0["sbits"], L0["out_bit"])
        outs.append(x)
        for L in self.layers[1:]:
            x = _lib.ultra_conv_int(x, 3, L["w"], L["cout"], L["inc"], L["bias"], L["sbits"], L["out_bit"], L["pool"])
            outs.append(x)
        head = _lib.ultra_conv(x, 1, self.head_w, 36, W_BIT[8], IN_BIT[8], None, self.head_bias, _lib.ULTRA_F32)
        outs.append(head)
        return outs

    @torch.no_grad()
    def __call__(self, img_u8: torch.Tensor):
        """(io [B, 6*ny*nx, 6], p [B, 6, ny, nx, 6]) as YOLOLayer.forward in eval (mymodel.py:47-60)."""
        head = self.features(img_u8)[-1]
        return self.yolo.decode_nhwc(head, img_u8.shape[-2:])
