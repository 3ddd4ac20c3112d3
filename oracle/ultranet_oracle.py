"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may
use it; the product never does). CPU fp32 restatement of the UltraNet 4-bit path:

  `4-bit quantization/quant_ultra.py`   uniform_quantize :8-27, weight_quantize_fn :30-56,
                                        activation_quantize_fn :59-73, conv2d_Q_fn :76-91
  `4-bit quantization/mymodel.py`       create_grids :7-21, YOLOLayer :23-60, UltraNetQua :62-144

Same op sequence as the reference in fp32 torch (torch.round = half-to-even, nn.BatchNorm2d in
eval mode). Pinned by KAT-2/KAT-4 (tests/test_oracle.py) and by the integer identities of
the reference's numpy deploy code (oracle/quantization_np.py); the float network itself has no
published vectors (parity of the reference's float conv rounding: unpinned).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

W_BIT = 4
A_BIT = 4
# (in, out, kernel, maxpool after) for layers.{0,4,8,...}: mymodel.py:71-124
CONV_SPECS: List[Tuple[int, int, int, bool]] = [
    (3, 16, 3, True), (16, 32, 3, True), (32, 64, 3, True), (64, 64, 3, True),
    (64, 64, 3, False), (64, 64, 3, False), (64, 64, 3, False), (64, 64, 3, False),
]
ANCHORS = [[20, 20]] * 6  # mymodel.py:130


def uniform_quantize(x: torch.Tensor, k: int) -> torch.Tensor:
    """quant_ultra.py:8-27 forward."""
    if k == 32:
        return x
    if k == 1:
        return torch.sign(x)
    n = float(2 ** k - 1)
    return torch.round(x * n) / n


def weight_quantize(w: torch.Tensor, w_bit: int = W_BIT) -> torch.Tensor:
    """quant_ultra.py:30-56 (weight_quantize_fn.forward)."""
    if w_bit == 32:
        return w
    if w_bit == 1:
        E = torch.mean(torch.abs(w))
        return (uniform_quantize(w / E, 0) + 1) / 2 * E   # k = w_bit - 1 = 0 -> n = 0: reference behaviour
    t = torch.tanh(w)
    t = t / torch.max(torch.abs(t))
    return uniform_quantize(t, w_bit - 1)


def weight_codes(w: torch.Tensor, w_bit: int = W_BIT) -> torch.Tensor:
    """Integer codes k with weight_quantize(w) == k / (2^(w_bit-1) - 1) (quantization.py:24-31 form)."""
    n = float(2 ** (w_bit - 1) - 1)
    t = torch.tanh(w)
    t = t / torch.max(torch.abs(t))
    return torch.round(t * n)


def activation_quantize(x: torch.Tensor, a_bit: int = A_BIT) -> torch.Tensor:
    """quant_ultra.py:59-73."""
    if a_bit == 32:
        return x
    return uniform_quantize(torch.clamp(x, 0, 1), a_bit)


def conv_q(x, w, b=None, stride=1, padding=0, w_bit: int = W_BIT):
    """Conv2d_Q.forward, quant_ultra.py:85-89."""
    return F.conv2d(x, weight_quantize(w, w_bit), b, stride, padding)


def batch_norm_eval(x, sd, prefix, eps=1e-5):
    """nn.BatchNorm2d in eval mode (running statistics)."""
    return F.batch_norm(x, sd[prefix + ".running_mean"], sd[prefix + ".running_var"], sd[prefix + ".weight"],
                        sd[prefix + ".bias"], False, 0.0, eps)


def layer_prefixes() -> List[Tuple[str, str]]:
    """(conv prefix, bn prefix) per quantized conv block in UltraNetQua.layers (mymodel.py:71-124)."""
    out, i = [], 0
    for (_, _, _, pool) in CONV_SPECS:
        out.append((f"layers.{i}", f"layers.{i + 1}"))
        i += 4 if pool else 3
    return out


HEAD_PREFIX = "layers.28"  # conv2d_q(64, 36, 1) (mymodel.py:124), after 4 pooled (4 modules) + 4 plain (3) blocks


def create_grids(img_size, ng, stride_from: int):
    nx, ny = ng
    yv, xv = torch.meshgrid([torch.arange(ny), torch.arange(nx)], indexing="ij")
    grid_xy = torch.stack((xv, yv), 2).float().view((1, 1, ny, nx, 2))
    stride = max(img_size) / max(ng)
    anchor_vec = torch.tensor(ANCHORS, dtype=torch.float32) / stride
    anchor_wh = anchor_vec.view(1, len(ANCHORS), 1, 1, 2)
    return grid_xy, anchor_wh, stride


def yolo_decode(p: torch.Tensor, img_size) -> Tuple[torch.Tensor, torch.Tensor]:
    """YOLOLayer.forward in eval mode (mymodel.py:32-60)."""
    bs, _, ny, nx = p.shape
    na, no = len(ANCHORS), 6
    grid_xy, anchor_wh, stride = create_grids(img_size, (nx, ny), 0)
    p = p.view(bs, na, no, ny, nx).permute(0, 1, 3, 4, 2).contiguous()
    io = p.clone()
    io[..., :2] = torch.sigmoid(io[..., :2]) + grid_xy
    io[..., 2:4] = torch.exp(io[..., 2:4]) * anchor_wh
    io[..., :4] *= stride
    torch.sigmoid_(io[..., 4:])
    return io.view(bs, -1, no), p


def ultranet_block(sd: Dict[str, torch.Tensor], k: int, x: torch.Tensor) -> torch.Tensor:
    """Quantized block k of UltraNetQua.layers alone (mymodel.py:71-124): Conv2d_Q -> BatchNorm2d (eval) ->
    activation_quantize_fn (-> MaxPool2d(2, 2) for k < 4), as ultranet_forward runs it. Values k/15."""
    (cp, bp), (_, _, ks, pool) = layer_prefixes()[k], CONV_SPECS[k]
    x = activation_quantize(batch_norm_eval(conv_q(x, sd[cp + ".weight"], None, 1, ks // 2), sd, bp))
    return F.max_pool2d(x, 2, 2) if pool else x


def ultranet_forward(sd: Dict[str, torch.Tensor], x: torch.Tensor, trace: list = None):
    """UltraNetQua.forward (mymodel.py:134-144), eval mode. Returns (io [B, na*ny*nx, 6], p).
    If `trace` is a list, the activation after every quantized block is appended (post act-quant,
    post maxpool where the block has one) — values k/15."""
    img_size = x.shape[-2:]
    for (cp, bp), (_, _, k, pool) in zip(layer_prefixes(), CONV_SPECS):
        x = conv_q(x, sd[cp + ".weight"], None, 1, k // 2)
        x = batch_norm_eval(x, sd, bp)
        x = activation_quantize(x)
        if pool:
            x = F.max_pool2d(x, 2, 2)
        if trace is not None:
            trace.append(x.clone())
    x = conv_q(x, sd[HEAD_PREFIX + ".weight"], sd[HEAD_PREFIX + ".bias"], 1, 0)
    if trace is not None:
        trace.append(x.clone())
    io, p = yolo_decode(x, img_size)
    return io, p
