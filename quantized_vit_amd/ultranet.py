"""Mirror of the reference's `4-bit quantization/mymodel.py` (UltraNetQua + YOLOLayer) with a fused
MI355X forward.

Same module tree as the reference (state_dict keys layers.{i}.*, yololayer attributes), so a reference
checkpoint loads unchanged. In eval mode on a ROCm device the network runs as 5 HIP launches at 416 x 416:

  layers.0-3   qvit_ultra_conv0  float image -> conv3x3 (W4) -> BN -> A4 quantizer -> maxpool -> NHWC codes
  layers.4-15  qvit_ultra_conv   codes -> implicit-GEMM conv on MFMA -> BN -> quantizer -> maxpool
  layers.16-28 qvit_ultra_tail   the four 26 x 26 blocks, the 1x1 head (acc/105 + bias) and the YOLO decode
  + yololayer                    in one launch, the maps resident in LDS (for larger maps: qvit_ultra_conv per
                                 layer, then qvit_yolo_decode)

Weight codes and BN constants are prepared once per parameter version (a plan cache, like the ViT
layers). Anything else (training mode, CPU tensors, non-reference layer stacks) runs module by module.
"""
from __future__ import annotations

import contextlib
from typing import Optional

import torch
import torch.nn as nn

from . import _lib
from .quant_ultra import activation_quantize_fn, conv2d_Q_fn
from .vit_model import _timed   # benchmark event hooks (vit_model.KERNEL_TIMING)


def create_grids(self, img_size=416, ng=(13, 13), device="cpu", type=torch.float32):
    """mymodel.py:7-21."""
    nx, ny = ng
    self.img_size = max(img_size)
    self.stride = self.img_size / max(ng)
    yv, xv = torch.meshgrid([torch.arange(ny), torch.arange(nx)], indexing="ij")
    self.grid_xy = torch.stack((xv, yv), 2).to(device).type(type).view((1, 1, ny, nx, 2))
    self.anchor_vec = self.anchors.to(device) / self.stride
    self.anchor_wh = self.anchor_vec.view(1, self.na, 1, 1, 2).to(device).type(type)
    self.ng = torch.Tensor(ng).to(device)
    self.nx = nx
    self.ny = ny


class YOLOLayer(nn.Module):
    """mymodel.py:23-60."""

    def __init__(self, anchors):
        super().__init__()
        self.anchors = torch.Tensor(anchors)
        self.na = len(anchors)
        self.no = 6
        self.nx = 0
        self.ny = 0

    def forward(self, p, img_size):
        bs, _, ny, nx = p.shape
        if (self.nx, self.ny) != (nx, ny):
            create_grids(self, img_size, (nx, ny), p.device, p.dtype)
        p = p.view(bs, self.na, self.no, self.ny, self.nx).permute(0, 1, 3, 4, 2).contiguous()
        if self.training:
            return p
        io = p.clone()
        io[..., :2] = torch.sigmoid(io[..., :2]) + self.grid_xy
        io[..., 2:4] = torch.exp(io[..., 2:4]) * self.anchor_wh
        io[..., :4] *= self.stride
        torch.sigmoid_(io[..., 4:])
        return io.view(bs, -1, self.no), p

    def decode_params(self, ny: int, nx: int, img_size, device):
        """(anchors on the device, na, no, stride) of the decode at an ny x nx grid (create_grids, mymodel.py:7-21)."""
        if (self.nx, self.ny) != (nx, ny):
            create_grids(self, img_size, (nx, ny), device, torch.float32)
        dev_anchors = getattr(self, "_dev_anchors", None)
        if dev_anchors is None or dev_anchors.device != device:
            dev_anchors = self.anchors.to(device, torch.float32).contiguous()
            self._dev_anchors = dev_anchors
        return dev_anchors, self.na, self.no, float(self.stride)

    def decode_nhwc(self, head: torch.Tensor, img_size):
        """The same decode on the device from the head conv's NHWC output (qvit_yolo_decode)."""
        bs, ny, nx, _ = head.shape
        anchors, na, no, stride = self.decode_params(ny, nx, img_size, head.device)
        return _lib.yolo_decode(head, na, no, anchors, stride)


W_BIT = 4
A_BIT = 4
TAIL_MAX = 26  # qvit_ultra_tail: maps up to 26 x 26 (416 x 416 images) stay in LDS


def _conv_stack(w_bit=W_BIT, a_bit=A_BIT):
    conv2d_q = conv2d_Q_fn(w_bit)
    mods = []
    for cin, cout, pool in ((3, 16, True), (16, 32, True), (32, 64, True), (64, 64, True), (64, 64, False),
                            (64, 64, False), (64, 64, False), (64, 64, False)):
        mods += [conv2d_q(cin, cout, kernel_size=3, stride=1, padding=1, bias=False), nn.BatchNorm2d(cout),
                 activation_quantize_fn(a_bit)]
        if pool:
            mods.append(nn.MaxPool2d(2, stride=2))
    mods.append(conv2d_q(64, 36, kernel_size=1, stride=1, padding=0))
    return nn.Sequential(*mods)


@contextlib.contextmanager
def _aten_batch_norm():
    """BatchNorm2d on ATen's own kernels: torch routes an fp32 batch norm to MIOpen while cudnn is enabled."""
    prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    try:
        yield
    finally:
        torch.backends.cudnn.enabled = prev


def _round_up(v, m):
    return (v + m - 1) // m * m


class UltraNetQua(nn.Module):
    """mymodel.py:62-144."""

    def __init__(self):
        super().__init__()
        self.layers = _conv_stack()
        self.yololayer = YOLOLayer([[20, 20], [20, 20], [20, 20], [20, 20], [20, 20], [20, 20]])
        self.yolo_layers = [self.yololayer]
        self._plan = None
        self._plan_key = None

    # ---- fused path ---------------------------------------------------------------------------
    def _blocks(self):
        """[(conv, bn, act, pool or None)] for the 8 quantized blocks, then the head conv."""
        mods = list(self.layers)
        blocks, i = [], 0
        while i < len(mods) - 1:
            conv, bn, act = mods[i], mods[i + 1], mods[i + 2]
            pool = mods[i + 3] if i + 3 < len(mods) and isinstance(mods[i + 3], nn.MaxPool2d) else None
            blocks.append((conv, bn, act, pool))
            i += 4 if pool is not None else 3
        return blocks, mods[-1]

    def fused_ok(self, x: torch.Tensor) -> bool:
        if self.training or not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] != 3:
            return False
        if x.shape[2] % 16 or x.shape[3] % 16:
            return False
        blocks, head = self._blocks()
        if len(blocks) != 8 or not isinstance(head, nn.Conv2d) or head.kernel_size != (1, 1):
            return False
        for k, (conv, bn, act, pool) in enumerate(blocks):
            if not (isinstance(conv, nn.Conv2d) and isinstance(bn, nn.BatchNorm2d)
                    and isinstance(act, activation_quantize_fn) and act.a_bit == A_BIT
                    and getattr(conv, "w_bit", None) == W_BIT and conv.kernel_size == (3, 3)
                    and conv.padding == (1, 1) and conv.stride == (1, 1) and conv.bias is None
                    and bn.track_running_stats and (pool is None) == (k >= 4)):
                return False
            if pool is not None and (pool.kernel_size not in (2, (2, 2)) or pool.stride not in (2, (2, 2))):
                return False
        return getattr(head, "w_bit", None) == W_BIT

    def _key(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters()) + tuple(
            (b.data_ptr(), b._version) for b in self.buffers())

    def _build_plan(self, dev):
        blocks, head = self._blocks()
        plan = []
        for k, (conv, bn, _, pool) in enumerate(blocks):
            cout, cin = conv.out_channels, conv.in_channels
            if k == 0:   # float-input layer: the fake-quant weight values feed a direct fp32 conv
                _, codes = _lib.ultra_weight_codes(conv.weight, W_BIT, 32, 16, values=True)
            else:
                codes = _lib.ultra_weight_codes(conv.weight, W_BIT, _round_up(9 * cin, 64), _round_up(cout, 16))
            alpha, shift = _lib.ultra_bn_fold(bn, dev)
            plan.append((codes, alpha, shift, cout, pool is not None))
        hcodes = _lib.ultra_weight_codes(head.weight, W_BIT, 64, 48)
        hbias = head.bias.detach().float().contiguous() if head.bias is not None else torch.zeros(
            head.out_channels, device=dev)
        return plan, (hcodes, hbias, head.out_channels)

    def forward_fused(self, x: torch.Tensor):
        key = self._key()
        if self._plan is None or self._plan_key != key:
            self._plan, self._plan_key = self._build_plan(x.device), key
        plan, (hcodes, hbias, hout) = self._plan
        img_size = x.shape[-2:]
        c0, a0, s0, _, _ = plan[0]
        with _timed("ultra_conv0"):
            h = _lib.ultra_conv0(x.contiguous(), c0, a0, s0, A_BIT)
        for k, (codes, alpha, shift, cout, pool) in enumerate(plan[1:], 1):
            if k == 4 and h.shape[1] <= TAIL_MAX and h.shape[2] <= TAIL_MAX and hout == self.yololayer.na * 6:
                # layers.16-28 (the four unpooled blocks and the head) and the YOLO decode in one launch, the maps
                # resident in LDS
                tail = plan[4:]
                dec = self.yololayer.decode_params(h.shape[1], h.shape[2], img_size, h.device)
                with _timed("ultra_tail"):
                    io, p = _lib.ultra_tail(h, [c for c, *_ in tail], [a for _, a, *_ in tail],
                                            [s for _, _, s, *_ in tail], hcodes, hbias, hout, W_BIT, A_BIT, decode=dec)
                return io, (p,)
            mode = _lib.ULTRA_CODES_POOL if pool else _lib.ULTRA_CODES
            with _timed(f"ultra_conv{k}"):
                h = _lib.ultra_conv(h, 3, codes, cout, W_BIT, A_BIT, alpha, shift, mode)
        else:
            with _timed("ultra_head"):
                head = _lib.ultra_conv(h, 1, hcodes, hout, W_BIT, A_BIT, None, hbias, _lib.ULTRA_F32)
        with _timed("ultra_decode"):
            io, p = self.yololayer.decode_nhwc(head, img_size)
        return io, (p,)   # = torch.cat((io,), 1): the single YOLO layer's output, already a fresh tensor

    # ---- reference forward ------------------------------------------------------------------
    def forward(self, x):
        if self.fused_ok(x):
            return self.forward_fused(x)
        return self.forward_modules(x)

    def forward_modules(self, x):
        """mymodel.py:134-144 module by module: Conv2d_Q on qvit_conv_wonly, activation_quantize_fn on the HIP
        quantizer; BatchNorm2d and MaxPool2d on ATen's own kernels (the MIOpen batch-norm route off, so no
        library kernel is on the path). In eval mode each Conv2d_Q -> BatchNorm2d -> activation_quantize_fn triple
        runs as one launch (Conv2d_Q.forward_bn_act: the BN applied as the fused network folds it, fma(y, alpha,
        shift), which is not ATen's (x - mean) * invstd * w + b bit for bit: a 4-bit code can flip at a rounding tie,
        inside the 1e-3 end-to-end bar) unless one of the three modules carries forward (pre-)hooks or global module
        hooks are registered, which then run module by module as usual; the Sequential's own forward hooks are not
        called on this walk. Any image size, training mode included; under autograd (grad mode on and a
        parameter or the input requiring grad) the Conv2d_Q layers take the reference's F.conv2d on the fake-quant
        weight instead, so gradients flow (the packed-codes kernels record no history)."""
        img_size = x.shape[-2:]
        yolo_out = []
        with _aten_batch_norm():
            mods, i = list(self.layers), 0
            while i < len(mods):
                m = mods[i]
                if hasattr(m, "forward_bn_act") and i + 2 < len(mods) and not _hooked(mods[i:i + 3]):
                    y = m.forward_bn_act(x, mods[i + 1], mods[i + 2])   # conv -> BN -> quantizer in one launch
                    if y is not None:
                        x, i = y, i + 3
                        continue
                x, i = m(x), i + 1
        x = self.yololayer(x, img_size)
        yolo_out.append(x)
        if self.training:
            return yolo_out
        io, p = zip(*yolo_out)
        return torch.cat(io, 1), p


def _hooked(mods) -> bool:
    """Whether a forward (pre-)hook would see any of these modules' calls (their own hooks or global ones): the
    fused conv -> BN -> quantizer launch would skip them."""
    from torch.nn.modules import module as _m
    if _m._global_forward_hooks or _m._global_forward_pre_hooks:
        return True
    return any(mod._forward_hooks or mod._forward_pre_hooks for mod in mods)


def synthetic_images_u8(batch: int, size: int = 416, seed: int = 0, device=None) -> torch.Tensor:
    """k/255 images (k uniform in [0, 255]): the exact uint8-derived inputs of SURVEY §8(d)."""
    g = torch.Generator().manual_seed(seed)
    img = torch.randint(0, 256, (batch, 3, size, size), generator=g).float() / 255.0
    return img.to(device) if device is not None else img


def random_ultranet(seed: int = 0, device: Optional[torch.device] = None, calib_batch: int = 2,
                    img_size: int = 416) -> UltraNetQua:
    """Random-init UltraNetQua (conv weights N(0, 0.1)) whose BatchNorm running statistics are the
    per-channel mean/variance of its own conv outputs on `calib_batch` synthetic k/255 images (what a
    trained network's BN holds), with gamma ~ U(0.15, 0.35) and beta ~ U(0.3, 0.7) so the 4-bit codes
    spread over [0, 15] instead of saturating. Calibration runs the per-module path on `device`
    (a ROCm device). Eval mode."""
    g = torch.Generator().manual_seed(seed)
    m = UltraNetQua()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, nn.Conv2d):
                mod.weight.copy_(torch.randn(mod.weight.shape, generator=g) * 0.1)
                if mod.bias is not None:
                    mod.bias.copy_(torch.randn(mod.bias.shape, generator=g) * 0.1)
            elif isinstance(mod, nn.BatchNorm2d):
                n = mod.num_features
                mod.weight.copy_(torch.rand(n, generator=g) * 0.2 + 0.15)
                mod.bias.copy_(torch.rand(n, generator=g) * 0.4 + 0.3)
        m = m.to(device).eval()
        x = synthetic_images_u8(calib_batch, img_size, seed + 1, device)
        with _aten_batch_norm():
            for mod in m.layers:
                if isinstance(mod, nn.BatchNorm2d):
                    mod.running_mean.copy_(x.mean(dim=(0, 2, 3)))
                    mod.running_var.copy_(x.var(dim=(0, 2, 3)).clamp_min(1e-3))
                x = mod(x)
    return m
