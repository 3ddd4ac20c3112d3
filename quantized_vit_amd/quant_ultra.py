"""Mirror of the reference's `4-bit quantization/quant_ultra.py` (DoReFa-style 4-bit quantizers of
UltraNet): same factory / class names and forward semantics, computed on the ROCm device.

  uniform_quantize(k)        quant_ultra.py:8-27   round(x * (2^k - 1)) / (2^k - 1)  (k = 1: sign, 32: identity)
  weight_quantize_fn(w_bit)  :30-56   tanh -> / max|tanh| -> (w_bit-1)-bit uniform quantizer (HIP codes)
  activation_quantize_fn     :59-73   clamp(x, 0, 1) -> a_bit uniform quantizer (HIP)
  conv2d_Q_fn(w_bit)         :76-91   Conv2d_Q: conv with quantized weights -- qvit_conv_wonly (implicit GEMM of the
                                      fp32 input against the int weight codes, d_w = 1/(2^(w_bit-1)-1); <= 64
                                      output channels: the narrow schedule); forward_bn_act fuses a following
                                      eval BatchNorm2d + activation_quantize_fn (qvit_conv_wonly_bn_act)
  linear_Q_fn(w_bit)         :210-222 Linear_Q -- qvit_gemm_wonly on the same codes
  batchNorm2d_Q_fn / batchNorm1d_Q_fn  :94-207 (not used by UltraNetQua; kept for API parity)

Conv2d_Q / Linear_Q with 2 <= w_bit <= 8 (UltraNet: 4) run on the hand-written kernels; their weight codes are
packed once per weight version. w_bit 32 (no quantization: a plain conv / linear) and w_bit 1 (the reference's
k = 0 quantizer divides by zero) keep the library call on the device, as do grouped or non-zero-padded convs.

The network-level fused path (conv + BN + quantizer + max pool on codes) is in ultranet.py; these
modules are the per-layer surface. Forward-only (inference): the reference's straight-through
backward is not provided.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib


def _check_gpu(x: torch.Tensor, what: str) -> None:
    if not x.is_cuda:
        raise _lib.QvitError(f"{what} on {x.device}: the UltraNet path runs on a ROCm device (no CPU fallback)")


def uniform_quantize(k):
    """quant_ultra.py:8-27. Returns the quantizer function (the reference returns an autograd apply)."""

    def qfn(x: torch.Tensor) -> torch.Tensor:
        if k == 32:
            return x
        if k == 1:
            return torch.sign(x)
        n = float(2 ** k - 1)
        return torch.round(x * n) / n

    return qfn


def _round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


def weight_codes(weight: torch.Tensor, w_bit: int, kpad: int = None, cout_pad: int = None) -> torch.Tensor:
    """Integer weight codes of weight_quantize_fn (HIP), [cout_pad][kpad] in K order (ky, kx, c)."""
    _check_gpu(weight, "weight")
    w4 = weight if weight.dim() == 4 else weight.reshape(weight.shape[0], -1, 1, 1)
    cout, cin, ks, _ = w4.shape
    kpad = kpad or _round_up(ks * ks * cin, 16)
    cout_pad = cout_pad or cout
    return _lib.ultra_weight_codes(w4, w_bit, kpad, cout_pad)


class weight_quantize_fn(nn.Module):
    """quant_ultra.py:30-56."""

    def __init__(self, w_bit):
        super().__init__()
        assert w_bit <= 8 or w_bit == 32
        self.w_bit = w_bit
        self.uniform_q = uniform_quantize(k=w_bit - 1)

    def forward(self, x):
        if self.w_bit == 32:
            return x
        if self.w_bit == 1:   # reference behaviour kept as is (its k = 0 quantizer divides by zero)
            E = torch.mean(torch.abs(x)).detach()
            return (self.uniform_q(x / E) + 1) / 2 * E
        _check_gpu(x, "weight")
        w4 = x if x.dim() == 4 else x.reshape(x.shape[0], -1, 1, 1)
        cout, cin, ks, _ = w4.shape
        _, vals = _lib.ultra_weight_codes(w4, self.w_bit, _round_up(ks * ks * cin, 16), cout, values=True)
        return vals.reshape(x.shape)   # round(.)/n (:20), divided on the device as IEEE fp32


class activation_quantize_fn(nn.Module):
    """quant_ultra.py:59-73."""

    def __init__(self, a_bit):
        super().__init__()
        assert a_bit <= 8 or a_bit == 32
        self.a_bit = a_bit
        self.uniform_q = uniform_quantize(k=a_bit)

    def forward(self, x):
        if self.a_bit == 32:
            return x
        _check_gpu(x, "activation")
        if self.a_bit > 7:   # levels beyond the int8 code range: the reference arithmetic on the device
            return self.uniform_q(torch.clamp(x, 0, 1))
        return _lib.fake_quant_f32(x, _lib.QT_ULTRA_ACT, None, None, None, 2 ** self.a_bit - 1).reshape(x.shape)


class _PackedCodes:
    """Packed weight codes of weight_quantize_fn for qvit_gemm_wonly / qvit_conv_wonly: the HIP quantizer's codes
    k (values k / n, n = 2^(w_bit-1) - 1) re-ordered to the weight's flattening (c, kh, kw), packed int4 (n <= 7)
    or int8, with d_w = 1/n. Rebuilt when the weight or bias changes (in place or replaced)."""

    def __init__(self):
        self.key = None

    def get(self, weight: torch.Tensor, bias, w_bit: int):
        key = (weight.data_ptr(), weight._version, tuple(weight.shape), weight.device,
               None if bias is None else (bias.data_ptr(), bias._version))
        if key == self.key:
            return self
        w4 = weight.detach() if weight.dim() == 4 else weight.detach().reshape(weight.shape[0], -1, 1, 1)
        cout, cin, kh, kw = w4.shape
        k = cin * kh * kw
        self.n, self.npad, self.kpad = cout, _round_up(cout, _lib.TILE_N), _round_up(k, _lib.TILE_K)
        codes = _lib.ultra_weight_codes(w4, w_bit, _round_up(k, 16), cout)       # (ky, kx, c) order
        codes = codes[:, :k].view(cout, kh, kw, cin).permute(0, 3, 1, 2).reshape(cout, k).float().contiguous()
        n_lvl = 2 ** (w_bit - 1) - 1
        dev = weight.device
        self.wfmt = _lib.W4 if n_lvl <= 7 else _lib.W8
        ovf = torch.zeros(1, dtype=torch.int32, device=dev)
        self.packed = _lib.pack_weight(codes, _lib.QT_LINEAR, torch.ones(1, device=dev),
                                       torch.full((1,), 1024.0, device=dev), None, self.wfmt, self.npad, self.kpad, ovf)
        self.d_wt = torch.full((1,), 1.0 / n_lvl, dtype=torch.float32, device=dev)
        self.bias_pad = _lib.pad_bias(bias, cout, self.npad, dev)
        self.key = key
        return self


def _codes_path(w_bit: int) -> bool:
    return 2 <= w_bit <= 8


def _needs_grad(module: nn.Module, input: torch.Tensor) -> bool:
    """Autograd wants this call's history: the packed-codes kernels record none, so such calls take the
    reference's own F.conv2d / F.linear on quantize_fn(weight) (quant_ultra.py:85-89, :219-222), gradients included."""
    return torch.is_grad_enabled() and (input.requires_grad or any(p.requires_grad for p in module.parameters()))


def conv2d_Q_fn(w_bit):
    """quant_ultra.py:76-91."""

    class Conv2d_Q(nn.Conv2d):
        def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                     bias=True):
            super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)
            self.w_bit = w_bit
            self.quantize_fn = weight_quantize_fn(w_bit=w_bit)
            self._codes = _PackedCodes()
            self._bn_fold = None   # (key, alpha, shift) of the BatchNorm2d forward_bn_act last fused

        def prepare(self):
            """Packs the weight codes now (cached per weight version; see QuantizeMixin.prepare)."""
            if _codes_path(self.w_bit) and self.weight.is_cuda:
                self._codes.get(self.weight, self.bias, self.w_bit)
            return self

        def invalidate(self):
            """Drops the packed codes (and the fused BatchNorm fold): needed only after editing the weight, bias or BN
            statistics through `.data` (which bypasses the version counter the caches key on; QuantizeMixin.invalidate
            alike)."""
            self._codes.key = None
            self._bn_fold = None
            return self

        def forward(self, input, order=None):
            if _codes_path(self.w_bit):
                _check_gpu(input, "input")
            if _codes_path(self.w_bit) and self.groups == 1 and self.padding_mode == "zeros" and \
                    not isinstance(self.padding, str) and input.dim() == 4 and not _needs_grad(self, input):
                c = self._codes.get(self.weight, self.bias, self.w_bit)
                return _lib.conv_wonly(input.detach(), self.kernel_size, self.stride, self.padding, self.dilation,
                                       c.packed, c.wfmt, c.n, c.npad, c.kpad, c.d_wt, c.bias_pad)
            weight_q = self.quantize_fn(self.weight)
            return F.conv2d(input, weight_q, self.bias, self.stride, self.padding, self.dilation, self.groups)

        def forward_bn_act(self, input, bn, act):
            """act(bn(self(input))) in one launch when `bn` is a BatchNorm2d in eval mode on running statistics and
            `act` an activation_quantize_fn with 1 <= a_bit <= 7 (UltraNet's conv -> BN -> quantizer blocks,
            mymodel.py:71-124): qvit_conv_wonly_bn_act, BN as y alpha + shift (alpha = gamma / sqrt(var + eps),
            shift = beta - mean alpha: the fused network's fold, ultra_bn_fold) and the quantizer's values
            round(clamp(., 0, 1) n) / n. Returns None when the three modules do not fit that launch (the caller then
            runs them one by one)."""
            if not (_codes_path(self.w_bit) and self.groups == 1 and self.padding_mode == "zeros"
                    and not isinstance(self.padding, str) and input.dim() == 4 and input.is_cuda
                    and isinstance(bn, nn.BatchNorm2d) and not bn.training and bn.track_running_stats
                    and bn.running_mean is not None and bn.running_var is not None
                    and bn.num_features == self.out_channels
                    and isinstance(act, activation_quantize_fn) and 1 <= act.a_bit <= 7
                    and not _needs_grad(self, input) and not _needs_grad(bn, input)):
                return None
            c = self._codes.get(self.weight, self.bias, self.w_bit)
            key = tuple((t.data_ptr(), t._version) for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)
                        if t is not None) + (bn.eps, input.device)
            if self._bn_fold is None or self._bn_fold[0] != key:
                self._bn_fold = (key, *_lib.ultra_bn_fold(bn, input.device))
            return _lib.conv_wonly_bn_act(input.detach(), self.kernel_size, self.stride, self.padding, self.dilation,
                                          c.packed, c.wfmt, c.n, c.npad, c.kpad, c.d_wt, c.bias_pad, self._bn_fold[1],
                                          self._bn_fold[2], 2 ** act.a_bit - 1)

    return Conv2d_Q


def batchNorm2d_Q_fn(w_bit):
    """quant_ultra.py:94-132 (BN with quantized folded scale/shift)."""

    class BatchNorm2d_Q(nn.BatchNorm2d):
        def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True):
            super().__init__(num_features, eps, momentum, affine, track_running_stats)
            self.w_bit = w_bit
            self.quantize_fn = uniform_quantize(k=w_bit)

        def forward(self, input):
            gamma, var, mean, eps, bias = self.weight, self.running_var, self.running_mean, self.eps, self.bias
            w = gamma / (torch.sqrt(var) + eps)
            b = bias - (mean / (torch.sqrt(var) + eps)) * gamma
            w = torch.clamp(w, -1, 1) / 2 + 0.5
            w_q = 2 * self.quantize_fn(w) - 1
            b = torch.clamp(b, -1, 1) / 2 + 0.5
            b_q = 2 * self.quantize_fn(b) - 1
            return F.batch_norm(input, running_mean=mean * 0, running_var=torch.sign(torch.abs(var) + 1),
                                weight=w_q, bias=b_q, eps=eps * 0)

    return BatchNorm2d_Q


def batchNorm1d_Q_fn(w_bit):
    """quant_ultra.py:135-207 (eval form)."""

    class BatchNorm1d_Q(nn.BatchNorm1d):
        def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True):
            super().__init__(num_features, eps, momentum, affine, track_running_stats)
            self.w_bit = w_bit
            self.quantize_fn = uniform_quantize(k=w_bit)

        def forward(self, input):
            self._check_input_dim(input)
            gamma, var, mean, eps, bias = self.weight, self.running_var, self.running_mean, self.eps, self.bias
            w = gamma / (torch.sqrt(var) + eps)
            b = bias - (mean / (torch.sqrt(var) + eps)) * gamma
            return F.batch_norm(input, mean * 0, torch.sign(var + 1), w, b,
                                self.training or not self.track_running_stats, self.momentum or 0.0, eps * 0)

    return BatchNorm1d_Q


def linear_Q_fn(w_bit):
    """quant_ultra.py:210-222."""

    class Linear_Q(nn.Linear):
        def __init__(self, in_features, out_features, bias=True):
            super().__init__(in_features, out_features, bias)
            self.w_bit = w_bit
            self.quantize_fn = weight_quantize_fn(w_bit=w_bit)
            self._codes = _PackedCodes()

        def prepare(self):
            """Packs the weight codes now (cached per weight version; see QuantizeMixin.prepare)."""
            if _codes_path(self.w_bit) and self.weight.is_cuda:
                self._codes.get(self.weight, self.bias, self.w_bit)
            return self

        def invalidate(self):
            """Drops the packed codes (see Conv2d_Q.invalidate)."""
            self._codes.key = None
            return self

        def forward(self, input):
            if not _codes_path(self.w_bit) or _needs_grad(self, input):
                return F.linear(input, self.quantize_fn(self.weight), self.bias)
            _check_gpu(input, "input")
            c = self._codes.get(self.weight, self.bias, self.w_bit)
            x2 = input.detach().reshape(-1, self.in_features)
            if (x2.dtype != torch.float32 or x2.stride(-1) != 1 or c.kpad != self.in_features or x2.stride(0) % 4
                    or x2.data_ptr() % 16):
                xp = torch.zeros((x2.shape[0], c.kpad), dtype=torch.float32, device=x2.device)
                xp[:, :self.in_features] = x2
                x2 = xp
            ldy = _round_up(c.n, 4)
            y = torch.empty((x2.shape[0], ldy), dtype=torch.float32, device=x2.device)
            _lib.gemm_wonly(x2, x2.shape[0], c.kpad, c.packed, c.wfmt, c.n, c.npad, c.d_wt, c.bias_pad, y)
            y = y if ldy == c.n else y[:, :c.n]
            return y.reshape(*input.shape[:-1], c.n)

    return Linear_Q
