"""QuantizeLinear / QuantizeConv2d for MI355X: the reference's module surface, HIP underneath.

Mirrors OTO/quantization/quant_layers.py (OTO = QViT_with_GETA/only_train_once): same class
names, constructor arguments, parameter names / state_dict keys (weight, bias, d_quant_wt, q_m_wt,
[t_quant_wt], [d_quant_act, q_m_act, t_quant_act]), enums, from_module(), weight_bit /
activation_bit and LAYER_TO_QUANTLAYER, so model_to_quantize_model and existing callers
(vit_model.py:100,133,151,172,175,327) work unchanged.

What differs is how forward() computes (quant_layers.py:495-499, 575-587). The reference
re-quantizes the fp32 master weight on every call and runs an fp32 F.linear on fake-quant
operands. Here, on a ROCm device:
  * weights are quantized once per parameter version into int4 (|level| <= 7) or int8 codes,
    packed for the MFMA kernel (qvit_pack_weight), and cached;
  * activations are quantized to int8 codes by a HIP kernel (qvit_quantize_act_i8);
  * the product is an exact int32 MFMA contraction with the fp32 epilogue
    d_act * d_wt * acc + bias (qvit_gemm) — mathematically the reference's F.linear on
    d_a*k_a and d_w*k_w, differing only in fp32 rounding.
Layers whose levels do not fit int8 (e.g. the 16/32-bit initial states, weight-only mode) run
the reference's fake-quant values (HIP kernel qvit_fake_quant_f32) through the library fp32
GEMM instead. CPU tensors are rejected: the product has no CPU fallback.

Inference only: the HIP path does not record autograd history (training / GETA is out of scope).
"""
from __future__ import annotations

import logging
import math
import os
import warnings
from dataclasses import dataclass, field
from enum import Enum
from typing import Optional, Tuple, Union

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

logger = logging.getLogger(__name__)


class NanInGradientError(Exception):
    """quant_layers.py:10-13 (raised by the reference's backward; kept for API parity)."""

    def __init__(self, message):
        self.message = message
        super().__init__(self.message)


class QuantizationType(Enum):
    """quant_layers.py:20-24."""
    SYMMETRIC_LINEAR = "symmetric+linear"
    SYMMETRIC_NONLINEAR = "symmetric+nonlinear"
    DGE = "dge"


class QuantizationMode(Enum):
    """quant_layers.py:27-29."""
    WEIGHT_ONLY = "weight_only"
    WEIGHT_AND_ACTIVATION = "weight_and_activation"


def _qtype_code(qt: QuantizationType) -> int:
    # DGEQuantizer.forward (quant_layers.py:217-246) is the linear quantizer's forward
    if qt in (QuantizationType.SYMMETRIC_LINEAR, QuantizationType.DGE):
        return _lib.QT_LINEAR
    if qt == QuantizationType.SYMMETRIC_NONLINEAR:
        return _lib.QT_NONLINEAR
    raise NotImplementedError(qt)


_warned_grad = False

# Parity instrumentation (tests): when CODE_TRACE is a dict, every int8 activation-code operand handed to
# a layer's contraction is recorded as CODE_TRACE[layer] = codes[:, :K] (a stream-ordered copy), so a
# checker can compare each quantizer boundary of a full forward with the reference's.
CODE_TRACE: Optional[dict] = None


def trace_codes(layer, codes: torch.Tensor, k: int) -> None:
    if CODE_TRACE is not None:
        CODE_TRACE[layer] = codes[:, :k].detach().clone()


def _warn_no_grad() -> None:
    global _warned_grad
    if not _warned_grad:
        _warned_grad = True
        warnings.warn("quantized_vit_amd: the HIP forward path records no autograd history "
                      "(inference only); run under torch.no_grad() to silence this warning.")


def _as_param_ptr(p: Optional[torch.Tensor], device: torch.device) -> Optional[torch.Tensor]:
    if p is None:
        return None
    t = p.detach()
    if t.device != device or t.dtype != torch.float32 or not t.is_contiguous():
        t = t.to(device=device, dtype=torch.float32).contiguous()
    return t


def saturation_level(qtype: int, d: float, q_m: float, t: float = 1.0) -> float:
    """Host copy of the device formula: rne(|q_m| / d) (linear, quant_layers.py:154,159) or
    rne(exp(t log(|q_m| + 1e-6)) / d) (nonlinear, :62,67), in fp32."""
    f = np.float32
    with np.errstate(all="ignore"):
        if qtype == _lib.QT_LINEAR:
            p = np.abs(f(q_m))
        else:
            p = np.exp(f(t) * np.log(np.abs(f(q_m)) + f(1e-6)), dtype=np.float32)
        q = f(p) / f(d)
    return float(np.rint(q)) if np.isfinite(q) else float("inf")


def _round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


# The int path's W4 GEMMs (qvit_gemm, qvit_gemm_qkv_split) take a register image of the packed codes (same
# results, each GEMM wave's weight rows loaded into registers instead of through LDS): "w4r" (qvit_pack_weight_w4r,
# the int4 bytes re-ordered; round 5: fc1 -2.6 % in the model) or "w8r" (qvit_pack_weight_w8r, the codes already
# unpacked to the MFMA's int8 operands: twice the bytes, no unpack in the main loop). QVIT_GEMM_WREG=w4 (or the
# older QVIT_GEMM_W4R=0) keeps the LDS-staged form (same-box A/B).
GEMM_WREG = os.environ.get("QVIT_GEMM_WREG", "w4r" if os.environ.get("QVIT_GEMM_W4R", "1") == "1" else "w4")
if GEMM_WREG not in ("w4", "w4r", "w8r"):
    raise ValueError(f"QVIT_GEMM_WREG={GEMM_WREG!r}: expected w4, w4r or w8r")
GEMM_W4R = GEMM_WREG != "w4"   # a register image is in use


@dataclass
class QuantPlan:
    """Per-layer device state derived from the parameters (rebuilt when any of them changes)."""
    key: tuple
    device: torch.device
    qtype: int
    n: int
    k: int
    npad: int
    kpad: int
    wfmt: int                       # _lib.W4 / _lib.W8 / 0 (fp32 fake-quant path)
    int_path: bool                  # activation codes fit int8 and the weight was packed
    level_wt: float
    level_act: float
    packed: Optional[torch.Tensor] = None
    bias_pad: Optional[torch.Tensor] = None
    w_fakequant: Optional[torch.Tensor] = None
    d_wt: Optional[torch.Tensor] = None
    qm_wt: Optional[torch.Tensor] = None
    t_wt: Optional[torch.Tensor] = None
    d_act: Optional[torch.Tensor] = None
    qm_act: Optional[torch.Tensor] = None
    t_act: Optional[torch.Tensor] = None
    extra: dict = field(default_factory=dict)

    def gemm_weights(self) -> Tuple[torch.Tensor, int]:
        """(image, wfmt) the int path's GEMM reads: the register image (W4R / W8R) of a W4 plan, else the packed
        codes. The register image is built on the first call and the packed codes it is made from are then
        released, so a layer holds its int4 weights once (conv layers and the fused qkv + attention kernel never
        call this and keep only the packed codes); `packed_codes()` re-packs them for a route that needs them."""
        if self.int_path and self.wfmt == _lib.W4 and GEMM_WREG != "w4" and "wreg" not in self.extra:
            src = self.packed_codes()
            pack = _lib.pack_weight_w4r if GEMM_WREG == "w4r" else _lib.pack_weight_w8r
            self.extra["wreg"] = (pack(src, self.npad, self.kpad), _lib.W4R if GEMM_WREG == "w4r" else _lib.W8R)
            if self.extra.get("repack") is not None:
                self.packed = None
        wreg = self.extra.get("wreg")
        return wreg if wreg is not None else (self.packed_codes(), self.wfmt)

    def packed_codes(self) -> torch.Tensor:
        """The packed weight codes (qvit_pack_weight layout), re-packed from the layer's weights if
        gemm_weights() released them (the same call that made them: deterministic, no overflow to re-check)."""
        if self.packed is None:
            self.packed = self.extra["repack"]()
        return self.packed


class QuantizeMixin:
    """quant_layers.py:303-410 — parameters, quantize_weight/quantize_act, bit-width properties."""

    def init_quantization(
        self,
        d_quant_init: float = 1.0,
        t_quant_init: float = 1.0,
        q_m_init: float = 1.0,
        quant_type: QuantizationType = QuantizationType.SYMMETRIC_LINEAR,
        quant_mode: QuantizationMode = QuantizationMode.WEIGHT_ONLY,
        weight_clip_val: Tuple[float, float] = (-2.0, 2.0),
        act_clip_val: Tuple[float, float] = (-2.0, 2.0),
    ):
        self.d_quant_wt = nn.Parameter(torch.tensor([d_quant_init]))
        self.q_m_wt = nn.Parameter(torch.tensor([q_m_init]))
        if quant_type == QuantizationType.SYMMETRIC_NONLINEAR:
            self.t_quant_wt = nn.Parameter(torch.tensor([t_quant_init]))
        if quant_mode == QuantizationMode.WEIGHT_AND_ACTIVATION:
            self.d_quant_act = nn.Parameter(torch.tensor([d_quant_init]))
            self.q_m_act = nn.Parameter(torch.tensor([q_m_init]))
            if quant_type == QuantizationType.SYMMETRIC_NONLINEAR:
                self.t_quant_act = nn.Parameter(torch.tensor([t_quant_init]))
        self.quant_type = quant_type
        self.quant_mode = quant_mode
        self.weight_clip_val = weight_clip_val
        self.act_clip_val = act_clip_val
        self._qplan: Optional[QuantPlan] = None
        self._weight_codes: Optional[Tuple[tuple, torch.Tensor]] = None

    # -- reference API: fake-quant fp32 tensors (quant_layers.py:332-381) -------------------
    def quantize_weight(self, weight: torch.Tensor) -> torch.Tensor:
        dev = weight.device
        return _lib.fake_quant_f32(weight.detach(), _qtype_code(self.quant_type),
                                   _as_param_ptr(self.d_quant_wt, dev), _as_param_ptr(self.q_m_wt, dev),
                                   _as_param_ptr(getattr(self, "t_quant_wt", None), dev))

    def quantize_act(self, activation: torch.Tensor) -> torch.Tensor:
        if self.quant_mode != QuantizationMode.WEIGHT_AND_ACTIVATION:
            return activation
        dev = activation.device
        return _lib.fake_quant_f32(activation.detach(), _qtype_code(self.quant_type),
                                   _as_param_ptr(self.d_quant_act, dev), _as_param_ptr(self.q_m_act, dev),
                                   _as_param_ptr(getattr(self, "t_quant_act", None), dev))

    @property
    def weight_bit(self) -> int:
        d = self.d_quant_wt.item()
        qmax = abs(self.q_m_wt.item())
        if self.quant_type == QuantizationType.SYMMETRIC_LINEAR:
            t = 1.0
        elif self.quant_type == QuantizationType.SYMMETRIC_NONLINEAR:
            t = self.t_quant_wt.item()
        else:
            raise NotImplementedError
        return round(math.log2(math.exp(t * math.log(qmax)) / abs(d) + 1) + 1)

    @property
    def activation_bit(self) -> int:
        if self.quant_mode != QuantizationMode.WEIGHT_AND_ACTIVATION:
            return 32
        d = self.d_quant_act.item()
        qmax = abs(self.q_m_act.item())
        if self.quant_type == QuantizationType.SYMMETRIC_LINEAR:
            t = 1.0
        elif self.quant_type == QuantizationType.SYMMETRIC_NONLINEAR:
            t = self.t_quant_act.item()
        else:
            raise NotImplementedError
        return round(math.log2(math.exp(t * math.log(qmax)) / abs(d) + 1) + 1)

    # -- MI355X state ---------------------------------------------------------------------------
    def prepare(self):
        """Packs the weight codes (and bias, code tables' inputs) on the device now instead of at the first
        forward: the reference re-quantizes on every call; here the packed form is cached per
        parameter version, so this only moves the one-time cost out of the first timed call. Returns self."""
        self.quant_plan()
        return self

    def invalidate(self) -> None:
        """Drops the cached quantized weight. Needed only after editing parameters through
        `.data` (which bypasses the version counter the cache keys on)."""
        self._qplan = None

    def load_weight_codes(self, codes: Optional[torch.Tensor]) -> None:
        """Uses the given integer weight codes k (quantize_weight(W) == d_quant_wt * k, quant_layers.py:332-354)
        instead of deriving them on the device — e.g. the codes the reference's own host computed, so that
        both sides run on identical int4 weights. The codes stay bound to the current parameter versions:
        editing any parameter drops them (the device derives the codes again). `None` unbinds them."""
        if codes is None:
            self._weight_codes = None
        else:
            c = torch.as_tensor(codes).detach()
            if c.is_floating_point() and not torch.equal(c, c.round()):
                raise ValueError("weight codes must be integers")
            if tuple(c.shape) != tuple(self.weight.shape):
                raise ValueError(f"weight codes of shape {tuple(c.shape)} for a weight of shape "
                                 f"{tuple(self.weight.shape)}")
            self._weight_codes = (self._plan_key(), c.reshape(c.shape[0], -1).to(torch.int16))
        self._qplan = None

    def _bound_weight_codes(self, key: tuple) -> Optional[torch.Tensor]:
        wc = self._weight_codes
        if wc is None:
            return None
        if (wc[0][0],) + wc[0][3:] != (key[0],) + key[3:]:   # type or a parameter changed since the load
            self._weight_codes = None
            return None
        return wc[1]

    def _quant_param_tensors(self):
        names = ["weight", "bias", "d_quant_wt", "q_m_wt", "t_quant_wt", "d_quant_act", "q_m_act", "t_quant_act"]
        return [getattr(self, n, None) for n in names]

    def _plan_key(self) -> tuple:
        key = [self.quant_type, self.quant_mode, self.training]
        for p in self._quant_param_tensors():
            key.append(None if p is None else (p.data_ptr(), p._version, p.device, p.dtype, tuple(p.shape)))
        return tuple(key)

    def _weight_2d(self) -> torch.Tensor:
        w = self.weight.detach()
        return w.reshape(w.shape[0], -1)

    def quant_plan(self) -> QuantPlan:
        """Builds (or returns the cached) device plan. Building syncs the host once (it reads the
        scalar quantizer parameters to choose int4 / int8 / fp32 storage)."""
        key = self._plan_key()
        plan = self._qplan
        if plan is not None and plan.key == key and not self.training:
            return plan
        plan = self._build_plan(key)
        self._qplan = plan
        return plan

    def _build_plan(self, key: tuple) -> QuantPlan:
        w2 = self._weight_2d()
        dev = w2.device
        if not w2.is_cuda:
            raise _lib.QvitError(f"{type(self).__name__}: weights are on {dev}; move the model to a ROCm "
                                 "device (the HIP path has no CPU fallback)")
        qt = _qtype_code(self.quant_type)
        n, k = w2.shape
        npad, kpad = _round_up(n, _lib.TILE_N), _round_up(k, _lib.TILE_K)
        d_wt = _as_param_ptr(self.d_quant_wt, dev)
        qm_wt = _as_param_ptr(self.q_m_wt, dev)
        t_wt = _as_param_ptr(getattr(self, "t_quant_wt", None), dev)
        wa = self.quant_mode == QuantizationMode.WEIGHT_AND_ACTIVATION
        d_act = _as_param_ptr(getattr(self, "d_quant_act", None), dev) if wa else None
        qm_act = _as_param_ptr(getattr(self, "q_m_act", None), dev) if wa else None
        t_act = _as_param_ptr(getattr(self, "t_quant_act", None), dev) if wa else None
        # one host sync: the scalar parameters decide the storage format
        bias_max = (self.bias.detach().abs().max().float().reshape(1).to(dev) if self.bias is not None
                    else torch.zeros(1, device=dev))
        scal = torch.stack([x.reshape(-1)[0] for x in (d_wt, qm_wt, t_wt if t_wt is not None else d_wt)]
                           + ([d_act.reshape(-1)[0], qm_act.reshape(-1)[0],
                               (t_act if t_act is not None else d_act).reshape(-1)[0]] if wa else [])
                           + [bias_max[0]]).cpu()
        s = scal.tolist()
        lw = saturation_level(qt, s[0], s[1], s[2] if t_wt is not None else 1.0)
        la = saturation_level(qt, s[3], s[4], s[5] if t_act is not None else 1.0) if wa else float("inf")
        plan = QuantPlan(key=key, device=dev, qtype=qt, n=n, k=k, npad=npad, kpad=kpad, wfmt=0, int_path=False,
                         level_wt=lw, level_act=la, d_wt=d_wt, qm_wt=qm_wt, t_wt=t_wt, d_act=d_act,
                         qm_act=qm_act, t_act=t_act)
        w32 = w2 if (w2.dtype == torch.float32 and w2.is_contiguous()) else w2.float().contiguous()
        act_ok = wa and abs(la) <= 127
        codes = self._bound_weight_codes(key)
        if codes is not None:
            cmax = int(codes.abs().max().item()) if codes.numel() else 0
            if cmax > abs(lw):
                raise ValueError(f"{type(self).__name__}: loaded weight code {cmax} exceeds the quantizer's "
                                 f"saturation level {lw}")
            plan.extra["weight_codes"] = True
            # packing integer values with the linear quantizer at d = 1 reproduces them exactly
            w32 = codes.to(device=dev, dtype=torch.float32).contiguous()
            qt_pack, d_pack = _lib.QT_LINEAR, torch.ones(1, device=dev)
            qm_pack, t_pack = torch.full((1,), 1024.0, device=dev), None
        else:
            qt_pack, d_pack, qm_pack, t_pack = qt, d_wt, qm_wt, t_wt
        if act_ok and abs(lw) <= 127:
            overflow = torch.zeros(1, dtype=torch.int32, device=dev)
            for wfmt in ((_lib.W4, _lib.W8) if abs(lw) <= 7 else (_lib.W8,)):
                overflow.zero_()
                packed = _lib.pack_weight(w32, qt_pack, d_pack, qm_pack, t_pack, wfmt, npad, kpad, overflow)
                if int(overflow.item()) == 0:
                    plan.packed, plan.wfmt, plan.int_path = packed, wfmt, True
                    if wfmt == _lib.W4:   # how gemm_weights() gets the packed codes back after releasing them
                        plan.extra["repack"] = self._repacker(w2, codes, (qt_pack, d_pack, qm_pack, t_pack),
                                                              wfmt, npad, kpad)
                    break
        if not plan.int_path and abs(lw) <= 65536:
            # fp32 activations against the packed weight codes (qvit_gemm_wonly, QuantizeLinear): the weight-only
            # mode (the reference's default) and W+A layers off the int path (levels beyond int8: their
            # activations are fake-quantized to fp32 first); int4 / int8 codes as on the int path, wider ones
            # (e.g. the default num_bits = 16) as balanced base-256 digits (W16 / W24)
            if abs(lw) <= 127:
                overflow = torch.zeros(1, dtype=torch.int32, device=dev)
                for wfmt in ((_lib.W4, _lib.W8) if abs(lw) <= 7 else (_lib.W8,)):
                    overflow.zero_()
                    packed = _lib.pack_weight(w32, qt_pack, d_pack, qm_pack, t_pack, wfmt, npad, kpad, overflow)
                    if int(overflow.item()) == 0:
                        plan.packed, plan.wfmt = packed, wfmt
                        plan.extra["wonly"] = True
                        break
            else:
                wc = codes.to(device=dev, dtype=torch.float32) if codes is not None else \
                    (_lib.fake_quant_f32(w32, qt, d_wt, qm_wt, t_wt) / d_wt).round()
                plan.packed, plan.wfmt = _lib.pack_weight_wide(wc, npad, kpad)
                plan.extra["wonly"] = True
        if plan.int_path or plan.extra.get("wonly"):
            bias = self.bias.detach() if self.bias is not None else None
            plan.bias_pad = _lib.pad_bias(bias, n, npad, dev)
            # |output| <= d_act d_wt sum_k |a_k||w_k| + |bias| <= d_act d_wt K L_a L_w + max|bias| (integer path
            # only: a weight-only plan has no activation scalars, and its output is unbounded a priori)
            plan.extra["out_bound"] = (abs(s[3] * s[0]) * k * abs(la) * abs(lw) + s[-1]) if plan.int_path \
                else float("inf")
        if wa:   # host copies of the activation quantizer's scalars (epilogue code tables of the producer)
            plan.extra["act_host"] = (qt, s[3], s[4], s[5] if t_act is not None else 1.0, la)
        if not plan.int_path and not plan.extra.get("wonly"):   # levels that fit neither int4 nor int8 (e.g. 16/32
            plan.w_fakequant = self._fake_quant_weight(plan)     # bits); the fp32 form is otherwise filled lazily
        return plan

    @staticmethod
    def _repacker(w2: torch.Tensor, codes: Optional[torch.Tensor], qargs: tuple, wfmt: int, npad: int, kpad: int):
        """A closure that repeats quant_plan's packing of these weights (the fp32 source is re-derived on the call,
        so the plan holds no fp32 copy)."""
        def repack() -> torch.Tensor:
            if codes is not None:
                src = codes.to(device=w2.device, dtype=torch.float32).contiguous()
            else:
                src = w2 if (w2.dtype == torch.float32 and w2.is_contiguous()) else w2.float().contiguous()
            overflow = torch.zeros(1, dtype=torch.int32, device=w2.device)
            return _lib.pack_weight(src, *qargs, wfmt, npad, kpad, overflow)
        return repack

    def _fake_quant_weight(self, plan: QuantPlan) -> torch.Tensor:
        """quantize_weight(W) on the device; with codes bound by load_weight_codes, d_w * k of exactly those
        codes (also when the plan is on the int path and the fp32 form is only filled later, e.g. for a
        grouped conv whose forward takes the library path)."""
        codes = self._bound_weight_codes(plan.key)
        if codes is not None:
            k = codes.to(device=plan.device, dtype=torch.float32)
            return (plan.d_wt * k).view_as(self.weight)      # d_w * k, as quantize_weight returns it
        return _lib.fake_quant_f32(self.weight.detach().float(), plan.qtype, plan.d_wt, plan.qm_wt, plan.t_wt)

    def weight_codes(self) -> torch.Tensor:
        """The integer weight codes the device path uses ([N, K] float32 on the device): the loaded ones
        (load_weight_codes) or the device quantizer's."""
        plan = self.quant_plan()
        wc = self._bound_weight_codes(plan.key)
        if wc is not None:
            return wc.to(device=plan.device, dtype=torch.float32)
        w = self._weight_2d().float().contiguous()
        if abs(plan.level_wt) > 127:
            return (_lib.fake_quant_f32(w, plan.qtype, plan.d_wt, plan.qm_wt, plan.t_wt) / plan.d_wt).round()
        codes = torch.empty((w.shape[0], plan.kpad), dtype=torch.int8, device=plan.device)
        _lib.quantize_act_i8(w, plan.qtype, plan.d_wt, plan.qm_wt, plan.t_wt, 0, codes, plan.kpad)
        return codes[:, :w.shape[1]].float()

    def _wonly_rows(self, x2: torch.Tensor, plan: QuantPlan) -> torch.Tensor:
        """[M, k] fp32 rows (or rows already zero-padded to kpad columns) @ quantize_weight(W)^T + b on
        qvit_gemm_wonly (weight-only / wide-level plans)."""
        M = x2.shape[0]
        if (x2.dtype != torch.float32 or x2.stride(-1) != 1 or x2.shape[1] < plan.kpad or x2.stride(0) % 4
                or x2.data_ptr() % 16):
            xp = torch.zeros((M, plan.kpad), dtype=torch.float32, device=x2.device)
            xp[:, :plan.k] = x2[:, :plan.k]
            x2 = xp
        ldy = _round_up(plan.n, 4)
        y = torch.empty((M, ldy), dtype=torch.float32, device=x2.device)
        _lib.gemm_wonly(x2, M, plan.kpad, plan.packed, plan.wfmt, plan.n, plan.npad, plan.d_wt, plan.bias_pad, y)
        return y if ldy == plan.n else y[:, :plan.n]

    def w_fakequant(self, plan: QuantPlan) -> torch.Tensor:
        """The reference's quantize_weight(W) (quant_layers.py:332-354), cached on the plan."""
        if plan.w_fakequant is None:
            plan.w_fakequant = self._fake_quant_weight(plan)
        return plan.w_fakequant

    def _check_input(self, x: torch.Tensor) -> None:
        if not x.is_cuda:
            raise _lib.QvitError(f"{type(self).__name__}: input on {x.device}; the HIP path needs a ROCm "
                                 "device tensor (no CPU fallback)")
        if torch.is_grad_enabled() and (x.requires_grad or any(
                p is not None and p.requires_grad for p in self._quant_param_tensors())):
            _warn_no_grad()

    def _act_codes(self, x2d: torch.Tensor, plan: QuantPlan) -> torch.Tensor:
        M = x2d.shape[0]
        codes = torch.empty((M, plan.kpad), dtype=torch.int8, device=x2d.device)
        _lib.quantize_act_i8(x2d, plan.qtype, plan.d_act, plan.qm_act, plan.t_act, 0, codes, plan.kpad)
        return codes

    def gemm_codes(self, codes: torch.Tensor, plan: QuantPlan, epilogue: int = _lib.EPI_F32,
                   out: Optional[torch.Tensor] = None, next_layer: Optional["QuantizeMixin"] = None) -> torch.Tensor:
        """Runs the contraction on activation codes (int8 [M, kpad]) with the given epilogue.
        EPI_I8 / EPI_I8_GELU quantize the result with `next_layer`'s activation quantizer."""
        M = codes.shape[0]
        dev = codes.device
        oq = dict(out_qtype=0)
        if epilogue in (_lib.EPI_I8, _lib.EPI_I8_GELU):
            nplan = next_layer.quant_plan()
            if out is None:
                out = torch.empty((M, _round_up(plan.n, 16)), dtype=torch.int8, device=dev)
            oq = dict(out_qtype=nplan.qtype, out_d=nplan.d_act, out_qm=nplan.qm_act, out_t=nplan.t_act,
                      epi_table=epilogue_table(nplan, epilogue))
        elif epilogue == _lib.EPI_I32:
            if out is None:
                out = torch.empty((M, _round_up(plan.n, 4)), dtype=torch.int32, device=dev)
        elif out is None:
            out = torch.empty((M, _round_up(plan.n, 4)), dtype=torch.float32, device=dev)
        wimg, wfmt = plan.gemm_weights()
        _lib.gemm(codes, M, plan.kpad, wimg, wfmt, plan.n, plan.npad, plan.d_act, plan.d_wt,
                  plan.bias_pad, epilogue, out, **oq)
        return out

    def a32_fits(self, plan: QuantPlan, epilogue: int) -> bool:
        """Whether gemm_codes_a32 runs this layer (qvit_gemm_a32_fits: the fc1 shape class)."""
        return _lib.gemm_a32_fits(plan.kpad, plan.wfmt, plan.n, plan.npad, epilogue)

    def gemm_codes_a32(self, codes_t32: torch.Tensor, M: int, plan: QuantPlan, epilogue: int, out: torch.Tensor,
                       next_layer: "QuantizeMixin") -> torch.Tensor:
        """gemm_codes for the int8-code epilogues on QVIT_ACT_T32 activation codes (qvit_gemm_a32: weight-stationary
        schedule, same codes as gemm_codes on the row-major codes)."""
        nplan = next_layer.quant_plan()
        _lib.gemm_a32(codes_t32, M, plan.kpad, plan.packed_codes(), plan.wfmt, plan.n, plan.npad, plan.d_act, plan.d_wt,
                      plan.bias_pad, epilogue, out, out_qtype=nplan.qtype, out_d=nplan.d_act, out_qm=nplan.qm_act,
                      out_t=nplan.t_act, epi_table=epilogue_table(nplan, epilogue))
        return out


_GELU_MAX_SLOPE = 1.1289   # max of d/dv [v Phi(v)] (at v ~ 1.41)


def _gelu(v: float) -> float:
    return 0.5 * v * (1.0 + math.erf(v / math.sqrt(2.0)))


def epilogue_table_geometry(qtype: int, d: float, qm: float, t: float, level: float, gelu: bool):
    """(v_lo, w, nb) of the int8-epilogue code table for an activation quantizer (host scalars), or None
    when the table would be too large (the GEMM then evaluates every element directly). Only the
    speed depends on this choice: the device validates the table and falls back on its own."""
    if qtype == _lib.QT_ULTRA_ACT or not (d > 0 and math.isfinite(d) and math.isfinite(qm) and qm != 0):
        return None
    L = int(abs(level))
    if L < 1 or L > 127:
        return None
    p = (lambda x: x) if qtype == _lib.QT_LINEAR else (lambda x: x ** (1.0 / t) if x > 0 else 0.0)
    if qtype == _lib.QT_NONLINEAR and not (t > 0 and math.isfinite(t)):
        return None
    # magnitude thresholds of the codes 1..L in x = gelu(v) (or v): x_k = p((k - 1/2) d), capped at |q_m|
    xs = [min(p((k - 0.5) * d), abs(qm)) for k in range(1, L + 1)]
    gaps = [b - a for a, b in zip(xs, xs[1:]) if b > a]
    min_gap = min(gaps + [2.0 * xs[0]])   # change points +-x_1 around the zero code are 2 x_1 apart
    x_sat, x_one = xs[-1], xs[0]
    if gelu:
        lo_v, hi_v = 0.0, max(1.0, x_sat)      # gelu(v) >= x_sat: v_hi
        while _gelu(hi_v) < x_sat * 1.02:
            hi_v *= 1.5
        v_hi = hi_v + 0.05
        if x_one >= 0.17:                       # min gelu = -0.17: no negative codes
            v_lo = -0.05
        else:                                   # most negative v with |gelu(v)| >= x_1
            a, b = -40.0, -0.7518
            for _ in range(80):
                mid = 0.5 * (a + b)
                if abs(_gelu(mid)) >= x_one * 0.98:
                    b = mid
                else:
                    a = mid
            v_lo = a - 0.05
        w = 0.8 * min_gap / _GELU_MAX_SLOPE
    else:
        v_hi, v_lo = x_sat * 1.02 + 1e-3, -(x_sat * 1.02 + 1e-3)
        w = 0.8 * min_gap
    nb = int(math.ceil((v_hi - v_lo) / w)) + 1
    if nb > _lib.EPI_TABLE_MAX_NB:
        return None
    return v_lo, w, nb


def epilogue_table(nplan: QuantPlan, epilogue: int) -> Optional[torch.Tensor]:
    """Device code table for a GEMM epilogue that quantizes with `nplan`'s activation quantizer (cached
    on that plan: it depends only on the quantizer's scalars)."""
    key = "epi_table_gelu" if epilogue == _lib.EPI_I8_GELU else "epi_table"
    if key not in nplan.extra:
        host = nplan.extra.get("act_host")
        geo = epilogue_table_geometry(*host, gelu=epilogue == _lib.EPI_I8_GELU) if host else None
        nplan.extra[key] = None if geo is None else _lib.epi_table_build(
            epilogue, nplan.qtype, nplan.d_act, nplan.qm_act, nplan.t_act, 0, geo[0], geo[1], geo[2], nplan.device)
    return nplan.extra[key]


def initialize_quant_layer(layer, num_bits: int = 16,
                           quant_type: QuantizationType = QuantizationType.SYMMETRIC_LINEAR,
                           quant_mode: QuantizationMode = QuantizationMode.WEIGHT_ONLY) -> None:
    """quant_layers.py:413-440: q_m = max|W|, d = q_m / (2^(b-1) - 1), t = 1; the activation
    parameters start from the same weight statistics (:436-438)."""
    if not isinstance(layer, (QuantizeConv2d, QuantizeLinear)):
        return
    num_bits = float(num_bits)
    t_quant_init = 1.0
    q_s = torch.tensor(0.0, device=layer.weight.device)
    qm_quant_init = torch.max(torch.abs(layer.weight))
    d_quant_init = (qm_quant_init - q_s) / (2 ** (num_bits - 1) - 1)
    nn.init.constant_(layer.d_quant_wt, d_quant_init)
    nn.init.constant_(layer.q_m_wt, qm_quant_init)
    if quant_type == QuantizationType.SYMMETRIC_NONLINEAR:
        nn.init.constant_(layer.t_quant_wt, t_quant_init)
    if quant_mode == QuantizationMode.WEIGHT_AND_ACTIVATION:
        nn.init.constant_(layer.d_quant_act, d_quant_init)
        nn.init.constant_(layer.q_m_act, qm_quant_init)
        if quant_type == QuantizationType.SYMMETRIC_NONLINEAR:
            nn.init.constant_(layer.t_quant_act, t_quant_init)
    layer.invalidate()


class QuantizeLinear(nn.Linear, QuantizeMixin):
    """quant_layers.py:443-499."""

    def __init__(self, in_features, out_features, bias=True, d_quant_init=1.0, t_quant_init=1.0, q_m_init=1.0,
                 quant_type=QuantizationType.SYMMETRIC_LINEAR, quant_mode=QuantizationMode.WEIGHT_ONLY):
        nn.Linear.__init__(self, in_features, out_features, bias)
        self.init_quantization(d_quant_init, t_quant_init, q_m_init, quant_type, quant_mode)

    @staticmethod
    def from_module(module=None, d_quant_init=1.0, t_quant_init=1.0, q_m_init=1.0,
                    quant_type=QuantizationType.SYMMETRIC_LINEAR, quant_mode=QuantizationMode.WEIGHT_ONLY,
                    quant_init_by_module=True, num_bits=8):
        q = QuantizeLinear(in_features=module.in_features, out_features=module.out_features,
                           bias=module.bias is not None, d_quant_init=d_quant_init, t_quant_init=t_quant_init,
                           q_m_init=q_m_init, quant_type=quant_type, quant_mode=quant_mode)
        q = q.to(device=module.weight.device)
        q.weight.data.copy_(module.weight.data)
        if module.bias is not None:
            q.bias.data.copy_(module.bias.data)
        if quant_init_by_module:
            initialize_quant_layer(q, num_bits=num_bits, quant_type=quant_type, quant_mode=quant_mode)
        return q

    def forward(self, input_: torch.Tensor) -> torch.Tensor:
        self._check_input(input_)
        plan = self.quant_plan()
        if plan.int_path:
            x2 = input_.detach().reshape(-1, plan.k)
            if x2.dtype != torch.float32 or x2.stride(-1) != 1:
                x2 = x2.float().contiguous()
            codes = self._act_codes(x2, plan)
            trace_codes(self, codes, plan.k)
            out = self.gemm_codes(codes, plan, _lib.EPI_F32)
            if out.shape[1] != plan.n:
                out = out[:, :plan.n].contiguous()
            return out.view(*input_.shape[:-1], plan.n)
        if plan.extra.get("wonly"):
            x = self.quantize_act(input_.float()) if self.quant_mode == QuantizationMode.WEIGHT_AND_ACTIVATION \
                else input_
            y = self._wonly_rows(x.detach().reshape(-1, plan.k), plan)
            return y.reshape(*input_.shape[:-1], plan.n)
        x = self.quantize_act(input_.float()) if self.quant_mode == QuantizationMode.WEIGHT_AND_ACTIVATION \
            else input_.float()
        return F.linear(x.detach(), self.w_fakequant(plan), None if self.bias is None else self.bias.detach())


class QuantizeConv2d(nn.Conv2d, QuantizeMixin):
    """quant_layers.py:502-587."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=1, dilation=1, groups=1,
                 bias=False, d_quant_init=1.0, t_quant_init=1.0, q_m_init=1.0,
                 quant_type=QuantizationType.SYMMETRIC_LINEAR, quant_mode=QuantizationMode.WEIGHT_ONLY):
        nn.Conv2d.__init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation, groups,
                           bias=bias)
        self.init_quantization(d_quant_init, t_quant_init, q_m_init, quant_type, quant_mode)

    @staticmethod
    def from_module(module=None, d_quant_init=1.0, t_quant_init=1.0, q_m_init=1.0,
                    quant_type=QuantizationType.SYMMETRIC_LINEAR, quant_mode=QuantizationMode.WEIGHT_ONLY,
                    quant_init_by_module=True, num_bits=8):
        q = QuantizeConv2d(in_channels=module.in_channels, out_channels=module.out_channels,
                           kernel_size=module.kernel_size, stride=module.stride, padding=module.padding,
                           dilation=module.dilation, groups=module.groups, bias=module.bias is not None,
                           d_quant_init=d_quant_init, t_quant_init=t_quant_init, q_m_init=q_m_init,
                           quant_type=quant_type, quant_mode=quant_mode)
        q = q.to(device=module.weight.device)
        q.weight.data.copy_(module.weight.data)
        if module.bias is not None:
            q.bias.data.copy_(module.bias.data)
        if quant_init_by_module:
            initialize_quant_layer(q, num_bits=num_bits, quant_type=quant_type, quant_mode=quant_mode)
        return q

    def _int_conv_ok(self) -> bool:
        return (self.groups == 1 and self.padding_mode == "zeros" and not isinstance(self.padding, str))

    def conv_codes_gemm(self, input_: torch.Tensor, epilogue: int = _lib.EPI_F32):
        """im2col + quantize + contraction. Returns ([B*OH*OW, Cout] NHWC rows, (B, OH, OW))."""
        plan = self.quant_plan()
        x = input_.detach()
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.float().contiguous()
        B, C, H, W = x.shape
        kh, kw = self.kernel_size
        sh, sw = self.stride
        ph, pw = self.padding
        dh, dw = self.dilation
        OH = (H + 2 * ph - dh * (kh - 1) - 1) // sh + 1
        OW = (W + 2 * pw - dw * (kw - 1) - 1) // sw + 1
        codes = torch.empty((B * OH * OW, plan.kpad), dtype=torch.int8, device=x.device)
        _lib.im2col_quant_i8(x, kh, kw, sh, sw, ph, pw, dh, dw, plan.qtype, plan.d_act, plan.qm_act, plan.t_act, 0,
                             codes, plan.kpad)
        trace_codes(self, codes, plan.k)
        out = self.gemm_codes(codes, plan, epilogue)
        return out, (B, OH, OW)

    def forward(self, input_: torch.Tensor) -> torch.Tensor:
        self._check_input(input_)
        plan = self.quant_plan()
        if plan.int_path and self._int_conv_ok():
            out, (B, OH, OW) = self.conv_codes_gemm(input_)
            n = plan.n
            return out[:, :n].reshape(B, OH, OW, n).permute(0, 3, 1, 2).contiguous()
        x = self.quantize_act(input_.float()) if self.quant_mode == QuantizationMode.WEIGHT_AND_ACTIVATION \
            else input_.float()
        if plan.extra.get("wonly") and self._int_conv_ok():
            # weight-only / wide levels: an implicit GEMM of the NCHW input against the packed codes
            # (qvit_conv_wonly: patches gathered in the kernel, NCHW out)
            return _lib.conv_wonly(x.detach(), self.kernel_size, self.stride, self.padding, self.dilation,
                                   plan.packed, plan.wfmt, plan.n, plan.npad, plan.kpad, plan.d_wt, plan.bias_pad)
        w = self.w_fakequant(plan).view_as(self.weight)
        return F.conv2d(x.detach(), w, None if self.bias is None else self.bias.detach(), self.stride,
                        self.padding, self.dilation, self.groups)


LAYER_TO_QUANTLAYER = {"Linear": QuantizeLinear, "Conv2d": QuantizeConv2d}
