"""Vision Transformer caller of the quantized path — mirrors QViT_with_GETA/vit_model.py.

Same classes, constructor arguments, attribute names and state_dict keys as the reference
(PatchEmbed 46-103, ViTAttention 106-153, Mlp 156-177, Block 180-208, VisionTransformer 211-328,
_init_vit_weights 331-346, factories 351-483), so reference checkpoints / state_dicts load as-is and
model_to_quantize_model swaps the same 50 layers (ViT-B/16).

When every GEMM site is a QuantizeLinear / QuantizeConv2d on its integer path and the input is on
a ROCm device, forward() runs the fused MI355X pipeline per block (one residual buffer, updated in
place by the GEMM epilogues):
    LayerNorm+act-quant -> qkv projection + attention + proj's act-quant in one kernel
    (qvit_qkv_attention, N <= 208; longer sequences: qkv GEMM to fp16 hi/lo head planes -> streaming
    attention) -> proj GEMM (+= residual) -> LayerNorm+act-quant -> fc1 GEMM with GELU and fc2's
    act-quant fused (int8 codes out) -> fc2 GEMM (+= residual)
Otherwise each module runs on its own (still the HIP kernels for every quantized layer).
"""
from __future__ import annotations

from collections import OrderedDict
from functools import partial
from typing import Optional

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import quant_layers as _ql
from .quant_layers import QuantizationMode, QuantizeConv2d, QuantizeLinear, epilogue_table, trace_codes

# The residual GEMMs (proj, fc2) run the following LayerNorm + quantizer behind their tiles (qvit_gemm_resid_ln)
# instead of as a separate launch when QVIT_FUSE_LN=1 (or FUSE_RESID_LN = True). Off by default: the fused
# form is bit-identical but measured slower (the LayerNorm of a 128-row block
# runs on the one workgroup that completes the block and stalls its tile pipeline).
FUSE_RESID_LN = os.environ.get("QVIT_FUSE_LN", "0") == "1"
# fc1 on the weight-stationary schedule (norm2 writes QVIT_ACT_T32 codes, qvit_gemm_a32) instead of the tile
# schedule when QVIT_FC1_A32=1 (or FC1_WEIGHT_STATIONARY = True). Off by default: bit-identical, faster on
# full-range random codes but 2-3 % slower on the model's own activations, and its LayerNorm 4 % slower
# (profiles/r05_fc1_weight_stationary_ab.txt).
FC1_WEIGHT_STATIONARY = os.environ.get("QVIT_FC1_A32", "0") == "1"

# Benchmark instrumentation: when KERNEL_TIMING[name] is a list (name in "fc1", "fc2", "proj",
# "qkv_attn", "ln"), the fused block appends a (start, end) HIP event pair recorded on the launch
# stream (torch's current stream, which every _lib entry point launches on) around each such launch.
KERNEL_TIMING: dict = {}


class _timed:
    __slots__ = ("ev", "e0")

    def __init__(self, name: str):
        self.ev = KERNEL_TIMING.get(name)

    def __enter__(self):
        if self.ev is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()

    def __exit__(self, *exc):
        if self.ev is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.ev.append((self.e0, e1))


def drop_path(x, drop_prob: float = 0., training: bool = False):
    """vit_model.py:14-30."""
    if drop_prob == 0. or not training:
        return x
    keep_prob = 1 - drop_prob
    shape = (x.shape[0],) + (1,) * (x.ndim - 1)
    random_tensor = keep_prob + torch.rand(shape, dtype=x.dtype, device=x.device)
    random_tensor.floor_()
    return x.div(keep_prob) * random_tensor


class DropPath(nn.Module):
    def __init__(self, drop_prob=None):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        return drop_path(x, self.drop_prob, self.training)


class PatchEmbed(nn.Module):
    """vit_model.py:46-103."""

    def __init__(self, img_size=224, patch_size=16, in_c=3, embed_dim=768, norm_layer=None):
        super().__init__()
        img_size = (img_size, img_size)
        patch_size = (patch_size, patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.grid_size = (img_size[0] // patch_size[0], img_size[1] // patch_size[1])
        self.num_patches = self.grid_size[0] * self.grid_size[1]
        self.proj = nn.Conv2d(in_c, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer else nn.Identity()

    def forward(self, x):
        B, C, H, W = x.shape
        if not torch.jit.is_tracing():
            assert H == self.img_size[0] and W == self.img_size[1], \
                f"Input image size ({H}*{W}) doesn't match model ({self.img_size[0]}*{self.img_size[1]})."
        if _conv_int_path(self.proj, x):
            # im2col+quant -> GEMM rows are already (b, patch) x embed: no flatten/transpose copy
            out, (B, OH, OW) = self.proj.conv_codes_gemm(x)
            n = self.proj.quant_plan().n
            x = out[:, :n].reshape(B, OH * OW, n)
        else:
            x = self.proj(x).flatten(2).transpose(1, 2)
        x = self.norm(x)
        return x


class ViTAttention(nn.Module):
    """vit_model.py:106-153."""

    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None, attn_drop_ratio=0., proj_drop_ratio=0.):
        super().__init__()
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.head_dim = head_dim
        self.scale = qk_scale or head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop_ratio)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop_ratio)

    def hip_ok(self, qkv: torch.Tensor) -> bool:
        return (qkv.is_cuda and qkv.dtype == torch.float32 and self.head_dim == 64 and qkv.dim() == 2
                and qkv.stride(1) == 1 and not (self.training and self.attn_drop.p > 0))

    def split_ok(self, p_qkv) -> bool:
        """The fused block can take the split-operand path (qvit_gemm_qkv_split -> qvit_attention_split)."""
        return (self.head_dim == 64 and p_qkv.n == 3 * self.num_heads * 64
                and not (self.training and self.attn_drop.p > 0))

    def core_hip(self, qkv: torch.Tensor, B: int, N: int, out: torch.Tensor, out_mode: int = _lib.ATT_F32,
                 in_scale: float = 1.0, plan=None) -> torch.Tensor:
        """The same op on the fused HIP kernel (qvit_attention); with out_mode ATT_I8 it also applies the
        activation quantizer of `plan` (the proj layer) and writes its int8 codes."""
        if out_mode == _lib.ATT_I8:
            return _lib.attention(qkv, B, N, self.num_heads, 64, self.scale, out, out_mode, in_scale, plan.qtype,
                                  plan.d_act, plan.qm_act, plan.t_act)
        return _lib.attention(qkv, B, N, self.num_heads, 64, self.scale, out, out_mode, in_scale)

    def core(self, qkv: torch.Tensor, B: int, N: int) -> torch.Tensor:
        """softmax(q k^T * scale) v on the qkv projection (vit_model.py:133-149), fp32."""
        if self.hip_ok(qkv.reshape(B * N, -1)):
            q2 = qkv.reshape(B * N, -1)
            out = torch.empty((B * N, self.num_heads * 64), dtype=torch.float32, device=qkv.device)
            amax = float(q2.abs().max()) if q2.numel() else 0.0   # unfused path: no plan bound, one sync
            scale = 1.0 if amax <= 16384.0 else 2.0 ** -math.ceil(math.log2(amax / 16384.0))
            return self.core_hip(q2, B, N, out, _lib.ATT_F32, scale).reshape(B, N, -1)
        qkv = qkv.reshape(B, N, 3, self.num_heads, -1).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        attn = (q @ k.transpose(-2, -1)) * self.scale
        attn = attn.softmax(dim=-1)
        attn = self.attn_drop(attn)
        return (attn @ v).transpose(1, 2).reshape(B, N, -1)

    def forward(self, x):
        B, N, C = x.shape
        x = self.core(self.qkv(x), B, N)
        x = self.proj(x)
        x = self.proj_drop(x)
        return x


class Mlp(nn.Module):
    """vit_model.py:156-177."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        x = self.fc1(x)
        x = self.act(x)
        x = self.drop(x)
        x = self.fc2(x)
        x = self.drop(x)
        return x


def attention_in_scale(p_qkv) -> float:
    """Power of two that keeps the qkv projection (|x| <= its plan's output bound) inside the fp16
    range of the attention kernel's hi/lo split (qvit_attention's in_scale)."""
    bound = p_qkv.extra.get("out_bound", float("inf"))
    if bound <= 16384.0:
        return 1.0
    if not math.isfinite(bound):
        raise _lib.QvitError("qkv projection has no finite output bound; cannot size the attention input scale")
    return 2.0 ** -math.ceil(math.log2(bound / 16384.0))


def _qlinear_int(m: nn.Module) -> bool:
    return (isinstance(m, QuantizeLinear) and m.quant_mode == QuantizationMode.WEIGHT_AND_ACTIVATION
            and m.quant_plan().int_path)


def _conv_int_path(m: nn.Module, x: torch.Tensor) -> bool:
    return (isinstance(m, QuantizeConv2d) and x.is_cuda and m.quant_mode == QuantizationMode.WEIGHT_AND_ACTIVATION
            and m._int_conv_ok() and m.quant_plan().int_path)


def _inactive(m: nn.Module) -> bool:
    """Dropout / DropPath / Identity that does nothing in the current mode."""
    if isinstance(m, nn.Identity):
        return True
    if isinstance(m, nn.Dropout):
        return m.p == 0.0 or not m.training
    if isinstance(m, DropPath):
        return not m.drop_prob or not m.training
    return False


class Block(nn.Module):
    """vit_model.py:180-208."""

    def __init__(self, dim, num_heads, mlp_ratio=4., qkv_bias=False, qk_scale=None, drop_ratio=0.,
                 attn_drop_ratio=0., drop_path_ratio=0., act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = ViTAttention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                 attn_drop_ratio=attn_drop_ratio, proj_drop_ratio=drop_ratio)
        self.drop_path = DropPath(drop_path_ratio) if drop_path_ratio > 0. else nn.Identity()
        self.norm2 = norm_layer(dim)
        mlp_hidden_dim = int(dim * mlp_ratio)
        self.mlp = Mlp(in_features=dim, hidden_features=mlp_hidden_dim, act_layer=act_layer, drop=drop_ratio)

    def fused_ok(self, x: torch.Tensor) -> bool:
        a, m = self.attn, self.mlp
        return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3
                and isinstance(self.norm1, nn.LayerNorm) and isinstance(self.norm2, nn.LayerNorm)
                and self.norm1.elementwise_affine and self.norm2.elementwise_affine
                and isinstance(m.act, nn.GELU) and m.act.approximate == "none"
                and _inactive(self.drop_path) and _inactive(a.attn_drop) and _inactive(a.proj_drop)
                and _inactive(m.drop)
                and all(_qlinear_int(l) for l in (a.qkv, a.proj, m.fc1, m.fc2)))

    def forward_fused_(self, x: torch.Tensor) -> torch.Tensor:
        """In-place fused block on a contiguous [B, N, C] fp32 residual buffer (owned by caller)."""
        return self.forward_fused_chain_(x)[0]

    def ln_fusable(self, x2: torch.Tensor, norm: nn.LayerNorm, p_res: QuantPlan) -> bool:
        """Whether the residual GEMM with plan p_res can run `norm` (+ the next quantizer) behind its tiles."""
        C = x2.shape[1]
        return (FUSE_RESID_LN and p_res.n == C and C % 4 == 0 and C <= 1024 and x2.stride(0) == C
                and x2.shape[0] * C * 4 < 2 ** 31 and norm.weight is not None and norm.bias is not None
                and norm.weight.is_contiguous() and norm.bias.is_contiguous())

    def resid_ln_(self, codes_in: torch.Tensor, p_res: QuantPlan, x2: torch.Tensor, norm: nn.LayerNorm,
                  p_next: QuantPlan) -> torch.Tensor:
        """x2 += layer(codes_in) (the proj / fc2 contraction), then norm(x2) quantized with p_next's activation
        quantizer -> int8 codes [M, p_next.kpad] (qvit_gemm_resid_ln: one launch)."""
        M, C = x2.shape
        out = torch.empty((M, p_next.kpad), dtype=torch.int8, device=x2.device)
        _lib.gemm_resid_ln(codes_in, M, p_res.kpad, p_res.packed_codes(), p_res.wfmt, p_res.n, p_res.npad, p_res.d_act,
                           p_res.d_wt, p_res.bias_pad, x2, norm.weight, norm.bias, norm.eps, p_next.qtype,
                           p_next.d_act, p_next.qm_act, p_next.t_act, 0, epilogue_table(p_next, _lib.EPI_I8), out,
                           p_next.kpad)
        return out

    def forward_fused_chain_(self, x: torch.Tensor, codes_in: Optional[torch.Tensor] = None,
                             next_block: Optional["Block"] = None):
        """forward_fused_ with the LayerNorms carried by the residual GEMMs: `codes_in` = this block's norm1
        codes when the previous block's fc2 produced them; with `next_block`, fc2 also produces that block's
        norm1 codes. Returns (x, next_block's norm1 codes or None)."""
        B, N, C = x.shape
        M = B * N
        x2 = x.view(M, C)
        a, m = self.attn, self.mlp
        # x + attn(norm1(x))
        p_qkv = a.qkv.quant_plan()
        if codes_in is not None:
            codes = codes_in
        else:
            codes = torch.empty((M, p_qkv.kpad), dtype=torch.int8, device=x.device)
            with _timed("ln"):
                _lib.layernorm_quant_i8(x2, self.norm1.weight, self.norm1.bias, self.norm1.eps, p_qkv.qtype,
                                        p_qkv.d_act, p_qkv.qm_act, p_qkv.t_act, 0, codes, p_qkv.kpad,
                                        code_table=epilogue_table(p_qkv, _lib.EPI_I8))
        trace_codes(a.qkv, codes, C)
        p_proj = a.proj.quant_plan()
        if (a.split_ok(p_qkv) and N <= _lib.QKV_ATT_MAX_N and p_qkv.wfmt == _lib.W4 and p_qkv.kpad <= 65536
                and p_qkv.kpad % 256 == 0 and a.num_heads * 64 <= _lib.QKV_ATT_MAX_C):
            # qkv projection + attention + proj's activation quantizer in one kernel (q/k/v stay on chip)
            out = torch.empty((M, p_proj.kpad), dtype=torch.int8, device=x.device)
            if p_proj.kpad != a.num_heads * 64:
                out[:, a.num_heads * 64:].zero_()
            in_scale, tab = attention_in_scale(p_qkv), epilogue_table(p_proj, _lib.EPI_I8)
            with _timed("qkv_attn"):
                _lib.qkv_attention(codes, B, N, p_qkv.kpad, p_qkv.packed_codes(), p_qkv.npad, p_qkv.d_act, p_qkv.d_wt,
                                   p_qkv.bias_pad, a.num_heads, a.scale, out, _lib.ATT_I8, in_scale,
                                   p_proj.qtype, p_proj.d_act, p_proj.qm_act, p_proj.t_act, epi_table=tab)
            trace_codes(a.proj, out, p_proj.k)
            p_fc1 = m.fc1.quant_plan()
            if self.ln_fusable(x2, self.norm2, p_proj):
                with _timed("proj"):
                    ln_codes = self.resid_ln_(out, p_proj, x2, self.norm2, p_fc1)
                return self._mlp_fused_(x, x2, M, ln_codes, next_block)
            with _timed("proj"):
                a.proj.gemm_codes(out, p_proj, _lib.EPI_F32_RESID, out=x2)
            return self._mlp_fused_(x, x2, M, None, next_block)
        if a.split_ok(p_qkv):
            # qkv as pre-scaled fp16 hi/lo head planes, then attention + proj's activation quantizer
            in_scale = attention_in_scale(p_qkv)
            hi = torch.empty(M * p_qkv.n, dtype=torch.float16, device=x.device)
            lo = torch.empty(M * p_qkv.n, dtype=torch.float16, device=x.device)
            wimg, wfmt = p_qkv.gemm_weights()
            _lib.gemm_qkv_split(codes, M, p_qkv.kpad, wimg, wfmt, p_qkv.n, p_qkv.npad, p_qkv.d_act,
                                p_qkv.d_wt, p_qkv.bias_pad, N, in_scale, hi, lo)
            codes = torch.empty((M, p_proj.kpad), dtype=torch.int8, device=x.device)
            if p_proj.kpad != a.num_heads * 64:
                codes[:, a.num_heads * 64:].zero_()
            _lib.attention_split(hi, lo, B, N, a.num_heads, 64, a.scale, codes, _lib.ATT_I8, in_scale,
                                 p_proj.qtype, p_proj.d_act, p_proj.qm_act, p_proj.t_act,
                                 epi_table=epilogue_table(p_proj, _lib.EPI_I8))
            trace_codes(a.proj, codes, p_proj.k)
            a.proj.gemm_codes(codes, p_proj, _lib.EPI_F32_RESID, out=x2)
            return self._mlp_fused_(x, x2, M, None, next_block)
        qkv = a.qkv.gemm_codes(codes, p_qkv, _lib.EPI_F32)
        if qkv.shape[1] != p_qkv.n:
            qkv = qkv[:, :p_qkv.n]
        if a.hip_ok(qkv):
            # attention core + proj's activation quantizer in one kernel: int8 codes for the proj GEMM
            codes = torch.empty((M, p_proj.kpad), dtype=torch.int8, device=x.device)
            if p_proj.kpad != a.num_heads * 64:
                codes[:, a.num_heads * 64:].zero_()
            a.core_hip(qkv, B, N, codes, _lib.ATT_I8, attention_in_scale(p_qkv), p_proj)
        else:
            h = a.core(qkv, B, N).reshape(M, -1)
            codes = a.proj._act_codes(h if h.is_contiguous() else h.contiguous(), p_proj)
        trace_codes(a.proj, codes, p_proj.k)
        a.proj.gemm_codes(codes, p_proj, _lib.EPI_F32_RESID, out=x2)
        return self._mlp_fused_(x, x2, M, None, next_block)

    def _mlp_fused_(self, x: torch.Tensor, x2: torch.Tensor, M: int, codes_in: Optional[torch.Tensor] = None,
                    next_block: Optional["Block"] = None):
        """x + mlp(norm2(x)) in place on the residual buffer (codes_in: norm2's codes, from the proj GEMM).
        Returns (x, next_block's norm1 codes when fc2 produced them, else None)."""
        m = self.mlp
        p_fc1 = m.fc1.quant_plan()
        p_fc2 = m.fc2.quant_plan()
        hid = torch.empty((M, p_fc2.kpad), dtype=torch.int8, device=x.device)
        if p_fc2.kpad != p_fc1.n:
            hid[:, p_fc1.n:].zero_()
        if (FC1_WEIGHT_STATIONARY and codes_in is None and m.fc1.a32_fits(p_fc1, _lib.EPI_I8_GELU)
                and self.norm2.weight.is_contiguous()):
            # norm2's codes in the MFMA operand order of the weight-stationary fc1 (qvit_gemm_a32): every fragment
            # load of the GEMM one contiguous KiB
            codes = torch.empty(_lib.t32_rows(M) * p_fc1.kpad, dtype=torch.int8, device=x.device)
            with _timed("ln"):
                _lib.layernorm_quant_i8_t32(x2, self.norm2.weight, self.norm2.bias, self.norm2.eps, p_fc1.qtype,
                                            p_fc1.d_act, p_fc1.qm_act, p_fc1.t_act, 0, codes, p_fc1.kpad,
                                            code_table=epilogue_table(p_fc1, _lib.EPI_I8))
            if _ql.CODE_TRACE is not None:
                trace_codes(m.fc1, _lib.t32_to_rows(codes, M, p_fc1.kpad), p_fc1.k)
            with _timed("fc1"):
                m.fc1.gemm_codes_a32(codes, M, p_fc1, _lib.EPI_I8_GELU, hid, m.fc2)
            return self._fc2_fused_(x, x2, hid, p_fc2, next_block)
        if codes_in is not None:
            codes = codes_in
        else:
            codes = torch.empty((M, p_fc1.kpad), dtype=torch.int8, device=x.device)
            with _timed("ln"):
                _lib.layernorm_quant_i8(x2, self.norm2.weight, self.norm2.bias, self.norm2.eps, p_fc1.qtype,
                                        p_fc1.d_act, p_fc1.qm_act, p_fc1.t_act, 0, codes, p_fc1.kpad,
                                        code_table=epilogue_table(p_fc1, _lib.EPI_I8))
        trace_codes(m.fc1, codes, p_fc1.k)
        with _timed("fc1"):
            m.fc1.gemm_codes(codes, p_fc1, _lib.EPI_I8_GELU, out=hid, next_layer=m.fc2)
        return self._fc2_fused_(x, x2, hid, p_fc2, next_block)

    def _fc2_fused_(self, x: torch.Tensor, x2: torch.Tensor, hid: torch.Tensor, p_fc2: QuantPlan,
                    next_block: Optional["Block"] = None):
        m = self.mlp
        trace_codes(m.fc2, hid, p_fc2.k)
        if next_block is not None and self.ln_fusable(x2, next_block.norm1, p_fc2):
            with _timed("fc2"):
                nxt = self.resid_ln_(hid, p_fc2, x2, next_block.norm1, next_block.attn.qkv.quant_plan())
            return x, nxt
        with _timed("fc2"):
            m.fc2.gemm_codes(hid, p_fc2, _lib.EPI_F32_RESID, out=x2)
        return x, None

    def forward(self, x):
        if self.fused_ok(x):
            return self.forward_fused_(x.contiguous().clone())
        x = x + self.drop_path(self.attn(self.norm1(x)))
        x = x + self.drop_path(self.mlp(self.norm2(x)))
        return x


class VisionTransformer(nn.Module):
    """vit_model.py:211-328."""

    def __init__(self, img_size=224, patch_size=16, in_c=3, num_classes=1000, embed_dim=768, depth=12,
                 num_heads=12, mlp_ratio=4.0, qkv_bias=True, qk_scale=None, representation_size=None,
                 distilled=False, drop_ratio=0., attn_drop_ratio=0., drop_path_ratio=0., embed_layer=PatchEmbed,
                 norm_layer=None, act_layer=None):
        super().__init__()
        self.num_classes = num_classes
        self.num_features = self.embed_dim = embed_dim
        self.num_tokens = 2 if distilled else 1
        norm_layer = norm_layer or partial(nn.LayerNorm, eps=1e-6)
        act_layer = act_layer or nn.GELU
        self.patch_embed = embed_layer(img_size=img_size, patch_size=patch_size, in_c=in_c, embed_dim=embed_dim)
        num_patches = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.dist_token = nn.Parameter(torch.zeros(1, 1, embed_dim)) if distilled else None
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches + self.num_tokens, embed_dim))
        self.pos_drop = nn.Dropout(p=drop_ratio)
        dpr = [x.item() for x in torch.linspace(0, drop_path_ratio, depth)]
        self.blocks = nn.Sequential(*[
            Block(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale,
                  drop_ratio=drop_ratio, attn_drop_ratio=attn_drop_ratio, drop_path_ratio=dpr[i],
                  norm_layer=norm_layer, act_layer=act_layer)
            for i in range(depth)
        ])
        self.norm = norm_layer(embed_dim)
        if representation_size and not distilled:
            self.has_logits = True
            self.num_features = representation_size
            self.pre_logits = nn.Sequential(OrderedDict([
                ("fc", nn.Linear(embed_dim, representation_size)),
                ("act", nn.Tanh())
            ]))
        else:
            self.has_logits = False
            self.pre_logits = nn.Identity()
        self.head = nn.Linear(self.num_features, num_classes) if num_classes > 0 else nn.Identity()
        self.head_dist = None
        if distilled:
            self.head_dist = nn.Linear(self.embed_dim, self.num_classes) if num_classes > 0 else nn.Identity()
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        if self.dist_token is not None:
            nn.init.trunc_normal_(self.dist_token, std=0.02)
        nn.init.trunc_normal_(self.cls_token, std=0.02)
        self.apply(_init_vit_weights)

    def forward_features(self, x):
        x = self.patch_embed(x)
        if x.is_cuda and _inactive(self.pos_drop):
            # cat((cls[, dist], x)) + pos_embed in one pass: the token rows are written straight into the
            # residual buffer (the same fp32 additions as the reference's cat-then-add)
            B, T, C = x.shape
            nt = self.num_tokens
            buf = torch.empty((B, T + nt, C), dtype=x.dtype, device=x.device)
            torch.add(x, self.pos_embed[:, nt:], out=buf[:, nt:])
            buf[:, 0] = self.cls_token[:, 0] + self.pos_embed[:, 0]
            if self.dist_token is not None:
                buf[:, 1] = self.dist_token[:, 0] + self.pos_embed[:, 1]
            x = buf
        else:
            cls_token = self.cls_token.expand(x.shape[0], -1, -1)
            if self.dist_token is None:
                x = torch.cat((cls_token, x), dim=1)
            else:
                x = torch.cat((cls_token, self.dist_token.expand(x.shape[0], -1, -1), x), dim=1)
            x = self.pos_drop(x + self.pos_embed)
        # the residual stream is a fresh buffer here, so fused blocks may update it in place; a fused block's
        # fc2 also runs the next fused block's norm1 (+ its qkv quantizer)
        blocks = list(self.blocks)
        codes = None
        for i, blk in enumerate(blocks):
            if isinstance(blk, Block) and blk.fused_ok(x):
                nb = blocks[i + 1] if i + 1 < len(blocks) else None
                nb = nb if isinstance(nb, Block) and nb.fused_ok(x) else None
                x, codes = blk.forward_fused_chain_(x.contiguous(), codes, nb)
            else:
                codes = None
                x = blk(x)
        # LayerNorm is per token: only the class (and distillation) token rows reach the heads
        if self.dist_token is None:
            return self.pre_logits(self.norm(x[:, 0]))
        else:
            x = self.norm(x[:, :2])
            return x[:, 0], x[:, 1]

    def forward(self, x):
        x = self.forward_features(x)
        if self.head_dist is not None:
            x, x_dist = self.head(x[0]), self.head_dist(x[1])
            if self.training and not torch.jit.is_scripting():
                return x, x_dist
            else:
                return (x + x_dist) / 2
        else:
            x = self.head(x)
        return x


def _init_vit_weights(m):
    """vit_model.py:331-346."""
    if isinstance(m, nn.Linear):
        nn.init.trunc_normal_(m.weight, std=.01)
        if m.bias is not None:
            nn.init.zeros_(m.bias)
    elif isinstance(m, nn.Conv2d):
        nn.init.kaiming_normal_(m.weight, mode="fan_out")
        if m.bias is not None:
            nn.init.zeros_(m.bias)
    elif isinstance(m, nn.LayerNorm):
        nn.init.zeros_(m.bias)
        nn.init.ones_(m.weight)


# ---- factories (vit_model.py:351-483) -------------------------------------------------------------
def vit_base_patch16_224(num_classes: int = 1000):
    return VisionTransformer(img_size=224, patch_size=16, embed_dim=768, depth=12, num_heads=12,
                             representation_size=None, num_classes=num_classes)


def vit_base_patch16_224_in21k(num_classes: int = 21843, has_logits: bool = True):
    return VisionTransformer(img_size=224, patch_size=16, embed_dim=768, depth=12, num_heads=12,
                             representation_size=768 if has_logits else None, num_classes=num_classes)


def vit_base_patch32_224(num_classes: int = 1000):
    return VisionTransformer(img_size=224, patch_size=32, embed_dim=768, depth=12, num_heads=12,
                             representation_size=None, num_classes=num_classes)


def vit_base_patch32_224_in21k(num_classes: int = 21843, has_logits: bool = True):
    return VisionTransformer(img_size=224, patch_size=32, embed_dim=768, depth=12, num_heads=12,
                             representation_size=768 if has_logits else None, num_classes=num_classes)


def vit_large_patch16_224(num_classes: int = 1000):
    return VisionTransformer(img_size=224, patch_size=16, embed_dim=1024, depth=24, num_heads=16,
                             representation_size=None, num_classes=num_classes)


def vit_large_patch16_224_in21k(num_classes: int = 21843, has_logits: bool = True):
    return VisionTransformer(img_size=224, patch_size=16, embed_dim=1024, depth=24, num_heads=16,
                             representation_size=1024 if has_logits else None, num_classes=num_classes)


def vit_large_patch32_224_in21k(num_classes: int = 21843, has_logits: bool = True):
    return VisionTransformer(img_size=224, patch_size=32, embed_dim=1024, depth=24, num_heads=16,
                             representation_size=1024 if has_logits else None, num_classes=num_classes)


def vit_huge_patch14_224_in21k(num_classes: int = 21843, has_logits: bool = True):
    return VisionTransformer(img_size=224, patch_size=14, embed_dim=1280, depth=32, num_heads=16,
                             representation_size=1280 if has_logits else None, num_classes=num_classes)


def vit_tiny_patch16_224(num_classes: int = 1000):
    """ViT-Tiny/16 (BASELINE config 1; no reference factory — built from VisionTransformer(...))."""
    return VisionTransformer(img_size=224, patch_size=16, embed_dim=192, depth=12, num_heads=3,
                             representation_size=None, num_classes=num_classes)


def vit_large_patch16_384(num_classes: int = 1000):
    """ViT-L/16 @384 (BASELINE config 4; no reference factory — built from VisionTransformer(...))."""
    return VisionTransformer(img_size=384, patch_size=16, embed_dim=1024, depth=24, num_heads=16,
                             representation_size=None, num_classes=num_classes)
