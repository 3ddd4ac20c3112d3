"""Checkpoint conversion and on-disk formats.

* ViT: a reference `state_dict` (QViT_with_GETA/vit_model.py after model_to_quantize_model,
  quant_model.py:15-82) -> this package's VisionTransformer with the same keys, including GETA-pruned
  shapes: whole heads removed from qkv/proj (operator.py:1208-1246) and arbitrary MLP neurons removed
  from fc1/fc2 (pruning_compression.py:64-131,217-291). Shapes, depth, quantizer type and mode are read
  from the tensors themselves; the weights are packed to int4/int8 MFMA operands on the first forward.
* The reference's predict.py:43 loads a whole pickled module (`torch.load(path)` of the compressed
  model, pruning_compression.py:385). Unpickling executes code from the file, so
  `load_reference_checkpoint` only accepts tensors (`torch.load(..., weights_only=True)`): a state_dict,
  or a dict holding one under 'state_dict' / 'model' / 'model_state_dict'. A whole-module file is
  rejected with the one-line recipe that turns it into a state_dict inside the reference's environment.
* UltraNet: the npz parameter export of torch_export.py:94-131 (`generate_params`: arr_0, arr_1, ... in
  module order: conv weight [, conv bias]; BatchNorm gamma, beta, running_mean, running_var, eps) in
  both directions, for this package's UltraNetQua mirror.
* FPGA memory format of qnn_mem_process.py: weight codes packed SIMD-per-word, LSB-first, two's
  complement per element (array_to_string :11-24), rows interleaved over PEs (w_to_hls_array :83-134),
  conv weights in (out, ky, kx, in) order (:155-160), inc/bias as [PE][tiles] (:137-147); and the
  inverse, so codes exported for the accelerator can be brought back to the GPU path.
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.nn as nn

from . import vit_model
from .quant_layers import QuantizationMode, QuantizationType, QuantizeConv2d, QuantizeLinear

StateDict = Dict[str, torch.Tensor]


# ---- ViT -----------------------------------------------------------------------------------------------

def vit_config_from_state_dict(sd: StateDict, head_dim: int = 64) -> dict:
    """Architecture of a (possibly pruned) reference ViT state_dict. head_dim is the unpruned
    embed_dim / num_heads (64 for every vit_model.py factory); pruning removes whole heads only."""
    w = sd["patch_embed.proj.weight"]
    embed_dim, in_c, patch, _ = w.shape
    num_tokens = 2 if "dist_token" in sd else 1
    num_patches = sd["pos_embed"].shape[1] - num_tokens
    grid = int(round(num_patches ** 0.5))
    if grid * grid != num_patches:
        raise ValueError(f"pos_embed holds {num_patches} patch positions, not a square grid")
    depth = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"blocks\.(\d+)\.", k)] if m)
    blocks = []
    for i in range(depth):
        nq = sd[f"blocks.{i}.attn.qkv.weight"].shape[0]
        if nq % (3 * head_dim):
            raise ValueError(f"blocks.{i}.attn.qkv has {nq} outputs, not 3 x heads x {head_dim}")
        blocks.append({"heads": nq // (3 * head_dim), "hidden": sd[f"blocks.{i}.mlp.fc1.weight"].shape[0],
                       "qkv_bias": f"blocks.{i}.attn.qkv.bias" in sd})
    has_pre = "pre_logits.fc.weight" in sd
    head_w = sd.get("head.weight")
    qtype = (QuantizationType.SYMMETRIC_NONLINEAR if "patch_embed.proj.t_quant_wt" in sd
             else QuantizationType.SYMMETRIC_LINEAR)
    qmode = (QuantizationMode.WEIGHT_AND_ACTIVATION if "patch_embed.proj.d_quant_act" in sd
             else QuantizationMode.WEIGHT_ONLY)
    return {
        "img_size": grid * patch, "patch_size": patch, "in_c": in_c, "embed_dim": embed_dim, "depth": depth,
        "num_heads": embed_dim // head_dim, "head_dim": head_dim, "blocks": blocks,
        "num_classes": head_w.shape[0] if head_w is not None else 0,
        "representation_size": sd["pre_logits.fc.weight"].shape[0] if has_pre else None,
        "distilled": num_tokens == 2, "quantized": "patch_embed.proj.d_quant_wt" in sd,
        "quant_type": qtype, "quant_mode": qmode,
    }


def _quantize_tree(model: nn.Module, qtype: QuantizationType, qmode: QuantizationMode) -> None:
    """Every Linear / Conv2d becomes its quantized twin (the reference's registry swap) with
    placeholder quantizer scalars; load_state_dict then overwrites them."""
    for name, mod in list(model.named_modules()):
        cls = {nn.Linear: QuantizeLinear, nn.Conv2d: QuantizeConv2d}.get(type(mod))
        if cls is None:
            continue
        q = cls.from_module(mod, quant_type=qtype, quant_mode=qmode, quant_init_by_module=False)
        parent = model.get_submodule(".".join(name.split(".")[:-1])) if "." in name else model
        setattr(parent, name.split(".")[-1], q)


def vit_from_state_dict(sd: StateDict, head_dim: int = 64, device: Optional[torch.device] = None,
                        strict: bool = True) -> vit_model.VisionTransformer:
    """Builds this package's ViT with the state_dict's exact (pruned) shapes and loads it."""
    cfg = vit_config_from_state_dict(sd, head_dim)
    model = vit_model.VisionTransformer(
        img_size=cfg["img_size"], patch_size=cfg["patch_size"], in_c=cfg["in_c"],
        num_classes=cfg["num_classes"], embed_dim=cfg["embed_dim"], depth=cfg["depth"],
        num_heads=cfg["num_heads"], representation_size=cfg["representation_size"],
        distilled=cfg["distilled"], qkv_bias=all(b["qkv_bias"] for b in cfg["blocks"]))
    C = cfg["embed_dim"]
    for blk, b in zip(model.blocks, cfg["blocks"]):
        h, hid = b["heads"], b["hidden"]
        a = blk.attn
        if h != a.num_heads:   # whole heads pruned: head_dim and the softmax scale stay
            a.qkv = nn.Linear(C, 3 * h * head_dim, bias=b["qkv_bias"])
            a.proj = nn.Linear(h * head_dim, C)
            a.num_heads = h
        if hid != blk.mlp.fc1.out_features:
            blk.mlp.fc1 = nn.Linear(C, hid)
            blk.mlp.fc2 = nn.Linear(hid, C)
    if cfg["quantized"]:
        _quantize_tree(model, cfg["quant_type"], cfg["quant_mode"])
    model.load_state_dict(sd, strict=strict)
    model.eval()
    return model.to(device) if device is not None else model


def load_reference_checkpoint(path: str, head_dim: int = 64, device: Optional[torch.device] = None
                              ) -> vit_model.VisionTransformer:
    """A ViT checkpoint file written by the reference (state_dict form) -> this package's model."""
    try:
        obj = torch.load(path, map_location="cpu", weights_only=True)
    except Exception as e:  # a pickled nn.Module (predict.py:43) needs the reference's classes to load
        raise ValueError(
            f"{path} is not a tensor-only checkpoint ({type(e).__name__}); it is probably a whole pickled "
            "module (pruning_compression.py:385). In the reference's environment run "
            "`torch.save(torch.load(path).state_dict(), 'sd.pt')` and convert 'sd.pt' instead.") from e
    if isinstance(obj, dict):
        for key in ("state_dict", "model_state_dict", "model"):
            if key in obj and isinstance(obj[key], dict):
                obj = obj[key]
                break
    if not isinstance(obj, dict) or not all(isinstance(v, torch.Tensor) for v in obj.values()):
        raise ValueError(f"{path} does not hold a state_dict of tensors")
    return vit_from_state_dict(obj, head_dim=head_dim, device=device)


def load_weight_codes(model: nn.Module, codes: Dict[str, torch.Tensor]) -> int:
    """Binds precomputed integer weight codes to the model's quantized layers (QuantizeMixin.load_weight_codes):
    `codes` maps a layer name ("blocks.0.mlp.fc1") or its state_dict-style key ("blocks.0.mlp.fc1.weight_codes")
    to k with quantize_weight(W) == d_quant_wt * k (quant_layers.py:332-354), e.g. exported next to a
    checkpoint by the reference's own host, so the device runs on exactly the reference's int4 weights.
    Returns the number of layers bound; an unknown name is an error."""
    from .quant_layers import QuantizeMixin
    layers = {n: m for n, m in model.named_modules() if isinstance(m, QuantizeMixin)}
    n = 0
    for key, c in codes.items():
        name = key[:-len(".weight_codes")] if key.endswith(".weight_codes") else key
        if name not in layers:
            raise KeyError(f"no quantized layer named {name!r}")
        layers[name].load_weight_codes(c)
        n += 1
    return n


# ---- UltraNet npz (torch_export.py:94-131) ------------------------------------------------------------

def _ultra_param_modules(model: nn.Module) -> List[nn.Module]:
    """Modules in the export's traversal order (torch_export.py:97-127): direct subclasses of Conv2d /
    Linear (the quantized Conv2d_Q / Linear_Q; a plain nn.Conv2d is not exported) and BatchNorm1d/2d."""
    out = []
    for m in model.modules():
        if type(m).__base__ in (nn.Conv2d, nn.Linear) or type(m) in (nn.BatchNorm2d, nn.BatchNorm1d):
            out.append(m)
    return out


def ultranet_to_npz(model: nn.Module) -> Dict[str, np.ndarray]:
    """generate_params(model): arr_i in module order (conv/linear weight [+ conv bias]; BN gamma, beta,
    running_mean, running_var, eps)."""
    d: Dict[str, np.ndarray] = {}
    cnt = 0

    def put(a):
        nonlocal cnt
        d[f"arr_{cnt}"] = np.asarray(a)
        cnt += 1

    for m in _ultra_param_modules(model):
        if isinstance(m, nn.Conv2d):
            put(m.weight.detach().cpu().numpy())
            if m.bias is not None:
                put(m.bias.detach().cpu().numpy())
        elif isinstance(m, nn.Linear):   # the export writes no Linear bias (torch_export.py:112-115)
            put(m.weight.detach().cpu().numpy())
        else:
            put(m.weight.detach().cpu().numpy())
            put(m.bias.detach().cpu().numpy())
            put(m.running_mean.cpu().numpy())
            put(m.running_var.cpu().numpy())
            put(np.float64(m.eps))
    return d


@torch.no_grad()
def ultranet_from_npz(npz: Union[str, Dict[str, np.ndarray]], model: Optional[nn.Module] = None) -> nn.Module:
    """Loads a generate_params npz into an UltraNetQua mirror (a fresh one unless given)."""
    from .ultranet import UltraNetQua
    arrs = np.load(npz, allow_pickle=False) if isinstance(npz, str) else npz
    model = model if model is not None else UltraNetQua()
    cnt = 0

    def take(shape=None):
        nonlocal cnt
        a = torch.from_numpy(np.array(arrs[f"arr_{cnt}"]))
        cnt += 1
        if shape is not None and tuple(a.shape) != tuple(shape):
            raise ValueError(f"arr_{cnt - 1}: shape {tuple(a.shape)}, expected {tuple(shape)}")
        return a

    for m in _ultra_param_modules(model):
        if isinstance(m, nn.Conv2d):
            m.weight.copy_(take(m.weight.shape))
            if m.bias is not None:
                m.bias.copy_(take(m.bias.shape))
        elif isinstance(m, nn.Linear):
            m.weight.copy_(take(m.weight.shape))
        else:
            m.weight.copy_(take(m.weight.shape))
            m.bias.copy_(take(m.bias.shape))
            m.running_mean.copy_(take(m.running_mean.shape))
            m.running_var.copy_(take(m.running_var.shape))
            m.eps = float(take())
    if f"arr_{cnt}" in arrs:
        raise ValueError(f"npz holds more arrays than the model's parameters (arr_{cnt} unused)")
    return model.eval()


# ---- FPGA weight memory (qnn_mem_process.py) -----------------------------------------------------------

def pack_simd_word(values: Sequence[int], elem_bit: int) -> int:
    """array_to_string (qnn_mem_process.py:11-24): element i in bits [i*elem_bit, (i+1)*elem_bit),
    negative values two's complement in elem_bit bits. Python int (may exceed 64 bits)."""
    val = 0
    for i, v in enumerate(values):
        v = int(v)
        if v < 0:
            v += 1 << elem_bit
        val += v << (elem_bit * i)
    return val


def unpack_simd_word(word: int, n: int, elem_bit: int) -> List[int]:
    """Inverse of pack_simd_word (elements sign-extended)."""
    mask, half = (1 << elem_bit) - 1, 1 << (elem_bit - 1)
    out = []
    for i in range(n):
        v = (word >> (elem_bit * i)) & mask
        out.append(v - (1 << elem_bit) if v >= half else v)
    return out


def hls_weight_matrix(codes: np.ndarray) -> np.ndarray:
    """Conv weight codes [out][in][ky][kx] -> [out][ky*kx*in] in (ky, kx, in) order
    (qnn_mem_process.py:155-160); 2-D linear codes pass through."""
    codes = np.asarray(codes)
    return codes.transpose(0, 2, 3, 1).reshape(codes.shape[0], -1) if codes.ndim == 4 else codes


def hls_pack_weights(w: np.ndarray, w_bit: int, pe: int, simd: int) -> List[List[int]]:
    """w_to_hls_array (qnn_mem_process.py:83-134): [out][K] codes -> [pe][tiles] SIMD words; output
    channel i*pe + p goes to PE p, its SIMD words in k order (a last partial word if simd does not
    divide K)."""
    w = np.asarray(w)
    if w.shape[0] % pe:
        raise ValueError("out_ch mod pe must 0")
    K = w.shape[1]
    words = [[pack_simd_word(row[i * simd:(i + 1) * simd], w_bit) for i in range(K // simd)] for row in w]
    if K % simd:
        for o, row in enumerate(w):
            words[o].append(pack_simd_word(row[K // simd * simd:], w_bit))
    per = len(words[0])
    res = [[0] * (per * (w.shape[0] // pe)) for _ in range(pe)]
    t = 0
    for i in range(w.shape[0] // pe):
        for j in range(per):
            for p in range(pe):
                res[p][t] = words[i * pe + p][j]
            t += 1
    return res


def hls_unpack_weights(res: List[List[int]], out_ch: int, K: int, w_bit: int, pe: int, simd: int) -> np.ndarray:
    """Inverse of hls_pack_weights: [pe][tiles] words -> int32 codes [out_ch][K]."""
    per = (K + simd - 1) // simd
    w = np.zeros((out_ch, K), dtype=np.int32)
    t = 0
    for i in range(out_ch // pe):
        for j in range(per):
            n = min(simd, K - j * simd)
            for p in range(pe):
                w[i * pe + p, j * simd:j * simd + n] = unpack_simd_word(res[p][t], n, w_bit)
            t += 1
    return w


def hls_inc_bias(inc: np.ndarray, bias: np.ndarray, pe: int) -> Tuple[np.ndarray, np.ndarray]:
    """inc_bias_to_hls_array (qnn_mem_process.py:137-147): per-channel vectors -> [pe][a_tiles]."""
    return np.asarray(inc).reshape(-1, pe).T, np.asarray(bias).reshape(-1, pe).T
