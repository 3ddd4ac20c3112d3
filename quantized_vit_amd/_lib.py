"""ctypes binding of libqvit_hip.so (include/qvit_hip.h) plus thin torch-tensor wrappers.

This is the only place the Python side touches the C-ABI. There is no fallback: if the
library is missing or a GPU is required and absent, calls raise. Tensors are passed as raw
device pointers; every call is enqueued on torch's current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# QVIT_LIB: another build of the library (diagnostic A/B runs of the same tests on one box)
LIB_PATH = os.environ.get("QVIT_LIB") or os.path.join(_HERE, "libqvit_hip.so")

# ---- constants mirrored from include/qvit_hip.h ---------------------------------------------
QT_LINEAR = 0
QT_NONLINEAR = 1
QT_ULTRA_ACT = 2
QT_FORCE_CAREFUL = 0x100  # test-only: disable the guarded fast path

W4 = 4
W8 = 8
W4R = 40  # qvit_gemm / qvit_gemm_qkv_split only: a W4 image re-ordered by qvit_pack_weight_w4r
W8R = 80  # qvit_gemm / qvit_gemm_qkv_split only: a W4 image as 16x-scaled int8 operands (qvit_pack_weight_w8r)
W16 = 16  # qvit_gemm_wonly only: balanced base-256 digits as W8 images, two (|k| <= 32639) or
W24 = 24  # three (|k| < 2^23)

EPI_F32 = 0
EPI_F32_RESID = 1
EPI_I8_GELU = 2
EPI_I8 = 3
EPI_I32 = 4
EPI_QKV_SPLIT = 5   # qvit_gemm_qkv_split only

ATT_F32 = 0
ATT_I8 = 1

ULTRA_CODES = 0
ULTRA_CODES_POOL = 1
ULTRA_F32 = 2

EPI_TABLE_MAX_NB = 3800

TILE_N = 256
TILE_K = 128

_c_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f32 = ctypes.c_float

# name -> argtypes (restype is int for all but the string getters)
_SIGNATURES = {
    "qvit_quantize_act_i8": [_c_p, _i64, _i64, _i64, _i32, _c_p, _c_p, _c_p, _i32, _c_p, _i64, _i64, _c_p],
    "qvit_fake_quant_f32": [_c_p, _i64, _i32, _c_p, _c_p, _c_p, _i32, _c_p, _c_p],
    "qvit_gelu_f32": [_c_p, _i64, _c_p, _c_p],
    "qvit_pack_weight": [_c_p, _i64, _i64, _i64, _i32, _c_p, _c_p, _c_p, _i32, _c_p, _i64, _i64, _c_p, _c_p],
    "qvit_pad_bias": [_c_p, _i64, _c_p, _i64, _c_p],
    "qvit_pack_weight_w4r": [_c_p, _i64, _i64, _c_p, _c_p],
    "qvit_pack_weight_w8r": [_c_p, _i64, _i64, _c_p, _c_p],
    "qvit_im2col_quant_i8": [_c_p, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                             _i32, _c_p, _c_p, _c_p, _i32, _c_p, _i64, _i64, _c_p],
    "qvit_layernorm_quant_i8": [_c_p, _i64, _i64, _i64, _c_p, _c_p, _f32, _i32, _c_p, _c_p, _c_p, _i32,
                                _c_p, _i64, _i64, _c_p, _c_p],
    "qvit_gemm": [_c_p, _i64, _i64, _i64, _c_p, _i32, _i64, _i64, _c_p, _c_p, _c_p, _i32, _c_p, _i64,
                  _i32, _c_p, _c_p, _c_p, _i32, _c_p, _c_p],
    "qvit_layernorm_quant_i8_t32": [_c_p, _i64, _i64, _i64, _c_p, _c_p, _f32, _i32, _c_p, _c_p, _c_p, _i32, _c_p,
                                    _i64, _c_p, _c_p],
    "qvit_gemm_a32_fits": [_i64, _i32, _i64, _i64, _i32],
    "qvit_gemm_a32": [_c_p, _i64, _i64, _c_p, _i32, _i64, _i64, _c_p, _c_p, _c_p, _i32, _c_p, _i64, _i32, _c_p, _c_p,
                      _c_p, _i32, _c_p, _c_p],
    "qvit_gemm_wonly": [_c_p, _i64, _i64, _i64, _c_p, _i32, _i64, _i64, _c_p, _c_p, _c_p, _i64, _c_p, _i64, _c_p],
    "qvit_conv_wonly": [_c_p, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _c_p, _i32,
                        _i64, _i64, _i64, _c_p, _c_p, _c_p, _c_p, _i64, _c_p],
    "qvit_conv_wonly_bn_act": [_c_p, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _c_p,
                               _i32, _i64, _i64, _i64, _c_p, _c_p, _c_p, _c_p, _i32, _c_p, _c_p],
    "qvit_conv_wonly_narrow": [_i32],
    "qvit_epi_table_build": [_i32, _i32, _c_p, _c_p, _c_p, _i32, _f32, _f32, _i64, _c_p, _c_p],
    "qvit_gemm_resid_ln": [_c_p, _i64, _i64, _i64, _c_p, _i32, _i64, _i64, _c_p, _c_p, _c_p, _c_p, _i64, _c_p, _c_p,
                           _f32, _i32, _c_p, _c_p, _c_p, _i32, _c_p, _c_p, _i64, _i64, _c_p, _c_p],
    "qvit_ultra_weight_codes": [_c_p, _i64, _i64, _i64, _i32, _c_p, _i64, _i64, _c_p, _c_p, _c_p],
    "qvit_ultra_bn_fold": [_c_p, _c_p, _c_p, _c_p, _f32, _i64, _c_p, _c_p, _c_p],
    "qvit_ultra_conv0": [_c_p, _i64, _i64, _i64, _c_p, _c_p, _c_p, _i32, _c_p, _c_p],
    "qvit_ultra_conv": [_c_p, _i64, _i64, _i64, _i64, _i64, _c_p, _i64, _i64, _i32, _i32, _c_p, _c_p, _i32, _c_p,
                        _i64, _c_p],
    "qvit_ultra_tail": [_c_p, _i64, _i64, _i64, _c_p, _i64, _c_p, _c_p, _c_p, _i64, _c_p, _i64, _i32, _i32, _c_p,
                        _i64, _c_p, _i64, _i64, _f32, _c_p, _c_p, _c_p],
    "qvit_ultra_conv0_int": [_c_p, _i64, _i64, _i64, _c_p, _c_p, _c_p, _i32, _i32, _c_p, _c_p],
    "qvit_ultra_conv_int": [_c_p, _i64, _i64, _i64, _i64, _i64, _c_p, _i64, _i64, _c_p, _c_p, _i32, _i32, _i32,
                            _c_p, _i64, _c_p],
    "qvit_yolo_decode": [_c_p, _i64, _i64, _i64, _i64, _i64, _i64, _c_p, _f32, _c_p, _c_p, _c_p],
    "qvit_attention": [_c_p, _i64, _i64, _i64, _i64, _i64, _f32, _f32, _i32, _c_p, _i64, _i32, _c_p, _c_p, _c_p,
                       _i32, _c_p],
    "qvit_gemm_qkv_split": [_c_p, _i64, _i64, _i64, _c_p, _i32, _i64, _i64, _c_p, _c_p, _c_p, _i64, _f32, _c_p,
                            _c_p, _c_p],
    "qvit_qkv_attention": [_c_p, _i64, _i64, _i64, _i64, _c_p, _i32, _i64, _c_p, _c_p, _c_p, _i64, _i64, _f32, _f32,
                           _i32, _c_p, _i64, _i32, _c_p, _c_p, _c_p, _i32, _c_p, _c_p],
    "qvit_attention_split": [_c_p, _c_p, _i64, _i64, _i64, _i64, _f32, _f32, _i32, _c_p, _i64, _i32, _c_p, _c_p,
                             _c_p, _i32, _c_p, _c_p],
}
# name -> argtypes of the entry points returning int64_t
INT64_FUNCS = {
}
STRING_FUNCS = {"qvit_strerror": [_i32], "qvit_version": []}
EXPORTED_SYMBOLS = sorted(list(_SIGNATURES) + list(INT64_FUNCS) + list(STRING_FUNCS))

_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None


class QvitError(RuntimeError):
    pass


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Loads libqvit_hip.so (no compute). Raises if it is absent: there is no fallback path."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise QvitError(
                f"{path} is missing: build it with `python -m quantized_vit_amd.build` "
                "(the HIP extension is required; there is no CPU fallback)")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGNATURES.items():
            if path != LIB_PATH and not hasattr(lib, name):
                continue  # an older build loaded for a same-box A/B (tools/lib_ab.sh): its entry points only
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        for name, args in INT64_FUNCS.items():
            if path != LIB_PATH and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int64
        for name, args in STRING_FUNCS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = ctypes.c_char_p
        _lib = lib
        return lib


def version() -> str:
    return load().qvit_version().decode()


def build_id(path: Optional[str] = None) -> Optional[str]:
    """Identity of a library build: the digest of its build inputs (sources, headers, build script, flags and
    defines; build.py writes it beside the library as <lib>.srcsha), so a rebuild from the same inputs keeps its
    id. Profile JSONs record the build they were measured on, and bench.py merges their counters
    only into a line timed on that same build. A library without a digest file falls back to its bytes' sha256."""
    import hashlib
    p = path or (getattr(_lib, "_name", None) if _lib is not None else None) or LIB_PATH
    try:
        with open(p + ".srcsha") as f:
            digest = f.read().strip()
        if digest:
            return "src-" + digest[:16]
    except OSError:
        pass
    try:
        with open(p, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def _check(code: int, what: str) -> None:
    if code != 0:
        msg = load().qvit_strerror(code).decode()
        raise QvitError(f"{what} failed: {msg} (status {code})")


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _require_gpu(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise QvitError(f"{name} must be a ROCm device tensor (got {t.device}); the HIP path has no CPU fallback")


# ---- wrappers -------------------------------------------------------------------------------
def quantize_act_i8(x2d: torch.Tensor, qtype: int, d: Optional[torch.Tensor], qm: Optional[torch.Tensor],
                    t: Optional[torch.Tensor], levels: int, out: torch.Tensor, kpad: int) -> torch.Tensor:
    _require_gpu(x2d, "input")
    assert x2d.dtype == torch.float32 and x2d.dim() == 2 and x2d.stride(1) == 1
    rows, cols = x2d.shape
    _check(load().qvit_quantize_act_i8(_ptr(x2d), rows, cols, x2d.stride(0), qtype, _ptr(d), _ptr(qm), _ptr(t),
                                       levels, _ptr(out), out.stride(0), kpad, _stream(x2d.device)),
           "qvit_quantize_act_i8")
    return out


def fake_quant_f32(x: torch.Tensor, qtype: int, d: Optional[torch.Tensor], qm: Optional[torch.Tensor],
                   t: Optional[torch.Tensor], levels: int = 0) -> torch.Tensor:
    _require_gpu(x, "input")
    xc = x.contiguous().float()
    y = torch.empty_like(xc)
    _check(load().qvit_fake_quant_f32(_ptr(xc), xc.numel(), qtype, _ptr(d), _ptr(qm), _ptr(t), levels, _ptr(y),
                                      _stream(x.device)), "qvit_fake_quant_f32")
    return y


def gelu_f32(x: torch.Tensor) -> torch.Tensor:
    """nn.GELU() bit-identical to torch's ATen CPU kernel (qvit_gelu_f32)."""
    _require_gpu(x, "input")
    xc = x.contiguous().float()
    y = torch.empty_like(xc)
    _check(load().qvit_gelu_f32(_ptr(xc), xc.numel(), _ptr(y), _stream(x.device)), "qvit_gelu_f32")
    return y


def pack_weight(w2d: torch.Tensor, qtype: int, d: torch.Tensor, qm: torch.Tensor, t: Optional[torch.Tensor],
                wfmt: int, npad: int, kpad: int, overflow: Optional[torch.Tensor]) -> torch.Tensor:
    _require_gpu(w2d, "weight")
    assert w2d.dtype == torch.float32 and w2d.stride(1) == 1
    n, k = w2d.shape
    nbytes = npad * kpad // 2 if wfmt == W4 else npad * kpad
    packed = torch.empty(nbytes, dtype=torch.uint8, device=w2d.device)
    _check(load().qvit_pack_weight(_ptr(w2d), n, k, w2d.stride(0), qtype, _ptr(d), _ptr(qm), _ptr(t), wfmt,
                                   _ptr(packed), npad, kpad, _ptr(overflow), _stream(w2d.device)),
           "qvit_pack_weight")
    return packed


def pack_weight_w4r(packed: torch.Tensor, npad: int, kpad: int) -> torch.Tensor:
    """The register-weight image (wfmt W4R) of a W4 image from pack_weight (qvit_pack_weight_w4r): same bytes,
    re-ordered per GEMM lane; qvit_gemm gives the W4 results on it."""
    _require_gpu(packed, "packed weights")
    assert packed.dtype == torch.uint8 and packed.is_contiguous() and packed.numel() == npad * kpad // 2
    out = torch.empty_like(packed)
    _check(load().qvit_pack_weight_w4r(_ptr(packed), npad, kpad, _ptr(out), _stream(packed.device)),
           "qvit_pack_weight_w4r")
    return out


def pack_weight_w8r(packed: torch.Tensor, npad: int, kpad: int) -> torch.Tensor:
    """The int8 register image (wfmt W8R) of a W4 image from pack_weight (qvit_pack_weight_w8r): npad * kpad
    bytes, each code as the byte 16 k in the GEMM lanes' operand order; qvit_gemm gives the W4 results on it."""
    _require_gpu(packed, "packed weights")
    assert packed.dtype == torch.uint8 and packed.is_contiguous() and packed.numel() == npad * kpad // 2
    out = torch.empty(npad * kpad, dtype=torch.uint8, device=packed.device)
    _check(load().qvit_pack_weight_w8r(_ptr(packed), npad, kpad, _ptr(out), _stream(packed.device)),
           "qvit_pack_weight_w8r")
    return out


def pack_weight_wide(codes: torch.Tensor, npad: int, kpad: int):
    """Packs integer weight codes beyond int8 ([n, k] float, on the device) for qvit_gemm_wonly as balanced
    base-256 digits, one W8 image per digit, most significant first: W16 (k = 256 h + l, |k| <= 32639) or W24
    (k = 65536 a + 256 h + l, |k| < 2^23). Returns (packed, wfmt)."""
    _require_gpu(codes, "weight codes")
    c = codes.detach().float().contiguous()
    cmax = float(c.abs().max()) if c.numel() else 0.0
    if cmax >= 2 ** 23:
        raise QvitError("pack_weight_wide: a weight code reaches 2^23")
    ndig = 2 if cmax <= 32639 else 3
    digits = []
    r = c
    for _ in range(ndig):
        d = torch.remainder(r + 128.0, 256.0) - 128.0   # in [-128, 127]
        digits.append(d)
        r = (r - d) / 256.0                              # exact: r - d is a multiple of 256
    if float(r.abs().max()) if r.numel() else 0.0:
        raise QvitError("pack_weight_wide: codes do not fit the digits")
    one = torch.ones(1, device=c.device)
    big = torch.full((1,), 1024.0, device=c.device)
    ovf = torch.zeros(1, dtype=torch.int32, device=c.device)
    imgs = [pack_weight(d.contiguous(), QT_LINEAR, one, big, None, W8, npad, kpad, ovf) for d in reversed(digits)]
    if int(ovf.item()) != 0:
        raise QvitError("pack_weight_wide: a digit left the int8 range")
    return torch.cat(imgs), (W16 if ndig == 2 else W24)


def pad_bias(bias: Optional[torch.Tensor], n: int, npad: int, device: torch.device) -> torch.Tensor:
    out = torch.empty(npad, dtype=torch.float32, device=device)
    b = None if bias is None else bias.detach().contiguous().float()
    _check(load().qvit_pad_bias(_ptr(b), n, _ptr(out), npad, _stream(device)), "qvit_pad_bias")
    return out


def im2col_quant_i8(x: torch.Tensor, kh: int, kw: int, sh: int, sw: int, ph: int, pw: int, dh: int, dw: int,
                    qtype: int, d, qm, t, levels: int, out: torch.Tensor, kpad: int) -> torch.Tensor:
    _require_gpu(x, "input")
    assert x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 4
    B, C, H, W = x.shape
    _check(load().qvit_im2col_quant_i8(_ptr(x), B, C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, qtype, _ptr(d),
                                       _ptr(qm), _ptr(t), levels, _ptr(out), out.stride(0), kpad,
                                       _stream(x.device)), "qvit_im2col_quant_i8")
    return out


def layernorm_quant_i8(x2d: torch.Tensor, gamma: Optional[torch.Tensor], beta: Optional[torch.Tensor], eps: float,
                       qtype: int, d, qm, t, levels: int, out: torch.Tensor, kpad: int,
                       code_table: Optional[torch.Tensor] = None) -> torch.Tensor:
    """LayerNorm + activation quantizer -> int8 codes (code_table: EPI_I8 table of the quantizer, optional)."""
    _require_gpu(x2d, "input")
    assert x2d.dtype == torch.float32 and x2d.stride(1) == 1
    rows, cols = x2d.shape
    _check(load().qvit_layernorm_quant_i8(_ptr(x2d), rows, cols, x2d.stride(0), _ptr(gamma), _ptr(beta), eps, qtype,
                                          _ptr(d), _ptr(qm), _ptr(t), levels, _ptr(out), out.stride(0), kpad,
                                          _ptr(code_table), _stream(x2d.device)), "qvit_layernorm_quant_i8")
    return out


def gemm(A: torch.Tensor, M: int, K: int, packed: torch.Tensor, wfmt: int, N: int, npad: int,
         d_act: Optional[torch.Tensor], d_wt: Optional[torch.Tensor], bias_pad: Optional[torch.Tensor],
         epilogue: int, C: torch.Tensor, out_qtype: int = 0, out_d=None, out_qm=None, out_t=None,
         out_levels: int = 0, epi_table: Optional[torch.Tensor] = None) -> torch.Tensor:
    _require_gpu(A, "codes")
    _check(load().qvit_gemm(_ptr(A), M, K, A.stride(0), _ptr(packed), wfmt, N, npad, _ptr(d_act), _ptr(d_wt),
                            _ptr(bias_pad), epilogue, _ptr(C), C.stride(0), out_qtype, _ptr(out_d), _ptr(out_qm),
                            _ptr(out_t), out_levels, _ptr(epi_table), _stream(A.device)), "qvit_gemm")
    return C


def t32_rows(M: int) -> int:
    """Rows a QVIT_ACT_T32 code buffer holds for M rows (whole 64-row wave tiles of qvit_gemm_a32)."""
    return (M + 63) // 64 * 64


def t32_to_rows(codes_t32: torch.Tensor, M: int, kpad: int) -> torch.Tensor:
    """QVIT_ACT_T32 codes -> row-major [M, kpad] (a view permutation; tests and code tracing only)."""
    R = t32_rows(M)
    t = codes_t32.view(-1)[:R * kpad].view(R // 32, kpad // 32, 2, 32, 16)   # [rb][kb][half][row][16]
    return t.permute(0, 3, 1, 2, 4).reshape(R, kpad)[:M]


def rows_to_t32(codes: torch.Tensor, kpad: int) -> torch.Tensor:
    """Row-major [M, >= kpad] codes -> a QVIT_ACT_T32 buffer (rows padded with zeros; tests only)."""
    M = codes.shape[0]
    R = t32_rows(M)
    full = torch.zeros((R, kpad), dtype=torch.int8, device=codes.device)
    full[:M] = codes[:, :kpad]
    return full.view(R // 32, 32, kpad // 32, 2, 16).permute(0, 2, 3, 1, 4).contiguous().view(-1)


def layernorm_quant_i8_t32(x2d: torch.Tensor, gamma: Optional[torch.Tensor], beta: Optional[torch.Tensor], eps: float,
                           qtype: int, d, qm, t, levels: int, out: torch.Tensor, kpad: int,
                           code_table: Optional[torch.Tensor] = None) -> torch.Tensor:
    """layernorm_quant_i8 with the codes in QVIT_ACT_T32 order (out: int8, >= t32_rows(M) * kpad bytes)."""
    _require_gpu(x2d, "input")
    assert x2d.dtype == torch.float32 and x2d.stride(1) == 1
    rows, cols = x2d.shape
    assert out.numel() >= t32_rows(rows) * kpad
    _check(load().qvit_layernorm_quant_i8_t32(_ptr(x2d), rows, cols, x2d.stride(0), _ptr(gamma), _ptr(beta), eps,
                                              qtype, _ptr(d), _ptr(qm), _ptr(t), levels, _ptr(out), kpad,
                                              _ptr(code_table), _stream(x2d.device)), "qvit_layernorm_quant_i8_t32")
    return out


def gemm_a32_fits(K: int, wfmt: int, N: int, npad: int, epilogue: int) -> bool:
    lib = load()
    if not hasattr(lib, "qvit_gemm_a32_fits"):  # (an older build in a same-box A/B)
        return False
    return bool(lib.qvit_gemm_a32_fits(K, wfmt, N, npad, epilogue))


def gemm_a32(A: torch.Tensor, M: int, K: int, packed: torch.Tensor, wfmt: int, N: int, npad: int, d_act, d_wt,
             bias_pad: Optional[torch.Tensor], epilogue: int, C: torch.Tensor, out_qtype: int = 0, out_d=None,
             out_qm=None, out_t=None, out_levels: int = 0, epi_table: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qvit_gemm_a32: the int8-code GEMM on QVIT_ACT_T32 activations (weight-stationary fc1 schedule)."""
    _require_gpu(A, "codes")
    assert A.numel() >= t32_rows(M) * K
    _check(load().qvit_gemm_a32(_ptr(A), M, K, _ptr(packed), wfmt, N, npad, _ptr(d_act), _ptr(d_wt), _ptr(bias_pad),
                                epilogue, _ptr(C), C.stride(0), out_qtype, _ptr(out_d), _ptr(out_qm), _ptr(out_t),
                                out_levels, _ptr(epi_table), _stream(A.device)), "qvit_gemm_a32")
    return C


WONLY_WS_MAX = 64 << 20   # bytes of split-K partials per call (small-M weight-only layers)


def wonly_workspace(device: torch.device, M: int, npad: int) -> Optional[torch.Tensor]:
    """Split-K workspace of qvit_gemm_wonly for M rows (at most 256 partial sets). A fresh buffer per call from
    torch's caching allocator, which ties it to the current stream: launches on different streams never share
    partials."""
    need = min(256 * M * npad * 4, WONLY_WS_MAX)
    return torch.empty(need // 4 + 4, dtype=torch.float32, device=device)


def gemm_wonly(X: torch.Tensor, M: int, K: int, packed: torch.Tensor, wfmt: int, N: int, npad: int,
               d_wt: torch.Tensor, bias_pad: Optional[torch.Tensor], Y: torch.Tensor, split: bool = True) -> torch.Tensor:
    """Y = d_wt * (X @ codes^T) + bias with fp32 X (qvit_gemm_wonly: weight-only QuantizeLinear); small M
    splits the K range over several workgroups through a cached workspace (split=False: never)."""
    _require_gpu(X, "activations")
    small = (npad // 256) * ((M + 63) // 64) < 128   # the kernel splits K only for fewer tiles than this
    ws = wonly_workspace(X.device, M, npad) if (split and small) else None
    _check(load().qvit_gemm_wonly(_ptr(X), M, K, X.stride(0), _ptr(packed), wfmt, N, npad, _ptr(d_wt),
                                  _ptr(bias_pad), _ptr(Y), Y.stride(0), _ptr(ws), 0 if ws is None else ws.numel() * 4,
                                  _stream(X.device)), "qvit_gemm_wonly")
    return Y


def conv_wonly(x: torch.Tensor, kernel_size, stride, padding, dilation, packed: torch.Tensor, wfmt: int, N: int,
               npad: int, kpad: int, d_wt: torch.Tensor, bias_pad: Optional[torch.Tensor],
               split: bool = True) -> torch.Tensor:
    """F.conv2d(x, d_wt * codes, bias) (groups 1, zero padding) with fp32 NCHW x on qvit_conv_wonly: an implicit
    GEMM against the packed codes ([N][C kh kw] in the weight's flattening order). Returns NCHW fp32. Few output
    pixels on the wide schedule split K through a workspace (split=False: never)."""
    _require_gpu(x, "activations")
    if x.dtype != torch.float32 or not x.is_contiguous():
        x = x.float().contiguous()
    B, C, H, W = x.shape
    (kh, kw), (sh, sw), (ph, pw), (dh, dw) = kernel_size, stride, padding, dilation
    OH = (H + 2 * ph - dh * (kh - 1) - 1) // sh + 1
    OW = (W + 2 * pw - dw * (kw - 1) - 1) // sw + 1
    y = torch.empty((B, N, OH, OW), dtype=torch.float32, device=x.device)
    M = B * OH * OW
    small = split and (npad // 256) * ((M + 63) // 64) < 128 and not narrow_conv_fits(wfmt, N, C * kh * kw, H, W)
    ws = wonly_workspace(x.device, M, npad) if small else None
    _check(load().qvit_conv_wonly(_ptr(x), B, C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, _ptr(packed), wfmt, N, npad,
                                  kpad, _ptr(d_wt), _ptr(bias_pad), _ptr(y), _ptr(ws),
                                  0 if ws is None else ws.numel() * 4, _stream(x.device)), "qvit_conv_wonly")
    return y


def conv_wonly_bn_act(x: torch.Tensor, kernel_size, stride, padding, dilation, packed: torch.Tensor, wfmt: int,
                      N: int, npad: int, kpad: int, d_wt: torch.Tensor, bias_pad: Optional[torch.Tensor],
                      bn_alpha: torch.Tensor, bn_shift: torch.Tensor, a_levels: int) -> Optional[torch.Tensor]:
    """conv_wonly -> BatchNorm2d(eval) as y alpha + shift (ultra_bn_fold) -> activation_quantize_fn values
    round(clamp(., 0, 1) levels) / levels, in one launch (qvit_conv_wonly_bn_act, the narrow schedule). None when
    the layer is outside that schedule (more than 64 channels, codes wider than int8, a weight panel past 24 KiB):
    the caller runs the modules one by one."""
    _require_gpu(x, "activations")
    (kh, kw), (sh, sw), (ph, pw), (dh, dw) = kernel_size, stride, padding, dilation
    if not narrow_conv_fits(wfmt, N, x.shape[1] * kh * kw, x.shape[2], x.shape[3]):
        return None
    if x.dtype != torch.float32 or not x.is_contiguous():
        x = x.float().contiguous()
    B, C, H, W = x.shape
    OH = (H + 2 * ph - dh * (kh - 1) - 1) // sh + 1
    OW = (W + 2 * pw - dw * (kw - 1) - 1) // sw + 1
    y = torch.empty((B, N, OH, OW), dtype=torch.float32, device=x.device)
    _check(load().qvit_conv_wonly_bn_act(_ptr(x), B, C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, _ptr(packed), wfmt, N,
                                       npad, kpad, _ptr(d_wt), _ptr(bias_pad), _ptr(bn_alpha), _ptr(bn_shift),
                                       a_levels, _ptr(y), _stream(x.device)), "qvit_conv_wonly_bn_act")
    return y


NARROW_W_MAX = 24 * 1024   # gemm_wonly.hip NW_WMAX: the narrow schedule's LDS weight panel
NARROW_K_MAX = 1024        # gemm_wonly.hip NW_KMAX: its tap table


def narrow_conv_fits(wfmt: int, N: int, kreal: int, H: int = 0, W: int = 0) -> bool:
    """Whether qvit_conv_wonly runs the narrow schedule (gemm_wonly.hip narrow_geo): N <= 64 channels, int4 / int8
    codes, the K stages up to C kh kw (<= NARROW_K_MAX taps) of 16 ceil(N / 16) rows within NARROW_W_MAX, input
    sides below 32767, the schedule enabled."""
    if N > 64 or wfmt not in (W4, W8) or not conv_wonly_narrow(-1) or H >= 32767 or W >= 32767:
        return False
    nke = (kreal + 63) // 64
    return (nke * 64 <= NARROW_K_MAX
            and nke * 16 * ((N + 15) // 16) * (32 if wfmt == W4 else 64) <= NARROW_W_MAX)


def conv_wonly_narrow(enable: int = -1) -> bool:
    """The narrow convolution schedule of qvit_conv_wonly (N <= 64) on (1) / off (0) for this process; -1 queries.
    Returns the previous setting (tests compare the two schedules)."""
    return bool(load().qvit_conv_wonly_narrow(int(enable)))


def resid_ln_counters(device: torch.device, rows: int, npad: int) -> torch.Tensor:
    """Arrival counters of qvit_gemm_resid_ln for `rows` rows: one int32 per 128-row block. The call zeroes them
    on its stream; a fresh buffer per call (caching allocator, stream-bound) so concurrent launches never share."""
    return torch.empty(max((rows + 127) // 128, 1), dtype=torch.int32, device=device)


def gemm_resid_ln(A: torch.Tensor, M: int, K: int, packed: torch.Tensor, wfmt: int, N: int, npad: int,
                  d_act, d_wt, bias_pad, C: torch.Tensor, gamma, beta, eps: float, out_qtype: int, out_d, out_qm,
                  out_t, out_levels: int, ln_table, codes: torch.Tensor, kpad_codes: int) -> torch.Tensor:
    """C += contraction (QVIT_EPI_F32_RESID), then LayerNorm + quantizer of the updated rows -> codes
    (qvit_gemm_resid_ln)."""
    _require_gpu(A, "codes")
    cnt = resid_ln_counters(A.device, M, npad)
    _check(load().qvit_gemm_resid_ln(_ptr(A), M, K, A.stride(0), _ptr(packed), wfmt, N, npad, _ptr(d_act),
                                     _ptr(d_wt), _ptr(bias_pad), _ptr(C), C.stride(0), _ptr(gamma), _ptr(beta), eps,
                                     out_qtype, _ptr(out_d), _ptr(out_qm), _ptr(out_t), out_levels, _ptr(ln_table),
                                     _ptr(codes), codes.stride(0), kpad_codes, _ptr(cnt), _stream(A.device)),
           "qvit_gemm_resid_ln")
    return codes


def epi_table_build(epilogue: int, out_qtype: int, out_d, out_qm, out_t, out_levels: int, v_lo: float, w: float,
                    nb: int, device: torch.device) -> torch.Tensor:
    """Code table of an int8 GEMM epilogue (qvit_epi_table_build); validity is decided on the device."""
    table = torch.zeros((16 + 8 * nb + 1023) // 1024 * 1024, dtype=torch.uint8, device=device)  # 1-KiB pieces
    _check(load().qvit_epi_table_build(epilogue, out_qtype, _ptr(out_d), _ptr(out_qm), _ptr(out_t), out_levels,
                                       v_lo, w, nb, _ptr(table), _stream(device)), "qvit_epi_table_build")
    return table


def attention(qkv: torch.Tensor, B: int, N: int, H: int, head_dim: int, scale: float, out: torch.Tensor,
              out_mode: int = ATT_F32, in_scale: float = 1.0, out_qtype: int = 0, out_d=None, out_qm=None,
              out_t=None, out_levels: int = 0) -> torch.Tensor:
    """softmax(q k^T * scale) v per (image, head) on a [B*N, >= 3*H*hd] fp32 qkv projection."""
    _require_gpu(qkv, "qkv")
    assert qkv.dtype == torch.float32 and qkv.stride(1) == 1
    _check(load().qvit_attention(_ptr(qkv), B, N, H, head_dim, qkv.stride(0), scale, in_scale, out_mode, _ptr(out),
                                 out.stride(0), out_qtype, _ptr(out_d), _ptr(out_qm), _ptr(out_t), out_levels,
                                 _stream(qkv.device)), "qvit_attention")
    return out


def gemm_qkv_split(A: torch.Tensor, M: int, K: int, packed: torch.Tensor, wfmt: int, N: int, npad: int,
                   d_act: torch.Tensor, d_wt: torch.Tensor, bias_pad: Optional[torch.Tensor], seq: int,
                   in_scale: float, hi: torch.Tensor, lo: torch.Tensor):
    """qkv projection as fp16 hi/lo planes [B][N/64][seq][64] of in_scale * x (qvit_gemm_qkv_split)."""
    _require_gpu(A, "codes")
    assert hi.dtype == torch.float16 and lo.dtype == torch.float16 and hi.is_contiguous() and lo.is_contiguous()
    assert hi.numel() >= M * N and lo.numel() >= M * N
    _check(load().qvit_gemm_qkv_split(_ptr(A), M, K, A.stride(0), _ptr(packed), wfmt, N, npad, _ptr(d_act),
                                      _ptr(d_wt), _ptr(bias_pad), seq, in_scale, _ptr(hi), _ptr(lo),
                                      _stream(A.device)), "qvit_gemm_qkv_split")
    return hi, lo


def attention_split(hi: torch.Tensor, lo: torch.Tensor, B: int, N: int, H: int, head_dim: int, scale: float,
                    out: torch.Tensor, out_mode: int = ATT_F32, in_scale: float = 1.0, out_qtype: int = 0,
                    out_d=None, out_qm=None, out_t=None, out_levels: int = 0,
                    epi_table: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qvit_attention on the split planes of gemm_qkv_split (epi_table: EPI_I8 code table of the output
    quantizer, optional)."""
    _require_gpu(hi, "qkv_hi")
    assert hi.dtype == torch.float16 and lo.dtype == torch.float16
    assert hi.numel() >= B * 3 * H * N * head_dim and lo.numel() >= B * 3 * H * N * head_dim
    _check(load().qvit_attention_split(_ptr(hi), _ptr(lo), B, N, H, head_dim, scale, in_scale, out_mode, _ptr(out),
                                       out.stride(0), out_qtype, _ptr(out_d), _ptr(out_qm), _ptr(out_t), out_levels,
                                       _ptr(epi_table), _stream(hi.device)), "qvit_attention_split")
    return out


QKV_ATT_MAX_N = 208
QKV_ATT_MAX_C = 768   # H * 64 (the bias of the qkv layer stays in LDS)


def qkv_attention(codes: torch.Tensor, B: int, N: int, K: int, packed: torch.Tensor, npad: int,
                  d_act: torch.Tensor, d_wt: torch.Tensor, bias_pad: Optional[torch.Tensor], H: int, scale: float,
                  out: torch.Tensor, out_mode: int = ATT_F32, in_scale: float = 1.0, out_qtype: int = 0,
                  out_d=None, out_qm=None, out_t=None, out_levels: int = 0,
                  epi_table: Optional[torch.Tensor] = None, wfmt: int = W4) -> torch.Tensor:
    """qkv projection (W4 codes) + attention core in one kernel (qvit_qkv_attention), N <= 208."""
    _require_gpu(codes, "codes")
    _check(load().qvit_qkv_attention(_ptr(codes), B, N, K, codes.stride(0), _ptr(packed), wfmt, npad, _ptr(d_act),
                                     _ptr(d_wt), _ptr(bias_pad), H, 64, scale, in_scale, out_mode, _ptr(out),
                                     out.stride(0), out_qtype, _ptr(out_d), _ptr(out_qm), _ptr(out_t), out_levels,
                                     _ptr(epi_table), _stream(codes.device)), "qvit_qkv_attention")
    return out


# ---- UltraNet ---------------------------------------------------------------------------------------
def ultra_weight_codes(w: torch.Tensor, w_bit: int, kpad: int, cout_pad: int, values: bool = False):
    """Conv weight [cout][cin][ks][ks] -> int8 codes [cout_pad][kpad] in K order (ky, kx, c)
    (and, with values=True, also the fake-quant weight k/(2^(w_bit-1)-1) in w's layout)."""
    _require_gpu(w, "weight")
    w = w.detach().float().contiguous()
    cout, cin, ks, ks2 = w.shape
    assert ks == ks2
    codes = torch.empty((cout_pad, kpad), dtype=torch.int8, device=w.device)
    vals = torch.empty_like(w) if values else None
    ws = torch.empty(1, dtype=torch.int32, device=w.device)
    _check(load().qvit_ultra_weight_codes(_ptr(w), cout, cin, ks, w_bit, _ptr(codes), kpad, cout_pad, _ptr(vals),
                                          _ptr(ws), _stream(w.device)), "qvit_ultra_weight_codes")
    return (codes, vals) if values else codes


def ultra_bn_fold(bn, device) -> tuple:
    n = bn.num_features
    alpha = torch.empty(n, device=device)
    shift = torch.empty(n, device=device)
    g = bn.weight.detach().float().contiguous() if bn.weight is not None else None
    b = bn.bias.detach().float().contiguous() if bn.bias is not None else None
    _check(load().qvit_ultra_bn_fold(_ptr(g), _ptr(b), _ptr(bn.running_mean), _ptr(bn.running_var), float(bn.eps), n,
                                     _ptr(alpha), _ptr(shift), _stream(device)), "qvit_ultra_bn_fold")
    return alpha, shift


def ultra_conv0(img: torch.Tensor, wvals: torch.Tensor, alpha, shift, a_bit: int) -> torch.Tensor:
    """Layer 0: float image NCHW -> conv3x3 with fake-quant weights wvals [16][3][3][3] -> BN -> quantizer
    -> 2x2 max pool -> NHWC codes [B][H/2][W/2][16]."""
    _require_gpu(img, "image")
    assert img.dtype == torch.float32 and img.is_contiguous() and img.shape[1] == 3
    assert wvals.shape == (16, 3, 3, 3) and wvals.is_contiguous()
    B, _, H, W = img.shape
    out = torch.empty((B, H // 2, W // 2, 16), dtype=torch.int8, device=img.device)
    _check(load().qvit_ultra_conv0(_ptr(img), B, H, W, _ptr(wvals), _ptr(alpha), _ptr(shift), a_bit, _ptr(out),
                                   _stream(img.device)), "qvit_ultra_conv0")
    return out


def ultra_conv(x: torch.Tensor, ks: int, wcodes: torch.Tensor, cout: int, w_bit: int, a_bit: int, alpha, shift,
               mode: int) -> torch.Tensor:
    """NHWC codes [B][H][W][cin] -> NHWC codes (mode ULTRA_CODES / ULTRA_CODES_POOL) or fp32 (ULTRA_F32)."""
    _require_gpu(x, "codes")
    assert x.dtype == torch.int8 and x.is_contiguous()
    B, H, W, cin = x.shape
    if mode == ULTRA_CODES_POOL:
        out = torch.empty((B, H // 2, W // 2, cout), dtype=torch.int8, device=x.device)
    elif mode == ULTRA_CODES:
        out = torch.empty((B, H, W, cout), dtype=torch.int8, device=x.device)
    else:
        out = torch.empty((B, H, W, cout), dtype=torch.float32, device=x.device)
    _check(load().qvit_ultra_conv(_ptr(x), B, H, W, cin, ks, _ptr(wcodes), wcodes.shape[1], cout, w_bit, a_bit,
                                  _ptr(alpha), _ptr(shift), mode, _ptr(out), cout, _stream(x.device)),
           "qvit_ultra_conv")
    return out


def ultra_tail(x: torch.Tensor, wcodes, alphas, shifts, hcodes: torch.Tensor, hbias: torch.Tensor, hout: int,
               w_bit: int, a_bit: int, decode=None):
    """UltraNet layers.16-28 in one launch (qvit_ultra_tail): NHWC codes [B][H][W][64] (H, W <= 26) through four
    3x3 64 -> 64 blocks and the 1x1 head -> fp32 NHWC [B][H][W][hout]; with decode = (anchors, na, no, stride)
    the YOLO decode runs in the kernel and (io [B, na*H*W, no], p [B, na, H, W, no]) is returned instead."""
    _require_gpu(x, "codes")
    assert x.dtype == torch.int8 and x.is_contiguous() and x.shape[3] == 64
    B, H, W, _ = x.shape
    arr = lambda ts: (ctypes.c_void_p * 4)(*[t.data_ptr() for t in ts])
    if decode is None:
        out = torch.empty((B, H, W, hout), dtype=torch.float32, device=x.device)
        io = p = anchors = None
        na = no = 0
        stride = 0.0
    else:
        anchors, na, no, stride = decode
        out = None
        io = torch.empty((B, na, H, W, no), device=x.device)
        p = torch.empty_like(io)
    _check(load().qvit_ultra_tail(_ptr(x), B, H, W, arr(wcodes), wcodes[0].shape[1], arr(alphas), arr(shifts),
                                  _ptr(hcodes), hcodes.shape[1], _ptr(hbias), hout, w_bit, a_bit, _ptr(out), hout,
                                  _ptr(anchors), na, no, float(stride), _ptr(io), _ptr(p), _stream(x.device)),
           "qvit_ultra_tail")
    return out if decode is None else (io.view(B, -1, no), p)


def ultra_conv0_int(img_u8: torch.Tensor, wcodes: torch.Tensor, inc: torch.Tensor, bias: torch.Tensor,
                    shift_bits: int, out_bit: int) -> torch.Tensor:
    """Integer deploy layer 0: uint8 image NCHW -> conv3x3 (weight codes [16][3][3][3]) -> integer BN/act
    threshold -> 2x2 max pool -> NHWC codes [B][H/2][W/2][16]."""
    _require_gpu(img_u8, "image")
    assert img_u8.dtype == torch.uint8 and img_u8.is_contiguous() and img_u8.shape[1] == 3
    assert wcodes.shape == (16, 3, 3, 3) and wcodes.dtype == torch.int8 and wcodes.is_contiguous()
    assert inc.dtype == torch.int32 and bias.dtype == torch.int32 and inc.numel() >= 16 and bias.numel() >= 16
    B, _, H, W = img_u8.shape
    out = torch.empty((B, H // 2, W // 2, 16), dtype=torch.int8, device=img_u8.device)
    _check(load().qvit_ultra_conv0_int(_ptr(img_u8), B, H, W, _ptr(wcodes), _ptr(inc), _ptr(bias), shift_bits,
                                       out_bit, _ptr(out), _stream(img_u8.device)), "qvit_ultra_conv0_int")
    return out


def ultra_conv_int(x: torch.Tensor, ks: int, wcodes: torch.Tensor, cout: int, inc: torch.Tensor, bias: torch.Tensor,
                   shift_bits: int, out_bit: int, pool: bool) -> torch.Tensor:
    """Integer deploy layers 1..7: NHWC codes [B][H][W][cin] -> NHWC codes (2x2 max-pooled when pool)."""
    _require_gpu(x, "codes")
    assert x.dtype == torch.int8 and x.is_contiguous()
    assert inc.dtype == torch.int32 and bias.dtype == torch.int32 and inc.numel() >= cout and bias.numel() >= cout
    B, H, W, cin = x.shape
    shape = (B, H // 2, W // 2, cout) if pool else (B, H, W, cout)
    out = torch.empty(shape, dtype=torch.int8, device=x.device)
    _check(load().qvit_ultra_conv_int(_ptr(x), B, H, W, cin, ks, _ptr(wcodes), wcodes.shape[1], cout, _ptr(inc),
                                      _ptr(bias), shift_bits, out_bit, 1 if pool else 0, _ptr(out), cout,
                                      _stream(x.device)), "qvit_ultra_conv_int")
    return out


def yolo_decode(head: torch.Tensor, na: int, no: int, anchors: torch.Tensor, stride: float):
    """head NHWC fp32 [B][ny][nx][na*no] -> (io [B, na*ny*nx, no], p [B, na, ny, nx, no])."""
    _require_gpu(head, "head")
    B, ny, nx, C = head.shape
    io = torch.empty((B, na, ny, nx, no), device=head.device)
    p = torch.empty_like(io)
    _check(load().qvit_yolo_decode(_ptr(head), B, ny, nx, na, no, C, _ptr(anchors), stride, _ptr(io), _ptr(p),
                                   _stream(head.device)), "qvit_yolo_decode")
    return io.view(B, -1, no), p
