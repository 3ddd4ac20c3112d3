"""The C-ABI library loads and exports exactly what include/qvit_hip.h declares; argument validation
follows the header's status conventions. No kernel is launched (runs without a GPU)."""
import ctypes
import os
import re

import pytest

from quantized_vit_amd import _lib, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "qvit_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(qvit_\w+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    build.build()
    return _lib.load()


def test_header_matches_binding():
    assert declared_functions() == _lib.EXPORTED_SYMBOLS


def test_library_exports_every_declared_symbol(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_version_and_strerror(lib):
    assert "gfx950" in _lib.version()
    assert lib.qvit_strerror(0) == b"ok"
    assert b"invalid" in lib.qvit_strerror(-1)
    assert b"NULL" in lib.qvit_strerror(-3)


def test_constants_match_header():
    text = open(HEADER).read()
    consts = dict(re.findall(r"#define\s+(QVIT_\w+)\s+(-?\d+)", text))
    assert int(consts["QVIT_QT_LINEAR"]) == _lib.QT_LINEAR
    assert int(consts["QVIT_QT_NONLINEAR"]) == _lib.QT_NONLINEAR
    assert int(consts["QVIT_QT_ULTRA_ACT"]) == _lib.QT_ULTRA_ACT
    assert int(consts["QVIT_W4"]) == _lib.W4 and int(consts["QVIT_W8"]) == _lib.W8
    assert int(consts["QVIT_W4R"]) == _lib.W4R
    for e in ("F32", "F32_RESID", "I8_GELU", "I8", "I32"):
        assert int(consts[f"QVIT_EPI_{e}"]) == getattr(_lib, f"EPI_{e}")
    assert int(consts["QVIT_TILE_N"]) == _lib.TILE_N and int(consts["QVIT_TILE_K"]) == _lib.TILE_K


def test_argument_validation_without_launch(lib):
    fake = ctypes.c_void_p(0x1000)   # never dereferenced: validation rejects before any launch
    # NULL operands
    assert lib.qvit_gemm(None, 16, 128, 128, fake, 4, 16, 256, fake, fake, None, 0, fake, 16, 0, None, None,
                         None, 0, None, None) == -3
    # K not a multiple of the tile
    assert lib.qvit_gemm(fake, 16, 100, 128, fake, 4, 16, 256, fake, fake, None, 0, fake, 16, 0, None, None,
                         None, 0, None, None) == -1
    # bad weight format
    assert lib.qvit_gemm(fake, 16, 128, 128, fake, 5, 16, 256, fake, fake, None, 0, fake, 16, 0, None, None,
                         None, 0, None, None) == -1
    # misaligned activation stride
    assert lib.qvit_gemm(fake, 16, 128, 136, fake, 4, 16, 256, fake, fake, None, 0, fake, 16, 0, None, None,
                         None, 0, None, None) == -2
    # bad quantizer enum
    assert lib.qvit_quantize_act_i8(fake, 4, 16, 16, 7, fake, fake, None, 0, fake, 16, 16, None) == -1
    # kpad not a multiple of 16
    assert lib.qvit_quantize_act_i8(fake, 4, 10, 16, 0, fake, fake, None, 0, fake, 16, 12, None) == -1
    # ULTRA activation quantizer needs a level count in [1, 127]
    assert lib.qvit_quantize_act_i8(fake, 4, 16, 16, 2, None, None, None, 0, fake, 16, 16, None) == -1
    # weight packing: npad must be a multiple of the tile
    assert lib.qvit_pack_weight(fake, 10, 128, 128, 0, fake, fake, None, 4, fake, 128, 128, None, None) == -1
    # register-weight image: npad a multiple of the tile, kpad of QVIT_TILE_K and <= 65536, 16-B aligned, not in place
    other = ctypes.c_void_p(0x2000)
    assert lib.qvit_pack_weight_w4r(fake, 100, 128, other, None) == -1
    assert lib.qvit_pack_weight_w4r(fake, 256, 100, other, None) == -1
    assert lib.qvit_pack_weight_w4r(fake, 256, 65536 + 128, other, None) == -1
    assert lib.qvit_pack_weight_w4r(fake, 256, 128, ctypes.c_void_p(0x2008), None) == -2
    assert lib.qvit_pack_weight_w4r(fake, 256, 128, fake, None) == -1
    assert lib.qvit_pack_weight_w4r(None, 256, 128, other, None) == -3
    # the int8 register image: the same argument rules
    assert lib.qvit_pack_weight_w8r(fake, 100, 128, other, None) == -1
    assert lib.qvit_pack_weight_w8r(fake, 256, 100, other, None) == -1
    assert lib.qvit_pack_weight_w8r(fake, 256, 65536 + 128, other, None) == -1
    assert lib.qvit_pack_weight_w8r(fake, 256, 128, ctypes.c_void_p(0x2008), None) == -2
    assert lib.qvit_pack_weight_w8r(fake, 256, 128, fake, None) == -1
    assert lib.qvit_pack_weight_w8r(None, 256, 128, other, None) == -3
    assert lib.qvit_gemm(fake, 16, 65536 + 128, 65536 + 128, fake, _lib.W8R, 16, 256, fake, fake, None, 0, fake, 16,
                         0, None, None, None, 0, None, None) == -1
    # QVIT_W4R: the int4 accumulation bound applies; the fused residual + LayerNorm GEMM takes W4 / W8 only
    assert lib.qvit_gemm(fake, 16, 65536 + 128, 65536 + 128, fake, _lib.W4R, 16, 256, fake, fake, None, 0, fake, 16,
                         0, None, None, None, 0, None, None) == -1
    # zero-size work is a no-op success
    assert lib.qvit_quantize_act_i8(fake, 0, 16, 16, 0, fake, fake, None, 0, fake, 16, 16, None) == 0


def test_conv_wonly_bn_act_rejects_offsets_past_the_tap_table(lib):
    """The narrow conv schedule keeps each tap's input offset in 32 bits and dy, dx in 16: inputs past
    those bounds are refused by the narrow-only fused entry (the module falls back to its unfused path) and take the
    wide schedule in qvit_conv_wonly. Checked before any launch."""
    fake = ctypes.c_void_p(0x1000)

    def call(C, H, W, kh=3, kw=3, ph=1, pw=1, dh=1, dw=1):
        return lib.qvit_conv_wonly_bn_act(fake, 1, C, H, W, kh, kw, 1, 1, ph, pw, dh, dw, fake, _lib.W4, 16, 256,
                                          (C * kh * kw + 127) // 128 * 128, fake, None, fake, fake, 15, fake, None)
    assert call(64, 5800, 5800) == -1                       # C H W >= 2^31: an int32 tap offset would overflow
    assert call(4, 100, 100, kh=2, dh=40000, ph=20000) == -1   # the tap's dy needs more than 15 bits
    assert call(4, 100, 100, kw=2, dw=40000, pw=20000) == -1   # dx likewise
    assert call(4, 100, 100, ph=32700) == -1                 # the zero-tap sentinel dy = 0x7fff could land inside
