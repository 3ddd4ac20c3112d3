"""Builds libqvit_hip.so (gfx950) in-tree with hipcc: one object per .hip, one shared library.

Usage: python -m quantized_vit_amd.build [--force] [--verbose]
The library is written next to this file so it travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libqvit_hip.so")
ARCH = "gfx950"

SOURCES = ["quant_kernels.hip", "gemm_w4a8.hip", "gemm_ws.hip", "gemm_wonly.hip", "attention.hip",
           "qkv_attention.hip", "ultra_conv.hip"]
# sources with inline-asm register loads: their device assembly is kept beside the objects (the very code in the
# library) for tools/asm_load_check.py (tests/test_asm_loads.py)
ASM_CHECKED = ["gemm_w4a8.hip", "ultra_conv.hip"]
HEADERS = ["qvit_common.h", "attn_common.h", "attn32.h", "ln_common.h", "diag_stamps.h"]

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-Wall",
    "-Wno-unused-function",
    "-fno-gpu-rdc",
    # keep IEEE fp32 division/sqrt: the quantizer's careful path depends on it
    "-fhip-fp32-correctly-rounded-divide-sqrt",
]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def source_digest(defines: tuple = ()) -> str:
    """sha256 of every input of the build (sources, headers, this script, flags and defines): a library
    is reused only when the digest recorded beside it matches, never on file times alone."""
    import hashlib
    h = hashlib.sha256()
    paths = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    paths += [os.path.join(INCLUDE, "qvit_hip.h"), os.path.abspath(__file__)]
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(HIPCC_FLAGS + [f"-D{d}" for d in defines]).encode())
    return h.hexdigest()


def is_stale(lib: str = LIB, defines: tuple = ()) -> bool:
    if not os.path.exists(lib):
        return True
    try:
        with open(lib + ".srcsha") as f:
            return f.read().strip() != source_digest(defines)
    except OSError:
        return True


def device_asm(src: str, build_dir: str = BUILD, name_only: bool = False) -> str:
    """The gfx950 device assembly hipcc -save-temps=obj kept for `src` (ASM_CHECKED)."""
    name = f"{os.path.splitext(src)[0]}-hip-amdgcn-amd-amdhsa-{ARCH}.s"
    return name if name_only else os.path.join(build_dir, name)


def build(force: bool = False, verbose: bool = False, defines: tuple = (), lib: str = LIB,
          build_dir: str = BUILD) -> str:
    """Builds the library. `defines`/`lib`/`build_dir` produce diagnostic variants (e.g. the
    QVIT_GEMM_STAMPS phase-timing build used by tools/gemm_stamps.py) without touching LIB."""
    if not force and not is_stale(lib, defines):
        return lib
    digest = source_digest(defines)
    hipcc = _hipcc()
    os.makedirs(build_dir, exist_ok=True)
    dflags = [f"-D{d}" for d in defines]

    def compile_one(src: str) -> str:
        obj = os.path.join(build_dir, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc, *HIPCC_FLAGS, *dflags, "-I", INCLUDE, "-c", os.path.join(CSRC, src), "-o", obj]
        keep_asm = src in ASM_CHECKED and build_dir == BUILD
        if keep_asm:
            cmd.insert(1, "-save-temps=obj")
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{res.stdout}\n{res.stderr}")
        if verbose and res.stderr.strip():
            print(res.stderr, file=sys.stderr)
        if keep_asm:   # keep the device assembly, drop the other temporaries
            stem = os.path.splitext(src)[0]
            for f in os.listdir(build_dir):
                if f.startswith(stem + "-") or f.startswith(stem + ".hip-"):
                    if f == device_asm(src, build_dir, name_only=True):
                        continue
                    os.remove(os.path.join(build_dir, f))
        return obj

    with ThreadPoolExecutor(max_workers=min(4, len(SOURCES))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed:\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, lib)
    with open(lib + ".srcsha", "w") as f:
        f.write(digest + "\n")
    return lib


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose))


if __name__ == "__main__":
    main()
