"""Builds a variant of libqvit_hip.so from another copy of the kernel sources (diagnostic A/B builds).

    python tools/build_variant.py NAME CSRC_DIR [-D DEF ...]

Compiles every source of quantized_vit_amd.build.SOURCES found in CSRC_DIR (else the package's csrc/; headers
from CSRC_DIR only: give it a full copy of csrc/) with the product flags plus the given defines, and links
tools/_diag/libqvit_hip_NAME.so. Used to run two builds of one kernel side by side on the same GPU box
(tools/lib_ab.sh); the product library is never touched.
"""
import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from quantized_vit_amd import build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("csrc")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "tools", "_diag", f"obj_{a.name}")
    os.makedirs(out_dir, exist_ok=True)
    hipcc = build._hipcc()

    def one(src):
        path = os.path.join(a.csrc, src)
        if not os.path.exists(path):
            path = os.path.join(build.CSRC, src)
        obj = os.path.join(out_dir, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc, *build.HIPCC_FLAGS, *[f"-D{d}" for d in a.defines], "-I", a.csrc, "-I", build.INCLUDE,
               "-c", path, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(f"{src}: {r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=4) as ex:
        objs = list(ex.map(one, build.SOURCES))
    lib = os.path.join(ROOT, "tools", "_diag", f"libqvit_hip_{a.name}.so")
    r = subprocess.run([hipcc, f"--offload-arch={build.ARCH}", "-shared", "-fPIC", "-o", lib, *objs],
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    print(lib)


if __name__ == "__main__":
    main()
