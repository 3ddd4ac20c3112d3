"""The inline-asm register loads against the compiler: tools/asm_load_check.py walks the
device assembly of every kernel that holds one and asserts that, on every control-flow path from each load, a
covering `s_waitcnt vmcnt(N)` comes before any instruction that reads, copies, spills or overwrites its
destination registers. The assembly is the one the library was assembled from
(build.py keeps it with -save-temps=obj); without it (a library built elsewhere) the sources are compiled to
assembly here with the product flags. CPU only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import asm_load_check  # noqa: E402
from quantized_vit_amd import build  # noqa: E402

# kernels (mangled-name fragments) that must be found holding asm loads: the check is not vacuous
EXPECT = {
    "gemm_w4a8.hip": ["gemm_kernelILi4ELi2ELi1ELi1E", "gemm_kernelILi4ELi2ELi1ELi2E",   # fc1: W4R, W8R
                      "gemm_kernelILi4ELi1ELi1ELi0E"],                                    # residual epilogue loads
    "ultra_conv.hip": ["ultra_tail_kernel"],
}


def _asm(src, tmp_path):
    path = build.device_asm(src)
    lib = build.LIB
    if (os.path.exists(path) and os.path.exists(lib) and not build.is_stale()
            and os.path.getmtime(path) <= os.path.getmtime(lib) + 1):
        return path
    out = str(tmp_path / (src + ".s"))
    cmd = [build._hipcc(), *build.HIPCC_FLAGS, "-I", build.INCLUDE, "--cuda-device-only", "-S",
           os.path.join(build.CSRC, src), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return out


@pytest.mark.parametrize("src", sorted(EXPECT))
def test_asm_loads_waited_before_use(src, tmp_path):
    counts, errs = asm_load_check.check_file(_asm(src, tmp_path))
    for frag in EXPECT[src]:
        assert any(frag in k for k in counts), f"no asm loads found in a kernel matching {frag}: {sorted(counts)}"
    assert not errs, "\n".join(errs[:20])


_BAD = """
_Zkernel:
	;;#ASMSTART
	; qvit_asm_load
	global_load_dwordx4 v[4:7], v1, s[2:3]
	;;#ASMEND
	global_load_dwordx4 v[8:11], v1, s[2:3]
	s_cbranch_scc1 .LBB0_2
	s_waitcnt vmcnt(1)
	s_branch .LBB0_3
.LBB0_2:
	s_waitcnt vmcnt(2)
	v_mov_b32_e32 v20, v5
.LBB0_3:
	;;#ASMSTART
	; qvit_pin v[4:7]
	;;#ASMEND
	s_endpgm
.Lfunc_end0:
"""


def test_checker_flags_a_copy_before_the_wait(tmp_path):
    """The checker itself: one path waits (vmcnt(1) covers the load: one younger operation), the other waits too
    little (vmcnt(2)) and copies a destination register: exactly that path is reported."""
    p = tmp_path / "bad.s"
    p.write_text(_BAD)
    counts, errs = asm_load_check.check_file(str(p))
    assert counts == {"_Zkernel": 1}
    assert len(errs) == 1 and "v_mov_b32_e32 v20, v5" in errs[0]
    p.write_text(_BAD.replace("vmcnt(2)", "vmcnt(1)"))
    assert asm_load_check.check_file(str(p))[1] == []
