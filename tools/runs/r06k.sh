# Round 6 k: fused qkv attention with one barrier per two projection k-steps (product build) vs the previous build
# (tools/_diag/libqvit_hip_base.so), and UltraNet conv0 with the next patch's fragment reads issued before this
# patch's MFMAs (c0pf: all three, c0pf2: hi / lo only). GPU suite on the product build first, the UltraNet tests
# on each conv0 variant, then same-box A/B lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in c0pf c0pf2; do
  QVIT_LIB=tools/_diag/libqvit_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ultranet.py tests/test_gpu_ultra_modules.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "$v tests failed"; tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
OUT=$O/ab SHAPES=proj ROUNDS=3 bash tools/lib_ab.sh tools/_diag/libqvit_hip_base.so quantized_vit_amd/libqvit_hip.so || exit 1
OUT=$O/uab ROUNDS=3 bash tools/ultra_ab.sh tools/_diag/libqvit_hip_base.so tools/_diag/libqvit_hip_c0pf.so tools/_diag/libqvit_hip_c0pf2.so || exit 1
