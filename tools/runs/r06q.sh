# Round 6 q: UltraNet conv0 VALU cuts. base = round-6 head, base2 = + BN sign folded into the weights (max pool
# only), product = + the staging hi/lo split on v_fma_mix + the code's rounding as the low byte of v + 2^23.
# UltraNet tests (with the new decreasing-BN conv0 test) on the product and on base, then a three-way A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ultranet.py tests/test_gpu_ultra_modules.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "product: $(tail -1 $O/tests.log)"
QVIT_LIB=tools/_diag/libqvit_hip_base.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ultranet.py -x -q --timeout 120 --timeout-method thread -k "conv0" > $O/tests_base.log 2>&1 || { tail -30 $O/tests_base.log; exit 1; }
echo "base conv0 tests: $(tail -1 $O/tests_base.log)"
OUT=$O/uab ROUNDS=3 bash tools/ultra_ab.sh tools/_diag/libqvit_hip_base.so tools/_diag/libqvit_hip_base2.so quantized_vit_amd/libqvit_hip.so || exit 1
