# Round 6 m: GPU suite on the lazy register-image plans (quant_layers.QuantPlan.gemm_weights / packed_codes), then
# UltraNet conv0 with ONE halo buffer (an extra barrier per tile; 13.5 KiB of LDS, 8 workgroups per CU instead of 6):
# the UltraNet tests on the variant, then same-box A/B against the product build.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
v=c0sb8
QVIT_LIB=tools/_diag/libqvit_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ultranet.py tests/test_gpu_ultra_modules.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "$v tests failed"; tail -30 $O/tests_$v.log; exit 1; }
echo "$v: $(tail -1 $O/tests_$v.log)"
OUT=$O/uab ROUNDS=3 bash tools/ultra_ab.sh quantized_vit_amd/libqvit_hip.so tools/_diag/libqvit_hip_c0sb8.so || exit 1
