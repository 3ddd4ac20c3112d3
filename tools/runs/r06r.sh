# Round 6 r (rerun with the sign mask from one ballot): the BN sign folded into the weights of the pooled UltraNet layers too (ultra_conv_kernel SW path,
# OUT 0). New tests: every layer stage-forced and end to end on a network with gamma < 0 in every other channel.
# Tests on the product and (decreasing-BN tests only) on the round-6 head library; then A/B: base2 (conv0 fold
# only) vs the product.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06r}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ultranet.py tests/test_gpu_ultra_modules.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "product: $(tail -1 $O/tests.log)"
QVIT_LIB=tools/_diag/libqvit_hip_base.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ultranet.py -x -q --timeout 120 --timeout-method thread -k "decreasing" > $O/tests_base.log 2>&1 || { tail -30 $O/tests_base.log; exit 1; }
echo "round-6 head, decreasing-BN tests: $(tail -1 $O/tests_base.log)"
OUT=$O/uab ROUNDS=3 bash tools/ultra_ab.sh tools/_diag/libqvit_hip_base2.so quantized_vit_amd/libqvit_hip.so || exit 1
