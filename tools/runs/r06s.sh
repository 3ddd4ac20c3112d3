# Round 6 s: the pooled-layer BN sign fold restricted to the staged kernels (conv1, conv2), tests on the product,
# then A/B: base2 (conv0 fold only) vs the product vs c0g2 (conv0 with two patches per MFMA group at 5 workgroups
# per CU; its other layers carry the unrestricted fold).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ultranet.py tests/test_gpu_ultra_modules.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "product: $(tail -1 $O/tests.log)"
QVIT_LIB=tools/_diag/libqvit_hip_c0g2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ultranet.py -x -q --timeout 120 --timeout-method thread -k "conv0 or decreasing or production" > $O/tests_c0g2.log 2>&1 || { tail -30 $O/tests_c0g2.log; exit 1; }
echo "c0g2: $(tail -1 $O/tests_c0g2.log)"
OUT=$O/uab ROUNDS=3 bash tools/ultra_ab.sh tools/_diag/libqvit_hip_base2.so quantized_vit_amd/libqvit_hip.so tools/_diag/libqvit_hip_c0g2.so || exit 1
