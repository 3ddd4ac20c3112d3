set -u
O=gpurun_out/${OUTD:-r05x}; mkdir -p $O; export TMPDIR=/tmp
QVIT_LIB=tools/_diag/libqvit_hip_c0t.so timeout -k 10 400 python -u -m pytest tests/test_gpu_ultranet.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_c0.log 2>&1 || { echo "c0t tests failed"; tail -30 $O/t_c0.log; exit 1; }
echo "c0t tests: $(tail -1 $O/t_c0.log)"
OUT=$O/uab ROUNDS=3 bash tools/ultra_ab.sh quantized_vit_amd/libqvit_hip.so tools/_diag/libqvit_hip_c0t.so || exit 1
