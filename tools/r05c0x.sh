set -u
O=gpurun_out/${OUTD:-r05c0x}; mkdir -p $O; export TMPDIR=/tmp
L=tools/_diag/libqvit_hip_c0x.so
QVIT_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_ultranet.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo "c0x tests failed"; tail -30 $O/t.log; exit 1; }
echo "c0x tests: $(tail -1 $O/t.log)"
OUT=$O/uab ROUNDS=3 bash tools/ultra_ab.sh quantized_vit_amd/libqvit_hip.so $L || exit 1
