set -u
O=gpurun_out/${OUTD:-r05d}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_ws.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_ws.log 2>&1 || { echo "ws tests failed"; tail -40 $O/t_ws.log; exit 1; }
echo "ws tests: $(tail -1 $O/t_ws.log)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_production.py -m gpu -x -q -k "gemm or epilogue" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_gemm.log 2>&1 || { echo "gemm tests failed"; tail -40 $O/t_gemm.log; exit 1; }
echo "gemm tests: $(tail -1 $O/t_gemm.log)"
OUT=$O/ab SHAPES=fc1,fc2,proj ROUNDS=2 bash tools/lib_ab.sh tools/_diag/libqvit_hip_base.so quantized_vit_amd/libqvit_hip.so
