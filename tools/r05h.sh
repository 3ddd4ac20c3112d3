set -u
O=gpurun_out/${OUTD:-r05h}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_ws.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_ws.log 2>&1 || { echo "ws tests failed"; tail -40 $O/t_ws.log; exit 1; }
echo "ws tests: $(tail -1 $O/t_ws.log)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py -m gpu -x -q -k "gelu_code" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_prod.log 2>&1 || { echo "prod tests failed"; tail -40 $O/t_prod.log; exit 1; }
echo "prod tests: $(tail -1 $O/t_prod.log)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_model.log 2>&1 || { echo "model tests failed"; tail -40 $O/t_model.log; exit 1; }
echo "model tests: $(tail -1 $O/t_model.log)"
MODEL=1 OUT=$O/ab SHAPES=fc1 ROUNDS=2 bash tools/lib_ab.sh tools/_diag/libqvit_hip_base.so quantized_vit_amd/libqvit_hip.so
