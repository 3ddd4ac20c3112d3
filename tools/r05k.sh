set -u
O=gpurun_out/${OUTD:-r05k}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_ws.py "tests/test_gpu_ultra_modules.py::test_conv2d_q_invalidate_and_grad" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_ws.log 2>&1 || { echo "ws tests failed"; tail -40 $O/t_ws.log; exit 1; }
echo "ws tests: $(tail -1 $O/t_ws.log)"
timeout -k 10 200 python tools/gemm_stamps.py --ws tools/_diag/libqvit_hip_wst2.so --shapes fc1_a32 --iters 10 > $O/ws.log 2>&1 || { echo "stamps failed"; tail -20 $O/ws.log; exit 1; }
grep -v amdgpu.ids $O/ws.log
MODEL=0 OUT=$O/g SHAPES=fc1_a32 ROUNDS=2 bash tools/lib_ab.sh tools/_diag/libqvit_hip_a32v1.so quantized_vit_amd/libqvit_hip.so || exit 1
MODEL=1 OUT=$O/ab SHAPES=fc1 ROUNDS=2 bash tools/lib_ab.sh tools/_diag/libqvit_hip_base.so tools/_diag/libqvit_hip_a32v1.so quantized_vit_amd/libqvit_hip.so
