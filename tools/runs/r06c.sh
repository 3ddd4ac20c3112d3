# two-ahead activation ring (L2) vs one-ahead (l1): GEMM tests on the product (L2), then same-box model A/B
set -u
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_w4r.py tests/test_gpu_kernels.py tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ACT_STD=25 OUT=$O/ab SHAPES=fc1,fc1_9r,fc2,proj ROUNDS=2 bash tools/lib_ab.sh tools/_diag/libqvit_hip_l1.so tools/_diag/libqvit_hip_l2.so
