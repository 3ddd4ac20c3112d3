set -u
O=gpurun_out/${OUTD:-r05w4off}; mkdir -p $O; export TMPDIR=/tmp
QVIT_GEMM_W4R=0 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
echo "tests (QVIT_GEMM_W4R=0): $(tail -1 $O/tests.log)"
QVIT_FUSE_LN=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_fuse_ln.log 2>&1 || { echo "fuse-ln tests failed"; tail -40 $O/tests_fuse_ln.log; exit 1; }
echo "model tests (QVIT_FUSE_LN=1, W4R on): $(tail -1 $O/tests_fuse_ln.log)"
