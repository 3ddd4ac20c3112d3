# Round 6 l: int8 GELU table epilogue with both FMAs of a column pair on v_pk_fma_f32 (product) vs the previous
# build (tools/_diag/libqvit_hip_base.so): GPU suite on the product, then same-box GEMM + model A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/ab SHAPES=fc1,fc1_9r,fc2 ROUNDS=3 bash tools/lib_ab.sh tools/_diag/libqvit_hip_base.so quantized_vit_amd/libqvit_hip.so || exit 1
