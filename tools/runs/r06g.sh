# activation lead 3 (ring of 5 x 8 KiB) vs lead 2 (product), same box: GEMM microbench (model-like codes) + model
set -u
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
ACT_STD=25 OUT=$O/ab SHAPES=fc1,fc2,proj ROUNDS=2 bash tools/lib_ab.sh tools/_diag/libqvit_hip_l2.so tools/_diag/libqvit_hip_al3.so
