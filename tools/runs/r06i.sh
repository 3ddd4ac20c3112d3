# tile pairing (QVIT_GEMM_PAIR=1: the two blocks of a CU on adjacent tiles of one activation panel) vs product
set -u
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
ACT_STD=25 OUT=$O/ab SHAPES=fc1,fc2,proj ROUNDS=2 bash tools/lib_ab.sh tools/_diag/libqvit_hip_l2.so tools/_diag/libqvit_hip_pair1.so
