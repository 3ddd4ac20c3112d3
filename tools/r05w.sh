set -u
O=gpurun_out/${OUTD:-r05w}; mkdir -p $O; export TMPDIR=/tmp
OUT=$O/uab ROUNDS=2 bash tools/ultra_ab.sh quantized_vit_amd/libqvit_hip.so tools/_diag/libqvit_hip_c0pk.so tools/_diag/libqvit_hip_c0p46.so || exit 1
