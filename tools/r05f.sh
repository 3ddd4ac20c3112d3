set -u
O=gpurun_out/${OUTD:-r05f}; mkdir -p $O; export TMPDIR=/tmp
for v in g2p2 g2p4; do
  timeout -k 10 200 python tools/gemm_stamps.py --ws tools/_diag/libqvit_hip_$v.so --shapes fc1,fc1_i8 --iters 10 > $O/ws_$v.log 2>&1 || { echo "stamps $v failed"; tail -20 $O/ws_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/ws_$v.log
done
MODEL=1 OUT=$O/ab SHAPES=fc1 ROUNDS=1 bash tools/lib_ab.sh tools/_diag/libqvit_hip_base.so tools/_diag/libqvit_hip_g2p2n.so tools/_diag/libqvit_hip_g2p4n.so
