set -u
O=gpurun_out/${OUTD:-r05b}; mkdir -p $O; export TMPDIR=/tmp
for v in cur nopip pip; do
  QVIT_LIB=tools/_diag/libqvit_hip_$v.so timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "gemm" -p no:cacheprovider > $O/t_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/t_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $O/t_$v.log)"
done
for v in base_ls cur_ls; do
  timeout -k 10 200 python tools/gemm_stamps.py --light tools/_diag/libqvit_hip_$v.so --shapes fc1,fc1_i32,fc2 --iters 10 > $O/ls_$v.log 2>&1 || { echo "stamps $v failed"; tail -20 $O/ls_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/ls_$v.log
done
OUT=$O/ab SHAPES=fc1,fc2,proj bash tools/lib_ab.sh tools/_diag/libqvit_hip_base.so tools/_diag/libqvit_hip_pip.so tools/_diag/libqvit_hip_cur.so tools/_diag/libqvit_hip_nopip.so
