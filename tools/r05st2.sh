set -u
O=gpurun_out/${OUTD:-r05st2}; mkdir -p $O; export TMPDIR=/tmp
for V in 0 1; do
  QVIT_GEMM_W4R=$V timeout -k 10 300 python tools/gemm_stamps.py --shapes fc1,fc2,proj --iters 5 > $O/st_$V.log 2>&1 || { echo "stamps $V failed"; tail -5 $O/st_$V.log; exit 1; }
  echo "== W4R=$V"; grep -E "^(fc1|fc2|proj) " $O/st_$V.log
done
