set -u
O=gpurun_out/${OUTD:-r05st}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/attn_bench.py --B 128 --N 577 --H 16 --split-only --iters 10 > $O/base.log 2>&1 || { echo "base failed"; tail -5 $O/base.log; exit 1; }
cat $O/base.log | grep split
timeout -k 10 300 python tools/attn_bench.py --B 128 --N 577 --H 16 --split-only --iters 5 --stamps --lib tools/_diag/libqvit_hip_attst.so > $O/st.log 2>&1 || { echo "stamps failed"; tail -5 $O/st.log; exit 1; }
cat $O/st.log | grep -E "split|per wave"
