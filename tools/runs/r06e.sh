# GEMM ablations (diagnostic builds from /tmp copies of csrc, numerics wrong by construction): which resource sets
# the fc1 / fc2 stage time? nomfma: MFMAs -> one VALU each; nodma: no global loads (LDS-DMA, register weights);
# noread: no LDS fragment reads; noepi: no int8 epilogue
set -u
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
for r in 1 2; do
  for v in l2 nomfma nodma noread noepi; do
    timeout -k 10 120 python tools/gemm_bench.py --iters 30 --act-std 25 --shapes fc1_1t,fc1,fc2 --lib tools/_diag/libqvit_hip_$v.so > $O/g_${v}_$r.log 2>&1 || { tail -5 $O/g_${v}_$r.log; exit 1; }
    echo "== $v $r"; grep -v '^{\|amdgpu.ids' $O/g_${v}_$r.log
  done
done
