# GEMM ablations, part 2: which load stream sets fc2's stage time? noact: no activation LDS-DMA; now: no register
# weight loads (diagnostic builds, numerics wrong by construction)
set -u
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
for r in 1 2; do
  for v in l2 nodma noact now; do
    timeout -k 10 120 python tools/gemm_bench.py --iters 30 --act-std 25 --shapes fc1,fc2,proj --lib tools/_diag/libqvit_hip_$v.so > $O/g_${v}_$r.log 2>&1 || { tail -5 $O/g_${v}_$r.log; exit 1; }
    echo "== $v $r"; grep -v '^{\|amdgpu.ids' $O/g_${v}_$r.log
  done
done
