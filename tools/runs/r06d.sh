# the round staircase of fc1 / fc2 (model-like activation codes): is a lone block faster than a full round?
set -u
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --iters 30 --act-std 25 --shapes fc1_1t,fc1_1r,fc1_9r,fc1,fc1_975r,fc2_1t,fc2_2r,fc2,fc2_3r > $O/g_$r.log 2>&1 || { tail -5 $O/g_$r.log; exit 1; }
  echo "== round $r"; grep -v '^{\|amdgpu.ids' $O/g_$r.log
done
# light per-tile stamps (head / main loop / epilogue cycles, in-kernel clock) of the shipped pipeline
timeout -k 10 200 python tools/gemm_stamps.py --light tools/_diag/libqvit_hip_lst.so --shapes fc1_1t,fc1_1r,fc1,fc2_1t,fc2 > $O/light.log 2>&1 || { tail -5 $O/light.log; exit 1; }
echo "== light stamps"; grep -v 'amdgpu.ids' $O/light.log
timeout -k 10 200 python tools/gemm_stamps.py --lib tools/_diag/libqvit_hip_stamps.so --shapes fc1,fc2 > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 1; }
echo "== stamps"; grep -v 'amdgpu.ids' $O/stamps.log
