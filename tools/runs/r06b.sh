# W8R (int8 register weight image) vs W4R: GEMM tests, then same-box model A/B and GEMM microbench
set -u
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_w4r.py tests/test_capi.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for w in w4r w8r; do
    QVIT_GEMM_WREG=$w timeout -k 10 200 python tools/gemm_bench.py --iters 30 --act-std 25 --shapes fc1,fc1_9r,fc2,proj > $O/g_${w}_$r.log 2>&1 || { tail -5 $O/g_${w}_$r.log; exit 1; }
    echo "== gemm $w $r"; grep -v '^{\|amdgpu.ids' $O/g_${w}_$r.log
  done
  for w in w4r w8r; do
    QVIT_GEMM_WREG=$w timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/b_${w}_$r.log 2>&1 || { tail -5 $O/b_${w}_$r.log; exit 1; }
    echo "== model $w $r: $(grep '^{' $O/b_${w}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "img/s", round(d["ms_per_step"], 3), "ms", {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
  done
done
