set -u
O=gpurun_out/${OUTD:-r05w4r}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for r in 1 2; do
  for V in 0 1; do
    QVIT_GEMM_W4R=$V timeout -k 10 240 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/b_${V}_$r.log 2>&1 || { echo "bench $V failed"; tail -5 $O/b_${V}_$r.log; exit 1; }
    echo "== vitb W4R=$V $r: $(grep '^{' $O/b_${V}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "img/s", round(d["ms_per_step"], 3), "ms", {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
  done
done
for V in 0 1; do
  QVIT_GEMM_W4R=$V timeout -k 10 300 python bench.py --model vit_large_patch16_384 --batch 128 --steps 10 --warmup 3 --no-cpu-baseline > $O/l_${V}.log 2>&1 || { echo "vitl $V failed"; tail -5 $O/l_${V}.log; exit 1; }
  echo "== vitl W4R=$V: $(grep '^{' $O/l_${V}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "img/s", round(d["ms_per_step"], 3), "ms", {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
done
