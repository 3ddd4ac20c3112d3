set -u
O=gpurun_out/${OUTD:-r05box}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  for V in 1 0; do
    QVIT_GEMM_W4R=$V timeout -k 10 240 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b_${V}_$r.log 2>&1 || { echo "bench failed"; tail -5 $O/b_${V}_$r.log; exit 1; }
    echo "== W4R=$V $r: $(grep '^{' $O/b_${V}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "img/s", round(d["ms_per_step"], 3), "ms frac", round(d["roofline"]["frac"], 4), {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
  done
done
