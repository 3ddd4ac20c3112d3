set -u
O=gpurun_out/${OUTD:-r05sp}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for X in quantized_vit_amd/libqvit_hip.so tools/_diag/libqvit_hip_sp0.so tools/_diag/libqvit_hip_sp3.so; do
    tag=$(basename $X .so)
    timeout -k 10 240 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --lib $X > $O/b_${tag}_$r.log 2>&1 || { echo "bench $tag failed"; tail -5 $O/b_${tag}_$r.log; exit 1; }
    echo "== model $tag $r: $(grep '^{' $O/b_${tag}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "img/s", round(d["ms_per_step"], 3), "ms", {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
  done
done
