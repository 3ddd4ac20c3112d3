set -u
O=gpurun_out/${OUTD:-r05pair}; mkdir -p $O; export TMPDIR=/tmp
L=tools/_diag/libqvit_hip_pair.so
QVIT_LIB=$L timeout -k 10 900 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_production.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_pair.log 2>&1 || { echo "pair tests failed"; tail -30 $O/t_pair.log; exit 1; }
echo "pair tests: $(tail -1 $O/t_pair.log)"
for r in 1 2 3; do
  for X in quantized_vit_amd/libqvit_hip.so $L; do
    tag=$(basename $X .so)
    timeout -k 10 300 python tools/attn_bench.py --B 128 --N 577 --H 16 --split-only --iters 10 --lib $X > $O/a_${tag}_$r.log 2>&1 || { echo "attn_bench $tag failed"; tail -5 $O/a_${tag}_$r.log; exit 1; }
    echo "== attn $tag $r: $(grep split $O/a_${tag}_$r.log | tr '\n' ' ')"
  done
done
for r in 1 2; do
  for X in quantized_vit_amd/libqvit_hip.so $L; do
    tag=$(basename $X .so)
    timeout -k 10 300 python bench.py --model vit_large_patch16_384 --batch 128 --steps 10 --warmup 3 --no-cpu-baseline --lib $X > $O/b_${tag}_$r.log 2>&1 || { echo "bench $tag failed"; tail -5 $O/b_${tag}_$r.log; exit 1; }
    echo "== vitl $tag $r: $(grep '^{' $O/b_${tag}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "img/s", round(d["ms_per_step"], 3), "ms")')"
  done
done
