set -u
O=gpurun_out/${OUTD:-r05qs}; mkdir -p $O; export TMPDIR=/tmp
L=tools/_diag/libqvit_hip_qs.so
QVIT_LIB=$L timeout -k 10 900 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_production.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_qs.log 2>&1 || { echo "qs tests failed"; tail -30 $O/t_qs.log; exit 1; }
echo "qs tests: $(tail -1 $O/t_qs.log)"
for r in 1 2; do
  for X in quantized_vit_amd/libqvit_hip.so $L; do
    tag=$(basename $X .so)
    timeout -k 10 300 python bench.py --model vit_large_patch16_384 --batch 128 --steps 10 --warmup 3 --no-cpu-baseline --lib $X > $O/b_${tag}_$r.log 2>&1 || { echo "bench $tag failed"; tail -5 $O/b_${tag}_$r.log; exit 1; }
    echo "== vitl $tag $r: $(grep '^{' $O/b_${tag}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "img/s", round(d["ms_per_step"], 3), "ms", {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
  done
done
for X in quantized_vit_amd/libqvit_hip.so $L; do
  tag=$(basename $X .so)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_$tag -o vitl -- python bench.py --model vit_large_patch16_384 --batch 128 --steps 3 --warmup 1 --no-cpu-baseline --lib $X > $O/rp_$tag.log 2>&1 || { echo "rocprof $tag failed"; tail -5 $O/rp_$tag.log; exit 1; }
  S=$(find $O/rp_$tag -name "*kernel_stats.csv" | head -1); echo "== $tag"; grep -E "gemm_kernel|attn_split" $S | cut -c1-160
done
