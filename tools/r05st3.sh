set -u
O=gpurun_out/${OUTD:-r05st3}; mkdir -p $O; export TMPDIR=/tmp
for L in tools/_diag/libqvit_hip_stamps.so tools/_diag/libqvit_hip_rw2st.so tools/_diag/libqvit_hip_rw3st.so; do
  tag=$(basename $L .so)
  timeout -k 10 300 python tools/gemm_stamps.py --shapes fc1,fc2 --iters 5 --lib $L > $O/st_$tag.log 2>&1 || { echo "stamps $tag failed"; tail -5 $O/st_$tag.log; exit 1; }
  echo "== $tag"; grep -E "^(fc1|fc2) " $O/st_$tag.log | cut -c1-250
done
QVIT_LIB=tools/_diag/libqvit_hip_rw3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_w4r.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t3.log 2>&1 || { echo "rw3 tests failed"; tail -30 $O/t3.log; exit 1; }
echo "rw3 tests: $(tail -1 $O/t3.log)"
for r in 1 2 3; do
  for X in quantized_vit_amd/libqvit_hip.so tools/_diag/libqvit_hip_rw2.so tools/_diag/libqvit_hip_rw3.so; do
    tag=$(basename $X .so)
    timeout -k 10 240 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --lib $X > $O/b_${tag}_$r.log 2>&1 || { echo "bench $tag failed"; tail -5 $O/b_${tag}_$r.log; exit 1; }
    echo "== model $tag $r: $(grep '^{' $O/b_${tag}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "img/s", round(d["ms_per_step"], 3), "ms", {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
  done
done
