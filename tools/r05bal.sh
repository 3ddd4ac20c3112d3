set -u
O=gpurun_out/${OUTD:-r05bal}; mkdir -p $O; export TMPDIR=/tmp
L=tools/_diag/libqvit_hip_bal.so
QVIT_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_bal.log 2>&1 || { echo "bal tests failed"; tail -30 $O/t_bal.log; exit 1; }
echo "bal tests: $(tail -1 $O/t_bal.log)"
for r in 1 2 3; do
  for X in quantized_vit_amd/libqvit_hip.so $L; do
    timeout -k 10 200 python tools/attn_bench.py --fused --split-only --iters 20 --lib $X > $O/att_$(basename $X .so)_$r.log 2>&1 || { echo "attn_bench failed"; tail -5 $O/att_$(basename $X .so)_$r.log; exit 1; }
    echo "== $(basename $X) $r: $(grep fused $O/att_$(basename $X .so)_$r.log | tr '\n' ' ')"
  done
done
OUT=$O/ab SHAPES=proj ROUNDS=2 bash tools/lib_ab.sh quantized_vit_amd/libqvit_hip.so $L || exit 1
