set -u
O=gpurun_out/${OUTD:-r05v}; mkdir -p $O; export TMPDIR=/tmp
QVIT_LIB=tools/_diag/libqvit_hip_c0pad.so timeout -k 10 400 python -u -m pytest tests/test_gpu_ultranet.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_c0.log 2>&1 || { echo "c0pad tests failed"; tail -30 $O/t_c0.log; exit 1; }
echo "c0pad tests: $(tail -1 $O/t_c0.log)"
OUT=$O/uab ROUNDS=2 bash tools/ultra_ab.sh quantized_vit_amd/libqvit_hip.so tools/_diag/libqvit_hip_c0pad.so || exit 1
for r in 1 2; do
  for L in quantized_vit_amd/libqvit_hip.so tools/_diag/libqvit_hip_qa_vm2.so; do
    timeout -k 10 200 python tools/attn_bench.py --fused --split-only --iters 20 --lib $L > $O/att_$(basename $L .so)_$r.log 2>&1 || { echo "attn_bench failed"; tail -5 $O/att_$(basename $L .so)_$r.log; exit 1; }
    echo "== $(basename $L) $r: $(grep fused $O/att_$(basename $L .so)_$r.log | tr '\n' ' ')"
  done
done
