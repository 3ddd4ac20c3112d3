# Round 6 t: the fused qkv + attention epilogue's fp16 hi/lo split of q, k, v on v_fma_mix (split8_mix, the same
# values as split8) vs the final build (base): attention tests on the product, then model A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "product: $(tail -1 $O/tests.log)"
OUT=$O/ab SHAPES=proj ROUNDS=3 bash tools/lib_ab.sh tools/_diag/libqvit_hip_base.so quantized_vit_amd/libqvit_hip.so || exit 1
