set -u
O=gpurun_out/${OUTD:-r05q}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ultra_modules.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo "tests failed"; tail -40 $O/t.log; exit 1; }
echo "tests: $(tail -1 $O/t.log)"
timeout -k 10 200 python tools/profile_ultra_modules.py > $O/mods.log 2>&1 || { echo "mods failed"; tail -20 $O/mods.log; exit 1; }
grep -v amdgpu.ids $O/mods.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rpm -o mods -- python tools/profile_ultra_modules.py > $O/mods_rp.log 2>&1 || { echo "rocprof mods failed"; tail -20 $O/mods_rp.log; exit 1; }
S=$(find $O/rpm -name "*kernel_stats.csv" | head -1); python tools/kstats.py $S 12
for r in 1 2; do
  for L in quantized_vit_amd/libqvit_hip.so tools/_diag/libqvit_hip_t16diag.so; do
    timeout -k 10 200 python tools/attn_bench.py --fused --split-only --iters 20 --lib $L > $O/att_$(basename $L .so)_$r.log 2>&1 || { echo "attn_bench failed"; tail -5 $O/att_$(basename $L .so)_$r.log; exit 1; }
    echo "== $(basename $L) $r: $(grep fused $O/att_$(basename $L .so)_$r.log | tr '\n' ' ')"
  done
done
