set -u
O=gpurun_out/${OUTD:-r05o}; mkdir -p $O; export TMPDIR=/tmp
# 2. stream-K + narrow conv tests, SK on/off model A/B
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_sk.py tests/test_gpu_ultra_modules.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo "tests failed"; tail -40 $O/t.log; exit 1; }
echo "tests: $(tail -1 $O/t.log)"
for r in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --iters 20 --shapes fc2,fc2_sk,proj,proj_sk > $O/g_$r.log 2>&1 || { echo "gemm_bench failed"; tail -20 $O/g_$r.log; exit 1; }
  grep -v amdgpu.ids $O/g_$r.log | grep -v '^{'
  for sk in 0 1; do
    QVIT_STREAM_K=$sk timeout -k 10 240 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/b_${sk}_$r.log 2>&1 || { echo "bench failed"; tail -5 $O/b_${sk}_$r.log; exit 1; }
    echo "== model SK=$sk round $r: $(grep '^{' $O/b_${sk}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "img/s", round(d["ms_per_step"], 3), "ms", {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
  done
done
# 3. module-level UltraNet profile
timeout -k 10 200 python tools/profile_ultra_modules.py > $O/mods.log 2>&1 || { echo "mods failed"; tail -20 $O/mods.log; exit 1; }
grep -v amdgpu.ids $O/mods.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rpm -o mods -- python tools/profile_ultra_modules.py > $O/mods_rp.log 2>&1 || { echo "rocprof mods failed"; tail -20 $O/mods_rp.log; exit 1; }
S=$(find $O/rpm -name "*kernel_stats.csv" | head -1); python tools/kstats.py $S 12
