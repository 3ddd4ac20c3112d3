set -u
O=gpurun_out/${OUTD:-r05r}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ultra_modules.py tests/test_gpu_model.py -k "ultra or conv or weight_stationary" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo "tests failed"; tail -40 $O/t.log; exit 1; }
echo "tests: $(tail -1 $O/t.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rpm -o mods -- python tools/profile_ultra_modules.py > $O/mods_rp.log 2>&1 || { echo "rocprof mods failed"; tail -20 $O/mods_rp.log; exit 1; }
grep "forward_modules" $O/mods_rp.log
S=$(find $O/rpm -name "*kernel_stats.csv" | head -1); python tools/kstats.py $S 8
