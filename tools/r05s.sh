set -u
O=gpurun_out/${OUTD:-r05s}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-400
QVIT_STEP_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp -o bench -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_rp.log 2>&1 || { echo "rocprof bench failed"; tail -20 $O/bench_rp.log; exit 1; }
T=$(find $O/rp -name "*kernel_trace.csv" | head -1); python tools/kstats.py --split $T 5 40 > $O/split.txt && head -25 $O/split.txt
