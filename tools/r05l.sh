set -u
O=gpurun_out/${OUTD:-r05l}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_gpu_model.py::test_vit_fc1_weight_stationary_bit_identical" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo "tests failed"; tail -40 $O/t.log; exit 1; }
echo "tests: $(tail -1 $O/t.log)"
timeout -k 10 200 python tools/attn_bench.py --fused --stamps --split-only --iters 10 --lib tools/_diag/libqvit_hip_attst.so > $O/attst.log 2>&1 || { echo "attst failed"; tail -20 $O/attst.log; exit 1; }
grep -v amdgpu.ids $O/attst.log
timeout -k 10 200 python tools/attn_bench.py --fused --stamps --split-only --iters 10 --lib tools/_diag/libqvit_hip_attlst.so > $O/attlst.log 2>&1 || { echo "attlst failed"; tail -20 $O/attlst.log; exit 1; }
grep -v amdgpu.ids $O/attlst.log
QVIT_STEP_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rp -o bench -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || { echo "rocprof bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
T=$(find $O/rp -name "*kernel_trace.csv" | head -1); python tools/kstats.py --split $T 5 40 > $O/split.txt && head -30 $O/split.txt
