# Round-6 evidence run on one box: GPU suite, bench line, rocprof kernel summary (timed steps split out),
# fc1 HBM traffic and model PMC passes, then the bench line again with the counters of this build merged in.
# Everything lands under gpurun_out/$TAG (profiles/ json copies included) for committing.
set -u
TAG=${TAG:-r06ev}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
OUT=$O bash tools/gpu_round.sh \
  "600|tests|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300|bench|python bench.py" \
  "400|rocprof|QVIT_STEP_MARKERS=1 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "600|fc1_traffic|OUT=$O/fc1 ROUND=r06 bash tools/profile_fc1.sh" \
  "900|pmc|OUT=$O/pmc ROUND=r06 bash tools/profile_model_pmc.sh" \
  "300|bench2|python bench.py" \
  "120|smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "400|bench_vitl|python bench.py --model vit_large_patch16_384 --batch 128" \
  "300|bench_ultra|python bench.py --model ultranet" || exit $?
cp profiles/fc1_traffic_r06.json profiles/fc1_traffic.json $O/ 2>/dev/null
cp $O/pmc/pmc_mfma.json $O/pmc_mfma_r06.json 2>/dev/null
f=$(find $O/rp -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python tools/kstats.py --split "$f" 5 > $O/kernel_summary_split.txt
f=$(find $O/rp -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python tools/kstats.py "$f" 25 > $O/kernel_summary.txt
rm -rf $O/rp $O/fc1/pmc_fetch_size $O/fc1/pmc_write_size
echo "== bench lines"; grep -h '^{' $O/bench.log $O/bench2.log $O/bench_vitl.log $O/bench_ultra.log | cut -c1-400
