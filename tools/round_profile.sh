#!/bin/bash
# Round evidence in one GPU call: default bench line (with the CPU baseline), rocprofv3 kernel-trace
# stats of the bench, fc1 HBM traffic from two PMC passes, and the bench line again with the traffic
# field filled. Everything lands in $OUT (under gpurun_out/, the directory that returns from the box);
# copy the files into profiles/ afterwards. Usage: ROUND=r01 tools/round_profile.sh
set -u
ROUND=${ROUND:-r01}
OUT=${OUT:-gpurun_out/round_$ROUND}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > "$OUT/bench_default.log" 2>&1 || { tail -5 "$OUT/bench_default.log"; exit 1; }
grep '^{' "$OUT/bench_default.log" | tail -1 > "$OUT/bench_default.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/stats.log" 2>&1 || { tail -5 "$OUT/stats.log"; exit 1; }
f=$(find "$OUT/stats" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/${ROUND}_bench_kernel_stats.csv"
python tools/kstats.py "$f" 30 > "$OUT/${ROUND}_bench_kernel_summary.txt"
for c in FETCH_SIZE WRITE_SIZE; do
  d="$OUT/pmc_${c,,}"
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$d" -o run -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$d.log" 2>&1 || { tail -5 "$d.log"; exit 1; }
done
PMC_OUT="$OUT" python tools/kstats.py --pmc "$OUT/pmc_fetch_size" "$OUT/pmc_write_size" --round "$ROUND" > /dev/null
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_traffic.log" 2>&1 || { tail -5 "$OUT/bench_traffic.log"; exit 1; }
grep '^{' "$OUT/bench_traffic.log" | tail -1 > "$OUT/bench_traffic.json"
rm -rf "$OUT/stats" "$OUT/pmc_fetch_size" "$OUT/pmc_write_size"
cat "$OUT/bench_default.json" "$OUT/${ROUND}_bench_kernel_summary.txt" "$OUT/fc1_traffic.json"
