#!/bin/bash
# HBM traffic of the fc1 kernel from rocprofv3 PMC counters, two separate passes over a short bench run
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950; no tracing domains beside --kernel-trace).
# Writes $OUT/pmc_fetch, $OUT/pmc_write and profiles/fc1_traffic_<round>.json (+ profiles/fc1_traffic.json).
set -u
OUT=${OUT:-gpurun_out}
ROUND=${ROUND:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  d="$OUT/pmc_${c,,}"
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$d" -o run -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$d.log" 2>&1
  rc=$?
  echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$d.log"; exit $rc; fi
done
python tools/kstats.py --pmc "$OUT/pmc_fetch_size" "$OUT/pmc_write_size" --round "$ROUND"
