#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout (exit >= 2 for pytest, != 0 otherwise)
# stops the script before any further GPU work.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
STEPS=${STEPS:-tests,bench,prof}

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a "$OUT/steps.log"
  tail -n 25 "$OUT/$name.log"
  return $rc
}

if [[ $STEPS == *tests* ]]; then
  run pytest_gpu 600 python -m pytest tests -m gpu -q -rf -p no:cacheprovider ${PYTEST_ARGS:-}
  rc=$?
  if [[ $rc -ge 2 ]]; then echo "pytest crashed/timed out (rc=$rc): stopping"; exit $rc; fi
fi
if [[ $STEPS == *bench* ]]; then
  run bench 360 python bench.py ${BENCH_ARGS:-} || exit $?
fi
if [[ $STEPS == *prof* ]]; then
  run rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline || exit $?
  find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/" \; 2>/dev/null
fi
echo ALL DONE
