#!/bin/bash
# Same-box A/B of library builds on the UltraNet @416 b256 workload (bench.py --model ultranet): bench lines
# alternating the builds, each under its own time limit; stops at the first failure.
# Usage: OUT=gpurun_out/x ROUNDS=2 tools/ultra_ab.sh libA.so libB.so [...]
set -u
OUT=${OUT:-gpurun_out/ultra_ab}
ROUNDS=${ROUNDS:-2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    tag=$(basename "$lib" .so)
    timeout -k 10 240 python bench.py --model ultranet --no-cpu-baseline --steps 20 --warmup 3 --lib "$lib" \
        > "$OUT/u_${tag}_$r.log" 2>&1 || { echo "bench $tag failed"; tail -5 "$OUT/u_${tag}_$r.log"; exit 1; }
    echo "== ultranet $tag round $r: $(grep '^{' "$OUT/u_${tag}_$r.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "img/s", round(d["ms_per_step"], 3), "ms", {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
  done
done
