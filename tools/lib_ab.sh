#!/bin/bash
# Same-box A/B of library builds: GEMM microbench (tools/gemm_bench.py) and model bench lines, alternating
# the builds, each run under its own time limit; stops at the first failure.
# Usage: OUT=gpurun_out/x SHAPES=fc1,fc2 tools/lib_ab.sh libA.so libB.so [...]
set -u
OUT=${OUT:-gpurun_out/lib_ab}
SHAPES=${SHAPES:-fc1,fc2,proj}
ROUNDS=${ROUNDS:-2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    tag=$(basename "$lib" .so)
    timeout -k 10 240 python tools/gemm_bench.py --iters 20 ${ACT_STD:+--act-std $ACT_STD} --shapes "$SHAPES" --lib "$lib" > "$OUT/g_${tag}_$r.log" 2>&1 \
      || { echo "gemm_bench $tag failed"; tail -5 "$OUT/g_${tag}_$r.log"; exit 1; }
    echo "== gemm $tag round $r"; grep -v '^{' "$OUT/g_${tag}_$r.log" | tail -8
  done
  if [ "${MODEL:-1}" = 1 ]; then
    for lib in "$@"; do
      tag=$(basename "$lib" .so)
      timeout -k 10 240 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --lib "$lib" > "$OUT/b_${tag}_$r.log" 2>&1 \
        || { echo "bench $tag failed"; tail -5 "$OUT/b_${tag}_$r.log"; exit 1; }
      echo "== model $tag round $r: $(grep '^{' "$OUT/b_${tag}_$r.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "img/s", round(d["ms_per_step"], 3), "ms", {k: round(v["launch_us"], 1) for k, v in d["kernels"].items()})')"
    done
  fi
done
