#!/bin/bash
# Round-3 evidence, part B: model PMC summary (pmc_mfma), UltraNet and ViT-L bench lines, UltraNet kernel stats.
set -u
OUT=gpurun_out/r03_final
mkdir -p "$OUT"
export TMPDIR=/tmp
OUT=$OUT/pmc ROUND=r03 bash tools/profile_model_pmc.sh > "$OUT/pmc.out" 2>&1 || { tail -20 "$OUT/pmc.out"; exit 1; }
tail -3 "$OUT/pmc.out"
timeout -k 10 300 python bench.py --model ultranet > "$OUT/ultranet.log" 2>&1 || { tail -5 "$OUT/ultranet.log"; exit 1; }
grep '^{' "$OUT/ultranet.log" | tail -1 > "$OUT/r03_ultranet416_b256_bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ustats" -o run -- \
    python bench.py --model ultranet --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/ustats.log" 2>&1 || { tail -5 "$OUT/ustats.log"; exit 1; }
f=$(find "$OUT/ustats" -name "*kernel_stats.csv" | head -1)
python tools/kstats.py "$f" 30 > "$OUT/r03_ultranet416_b256_kernel_summary.txt"
rm -rf "$OUT/ustats"
timeout -k 10 400 python bench.py --model vit_large_patch16_384 --batch 128 --steps 10 --warmup 3 --cpu-batch 2 --cpu-iters 1 > "$OUT/vitl.log" 2>&1 || { tail -5 "$OUT/vitl.log"; exit 1; }
grep '^{' "$OUT/vitl.log" | tail -1 > "$OUT/r03_vitl384_b128_bench_line.json"
cat "$OUT/r03_ultranet416_b256_bench.json" | head -c 600; echo
cat "$OUT/r03_vitl384_b128_bench_line.json" | head -c 400; echo
