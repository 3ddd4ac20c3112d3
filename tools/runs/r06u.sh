# Round 6 u: rocprofv3 kernel summaries of the UltraNet @416 b256 and ViT-L/16 @384 b128 bench lines (final build).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rpu -o run -- python bench.py --model ultranet --steps 5 --warmup 2 --no-cpu-baseline > $O/ultra.log 2>&1 || { tail -20 $O/ultra.log; exit 1; }
f=$(find $O/rpu -name "*kernel_stats.csv" | head -1); python tools/kstats.py "$f" 25 > $O/ultra_kernel_summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rpl -o run -- python bench.py --model vit_large_patch16_384 --batch 128 --steps 3 --warmup 1 --no-cpu-baseline > $O/vitl.log 2>&1 || { tail -20 $O/vitl.log; exit 1; }
f=$(find $O/rpl -name "*kernel_stats.csv" | head -1); python tools/kstats.py "$f" 25 > $O/vitl_kernel_summary.txt
rm -rf $O/rpu $O/rpl
head -12 $O/ultra_kernel_summary.txt; head -12 $O/vitl_kernel_summary.txt
