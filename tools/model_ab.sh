#!/bin/bash
# Model-level A/B of the in-tree library against another build of it on ONE box (box-to-box spread is ~8 %):
# bench lines alternating A, B, A, B, then a rocprofv3 kernel-trace summary of each. The in-tree library is
# restored at the end. Usage: tools/model_ab.sh path/to/other_libqvit_hip.so [OUT]
set -u
ALT=$1
O=${2:-gpurun_out/model_ab}
mkdir -p "$O"
export TMPDIR=/tmp
LIB=quantized_vit_amd/libqvit_hip.so
cp "$LIB" "$O/lib_a.so.keep"
use() { if [ "$1" = b ]; then cp "$ALT" "$LIB"; else cp "$O/lib_a.so.keep" "$LIB"; fi; }
rc=0
for tag in a b a b; do
  use $tag
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > "$O/b_$tag.log" 2>&1 || { tail -5 "$O/b_$tag.log"; rc=1; break; }
  echo "$tag $(grep '^{' "$O/b_$tag.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
if [ $rc -eq 0 ]; then
  for tag in a b; do
    use $tag
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/s_$tag" -o run -- \
        python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$O/s_$tag.log" 2>&1 || { tail -5 "$O/s_$tag.log"; rc=1; break; }
    f=$(find "$O/s_$tag" -name "*kernel_stats.csv" | head -1)
    echo "== $tag"; python tools/kstats.py "$f" 8
  done
fi
use a
rm -f "$O/lib_a.so.keep"
exit $rc
