# Phase budget of the fused qkv + attention kernel at b256 (ViT-B): light stamps (unit phase boundaries only) and
# full stamps (per k-step marks too), random data; tools/attn_bench.py --fused --stamps on diagnostic builds
set -u
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
for v in attlst attst; do
  timeout -k 10 200 python tools/attn_bench.py --fused --stamps --split-only --lib tools/_diag/libqvit_hip_$v.so > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  echo "== $v"; grep -v 'amdgpu.ids' $O/$v.log
done
timeout -k 10 200 python tools/attn_bench.py --fused --split-only > $O/product.log 2>&1 || { tail -5 $O/product.log; exit 1; }
echo "== product"; grep -v 'amdgpu.ids' $O/product.log
