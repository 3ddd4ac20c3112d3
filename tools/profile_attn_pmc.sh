#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over the fused qkv + attention
# microbenchmark (tools/attn_bench.py --fused), then a per-kernel summary. Usage: tools/profile_attn_pmc.sh OUTDIR [--lib L]
# ATTN_ARGS replaces the benchmark's shape/mode arguments (default "--fused --split-only"; the ViT-L split kernel:
# ATTN_ARGS="--split-only --B 128 --N 577 --H 16").
set -u
OUT=${1:-gpurun_out/attn_pmc}
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in \
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
  "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "FETCH_SIZE" \
  "TCC_HIT TCC_MISS" \
  "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o p -- \
      python tools/attn_bench.py ${ATTN_ARGS:---fused --split-only} --iters 3 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
head -80 "$OUT/summary.txt"
