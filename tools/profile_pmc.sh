#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over the GEMM microbenchmark,
# then a per-kernel summary (tools/pmc_summary.py). Usage: tools/profile_pmc.sh OUTDIR "shapes"
set -u
OUT=${1:-gpurun_out/pmc}
SHAPES=${2:-fc1}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in \
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
  "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES" \
  "TCP_TOTAL_CACHE_ACCESSES TCP_CACHE_MISS TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES" \
  "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TA_FLAT_READ_LDS_WAVEFRONTS" \
  "TD_TD_BUSY TD_TC_STALL TD_LOAD_WAVEFRONT" \
  "TCC_HIT TCC_MISS TCC_BUSY TCC_TAG_STALL" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o p -- \
      python tools/gemm_bench.py --iters 3 --shapes "$SHAPES" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python tools/pmc_summary.py "$OUT"
