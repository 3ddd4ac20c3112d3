#!/bin/bash
# rocprofv3 PMC passes over the bench workload (tools/pmc_model.py), one counter group per run with
# --kernel-trace only (no other trace domains), each under its own hard time limit; then the per-kernel
# summary pmc_mfma.json (tools/pmc_model_summary.py) in $OUT. Copy it into profiles/ afterwards.
# Usage: OUT=gpurun_out/pmc ROUND=r02 tools/profile_model_pmc.sh [--model M --batch B]
set -u
OUT=${OUT:-gpurun_out/pmc_model}
ROUND=${ROUND:-r02}
MODEL=${MODEL:-vit_base_patch16_224}
BATCH=${BATCH:-256}
DEPTH=${DEPTH:-12}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in \
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
  "FETCH_SIZE" \
  "WRITE_SIZE" \
  "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" ; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python tools/pmc_model.py --model "$MODEL" --batch "$BATCH" --iters 2 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python tools/pmc_model_summary.py "$OUT" --model "$MODEL" --batch "$BATCH" --depth "$DEPTH" --iters 2 --round "$ROUND"
rc=$?
# keep only the summaries (the raw per-dispatch CSVs are large)
find "$OUT" -mindepth 1 -maxdepth 1 -type d -name 'p*' -exec rm -rf {} +
exit $rc
