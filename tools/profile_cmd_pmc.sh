#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only, each under a hard time limit) over any
# python command, then the per-kernel summary (tools/pmc_summary.py). Usage: tools/profile_cmd_pmc.sh OUTDIR script.py [args]
set -u
OUT=$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in \
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
  "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_INSTS_BRANCH" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o p -- python "$@" \
      > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
find "$OUT" -mindepth 1 -maxdepth 1 -type d -name 'p*' -exec rm -rf {} +
