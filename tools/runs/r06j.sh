# UltraNet layer 0 (ultra_conv0_mfma_kernel, b256 @416 fused forward): which LDS access class conflicts? One PMC pass
# per diagnostic build that drops one class (numerics wrong by construction): c0nostage (halo staging writes after
# the first tile), c0nocodes (the pooled-code byte writes), c0nofrag (all fragment reads), c0nox1 (tap (2,2) reads),
# c0nolo (lo-plane reads); l2 = the product. Then the per-kernel medians (tools/pmc_summary.py) for each.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
for v in l2 c0nostage c0nocodes c0nofrag c0nox1 c0nolo; do
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/$v -o p -- python tools/pmc_ultra.py --iters 2 --lib tools/_diag/libqvit_hip_$v.so > $O/$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/$v.log; exit $rc; fi
  python tools/pmc_summary.py $O/$v > $O/${v}_summary.txt
  grep -A12 "ultra_conv0_mfma_kernel" $O/${v}_summary.txt | head -12
  f=$(find $O/$v -name "*kernel_trace.csv" | head -1)
  python - "$f" <<'PY'
import csv, statistics, sys
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(sys.argv[1])) if "ultra_conv0_mfma" in r["Kernel_Name"]]
print("   conv0 duration median us", statistics.median(d) / 1000 if d else None, "n", len(d))
PY
  rm -rf $O/$v
done
