set -u
O=gpurun_out/${OUTD:-r05i}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python tools/gemm_stamps.py --ws tools/_diag/libqvit_hip_wst.so --shapes fc1_a32 --iters 10 > $O/ws.log 2>&1 || { echo "stamps failed"; tail -20 $O/ws.log; exit 1; }
grep -v amdgpu.ids $O/ws.log
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc_$i -o p -- python tools/gemm_bench.py --iters 5 --shapes fc1_a32 > $O/pmc_$i.log 2>&1
  echo "pmc pass $i rc=$?"
done
python tools/pmc_kernel.py 'gemm_ws' $O/pmc_* > $O/pmc.txt 2>&1; cat $O/pmc.txt
