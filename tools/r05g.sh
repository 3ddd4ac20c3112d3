set -u
O=gpurun_out/${OUTD:-r05g}; mkdir -p $O; export TMPDIR=/tmp
for v in dhot dnoload; do
  timeout -k 10 200 python tools/gemm_stamps.py --ws tools/_diag/libqvit_hip_$v.so --shapes fc1 --iters 10 > $O/ws_$v.log 2>&1 || { echo "stamps $v failed"; tail -20 $O/ws_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/ws_$v.log
done
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
grep -oE "(TCC|TCP|TA|TD)_[A-Z0-9_]+" $O/counters.txt | sort -u > $O/counters_short.txt
for lib in base g2p2n; do
  i=0
  for grp in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM" \
             "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
             "TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc_${lib}_$i -o p -- python tools/gemm_bench.py --iters 5 --shapes fc1 --lib tools/_diag/libqvit_hip_$lib.so > $O/pmc_${lib}_$i.log 2>&1
    echo "pmc $lib pass $i rc=$?"
  done
  python tools/pmc_kernel.py 'gemm' $O/pmc_${lib}_* > $O/pmc_${lib}.txt 2>&1; cat $O/pmc_${lib}.txt
done
