set -u
O=gpurun_out/${OUTD:-r05z}; mkdir -p $O; export TMPDIR=/tmp
OUT=$O/pmc_model ROUND=r05 bash tools/profile_model_pmc.sh > $O/pmc_model.log 2>&1 || { echo "pmc model failed"; tail -20 $O/pmc_model.log; exit 1; }
tail -8 $O/pmc_model.log
cp $O/pmc_model/pmc_mfma.json $O/pmc_model/pmc_mfma_r05.json profiles/
ROUND=r05 OUT=$O/round bash tools/round_profile.sh > $O/round.log 2>&1 || { echo "round profile failed"; tail -20 $O/round.log; exit 1; }
cut -c1-600 $O/round/bench_traffic.json
