set -u
O=gpurun_out/${OUTD:-r05final3}; mkdir -p $O; export TMPDIR=/tmp
(while sleep 50; do date >> $O/heartbeat.txt; done) & HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
OUT=$O/pmc_model ROUND=r05 bash tools/profile_model_pmc.sh > $O/pmc_model.log 2>&1 || { echo "pmc model failed"; tail -20 $O/pmc_model.log; exit 1; }
tail -6 $O/pmc_model.log
cp $O/pmc_model/pmc_mfma.json $O/pmc_model/pmc_mfma_r05.json profiles/
ROUND=r05 OUT=$O/round bash tools/round_profile.sh > $O/round.log 2>&1 || { echo "round profile failed"; tail -20 $O/round.log; exit 1; }
cut -c1-400 $O/round/bench_traffic.json
timeout -k 10 900 python bench.py --model vit_large_patch16_384 --batch 128 > $O/vitl.log 2>&1 || { echo "vitl bench failed"; tail -20 $O/vitl.log; exit 1; }
grep '^{' $O/vitl.log > $O/vitl.json; cut -c1-300 $O/vitl.json
