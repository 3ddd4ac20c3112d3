set -u
O=gpurun_out/${OUTD:-r05z}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
OUT=$O/pmc_model ROUND=r05 bash tools/profile_model_pmc.sh > $O/pmc_model.log 2>&1 || { echo "pmc model failed"; tail -20 $O/pmc_model.log; exit 1; }
tail -8 $O/pmc_model.log
ROUND=r05 OUT=$O/round bash tools/round_profile.sh > $O/round.log 2>&1 || { echo "round profile failed"; tail -20 $O/round.log; exit 1; }
cut -c1-600 $O/round/bench_traffic.json
