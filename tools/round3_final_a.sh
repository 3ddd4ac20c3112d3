#!/bin/bash
# Round-3 evidence, part A: the full -m gpu suite, then tools/round_profile.sh (default bench line with the
# CPU baseline, rocprofv3 kernel stats, fc1 PMC traffic, the bench line with traffic). Output: gpurun_out/r03_final2
set -u
OUT=gpurun_out/r03_final2
mkdir -p "$OUT"
export TMPDIR=/tmp
OUT=$OUT/tests TESTS_TIMEOUT=700 TEST_TIMEOUT=120 bash tools/gpu_tests.sh -x -q > /dev/null 2>&1
rc=$?
tail -3 "$OUT/tests/pytest.log"
[ $rc -eq 0 ] || exit $rc
ROUND=r03 OUT=$OUT bash tools/round_profile.sh > "$OUT/round_profile.out" 2>&1
rc=$?
tail -40 "$OUT/round_profile.out"
exit $rc
