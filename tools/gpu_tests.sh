#!/bin/bash
# GPU tests only, one pytest process, each test under a thread timeout; stops on a crash.
# Usage: OUT=gpurun_out/x tools/gpu_tests.sh [pytest args...]
set -u
OUT=${OUT:-gpurun_out/tests}
mkdir -p "$OUT"
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest -m gpu -v -rf -p no:cacheprovider --timeout ${TEST_TIMEOUT:-300} \
    --timeout-method thread --durations=15 "$@" > "$OUT/pytest.log" 2>&1
rc=$?
tail -n 40 "$OUT/pytest.log"
exit $rc
