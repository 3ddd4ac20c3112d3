#!/bin/bash
# One GPU call of several steps. Each step runs under its own time limit; a step that ends in anything but
# success or ordinary test failures (pytest rc 1) -- a time limit, an abort, a crash, a fault -- ends the call.
# Usage: OUT=gpurun_out/x tools/gpu_round.sh "<step 1 command>" "<step 2 command>" ...
#   each step: "<seconds>|<log name>|<command>"
set -u
OUT=${OUT:-gpurun_out/round}
mkdir -p "$OUT"
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for step in "$@"; do
  secs=${step%%|*}; rest=${step#*|}
  name=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping: $name ended with status $rc"
    exit $rc
  fi
  # a GPU fault inside a test shows up as an ordinary failure (rc 1): stop on its signature too
  if grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|HSA_STATUS_ERROR|GPU Hang|hipErrorLaunchFailure" "$OUT/$name.log"; then
    echo "== stopping: $name hit a GPU fault"
    exit 3
  fi
done
