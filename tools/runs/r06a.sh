set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06a/tests.log 2>&1 || { tail -30 gpurun_out/r06a/tests.log; exit 1; }
tail -3 gpurun_out/r06a/tests.log
OUT=gpurun_out/r06a/ab SHAPES=fc1,fc1_9r,fc1_975r,fc2,proj ROUNDS=2 bash tools/lib_ab.sh tools/_diag/libqvit_hip_base.so tools/_diag/libqvit_hip_lane.so
