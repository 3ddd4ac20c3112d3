# Round 6 n: probe of a captured HIP graph for the ViT-B b256 forward (tools/experiments/graph_probe.py).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06n
timeout -k 10 300 python -u tools/experiments/graph_probe.py > gpurun_out/r06n/probe.log 2>&1; rc=$?
tail -8 gpurun_out/r06n/probe.log; exit $rc
