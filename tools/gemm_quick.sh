#!/bin/bash
# GEMM parity tests + microbenchmark on the GPU box (one call, stops at the first failure).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider -k "gemm" \
  > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
timeout -k 10 180 python tools/gemm_bench.py --iters 20 --json gpurun_out/gemm_bench.json 2>&1 | grep -v amdgpu.ids
