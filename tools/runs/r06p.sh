# Round 6 p: UltraNet conv0 with the BN sign folded into the weights (a decreasing channel's B column negated, so
# every lane max-pools: no min pool, no select) vs the previous build: UltraNet tests on the product, then A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ultranet.py tests/test_gpu_ultra_modules.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
OUT=$O/uab ROUNDS=3 bash tools/ultra_ab.sh tools/_diag/libqvit_hip_base.so quantized_vit_amd/libqvit_hip.so || exit 1
