"""bench.py's real N-rank branch (bench.py main: process-group init, rank-0 build + barrier, the sharded ViT-B
forward, the logits all-gather, the MAX-over-ranks timing, one JSON line) executed on a one-GPU box
(VERDICT r02 #5): QVIT_BENCH_ONE_DEVICE=1 maps every rank to cuda:0 and uses gloo (RCCL needs one GPU per
rank), staging the logits through the host only for gloo. The 8-GPU node then exercises RCCL itself first.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_one_device(dev):
    env = dict(os.environ, QVIT_BENCH_ONE_DEVICE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "QVIT_BENCH_DRYRUN"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--batch", "8", "--no-cpu-baseline"], capture_output=True, text=True, env=env, cwd=ROOT,
                       timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 only
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["config"]["global_batch"] == 16 and j["config"]["parallelism"] == "dp2"
    assert "rehearsal" in j["config"]
    assert j["gather_check"] is True                  # gathered rows == each rank's own forward
    assert j["value"] > 0 and j["roofline"]["launch_ms"] > 0
