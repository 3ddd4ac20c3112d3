"""bench.py's multi-rank plumbing on the CPU (QVIT_BENCH_DRYRUN=1: gloo, stand-in per-image model).

`python bench.py --gpus N` without a launcher must start N ranks itself and rank 0 must print one
JSON line with n_gpus == N and the global batch N * batch; a launcher whose WORLD_SIZE disagrees
with --gpus is an error (VERDICT r01 Missing #1)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=240):
    env = dict(os.environ, QVIT_BENCH_DRYRUN="1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_gpus_flag_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--steps", "3", "--warmup", "1", "--batch", "4"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    j = json.loads(lines[0])
    assert j["n_gpus"] == n
    assert j["config"]["global_batch"] == 4 * n
    assert j["config"]["parallelism"] == f"dp{n}"
    assert j["steps"] == 3 and j["value"] > 0 and j["scaling"] == "weak"


def test_bench_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"],
             extra_env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in (r.stderr + r.stdout)


def test_metric_names_the_workload_run():
    """The headline workload carries BASELINE.json's metric verbatim; any other workload names itself."""
    import json
    import os
    import bench
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "BASELINE.json")) as f:
        base = json.load(f)
    assert bench.metric_for("vit_base_patch16_224", 224, 256) == bench.METRIC == base["metric"]
    m = bench.metric_for("vit_large_patch16_384", 384, 128)
    assert "vit_large_patch16_384" in m and "batch 128" in m and m != bench.METRIC
