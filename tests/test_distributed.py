"""The N>1 path (batch shard + logits all-gather) with world_size 2 on the CPU (gloo)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from quantized_vit_amd.distributed import ShardedInference, gather_logits, shard_bounds


def test_shard_bounds_cover_batch():
    for gb in (1, 7, 256, 2048, 2049):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(gb, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == gb
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, global_batch, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        images = torch.randn(global_batch, 3, 8, 8)
        w = torch.randn(3 * 8 * 8, 10)

        def model(x):   # stand-in for the GPU model: per-image logits
            return x.flatten(1) @ w + rank * 0.0

        out = ShardedInference(model)(images)
        ref = images.flatten(1) @ w
        q.put((rank, torch.allclose(out, ref, atol=1e-5), tuple(out.shape)))
        # direct gather with ragged shards
        s, e = shard_bounds(global_batch, world, rank)
        g = gather_logits(torch.full((e - s, 4), float(rank)), global_batch)
        expect = torch.cat([torch.full((shard_bounds(global_batch, world, r)[1] - shard_bounds(global_batch, world, r)[0], 4),
                                       float(r)) for r in range(world)])
        q.put((rank, torch.equal(g, expect), tuple(g.shape)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("global_batch", [8, 7])
def test_sharded_inference_gloo_world2(global_batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, global_batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = [q.get(timeout=10) for _ in range(4)]
    assert all(ok for _, ok, _ in res), res
    assert all(shape[0] == global_batch for _, _, shape in res)
