"""GPU runs of the paths either side of the hot path:

* F3: a GETA-shaped pruned ViT state_dict (different head counts per block, arbitrary MLP widths;
  pruning_compression.py:64-131,217-291) written to disk, loaded tensor-only by
  convert.load_reference_checkpoint (predict.py:43's role), run on the GPU and held to the same parity
  bars as the factory models (teacher-forced blocks + tie-resolved end-to-end logits);
* configs[2]'s batch shard: two ranks (gloo, both on cuda:0 — RCCL needs one GPU per rank) each run the
  REAL quantized ViT on their shard and all-gather the logits through distributed.ShardedInference; the
  gathered logits must equal a single-process forward of the whole batch.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn

from oracle import quant_oracle as O

pytestmark = pytest.mark.gpu


def _pruned_state_dict(seed=9):
    from quantized_vit_amd import vit_model
    from quantized_vit_amd.calibrate import collect_input_absmax, set_activation_quant, synthetic_images
    from quantized_vit_amd.quant_model import model_to_quantize_model
    torch.manual_seed(seed)
    m = vit_model.VisionTransformer(embed_dim=192, depth=3, num_heads=3, num_classes=37)
    for blk, heads, hid in zip(m.blocks, (2, 3, 1), (500, 333, 768)):
        a = blk.attn
        if heads != a.num_heads:
            a.qkv = nn.Linear(192, 3 * heads * 64)
            a.proj = nn.Linear(heads * 64, 192)
            a.num_heads = heads
        if hid != blk.mlp.fc1.out_features:
            blk.mlp.fc1 = nn.Linear(192, hid)
            blk.mlp.fc2 = nn.Linear(hid, 192)
    m.apply(vit_model._init_vit_weights)
    m.eval()
    absmax = collect_input_absmax(m, synthetic_images(2, 224, seed=1))
    m = model_to_quantize_model(m, num_bits=4, quant_type="symmetric+nonlinear", quant_mode="weight_and_activation")
    set_activation_quant(m, absmax)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def test_converted_pruned_checkpoint_on_gpu(dev, tmp_path):
    from quantized_vit_amd import convert
    from quantized_vit_amd.calibrate import synthetic_images
    from test_gpu_model import check_vit_parity
    sd = _pruned_state_dict()
    path = os.path.join(tmp_path, "pruned_vit_sd.pt")
    torch.save(sd, path)
    model = convert.load_reference_checkpoint(path, device=dev)
    heads = [b.attn.num_heads for b in model.blocks]
    hidden = [b.mlp.fc1.out_features for b in model.blocks]
    assert heads == [2, 3, 1] and hidden == [500, 333, 768]
    img = synthetic_images(3, 224, seed=4)
    cfg = O.ViTConfig(embed_dim=192, depth=3, num_heads=3, num_classes=37)
    check_vit_parity(model, cfg, img, dev)
    # precomputed weight codes through the converter bind exactly
    from parity_tools import oracle_weight_codes
    codes = {f"{n}.weight_codes": oracle_weight_codes(sd, n, cfg.quant_type, cfg.quant_mode)
             for n in ("blocks.0.attn.qkv", "blocks.2.mlp.fc2")}
    assert convert.load_weight_codes(model, codes) == 2
    assert torch.equal(model.blocks[0].attn.qkv.weight_codes().cpu(), codes["blocks.0.attn.qkv.weight_codes"].float())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dist_worker(rank, world, port, global_batch, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quantized_vit_amd import _lib
        from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images
        from quantized_vit_amd.distributed import ShardedInference
        _lib.load()
        dev = torch.device("cuda:0")
        model = build_quantized_vit("vit_tiny_patch16_224", seed=3, depth=3).to(dev)
        images = synthetic_images(global_batch, 224, seed=6)
        with torch.no_grad():
            out = ShardedInference(lambda x: model(x.to(dev)).cpu())(images)
            whole = model(images.to(dev)).cpu()
        q.put((rank, tuple(out.shape), ((out - whole).abs().max() / whole.abs().max()).item()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("global_batch", [6, 5])
def test_sharded_quantized_vit_two_ranks(dev, global_batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, global_batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    res = [q.get(timeout=10) for _ in range(2)]
    for rank, shape, err in res:
        assert shape == (global_batch, 1000), (rank, shape)
        # per-image work is independent of the batch it runs in; the head's library GEMM may pick another
        # kernel for another M, so allow fp32 rounding
        assert err <= 1e-5, (rank, err)


def test_rccl_world1_all_gather_on_device(dev):
    """RCCL itself (backend "nccl") on one rank: librccl loads, the communicator initialises on the device, and
    all_gather_into_tensor moves device buffers, the collective distributed.gather_logits issues on the 8-GPU node
    (configs[2]). The ragged-shard padding path of gather_logits is checked with a world-1 group as well."""
    import torch.distributed as dist
    from quantized_vit_amd import distributed as qd
    assert not dist.is_initialized()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device(dev))
    try:
        assert dist.get_backend() == "nccl"
        x = torch.randn(256, 1000, device=dev)
        out = torch.empty_like(x)
        dist.all_gather_into_tensor(out, x)
        torch.cuda.synchronize()
        assert torch.equal(out, x)
        # a world-1 group through the module's collective path (world == 1 short-circuits the gather)
        assert torch.equal(qd.gather_logits(x, 256), x)
        y = torch.randn(5, 10, device=dev)
        big = torch.empty(5, 10, device=dev)
        dist.all_gather_into_tensor(big, y.contiguous())
        torch.cuda.synchronize()
        assert torch.equal(big, y)
    finally:
        dist.destroy_process_group()
