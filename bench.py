"""Headline benchmark: images/sec of the ViT-B/16 int4-weight / int8-activation forward at batch 256
per GPU (BASELINE.json configs[1]; N > 1 = configs[2], batch-sharded with an RCCL all-gather of logits).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 256] [--no-cpu-baseline]
    torchrun --nproc-per-node N bench.py --gpus N ...

A step = one forward of the quantized ViT-B/16 over one batch of synthetic 224x224 images already
resident in HBM (+ the logits all-gather when N > 1). Rank 0 prints ONE JSON line.

roofline: the dominant kernel is the fc1 GEMM (W4A8 contraction with the fused GELU + fc2
activation-quantizer epilogue). achieved = 2*M*N*K int8 ops per launch / its mean duration measured
with HIP events around every fc1 launch inside the timed region (events on the launch stream);
peak = gfx950 dense int8 MFMA rate; traffic = HBM bytes per launch from rocprofv3 PMC counters
(profiles/fc1_traffic.json, written by tools/profile_fc1.sh) or null.
cpu_baseline: the CPU oracle's fp32 fake-quant forward (the reference's op sequence restated,
oracle/quant_oracle.py) on a bounded sample of the same workload, rank 0 only, N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from quantized_vit_amd import _lib, build as qbuild, vit_model  # noqa: E402
from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images  # noqa: E402

METRIC = "images/sec ViT-B/16 int4 @224 batch 256; % int8-MFMA roofline"
# gfx950 dense int8 MFMA: 256 CU x 4 SIMD x (16*16*64*2 ops / 16 clk) x 2.4 GHz
INT8_PEAK_TOPS = 256 * 4 * 2048 * 2.4e9 / 1e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--model", default="vit_base_patch16_224")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=8)
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--lib", default="", help=argparse.SUPPRESS)  # diagnostic: A/B another build of the library
    return ap.parse_args()


def cpu_baseline(model, model_name: str, x_gpu_logits_fn, img_size: int, batch: int, iters: int):
    """Times the oracle's fp32 fake-quant forward on the host cores (bounded sample) and checks the
    GPU logits on the same images against it."""
    from oracle import quant_oracle as O
    from quantized_vit_amd.calibrate import VIT_CONFIGS
    mc = VIT_CONFIGS[model_name]
    cfg = O.ViTConfig(img_size=mc["img_size"], patch_size=mc["patch_size"], embed_dim=mc["embed_dim"],
                      depth=mc["depth"], num_heads=mc["num_heads"])
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    img = synthetic_images(batch, img_size, seed=12345)
    torch.set_num_threads(max(1, torch.get_num_threads()))
    with torch.no_grad():
        ref = O.vit_forward(sd, cfg, img)  # warm-up (also the parity reference)
        times = []
        for _ in range(iters):
            t0 = time.perf_counter()
            O.vit_forward(sd, cfg, img)
            times.append(time.perf_counter() - t0)
        gpu = x_gpu_logits_fn(img)
    times.sort()
    med = times[len(times) // 2]
    rel = ((gpu.double().cpu() - ref.double()).norm() / ref.double().norm()).item()
    # the same fp32 oracle against itself in fp64: quantizer rounding ties resolve differently and the
    # flips compound over the blocks, so this distance is the floor any fp32 implementation sits at
    with torch.no_grad():
        ref64 = O.vit_forward({k: v.double() for k, v in sd.items()}, cfg, img.double())
    floor = ((ref.double() - ref64).norm() / ref64.norm()).item()
    cpu_model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": batch / med, "unit": "img/s", "cores": torch.get_num_threads(), "kind": "port",
        "sample": f"oracle fp32 fake-quant {model_name} forward, batch {batch}, median of {iters} after 1 warm-up "
                  f"({cpu_model})",
    }, rel, floor


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if rank == 0:
        qbuild.build()
    if world > 1:
        dist.barrier()
    _lib.load(args.lib) if args.lib else _lib.load()

    img_size = {"vit_base_patch16_224": 224, "vit_large_patch16_384": 384, "vit_tiny_patch16_224": 224}[args.model]
    model = build_quantized_vit(args.model, seed=args.seed, device=dev)
    B = args.batch
    x = synthetic_images(B, img_size, seed=1000 + rank, device=dev)
    ncls = model.head.out_features
    gathered = torch.empty((world * B, ncls), device=dev) if world > 1 else None

    def step():
        logits = model(x)
        if world > 1:
            dist.all_gather_into_tensor(gathered, logits)
        return logits

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        # fc1 launch timing inside the timed region
        vit_model.KERNEL_TIMING["fc1"] = []
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        ev = vit_model.KERNEL_TIMING.pop("fc1")
    fc1_ms = sum(s.elapsed_time(e) for s, e in ev) / max(1, len(ev))

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    blk = model.blocks[0]
    M = B * (model.patch_embed.num_patches + 1)
    fc1 = blk.mlp.fc1
    ops = 2.0 * M * fc1.out_features * fc1.in_features
    achieved = ops / (fc1_ms * 1e-3) / 1e12
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "fc1_traffic.json")
    if os.path.exists(tpath):
        try:
            with open(tpath) as f:
                tj = json.load(f)
            if tj.get("batch") == B and tj.get("model") == args.model:
                traffic = tj.get("traffic_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    result = {
        "metric": METRIC,
        "value": world * B * args.steps / elapsed,
        "unit": "img/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": f"synthetic uniform[-1,1) {img_size}x{img_size} images; random-init {args.model} (reference init), "
                "W4 (nonlinear quantizer, t=1) / A8 calibrated",
        "config": {"workload": f"{args.model} int4w/int8a forward, batch {B} per GPU"
                               + (", RCCL all-gather of logits" if world > 1 else ""),
                   "model": args.model, "global_batch": world * B, "seq_len": model.patch_embed.num_patches + 1,
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "mfma", "kernel": "fc1 gemm_kernel<W4, EPI_I8_GELU>",
                     "achieved": achieved, "peak": INT8_PEAK_TOPS, "unit": "TFLOP/s",
                     "frac": achieved / INT8_PEAK_TOPS, "traffic": traffic,
                     "ops_per_launch": ops, "launch_ms": fc1_ms,
                     "note": "int8 ops (TOPS) counted as 2*M*N*K"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        def gpu_logits(img):
            return model(img.to(dev)).cpu()
        cb, rel, floor = cpu_baseline(model, args.model, gpu_logits, img_size, args.cpu_batch, args.cpu_iters)
        result["cpu_baseline"] = cb
        result["parity_rel_err_vs_oracle"] = rel
        result["parity_oracle_fp32_vs_fp64"] = floor
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
