"""Headline benchmark: images/sec of the ViT-B/16 int4-weight / int8-activation forward at batch 256
per GPU (BASELINE.json configs[1]; N > 1 = configs[2], batch-sharded with an RCCL all-gather of logits).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 256] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment starts the N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU) and exits with its code.
Under a launcher, WORLD_SIZE must equal --gpus.

A step = one forward of the quantized ViT-B/16 over this rank's batch of synthetic 224x224 images
already resident in HBM, plus the logits all-gather when N > 1 (distributed.ShardedInference).
Rank 0 prints ONE JSON line; `value` = all ranks' images / the max over ranks of the timed region.

roofline: the dominant GEMM, fc1 (W4A8 contraction with the fused GELU + fc2 activation-quantizer
epilogue). achieved = 2*M*N*K int8 ops per launch / its mean duration measured with HIP events
around every fc1 launch inside the timed region (events on the launch stream); peak = gfx950 dense
int8 MFMA rate; traffic = HBM bytes per launch from rocprofv3 PMC counters (profiles/fc1_traffic.json,
written by tools/profile_fc1.sh) or null. `kernels` gives the same event timing for every hot kernel
of the block (fused qkv+attention, proj, fc2, LayerNorm) with its algorithmic work, taken in a second,
untimed pass of the same steps (so the timed region carries only fc1's events); `model_frac` is the
whole forward's int8 GEMM ops / ms_per_step / peak. `parity` (N = 1, after timing, parity_report): on the
seed-12345 b2 images, the untied distance to the oracle split into weight-code and activation-code sources, and
the tie-resolved check (every quantizer boundary against the oracle's, oracle/ties.py) whose `pass` is the
tests' criterion.
cpu_baseline: the CPU oracle's fp32 fake-quant forward (the reference's op sequence restated,
oracle/quant_oracle.py) on a bounded sample of the same workload, rank 0 only, N = 1 only, with as
many intra-op threads as this process may run on (affinity, capped by a cgroup CPU quota).

QVIT_BENCH_DRYRUN=1 (tests only): gloo on the CPU, a stand-in per-image model instead of the ViT, so
the launcher / sharding / timing / JSON plumbing is testable without a GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from quantized_vit_amd.distributed import ShardedInference  # noqa: E402

METRIC = "images/sec ViT-B/16 int4 @224 batch 256; % int8-MFMA roofline"


def metric_for(model: str, img_size: int, batch: int) -> str:
    """BASELINE.json's metric for the headline workload; the same metric named for the workload actually run
    otherwise (e.g. configs[3], ViT-L/16 @384 b128), so a non-headline line never carries the headline name."""
    if (model, img_size, batch) == ("vit_base_patch16_224", 224, 256):
        return METRIC
    return f"images/sec {model} int4 @{img_size} batch {batch}; % int8-MFMA roofline"
# gfx950 dense int8 MFMA: 256 CU x 4 SIMD x (16*16*64*2 ops / 16 clk) x 2.4 GHz
INT8_PEAK_TOPS = 256 * 4 * 2048 * 2.4e9 / 1e12
# dense fp16 MFMA (v_mfma_f32_16x16x32_f16): half the int8 rate
FP16_PEAK_TFLOPS = INT8_PEAK_TOPS / 2
HBM_PEAK_GBS = 8000.0
DRYRUN = os.environ.get("QVIT_BENCH_DRYRUN") == "1"
ONE_DEVICE = os.environ.get("QVIT_BENCH_ONE_DEVICE") == "1"


def _step_marker() -> None:
    """With QVIT_STEP_MARKERS=1 (profiling runs only): one tiny torch spin kernel just before and just after the
    timed steps, OUTSIDE the timed region, so tools/kstats.py --split can tell the timed steps' dispatches in a
    rocprofv3 kernel trace from setup, calibration, event-timed and parity launches."""
    if os.environ.get("QVIT_STEP_MARKERS") == "1":
        torch.cuda._sleep(64)
        torch.cuda.synchronize()


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--model", default="vit_base_patch16_224")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=8, help="CPU baseline sample (images)")
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--lib", default="", help=argparse.SUPPRESS)  # diagnostic: A/B another build of the library
    return ap.parse_args(argv)


def _wreg() -> str:
    """The weight image the int path's W4 GEMMs run on (quant_layers.GEMM_WREG), and the two-ahead activation ring
    the register-weight GEMMs take at K >= 256: ", W4R, L2>", ", W8R, L2>" or ">"."""
    from quantized_vit_amd import quant_layers
    return {"w4r": ", W4R, L2>", "w8r": ", W8R, L2>"}.get(quant_layers.GEMM_WREG, ">")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args, argv) -> int:
    """Starts `args.gpus` ranks of this script under torch.distributed.run (one process per GPU) as a
    child process and returns its exit code. Called before any GPU call in this process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def usable_cores() -> dict:
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2/v1 CPU quota."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0:
                quota = max(1, q // p)
        except (OSError, ValueError):
            pass
    use = min(aff, quota) if quota else aff
    return {"threads": use, "affinity": aff, "cgroup_quota": quota, "cpu_count": os.cpu_count()}


def cpu_model_name() -> str:
    name = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return name


def cpu_baseline(model, model_name: str, x_gpu_logits_fn, img_size: int, batch: int, iters: int):
    """Times the oracle's fp32 fake-quant forward on the host cores (bounded sample) and checks the
    GPU logits on the same images against it."""
    from oracle import quant_oracle as O
    from quantized_vit_amd.calibrate import VIT_CONFIGS, synthetic_images
    mc = VIT_CONFIGS[model_name]
    cfg = O.ViTConfig(img_size=mc["img_size"], patch_size=mc["patch_size"], embed_dim=mc["embed_dim"],
                      depth=mc["depth"], num_heads=mc["num_heads"])
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    img = synthetic_images(batch, img_size, seed=12345)
    cores = usable_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores["threads"])
    try:
        with torch.no_grad():
            ref = O.vit_forward(sd, cfg, img)  # warm-up (also the parity reference)
            times = []
            for _ in range(iters):
                t0 = time.perf_counter()
                O.vit_forward(sd, cfg, img)
                times.append(time.perf_counter() - t0)
            gpu = x_gpu_logits_fn(img)
            # the same fp32 oracle against itself in fp64: quantizer rounding ties resolve differently
            # and the flips compound over the blocks, so this is the floor any fp32 implementation sits at
            ref64 = O.vit_forward({k: v.double() for k, v in sd.items()}, cfg, img.double())
        used = torch.get_num_threads()
    finally:
        torch.set_num_threads(prev)
    times.sort()
    med = times[len(times) // 2]
    rel = ((gpu.double().cpu() - ref.double()).norm() / ref.double().norm()).item()
    floor = ((ref.double() - ref64).norm() / ref64.norm()).item()
    return {
        "value": batch / med, "unit": "img/s", "cores": used, "kind": "port",
        "sample": f"oracle fp32 fake-quant {model_name} forward, batch {batch}, median of {iters} after 1 warm-up "
                  f"({cpu_model_name()}; {used} intra-op threads = affinity {cores['affinity']}"
                  f"{', cgroup quota ' + str(cores['cgroup_quota']) if cores['cgroup_quota'] else ''}"
                  f", os.cpu_count() {cores['cpu_count']})",
    }, rel, floor


PARITY_SEED = 12345   # the bench's parity images (tests/test_gpu_bench_parity.py checks the same ones)
PARITY_BATCH = 2


def parity_report(model, model_name: str, img_size: int, dev) -> dict:
    """After the timed region, on the bench's own b2 parity images (seed 12345):

    * `untied`: the logits' distance to the oracle with nothing shared, split by source:
      `rel_device_weights` (the timed configuration: the device's own weight codes), `weight_code_flips` (device
      weight codes that differ from the oracle's, and how many of those the correctly rounded quantizer
      explains, oracle/ties.py:cr_codes), `rel_oracle_weights` (the oracle's weight codes bound: what remains is
      the activation codes' contribution), `floor_fp32_vs_fp64` (the oracle against itself in fp64), and
      `default_gelu`: the same distances to the oracle run with torch's default (oneDNN) GELU instead of the pinned
      ATen kernel — what a default-configured reference would see (reported; not a criterion).
    * `tie_resolved`: with the oracle's weight codes bound, every quantizer boundary of the GPU forward against
      the oracle's (oracle/ties.py). A differing code must be a proven rounding tie, and no layer may flip more
      than the tests' 1e-4 budget of its codes; with ties resolved alike `rel` is the logits' distance. `pass`
      is exactly the tests' criterion (tests/test_gpu_bench_parity.py)."""
    from oracle import quant_oracle as O
    from oracle.ties import cr_codes, load_oracle_weight_codes, oracle_weight_codes, tie_resolved_vit_check
    from quantized_vit_amd.calibrate import VIT_CONFIGS, synthetic_images
    from quantized_vit_amd.quant_layers import QuantizeMixin
    mc = VIT_CONFIGS[model_name]
    cfg = O.ViTConfig(img_size=mc["img_size"], patch_size=mc["patch_size"], embed_dim=mc["embed_dim"],
                      depth=mc["depth"], num_heads=mc["num_heads"])
    img = synthetic_images(PARITY_BATCH, img_size, seed=PARITY_SEED)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}

    def rel(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm()).item()
    with torch.no_grad():
        ref = O.vit_forward(sd, cfg, img)
        ref64 = O.vit_forward({k: v.double() for k, v in sd.items()}, cfg, img.double())
        y_dev = model(img.to(dev)).cpu()
        wflips, wcr, wtot, wlayers = 0, 0, 0, {}
        for name, m in model.named_modules():
            if not isinstance(m, QuantizeMixin):
                continue
            q = O.LayerQ.from_state(sd, name + ".", cfg.quant_type, cfg.quant_mode)
            own = oracle_weight_codes(sd, name, cfg.quant_type, cfg.quant_mode).float()
            got = m.weight_codes().cpu().reshape(own.shape)
            diff = got != own
            n = int(diff.sum())
            wtot += own.numel()
            if n:
                w = sd[name + ".weight"].reshape(own.shape)[diff]
                c = int((cr_codes(w, cfg.quant_type, q.d_wt, q.q_m_wt, q.t_wt) == got[diff]).sum())
                wflips, wcr = wflips + n, wcr + c
                wlayers[name] = {"flips": n, "cr_explained": c}
        load_oracle_weight_codes(model, cfg)
        y_ow = model(img.to(dev)).cpu()
        with O.torch_default_gelu():
            ref_def = O.vit_forward(sd, cfg, img)
    untied = {"rel_device_weights": rel(y_dev, ref), "rel_oracle_weights": rel(y_ow, ref),
              "floor_fp32_vs_fp64": rel(ref, ref64),
              # reported, not a criterion: against a reference run in torch's default configuration (oneDNN GELU)
              "default_gelu": {"rel_device_weights": rel(y_dev, ref_def), "rel_oracle_weights": rel(y_ow, ref_def),
                               "oracle_pinned_vs_default": rel(ref, ref_def)},
              "weight_code_flips": {"flips": wflips, "cr_explained": wcr, "codes": wtot, "layers": wlayers}}
    r = tie_resolved_vit_check(model, cfg, img, dev)
    non_ties = sum(s.get("non_ties", 0) for s in r["stats"].values())
    missing = list(r["missing"])
    over = {p: {"flips": s["flips"], "total": s["total"], "cr_explained": s.get("cr_explained", 0),
                "max_tie_dist_code_units": s["max_dist"]} for p, s in r["bad"].items()}
    flipped = {p: {"flips": s["flips"], "cr_explained": s.get("cr_explained", 0)}
               for p, s in r["stats"].items() if s.get("flips", 0)}
    tied = {"rel": r["rel"], "tie_flips": r["flips"], "cr_explained": r["cr_explained"], "codes": r["codes"],
            "non_tie_differences": non_ties, "missing_layers": missing, "layers_over_budget": over,
            "flips_by_layer": flipped,
            "pass": bool(not missing and not r["bad"] and non_ties == 0 and r["rel"] <= 1e-3),
            "bound": "north star 1e-3 on identical int4 weights; every flip a proven tie; <= 1e-4 flips per layer"}
    return {"batch": PARITY_BATCH, "seed": PARITY_SEED, "untied": untied, "tie_resolved": tied,
            "weights": "device-derived weight codes in the timed steps; the oracle's bound after them"}


def model_gemm_ops(model, B: int) -> float:
    """Sum of 2*M*N*K over the forward's quantized GEMMs (patch embed, 4 per block, head)."""
    pe = model.patch_embed
    P = pe.num_patches
    T = P + model.num_tokens
    k_pe = pe.proj.in_channels * pe.proj.kernel_size[0] * pe.proj.kernel_size[1]
    ops = 2.0 * B * P * pe.proj.out_channels * k_pe
    for blk in model.blocks:
        for lin in (blk.attn.qkv, blk.attn.proj, blk.mlp.fc1, blk.mlp.fc2):
            ops += 2.0 * B * T * lin.out_features * lin.in_features
    if hasattr(model.head, "in_features"):
        ops += 2.0 * B * model.head.out_features * model.head.in_features
    return ops


def kernel_work(model, B: int) -> dict:
    """Algorithmic work of one launch of each timed kernel."""
    blk = model.blocks[0]
    T = model.patch_embed.num_patches + model.num_tokens
    M = B * T
    C = blk.attn.qkv.in_features
    H = blk.attn.num_heads
    hid = blk.mlp.fc1.out_features

    def gemm(lin):
        return 2.0 * M * lin.out_features * lin.in_features
    attn_flops = 4.0 * B * H * T * T * 64    # S = q k^T and O = P v, 2 flops per MAC
    return {
        "fc1": {"int8_ops": gemm(blk.mlp.fc1), "bytes": M * C + hid * C / 2 + M * hid},
        "fc2": {"int8_ops": gemm(blk.mlp.fc2), "bytes": M * hid + C * hid / 2 + 2 * 4 * M * C},
        "proj": {"int8_ops": gemm(blk.attn.proj), "bytes": M * C + C * C / 2 + 2 * 4 * M * C},
        "qkv_attn": {"int8_ops": gemm(blk.attn.qkv), "fp32_attn_flops": attn_flops, "bytes": M * C + 3 * C * C / 2 + M * C},
        "ln": {"bytes": 4 * M * C + M * C},
    }


def load_profile_json(name: str, model_name: str, B: int):
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            j = json.load(f)
    except (OSError, ValueError):
        return None
    if j.get("batch") != B or j.get("model") != model_name:
        return None
    # counters measured on another build of the library are not this line's numbers
    from quantized_vit_amd import _lib
    if j.get("lib_build_id") is None or j.get("lib_build_id") != _lib.build_id():
        return None
    return j


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
                         f"--nproc-per-node equal to --gpus (or without a launcher: python bench.py --gpus N)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if DRYRUN:
        return dryrun_main(args, world, rank)

    from quantized_vit_amd import _lib, build as qbuild, vit_model
    from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images
    # QVIT_BENCH_ONE_DEVICE=1 (tests/test_gpu_bench_ranks.py): every rank on cuda:0 and the gloo backend
    # (RCCL needs one GPU per rank), so this N-rank branch runs end to end on a one-GPU box; the logits are
    # staged through the host only for gloo (distributed.gather_logits)
    one_device = ONE_DEVICE and world > 1
    backend = "gloo" if one_device else "nccl"
    if world > 1:
        dist.init_process_group(backend, init_method="env://")
    if one_device:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if rank == 0:
        qbuild.build()
    if world > 1:
        dist.barrier()
    _lib.load(args.lib) if args.lib else _lib.load()

    if args.model == "ultranet":
        return ultranet_main(args, world, rank, dev, backend, one_device)
    img_size = {"vit_base_patch16_224": 224, "vit_large_patch16_384": 384, "vit_tiny_patch16_224": 224}[args.model]
    model = build_quantized_vit(args.model, seed=args.seed, device=dev)
    B = args.batch
    x = synthetic_images(B, img_size, seed=1000 + rank, device=dev)   # this rank's shard, made on-device
    sharded = ShardedInference(model)
    global_batch = world * B

    def step():
        return sharded.forward_shard(x, global_batch)

    names = ("fc1", "fc2", "proj", "qkv_attn", "ln")
    with torch.no_grad():
        for _ in range(args.warmup):
            out = step()
        torch.cuda.synchronize()
        assert out.shape == (global_batch, model.head.out_features), out.shape
        # timed region: only the roofline kernel (fc1) carries HIP events
        vit_model.KERNEL_TIMING["fc1"] = []
        _step_marker()
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
        _step_marker()
        events = {"fc1": vit_model.KERNEL_TIMING.pop("fc1")}
        # the other hot kernels: the same steps again with events around each of their launches (untimed)
        for n in names[1:]:
            vit_model.KERNEL_TIMING[n] = []
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        for n in names[1:]:
            events[n] = vit_model.KERNEL_TIMING.pop(n)
        gather_ok = None
        if world > 1:   # untimed: the gathered rows of this rank are exactly its own forward
            from quantized_vit_amd.distributed import shard_bounds
            s, e = shard_bounds(global_batch, world, rank)
            ok = torch.tensor([1 if torch.equal(step()[s:e], model(x)) else 0], dtype=torch.int32,
                              device="cpu" if backend == "gloo" else dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            gather_ok = bool(ok.item())
    launch_ms = {n: (sum(s.elapsed_time(e) for s, e in ev) / len(ev)) if ev else None for n, ev in events.items()}

    t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if backend == "gloo" else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3

    work = kernel_work(model, B)
    fc1_ms = launch_ms["fc1"]
    ops = work["fc1"]["int8_ops"]
    achieved = ops / (fc1_ms * 1e-3) / 1e12
    tj = load_profile_json("fc1_traffic.json", args.model, B)
    traffic = tj.get("traffic_bytes_per_launch") if tj else None
    pmc = load_profile_json("pmc_mfma.json", args.model, B)

    kernels = {}
    for n in names:
        ms = launch_ms[n]
        if ms is None:
            continue
        w = work[n]
        k = {"launch_us": ms * 1e3, "launches_per_step": len(events[n]) / args.steps,
             "hbm_GBs_algorithmic": w["bytes"] / (ms * 1e-3) / 1e9}
        if "int8_ops" in w:
            k["int8_TOPS"] = w["int8_ops"] / (ms * 1e-3) / 1e12
            k["frac_int8_peak"] = k["int8_TOPS"] / INT8_PEAK_TOPS
        if "fp32_attn_flops" in w:
            # bound of the fused kernel: its int8 projection at the int8 peak plus the attention's
            # fp32-equivalent flops as 3 fp16 MFMA passes (hi*hi + hi*lo + lo*hi) at the fp16 peak
            bound_s = w["int8_ops"] / (INT8_PEAK_TOPS * 1e12) + 3 * w["fp32_attn_flops"] / (FP16_PEAK_TFLOPS * 1e12)
            k["frac_of_mfma_bound"] = bound_s / (ms * 1e-3)
        if n == "ln":
            k["frac_hbm_peak"] = k["hbm_GBs_algorithmic"] / HBM_PEAK_GBS
        if pmc and n in pmc.get("kernels", {}):
            k["pmc"] = pmc["kernels"][n]
            tb = k["pmc"].get("traffic_bytes")
            if tb:   # HBM bytes per launch (PMC) over the algorithmic bytes: re-reads show up as > 1
                k["traffic_over_algorithmic"] = tb / w["bytes"]
        kernels[n] = k
    total_ops = model_gemm_ops(model, B)

    result = {
        "metric": metric_for(args.model, img_size, B),
        "value": global_batch * args.steps / elapsed,
        "unit": "img/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": f"synthetic uniform[-1,1) {img_size}x{img_size} images; random-init {args.model} (reference init), "
                "W4 (nonlinear quantizer, t=1) / A8 calibrated",
        "config": {"workload": f"{args.model} int4w/int8a forward, batch {B} per GPU"
                               + (", RCCL all-gather of logits" if world > 1 else ""),
                   "model": args.model, "global_batch": global_batch, "seq_len": model.patch_embed.num_patches + 1,
                   "parallelism": f"dp{world}"}
                  | ({"rehearsal": f"{world} ranks on one device, gloo, logits gathered through the host "
                                   "(QVIT_BENCH_ONE_DEVICE=1; not a scaling measurement)"} if one_device else {}),
        "roofline": {"bound": "mfma", "kernel": "fc1 gemm_kernel<W4, EPI_I8_GELU" + _wreg(),
                     "achieved": achieved, "peak": INT8_PEAK_TOPS, "unit": "TFLOP/s",
                     "frac": achieved / INT8_PEAK_TOPS, "traffic": traffic,
                     "ops_per_launch": ops, "launch_ms": fc1_ms,
                     "mfma_util": (pmc or {}).get("kernels", {}).get("fc1", {}).get("mfma_busy_frac"),
                     "note": "int8 ops (TOPS) counted as 2*M*N*K; mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / "
                             "(GRBM_GUI_ACTIVE x CUs) from profiles/pmc_mfma.json; traffic from "
                             "profiles/fc1_traffic.json; both only when measured on this library build "
                             "(lib_build_id), else null",
                     "lib_build_id": _lib.build_id()},
        "model_frac": {"int8_ops_per_step": total_ops, "achieved_TOPS": total_ops / (ms_per_step * 1e-3) / 1e12,
                       "frac": total_ops / (ms_per_step * 1e-3) / 1e12 / INT8_PEAK_TOPS},
        "kernels": kernels,
    }
    if gather_ok is not None:
        result["gather_check"] = gather_ok
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        def gpu_logits(img):
            return model(img.to(dev)).cpu()
        cb, rel, floor = cpu_baseline(model, args.model, gpu_logits, img_size, args.cpu_batch, args.cpu_iters)
        result["cpu_baseline"] = cb
        result["parity_rel_err_vs_oracle"] = rel
        result["parity_oracle_fp32_vs_fp64"] = floor
        result["parity"] = parity_report(model, args.model, img_size, dev)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


ULTRA_LAYERS = [  # (name, cin, cout, input size divisor, pooled): mymodel.py:71-124 at 416 x 416
    ("ultra_conv0", 3, 16, 1, True), ("ultra_conv1", 16, 32, 2, True), ("ultra_conv2", 32, 64, 4, True),
    ("ultra_conv3", 64, 64, 8, True), ("ultra_conv4", 64, 64, 16, False), ("ultra_conv5", 64, 64, 16, False),
    ("ultra_conv6", 64, 64, 16, False), ("ultra_conv7", 64, 64, 16, False)]


def ultranet_work(size: int = 416) -> dict:
    """Algorithmic work per image of each UltraNet launch: conv ops 2 H W cout cin 9; bytes =
    input read once (fp32 image for layer 0, int8 codes after) + output codes written once (pooled)."""
    work = {}
    for name, cin, cout, div, pool in ULTRA_LAYERS:
        hw = (size // div) ** 2
        out_hw = hw // 4 if pool else hw
        in_b = hw * cin * (4 if name == "ultra_conv0" else 1)
        work[name] = {"ops": 2.0 * hw * cout * cin * 9, "bytes": in_b + out_hw * cout}
    g = (size // 16) ** 2
    work["ultra_head"] = {"ops": 2.0 * g * 36 * 64, "bytes": g * 64 + g * 36 * 4}
    work["ultra_decode"] = {"ops": 0.0, "bytes": g * 36 * 4 + 2 * g * 36 * 4}   # head in, io and p out
    # qvit_ultra_tail (layers.16-28 + the YOLO decode in one launch, maps in LDS): layer 4's codes in, io and p out
    work["ultra_tail"] = {"ops": sum(work[f"ultra_conv{k}"]["ops"] for k in range(4, 8)) + work["ultra_head"]["ops"],
                          "bytes": g * 64 + 2 * g * 36 * 4}
    return work


def ultranet_main(args, world: int, rank: int, dev, backend: str, one_device: bool) -> None:
    """BASELINE.json configs[4]: the UltraNetQua W4A4 forward (4-bit quantization/mymodel.py:62-144) at 416 x 416
    on synthetic k/255 images, batch-sharded like the ViT. roofline: the dominant launch, layer 0 (float image
    -> conv3x3 + BN + A4 quantizer + max pool -> codes), against HBM (UltraNet is HBM-bound)."""
    from quantized_vit_amd import _lib, vit_model
    from quantized_vit_amd.ultranet import random_ultranet, synthetic_images_u8
    size = 416
    model = random_ultranet(seed=args.seed, device=dev)
    B = args.batch
    x = synthetic_images_u8(B, size, seed=1000 + rank, device=dev)
    assert model.fused_ok(x)
    sharded = ShardedInference(lambda im: model(im)[0].flatten(1))
    global_batch = world * B
    names = [n for n, *_ in ULTRA_LAYERS] + ["ultra_head", "ultra_tail", "ultra_decode"]
    with torch.no_grad():
        for _ in range(args.warmup):
            out = sharded.forward_shard(x, global_batch)
        torch.cuda.synchronize()
        assert out.shape[0] == global_batch, out.shape
        vit_model.KERNEL_TIMING["ultra_conv0"] = []
        _step_marker()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            sharded.forward_shard(x, global_batch)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        _step_marker()
        events = {"ultra_conv0": vit_model.KERNEL_TIMING.pop("ultra_conv0")}
        for n in names[1:]:
            vit_model.KERNEL_TIMING[n] = []
        for _ in range(args.steps):
            sharded.forward_shard(x, global_batch)
        torch.cuda.synchronize()
        for n in names[1:]:
            events[n] = vit_model.KERNEL_TIMING.pop(n)
    launch_ms = {n: sum(s.elapsed_time(e) for s, e in ev) / len(ev) for n, ev in events.items() if ev}
    t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if backend == "gloo" else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    work = ultranet_work(size)
    kernels = {}
    for n, ms in launch_ms.items():
        w = work[n]
        kernels[n] = {"launch_us": ms * 1e3, "hbm_GBs_algorithmic": w["bytes"] * B / (ms * 1e-3) / 1e9,
                      "int8_TOPS": w["ops"] * B / (ms * 1e-3) / 1e12}
    k0 = kernels["ultra_conv0"]
    # the launches that actually ran: with qvit_ultra_tail the layers 4..7, the head and the decode are
    # one launch moving the tail's own bytes (layer 4's codes in, io and p out), not the per-layer sum
    if "ultra_tail" in launch_ms:
        per_layer = [n for n, *_ in ULTRA_LAYERS[:4]] + ["ultra_tail"]
    else:
        per_layer = [n for n, *_ in ULTRA_LAYERS] + ["ultra_head", "ultra_decode"]
    img_bytes = sum(work[n]["bytes"] for n in per_layer)
    img_ops = sum(work[n]["ops"] for n in per_layer)
    value = global_batch * args.steps / elapsed
    result = {
        "metric": f"images/sec UltraNet int4 @{size} batch {B}; % HBM roofline",
        "value": value, "unit": "img/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int8",
        "data": f"synthetic k/255 {size}x{size} images; random-init UltraNetQua (BN statistics calibrated on its own "
                "outputs), W4 weights / A4 activations, fused HIP forward",
        "config": {"workload": f"UltraNetQua W4A4 forward @{size}, batch {B} per GPU"
                               + (", RCCL all-gather of the detections" if world > 1 else ""),
                   "model": "ultranet", "global_batch": global_batch, "img_size": size, "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "kernel": "ultra_conv0 (layer 0: fp32 image in, pooled codes out)",
                     "achieved": k0["hbm_GBs_algorithmic"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": k0["hbm_GBs_algorithmic"] / HBM_PEAK_GBS, "traffic": None,
                     "bytes_per_launch": work["ultra_conv0"]["bytes"] * B, "launch_ms": launch_ms["ultra_conv0"]},
        "model_frac": {"launches": per_layer, "algorithmic_bytes_per_img": img_bytes, "int8_ops_per_img": img_ops,
                       "hbm_GBs": img_bytes * value / world / 1e9,
                       "frac_hbm_peak": img_bytes * value / world / 1e9 / HBM_PEAK_GBS},
        "kernels": kernels,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import ultranet_oracle as U
        sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        img = synthetic_images_u8(args.cpu_batch, size, seed=12345)
        cores = usable_cores()
        prev = torch.get_num_threads()
        torch.set_num_threads(cores["threads"])
        try:
            with torch.no_grad():
                ref, _ = U.ultranet_forward(sd, img)          # warm-up, and the parity reference
                times = []
                for _ in range(args.cpu_iters):
                    t1 = time.perf_counter()
                    U.ultranet_forward(sd, img)
                    times.append(time.perf_counter() - t1)
                gpu = model(img.to(dev))[0].cpu()
            used = torch.get_num_threads()
        finally:
            torch.set_num_threads(prev)
        med = sorted(times)[len(times) // 2]
        result["cpu_baseline"] = {
            "value": img.shape[0] / med, "unit": "img/s", "cores": used, "kind": "port",
            "sample": f"oracle fp32 fake-quant UltraNetQua forward (oracle/ultranet_oracle.py), batch {img.shape[0]}, "
                      f"median of {args.cpu_iters} after 1 warm-up ({cpu_model_name()}; {used} intra-op threads)"}
        result["parity_rel_err_vs_oracle"] = ((gpu.double() - ref.double()).norm() / ref.double().norm()).item()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dryrun_main(args, world: int, rank: int) -> None:
    """QVIT_BENCH_DRYRUN=1: the same launcher / shard / gather / max-over-ranks timing on gloo + CPU with
    a stand-in per-image model (tests/test_bench_launcher.py)."""
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    B = args.batch
    g = torch.Generator().manual_seed(1000 + rank)
    x = torch.rand(B, 3, 8, 8, generator=g)
    w = torch.ones(3 * 8 * 8, 10)
    sharded = ShardedInference(lambda im: im.flatten(1) @ w)
    global_batch = world * B
    for _ in range(args.warmup):
        out = sharded.forward_shard(x, global_batch)
    assert out.shape == (global_batch, 10), out.shape
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sharded.forward_shard(x, global_batch)
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": global_batch * args.steps / elapsed, "unit": "img/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "fp32", "data": "dry run (stand-in model, CPU, gloo)",
                          "config": {"workload": "dry run", "global_batch": global_batch,
                                     "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
