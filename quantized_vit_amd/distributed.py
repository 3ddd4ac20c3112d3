"""Batch-sharded inference across the GPUs of one node (BASELINE.json configs[2]).

Images are independent in the reference's eval forward (no BatchNorm in the ViT, LayerNorm is per
token), so the path partitions by image: rank r owns global images [r*b, (r+1)*b) and holds a full
model replica (ViT-B int4 ~ 43 MB). The only exchange is one all-gather of the fp32 logits
(RCCL over xGMI with backend "nccl"; ~1 MB per rank at b=256, C=1000). One process per GPU.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard_bounds(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """[start, end) of rank's images; the first global_batch % world ranks get one extra image."""
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_logits(local: torch.Tensor, global_batch: int, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """All-gathers every rank's [b_r, C] logits into [global_batch, C] in global image order.
    Ragged shards are padded to the largest shard for the collective and trimmed afterwards."""
    world = dist.get_world_size(group)
    if world == 1:
        return local
    if local.is_cuda and dist.get_backend(group) == "gloo":
        # gloo moves host buffers only (the one-device rehearsal of the N-rank path);
        # RCCL ("nccl") gathers device buffers in place
        return gather_logits(local.cpu(), global_batch, group).to(local.device)
    per = -(-global_batch // world)
    C = local.shape[1]
    buf = local
    if local.shape[0] != per:
        buf = torch.zeros((per, C), dtype=local.dtype, device=local.device)
        buf[: local.shape[0]] = local
    out = torch.empty((world * per, C), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf.contiguous(), group=group)
    if per * world == global_batch:
        return out
    keep = []
    for r in range(world):
        s, e = shard_bounds(global_batch, world, r)
        keep.append(out[r * per: r * per + (e - s)])
    return torch.cat(keep, 0)


class ShardedInference:
    """Runs `model` on this rank's shard of a global batch and returns all logits on every rank."""

    def __init__(self, model: Callable[[torch.Tensor], torch.Tensor], group: Optional[dist.ProcessGroup] = None):
        self.model = model
        self.group = group

    def world_rank(self) -> Tuple[int, int]:
        if not dist.is_initialized():
            return 1, 0
        return dist.get_world_size(self.group), dist.get_rank(self.group)

    @torch.no_grad()
    def __call__(self, global_images: torch.Tensor) -> torch.Tensor:
        world, rank = self.world_rank()
        s, e = shard_bounds(global_images.shape[0], world, rank)
        return self.forward_shard(global_images[s:e], global_images.shape[0])

    @torch.no_grad()
    def forward_shard(self, local_images: torch.Tensor, global_batch: int) -> torch.Tensor:
        """This rank's images (already resident on its device, e.g. generated there) -> all logits."""
        world, rank = self.world_rank()
        s, e = shard_bounds(global_batch, world, rank)
        if local_images.shape[0] != e - s:
            raise ValueError(f"rank {rank} of {world}: shard of {local_images.shape[0]} images, but images "
                             f"[{s}, {e}) of the global batch {global_batch} belong to it")
        local = self.model(local_images)
        if world == 1:
            return local
        return gather_logits(local, global_batch, self.group)
