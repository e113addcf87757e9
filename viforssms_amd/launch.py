"""Process/device setup shared by the drivers: one process per GPU, torch.distributed over
RCCL ("nccl" backend on ROCm) when launched by torchrun, gloo on CPU-only hosts."""
from __future__ import annotations

import os

import torch

from .vi_ssm import DistCtx


def init_distributed() -> DistCtx:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        if torch.cuda.is_available():
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        return DistCtx()
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        backend = "nccl"
    else:
        backend = "gloo"
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return DistCtx(dist.get_rank(), dist.get_world_size())


def barrier(ctx: DistCtx):
    if ctx.world > 1:
        import torch.distributed as dist
        dist.barrier()
