"""Process/device setup shared by the drivers: one process per GPU, torch.distributed over
RCCL ("nccl" backend on ROCm) when launched by torchrun, gloo on CPU-only hosts."""
from __future__ import annotations

import os

import torch

from .vi_ssm import DistCtx


def init_distributed() -> DistCtx:
    """One process per GPU: rank r -> device LOCAL_RANK (mod the visible count, so a one-GPU box can
    rehearse several ranks), RCCL ("nccl") for GPU tensors unless VISSM_DIST_BACKEND says otherwise
    (gloo: the CPU tests and the single-GPU multi-rank rehearsal)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = torch.cuda.device_count()
    if world <= 1:
        if n_dev > 0:
            torch.cuda.set_device(local % n_dev)
        return DistCtx()
    import torch.distributed as dist
    if n_dev > 0:
        torch.cuda.set_device(local % n_dev)
        backend = os.environ.get("VISSM_DIST_BACKEND", "nccl")
    else:
        backend = "gloo"
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return DistCtx(dist.get_rank(), dist.get_world_size())


def barrier(ctx: DistCtx):
    if ctx.world > 1:
        import torch.distributed as dist
        dist.barrier()
