"""Process/device setup shared by the drivers: one process per GPU, torch.distributed over
RCCL ("nccl" backend on ROCm) when launched by torchrun, gloo on CPU-only hosts."""
from __future__ import annotations

import glob
import os
import socket
import subprocess
import sys
from typing import List, Optional

import torch

from .vi_ssm import DistCtx


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count() -> Optional[int]:
    """GPUs this process could hand to its ranks, WITHOUT touching the GPU runtime (torch.cuda.device_count() may
    initialise HIP on this torch build, and a launcher must not spawn its ranks from a process that did): the
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES list when one is set (an empty list is zero
    devices), else the AMD (vendor 0x1002) DRM render nodes.  None = unknown."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() != ""])
    n = 0
    for node in glob.glob("/sys/class/drm/renderD*"):
        try:
            with open(os.path.join(node, "device", "vendor")) as f:
                n += int(f.read().strip(), 16) == 0x1002
        except (OSError, ValueError):
            continue
    return n or None


def rank_launch_cmd(gpus: int, script: str, argv: List[str], port: Optional[int] = None) -> List[str]:
    """The torchrun command that runs `script argv` as `gpus` ranks on this node (rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port or _free_port()), script] + list(argv)


def ensure_world(gpus: int, script: str, argv: List[str]) -> Optional[int]:
    """`--gpus N` of bench.py / main.py.  Under torchrun (WORLD_SIZE set) the launched world must be N: a mismatch
    exits non-zero.  Without WORLD_SIZE and N > 1 this process becomes a launcher: it starts N rank processes
    with torchrun BEFORE any GPU call (no torch.cuda use here: a process that initialised the GPU must not be
    replaced, and its children get the devices) and returns their exit code for the caller to exit with.
    Returns None when this process is itself the (only) rank and should run the work."""
    if gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {gpus})")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != gpus:
            raise SystemExit(f"--gpus {gpus} but the launcher started WORLD_SIZE={env_world} ranks")
        return None
    if gpus == 1:
        return None
    n_dev = visible_gpu_count()   # no torch.cuda here: the ranks are spawned from this process
    backend = os.environ.get("VISSM_DIST_BACKEND", "nccl")
    if n_dev is not None and n_dev < gpus and backend != "gloo":
        raise SystemExit(f"--gpus {gpus} needs {gpus} visible GPUs for RCCL, found {n_dev} "
                         "(VISSM_DIST_BACKEND=gloo rehearses several ranks on one GPU)")
    return subprocess.call(rank_launch_cmd(gpus, script, argv))


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
