"""The ELBO training step captured once as a HIP graph and replayed.

The reference runs one TF session call per step (AR.py:300-301); its eager equivalent here is
~750 kernel launches per step, so at the paper's sizes (p = 50 windows of M = 50) the step is
bound by launch overhead, not by the GPU.  A captured graph removes that: every step after the
first few replays the same kernels with the same buffers.

What changes between steps is kept in device buffers the graph reads:
  * the sample -> window map: the window-shared parts (features, conv over features, ELBO feeds)
    are computed for every window start the reference can draw (arange(0, T, M)), and one int32
    per sample selects its window (one small host -> device copy per step);
  * the Philox row base of the step (step * p + rank * p_local), read by vissm_normal_base_dev.
Everything else (parameters, Adamax slots, gradients, workspaces from the graph's private pool)
is at fixed addresses.  Results equal the eager step's up to the summation order of the
window-shared GEMMs (their extra windows contribute exact zeros).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Optional

import numpy as np
import torch

from .nma import Batch


class GraphedStep:
    """model.elbo_step(batch_for(starts), step) with the step captured on its `warmup + 1`-th call."""

    def __init__(self, model, warmup: int = 2):
        self.m = model
        self.warmup = int(warmup)
        eng = model.engine
        dev = eng.device
        self.universe = np.arange(0, int(model.target_len()), int(model.batch_dims), dtype=np.int64)
        B = model.p_local
        base = eng.make_batch(self.universe)
        self.win: Optional[torch.Tensor] = None
        if len(self.universe) > 1:
            self.win = torch.zeros(B, dtype=torch.int32, device=dev)
            # two pinned staging buffers, each reused only after the event behind its last copy has
            # completed: the host may run steps ahead of the GPU (no per-step synchronize)
            self._win_host = [torch.zeros(B, dtype=torch.int32).pin_memory() for _ in range(2)]
            self._win_done = [None, None]
            self._slot = 0
        feeds = dataclasses.replace(base.feeds, win=self.win, n_win=len(self.universe))
        self.batch = Batch(np.zeros(B, dtype=np.int64), base.uniq, base.ts, self.win, feeds, base.host_feeds)
        self.row0 = torch.zeros(1, dtype=torch.int64, device=dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out: Optional[Dict[str, torch.Tensor]] = None
        self.calls = 0
        self._side = torch.cuda.Stream(device=dev)

    def _inputs(self, starts_global: np.ndarray, step: int):
        m = self.m
        r, pl = m.dist.rank, m.p_local
        local = np.asarray(starts_global[r * pl:(r + 1) * pl], dtype=np.int64)
        if self.win is not None:
            idx = np.searchsorted(self.universe, local)
            if not np.array_equal(self.universe[idx], local):
                raise ValueError("window start outside arange(0, T, M)")
            i, self._slot = self._slot, self._slot ^ 1
            if self._win_done[i] is not None:
                self._win_done[i].synchronize()
            self._win_host[i].numpy()[:] = idx.astype(np.int32)
            self.win.copy_(self._win_host[i], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._win_done[i] = ev
        self.row0.fill_(step * m.p + r * pl)

    def step(self, starts_global: np.ndarray, step: int) -> Dict[str, torch.Tensor]:
        """One training step; returns the step's outputs (static tensors: read them before the next call)."""
        m = self.m
        self._inputs(starts_global, step)
        self.calls += 1
        if self.graph is not None:
            self.graph.replay()
            return self.out
        if self.calls <= self.warmup:  # eager warm-up on a side stream (allocator pools, library state)
            self._side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self._side):
                out = m.elbo_step(self.batch, step, row0_dev=self.row0)
            torch.cuda.current_stream().wait_stream(self._side)
            return out
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # captured on the warm-up stream: autograd's per-parameter accumulation nodes run on the
        # stream of the backward that created them
        self._side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g, stream=self._side):
            self.out = m.elbo_step(self.batch, step, row0_dev=self.row0)
        torch.cuda.current_stream().wait_stream(self._side)
        self.graph = g
        g.replay()
        return self.out
