"""AdamaxOptimizer with the reference's constructor and methods (optimisers/adamax.py:11-61), over
torch tensors.  The update is the reference's Adamax without bias correction:
    v <- beta1 v + (1 - beta1) g ;  m <- max(beta2 m + eps, |g|) ;  var <- var - lr v / m
with eps = 1e-8 (1e-7 for fp16 variables), slots "v" (first moment) and "m" (inf-norm) starting
at zero.  apply_gradients runs one fused HIP kernel per variable (or one over the whole flat
buffer when the variables are views of a viforssms_amd ParamStore, as VI_SSM does);
clip_norm reproduces tf.clip_by_global_norm inside the same kernel.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from .ops import AdamaxKernel


class AdamaxOptimizer:
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, use_locking=False, name="Adamax"):
        self._lr = learning_rate
        self._beta1 = beta1
        self._beta2 = beta2
        self._name = name
        self._slots: Dict[int, Dict[str, torch.Tensor]] = {}
        self._kernels: Dict[int, AdamaxKernel] = {}

    # -- slots --------------------------------------------------------------------------
    def _create_slots(self, var_list):
        for v in var_list:
            if id(v) not in self._slots:
                self._slots[id(v)] = {"m": torch.zeros_like(v, memory_format=torch.contiguous_format),
                                      "v": torch.zeros_like(v, memory_format=torch.contiguous_format)}

    def get_slot(self, var, name):
        return self._slots.get(id(var), {}).get(name)

    def get_slot_names(self):
        return ["m", "v"]

    # -- TF-style API -----------------------------------------------------------------
    def compute_gradients(self, loss: torch.Tensor, var_list: Optional[Sequence[torch.Tensor]] = None):
        """Gradient of sum(loss) (a vector loss is summed, as tf.gradients does) -> [(grad, var)]."""
        if var_list is None:
            raise ValueError("var_list is required (no global trainable-variable collection in torch)")
        var_list = list(var_list)
        if loss.dim() > 0:
            loss = loss.sum()
        grads = torch.autograd.grad(loss, var_list, allow_unused=True)
        return list(zip(grads, var_list))

    def apply_gradients(self, grads_and_vars: Iterable[Tuple[Optional[torch.Tensor], torch.Tensor]],
                        global_step=None, name=None, clip_norm: float = 0.0):
        pairs = [(g, v) for g, v in grads_and_vars if g is not None]
        if not pairs:
            raise ValueError("No gradients provided for any variable")
        self._create_slots([v for _, v in pairs])
        if clip_norm and clip_norm > 0:
            # one global norm across all variables: scale the gradients once, then update unclipped
            gn = torch.sqrt(sum((g.float() ** 2).sum() for g, _ in pairs))
            scale = clip_norm * torch.minimum(1.0 / gn, torch.tensor(1.0 / clip_norm, device=gn.device))
            if not torch.isfinite(gn):
                scale = torch.tensor(float("nan"), device=gn.device)
            pairs = [(g * scale, v) for g, v in pairs]
        with torch.no_grad():
            for g, v in pairs:
                s = self._slots[id(v)]
                eps = 1e-7 if v.dtype == torch.float16 else 1e-8
                k = self._kernels.get(v.numel())
                if k is None:
                    k = self._kernels[v.numel()] = AdamaxKernel(v.numel(), v.device)
                target = v.detach()
                k.step(target.view(-1), g.detach().contiguous().view(-1), s["v"].view(-1), s["m"].view(-1),
                       self._lr, self._beta1, self._beta2, eps, 0.0)
        if global_step is not None and torch.is_tensor(global_step):
            global_step.add_(1)

    def minimize(self, loss, global_step=None, var_list=None, name=None):
        return self.apply_gradients(self.compute_gradients(loss, var_list), global_step=global_step)

    def _apply_sparse(self, grad, var):
        raise NotImplementedError("Sparse gradient updates are not supported.")
