"""Flat parameter store.

All trainable variables of a model live in ONE contiguous fp32 device buffer
(and their gradients in a second one), so the gradient all-reduce and the fused
clip+Adamax kernel each see a single buffer.  Each variable is exposed as a
leaf tensor sharing that storage; its ``.grad`` is a view of the flat gradient
buffer, so autograd accumulates straight into it.

Initialisers follow the TF 1.8 defaults the reference relies on
(tf.layers.dense / conv1d: glorot-uniform kernels, zero biases;
batch_normalization: gamma 1, beta 0; masked_dense: glorot-normal x mask).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch


def glorot_uniform(shape, fan_in, fan_out, rng: np.random.Generator):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape)


def glorot_normal(shape, fan_in, fan_out, rng: np.random.Generator):
    sd = math.sqrt(2.0 / (fan_in + fan_out)) / 0.87962566103423978  # truncated-normal correction
    x = rng.standard_normal(size=shape)
    while True:
        bad = np.abs(x) > 2.0
        if not bad.any():
            break
        x[bad] = rng.standard_normal(size=int(bad.sum()))
    return x * sd


class ParamStore:
    def __init__(self):
        self._specs: "OrderedDict[str, Tuple[tuple, np.ndarray]]" = OrderedDict()
        self.flat: Optional[torch.Tensor] = None
        self.grad: Optional[torch.Tensor] = None
        self.tensors: Dict[str, torch.Tensor] = {}
        self.offsets: Dict[str, Tuple[int, int]] = {}

    def add(self, name: str, value: np.ndarray):
        if name in self._specs:
            raise KeyError(f"duplicate variable {name}")
        self._specs[name] = (tuple(value.shape), np.asarray(value, dtype=np.float64))

    def names(self) -> List[str]:
        return list(self._specs)

    @property
    def numel(self) -> int:
        return sum(int(np.prod(s)) if len(s) else 1 for s, _ in self._specs.values())

    def finalize(self, device) -> "ParamStore":
        n = self.numel
        flat = torch.empty(n, dtype=torch.float32, device=device)
        grad = torch.zeros(n, dtype=torch.float32, device=device)
        off = 0
        host = np.empty(n, dtype=np.float32)
        for name, (shape, val) in self._specs.items():
            sz = int(np.prod(shape)) if len(shape) else 1
            host[off:off + sz] = val.reshape(-1)
            self.offsets[name] = (off, sz)
            off += sz
        flat.copy_(torch.from_numpy(host))
        self.flat, self.grad = flat, grad
        for name, (shape, _) in self._specs.items():
            a, sz = self.offsets[name]
            t = flat[a:a + sz].view(shape).detach()
            t.requires_grad_(True)
            t.grad = grad[a:a + sz].view(shape)
            self.tensors[name] = t
        return self

    def __getitem__(self, name) -> torch.Tensor:
        return self.tensors[name]

    def __contains__(self, name) -> bool:
        return name in self._specs

    def zero_grad(self):
        self.grad.zero_()
        # autograd may have replaced a .grad (e.g. if a variable received no gradient it stays)
        for name, t in self.tensors.items():
            a, sz = self.offsets[name]
            g = t.grad
            if g is None or g.data_ptr() != self.grad[a:a + sz].data_ptr():
                t.grad = self.grad[a:a + sz].view(t.shape)

    def release_grads(self):
        """Drop every variable's .grad view before a backward whose gradients nobody reads until sync_grads: autograd
        then keeps each variable's incoming gradient tensor as its .grad (no kernel) instead of adding it into the
        zeroed flat view (one element-wise launch per variable: ~160 per SV step, ~0.7 ms); sync_grads moves them
        into the flat buffer in a few multi-tensor copies.  The flat buffer is already zero (zero_grad), so a
        variable that receives no gradient keeps its zero slice."""
        for t in self.tensors.values():
            t.grad = None

    def sync_grads(self):
        """Copy any .grad that autograd re-allocated (or that release_grads let it allocate) back into the flat
        buffer, batched into multi-tensor copies, and point the .grad at the flat views again."""
        dst, src = [], []
        for name, t in self.tensors.items():
            a, sz = self.offsets[name]
            g = t.grad
            if g is None:   # no gradient reached it (released view): its flat slice is still zero_grad's zeros
                t.grad = self.grad[a:a + sz].view(t.shape)
            elif g.data_ptr() != self.grad[a:a + sz].data_ptr():
                v = self.grad[a:a + sz].view(t.shape)
                dst.append(v)
                src.append(g)
                t.grad = v
        if dst:
            torch._foreach_copy_(dst, src)

    def state_numpy(self) -> Dict[str, np.ndarray]:
        return {n: self.tensors[n].detach().cpu().numpy() for n in self._specs}

    def load_numpy(self, values: Dict[str, np.ndarray], strict: bool = True):
        with torch.no_grad():
            for name in self._specs:
                if name not in values:
                    if strict:
                        raise KeyError(f"missing variable {name}")
                    continue
                v = np.asarray(values[name], dtype=np.float32)
                t = self.tensors[name]
                if tuple(v.shape) != tuple(t.shape):
                    raise ValueError(f"{name}: shape {v.shape} != {tuple(t.shape)}")
                t.copy_(torch.from_numpy(v))
