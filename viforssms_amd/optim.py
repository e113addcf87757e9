"""AdamaxOptimizer with the reference's constructor and methods (optimisers/adamax.py:11-61), over
torch tensors.  The update is the reference's Adamax without bias correction:
    v <- beta1 v + (1 - beta1) g ;  m <- max(beta2 m + eps, |g|) ;  var <- var - lr v / m
with eps = 1e-8 (1e-7 for fp16 variables), slots "v" (first moment) and "m" (inf-norm) starting
at zero.

apply_gradients runs ONE fused HIP launch pair (vissm_adamax_step: fixed-order global norm, then the
update) over a flat fp32 image of every variable of a dtype: the variables' slots live in one flat
buffer per dtype (get_slot returns views of it); gradients and values are packed into flat buffers,
updated, and written back -- or updated in place when the variables already are consecutive views
of one buffer (a viforssms_amd ParamStore, as VI_SSM's are).  Variables of any layout (non-contiguous
views included) and fp16 variables (updated in fp32, rounded back) are accepted.  clip_norm > 0 is
tf.clip_by_global_norm over all the variables: fused into the kernel for one dtype group, a device
scale from vissm_sqnorm otherwise (no host synchronisation either way).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from .ops import AdamaxKernel, sqnorm


class _Group:
    """The variables of one dtype / device in one apply_gradients call: flat slots and a kernel."""

    def __init__(self, vars_: List[torch.Tensor]):
        self.vars = vars_
        self.sizes = [v.numel() for v in vars_]
        n = sum(self.sizes)
        dev = vars_[0].device
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.kernel = AdamaxKernel(n, dev)
        self.eps = 1e-7 if vars_[0].dtype == torch.float16 else 1e-8
        self.flat_view = self._consecutive_view()

    def _consecutive_view(self) -> Optional[torch.Tensor]:
        """A flat fp32 view covering every variable when they are contiguous, in order and adjacent in one
        storage (then the update runs in place); None otherwise."""
        v0 = self.vars[0]
        if v0.dtype != torch.float32:
            return None
        ptr = v0.data_ptr()
        st = v0.untyped_storage().data_ptr()
        for v, sz in zip(self.vars, self.sizes):
            if not v.is_contiguous() or v.data_ptr() != ptr or v.untyped_storage().data_ptr() != st:
                return None
            ptr += 4 * sz
        base = v0.detach()
        return torch.as_strided(base, (sum(self.sizes),), (1,), base.storage_offset())

    def slot_views(self, name: str) -> List[torch.Tensor]:
        buf = self.v if name == "v" else self.m
        out, a = [], 0
        for var, sz in zip(self.vars, self.sizes):
            out.append(buf[a:a + sz].view(var.shape))
            a += sz
        return out


class AdamaxOptimizer:
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, use_locking=False, name="Adamax"):
        self._lr = learning_rate
        self._beta1 = beta1
        self._beta2 = beta2
        self._name = name
        self._groups: Dict[tuple, _Group] = {}
        self._slot_of: Dict[int, Dict[str, torch.Tensor]] = {}

    # -- slots --------------------------------------------------------------------------
    def _group_for(self, vars_: List[torch.Tensor]) -> _Group:
        """The flat-slot group of exactly these variables.  A variable first seen in another grouping (a None
        gradient on one call, a changed var_list) keeps its Adamax state, as TF keeps one slot pair per variable
        (optimisers/adamax.py:36-40): _slot_of[id(var)] is the single record of where a variable's live slots
        are, and whenever it points outside the group about to run (a new group, or a cached one another
        grouping has run since), the current values are copied into the group's flat buffers and the record
        repointed.  Groups hold their variables, so the ids in a key cannot be reused while the group exists."""
        key = tuple(id(v) for v in vars_)
        g = self._groups.get(key)
        if g is None or any(a is not b for a, b in zip(g.vars, vars_)):
            g = self._groups[key] = _Group(vars_)
        with torch.no_grad():
            for var, sv, sm in zip(vars_, g.slot_views("v"), g.slot_views("m")):
                old = self._slot_of.get(id(var))
                if old is not None and old["var"] is var and old["v"].data_ptr() == sv.data_ptr():
                    continue   # the group's own views are the live slots
                if old is not None and old["var"] is var:
                    sv.copy_(old["v"])
                    sm.copy_(old["m"])
                self._slot_of[id(var)] = {"var": var, "v": sv, "m": sm}
        return g

    def get_slot(self, var, name):
        rec = self._slot_of.get(id(var))
        if rec is None or rec["var"] is not var or name not in ("v", "m"):
            return None
        return rec[name]

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
        by: Dict[tuple, List[Tuple[torch.Tensor, torch.Tensor]]] = {}
        for g, v in pairs:
            if v.dtype not in (torch.float32, torch.float16):
                raise TypeError(f"Adamax: unsupported variable dtype {v.dtype}")
            by.setdefault((v.dtype, v.device), []).append((g, v))
        clip = float(clip_norm) if clip_norm and clip_norm > 0 else 0.0
        with torch.no_grad():
            flat_g = {k: torch.cat([g.detach().reshape(-1).float() for g, _ in ps]) for k, ps in by.items()}
            if clip > 0 and len(by) > 1:
                # one global norm across the dtype groups: the clip scale on the device, applied up front
                sq = sum(sqnorm(fg) for fg in flat_g.values())
                gn = torch.sqrt(sq)
                scale = torch.where(torch.isfinite(gn), clip * torch.minimum(1.0 / gn, torch.full_like(gn, 1.0 / clip)),
                                    torch.full_like(gn, float("nan")))
                flat_g = {k: fg * scale for k, fg in flat_g.items()}
                clip = 0.0
            for k, ps in by.items():
                grp = self._group_for([v for _, v in ps])
                P = grp.flat_view
                inplace = P is not None
                if not inplace:
                    P = torch.cat([v.detach().reshape(-1).float() for _, v in ps])
                grp.kernel.step(P, flat_g[k], grp.v, grp.m, self._lr, self._beta1, self._beta2, grp.eps, clip)
                if not inplace:
                    a = 0
                    for (_, v), sz in zip(ps, grp.sizes):
                        v.copy_(P[a:a + sz].view(v.shape))
                        a += sz
        if global_step is not None and torch.is_tensor(global_step):
            global_step.add_(1)

    def minimize(self, loss, global_step=None, var_list=None, name=None):
        return self.apply_gradients(self.compute_gradients(loss, var_list), global_step=global_step)

    def _apply_sparse(self, grad, var):
        raise NotImplementedError("Sparse gradient updates are not supported.")
