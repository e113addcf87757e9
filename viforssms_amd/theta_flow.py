"""q(theta): TransformedDistribution(Normal(loc, scale), Chain(reversed([IMAF_0, P_0, ..., IMAF_n])))
with event_shape [P_theta] (AR.py:376-391; lotka_volterra_partial.py:494-508;
SV_dense.py:428-442 (relu); fitz_nag_NVP.py:480-494).

Each IMAF is tfb.Invert(tfb.MaskedAutoregressiveFlow(masked_autoregressive_default_template(
hidden_layers=[5, 5, 5], activation))):  Invert(MAF).forward(z) = (z - shift(z)) * exp(-log_scale(z)),
a single parallel pass, with forward log-det = -sum(log_scale(z)).  log q(theta) at a sample is the
base log-prob of the base draw minus the summed forward log-dets (TransformedDistribution.log_prob
through the bijector cache; identical in value and gradient to the explicit inverse).

The MADE masks restate TF 1.8's masked_autoregressive._gen_slices/_gen_mask; log_scale is clipped
to [-5, 3] with a straight-through gradient (_clip_by_value_preserve_grad).  These defaults are
recalled from TF 1.8 and cannot be checked against TF offline.
Tiny (P_theta <= 5, 580 parameters for P = 3): the training step's sample and log q and their
backward run as one HIP launch each (ops.ThetaFlowFn -> vissm_theta_fwd / vissm_theta_bwd, csrc/
theta.hip) instead of ~150 small tensor kernels; `sample_and_log_prob_torch` keeps the tensor-op
restatement, the tests' reference for the kernels.
"""
from __future__ import annotations

import math
from typing import List, Sequence

import numpy as np
import torch

from .params import ParamStore, glorot_normal
from .linalg import linear

HIDDEN = (5, 5, 5)


def gen_mask(num_blocks: int, n_in: int, n_out: int, exclusive: bool) -> np.ndarray:
    """[n_out, n_in] mask of TF's _gen_mask."""
    mask = np.zeros((n_out, n_in))
    d_in, d_out = n_in // num_blocks, n_out // num_blocks
    row = d_out if exclusive else 0
    col = 0
    for _ in range(num_blocks):
        mask[row:, col:col + d_in] = 1.0
        col += d_in
        row += d_out
    return mask


def made_masks(D: int, hidden: Sequence[int] = HIDDEN) -> List[np.ndarray]:
    """Dense-kernel masks [in, out] of the default template for event size D."""
    out, n_in = [], D
    for i, units in enumerate(hidden):
        out.append(gen_mask(D, n_in, units, exclusive=(i == 0)).T)
        n_in = units
    out.append(gen_mask(D, n_in, 2 * D, exclusive=False).T)
    return out


class ThetaFlow:
    """The variational posterior over the SDE parameters."""

    def __init__(self, store: ParamStore, P_theta: int, n_bijectors: int, perms: Sequence[Sequence[int]],
                 base_loc: float, base_scale: float, activation: str = "elu", rng=None, prefix: str = "theta"):
        if len(perms) != n_bijectors - 1:
            raise ValueError("need n_bijectors - 1 permutations")
        self.P = P_theta
        self.n = n_bijectors
        self.perms = [list(map(int, p)) for p in perms]
        self.base_loc = float(base_loc)
        self.base_scale = float(base_scale)
        self.act = torch.relu if activation == "relu" else torch.nn.functional.elu
        self.prefix = prefix
        self.masks_np = made_masks(P_theta)
        rng = rng if rng is not None else np.random.default_rng(0)
        for i in range(n_bijectors):
            for j, m in enumerate(self.masks_np):
                w = glorot_normal(m.shape, m.shape[0], m.shape[1], rng) * m
                store.add(f"{prefix}/maf{i}/dense{j}/kernel", w)
                store.add(f"{prefix}/maf{i}/dense{j}/bias", np.zeros(m.shape[1]))
        self.store = store
        self._masks = None

    def _dev_masks(self, device):
        if self._masks is None or self._masks[0].device != device:
            self._masks = [torch.tensor(m, dtype=torch.float32, device=device) for m in self.masks_np]
        return self._masks

    def _perm_matrix(self, i: int, z: torch.Tensor) -> torch.Tensor:
        """one-hot [P, P] with (z @ M)[..., d] = z[..., perms[i][d]]"""
        key = (i, z.device, z.dtype)
        cache = self.__dict__.setdefault("_pm", {})
        if key not in cache:
            m = torch.zeros(self.P, self.P, dtype=z.dtype, device=z.device)
            m[self.perms[i], torch.arange(self.P)] = 1.0
            cache[key] = m
        return cache[key]

    def _shift_log_scale(self, i: int, z: torch.Tensor):
        masks = self._dev_masks(z.device)
        h = z
        nl = len(masks)
        for j in range(nl):
            w = self.store[f"{self.prefix}/maf{i}/dense{j}/kernel"] * masks[j]
            h = linear(h, w, self.store[f"{self.prefix}/maf{i}/dense{j}/bias"])
            if j < nl - 1:
                h = self.act(h)
        h = h.reshape(*z.shape, 2)
        shift, ls = h[..., 0], h[..., 1]
        ls = ls + (torch.clamp(ls, -5.0, 3.0) - ls).detach()
        return shift, ls

    def _packed(self, device):
        """(w, grad, mask, anchor): the MAF variables as one contiguous slice of the parameter store (the
        kernels' layout), its gradient slice, the MADE masks packed the same way, one variable of the slice."""
        names = [f"{self.prefix}/maf{i}/dense{j}/{v}" for i in range(self.n) for j in range(len(self.masks_np))
                 for v in ("kernel", "bias")]
        st = self.store
        a = st.offsets[names[0]][0]
        b = st.offsets[names[-1]][0] + st.offsets[names[-1]][1]
        if b - a != sum(st.offsets[n][1] for n in names) or any(
                st.offsets[names[i + 1]][0] != st.offsets[names[i]][0] + st.offsets[names[i]][1]
                for i in range(len(names) - 1)):
            raise RuntimeError("q(theta) variables are not contiguous in the parameter store")
        cache = self.__dict__.setdefault("_mask_dev", {})
        if device not in cache:
            parts = []
            for _ in range(self.n):
                for m in self.masks_np:
                    parts += [m.reshape(-1), np.ones(m.shape[1])]
            cache[device] = torch.tensor(np.concatenate(parts), dtype=torch.float32, device=device)
        return st.flat[a:b], st.grad[a:b], cache[device], st.tensors[names[0]]

    def sample_and_log_prob(self, x0: torch.Tensor):
        """x0: base draw [p, P] ~ N(base_loc, base_scale).  Returns theta [p, P], log q(theta) [p]
        (vissm_theta_fwd; the backward adds the MAF variables' gradient into the store's flat gradient)."""
        from .ops import ThetaFlowFn
        w, g, mask, anchor = self._packed(x0.device)
        args = (self.n, self.act is torch.relu, self.base_loc, self.base_scale, self.perms)
        return ThetaFlowFn.apply(args, w, mask, g, x0.float().contiguous(), anchor)

    def sample_and_log_prob_torch(self, x0: torch.Tensor):
        """The same as tensor ops (the reference of the kernels in the tests)."""
        z = x0
        lq = (-0.5 * ((x0 - self.base_loc) / self.base_scale) ** 2 - math.log(self.base_scale)
              - 0.5 * math.log(2 * math.pi)).sum(-1)
        for i in range(self.n):
            shift, ls = self._shift_log_scale(i, z)
            z = (z - shift) * torch.exp(-ls)
            lq = lq + ls.sum(-1)
            if i < self.n - 1:
                z = z @ self._perm_matrix(i, z)  # exact; its backward is a product, not a scatter
        return z, lq

    def log_prob(self, theta: torch.Tensor):
        """log q at arbitrary theta via the iterative inverse (Invert(MAF).inverse = MAF.forward)."""
        y = theta
        ldj = torch.zeros(theta.shape[:-1], dtype=theta.dtype, device=theta.device)
        for i in reversed(range(self.n)):
            if i < self.n - 1:
                inv = np.argsort(self.perms[i])
                y = y[..., list(inv)]
            # MAF.forward(y): x_d = y_d * exp(ls_d(x)) + shift_d(x), autoregressive over P steps
            x = torch.zeros_like(y)
            for _ in range(self.P):
                shift, ls = self._shift_log_scale(i, x)
                x = y * torch.exp(ls) + shift
            shift, ls = self._shift_log_scale(i, x)
            ldj = ldj + ls.sum(-1)
            y = x
        base = (-0.5 * ((y - self.base_loc) / self.base_scale) ** 2 - math.log(self.base_scale)
                - 0.5 * math.log(2 * math.pi)).sum(-1)
        return base + ldj
