"""Rounding model of the reduced-precision flow products (bf16 / bf16x2f / bf16x2), as an emulation on the
float64 oracle.

TEST INFRASTRUCTURE ONLY (as nma_oracle): tests and scripts use it to DERIVE the tolerances of the reduced-precision
modes from the modes' own rounding, instead of holding a kernel to its last measurement.

Every flow product of the AR flows (nma_oracle.iaf_flow: the first conv's sample channel, the hidden layers, the
head) runs through a custom autograd function that rounds (bf16, round to nearest even, the accumulation exact)
exactly the operands the HIP kernels round in a mode (flow_v5.hip; include/vissm.h VISSM_PREC_*):

  fwd_x   forward / recompute activations (u taps, ELU outputs)           every bf16 mode
  fwd_w   forward / recompute weights                                      bf16 (split modes: w_hi x + w_lo x, exact
                                                                           to ~2^-16: off)
  bwd_g   backward-chain gradient operands (dI = W dZ, dcon = w_eps dA0, head backward (g_mu, g_r)); the window-
          shared dC and d theta_term sum the bf16 dA0 image                every bf16 mode
  bwd_w   backward-chain weights                                           bf16, bf16x2f (off in bf16x2)
  wg_x    the weight-gradient products' activation operands (dW = I dZ^T reads the bf16 images)   every bf16 mode

The emulation covers the one-hidden-layer AR flows (the modes' kernels: bwd2_kernel / fwd2_kernel / the fused last
flow); the three-hidden-layer families' BN / stride-2 heads run the plain oracle.
"""
from __future__ import annotations

import contextlib

import torch

from . import nma_oracle as O

MODES = {
    "bf16": dict(fwd_x=1, fwd_w=1, bwd_g=1, bwd_w=1, wg_x=1),
    "bf16x2f": dict(fwd_x=1, fwd_w=0, bwd_g=1, bwd_w=1, wg_x=1),
    "bf16x2": dict(fwd_x=1, fwd_w=0, bwd_g=1, bwd_w=0, wg_x=1),
}
# the product-side precision names (viforssms_amd._lib.TRAIN_PRECISIONS) -> rounding mode
PRECISION_MODE = {1: "bf16", 17: "bf16x2f", 3: "bf16x2"}

MODE = {}
# Realisations.  The kernels round the same operands in a scaled domain -- activations and weights carry log2(e)
# (flow_v5.hip: ELU on v_exp_f32), the theta fold splits its rows -- so their rounding errors are another draw of the
# same distribution, not the emulation's bit pattern.  Realisation s > 0 rounds every operand tensor as bf16(c x) / c
# with c uniform in [1, 2) drawn per rounding (REAL[1] seeded by s): the same rounding model, other error patterns.
REAL = [False, None]   # [on, torch.Generator]


def rb(x):
    if REAL[0]:
        c = 1.0 + float(torch.rand((), generator=REAL[1], dtype=torch.float64))
        return (x * c).float().bfloat16().double() / c
    return x.float().bfloat16().double()


def R(x, key):
    return rb(x) if MODE.get(key, False) else x


class BMM(torch.autograd.Function):
    """y = x @ W with the kernel's operand roundings (x activations [..., K], W weights [K, N])."""

    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(x, W)
        return R(x, "fwd_x") @ R(W, "fwd_w")

    @staticmethod
    def backward(ctx, gy):
        x, W = ctx.saved_tensors
        g = R(gy, "bwd_g")
        gx = g @ R(W, "bwd_w").t()
        xr = R(R(x, "fwd_x"), "wg_x")     # the kernels' weight-gradient products read the bf16 images
        gW = (xr.reshape(-1, x.shape[-1]).t() @ g.reshape(-1, g.shape[-1]))
        return gx, gW


class GradRound(torch.autograd.Function):
    """identity; the backward rounds the gradient (dC and d theta_term sum the bf16 dA0 image)"""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return R(g, "bwd_g")


def iaf_flow_emul(u, CF, theta, P, cfg):
    """nma_oracle.iaf_flow (AR.py:58-89) with the products of bf16_mode's rounding points (one hidden layer or more,
    no BN, stride 1)."""
    if cfg.bn or cfg.stride2:
        return _PLAIN(u, CF, theta, P, cfg)
    w = P["conv_w"][:, 0, :]                       # [k, H]
    k = w.shape[0]
    x = u[:, :-1]
    U = x.unfold(1, k, 1)                           # [p, n_out, k]
    a = BMM.apply(U, w) + GradRound.apply(CF + O.theta_term(theta, P)[:, None, :])
    h = O.elu(a)
    for l in range(cfg.n_hidden):
        h = O.elu(BMM.apply(h, P[f"hid_w{l}"]) + P[f"hid_b{l}"])
    head = BMM.apply(h, P["head_w"]) + P["head_b"]
    mu, sig = head[..., 0], O.softplus(head[..., 1]) + 1e-10
    return u[:, cfg.k:] * sig + mu, torch.log(sig[:, -cfg.n_logsig:])


_PLAIN = O.iaf_flow


@contextlib.contextmanager
def emulate(mode, realisation: int = 0):
    """Within the block every nma_oracle flow evaluation rounds as precision `mode` ("bf16", "bf16x2f", "bf16x2";
    a dict of rounding switches; None: exact); realisation > 0: a scaled-domain realisation of the rounding (REAL)."""
    MODE.clear()
    REAL[0], REAL[1] = (True, torch.Generator().manual_seed(realisation)) if realisation else (False, None)
    if mode is not None:
        MODE.update({k: bool(v) for k, v in (MODES[mode] if isinstance(mode, str) else mode).items()})
    O.iaf_flow = iaf_flow_emul if mode is not None else _PLAIN
    try:
        yield
    finally:
        O.iaf_flow = _PLAIN
        MODE.clear()
        REAL[0], REAL[1] = False, None
