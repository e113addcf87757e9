"""CPU restatement of the reference NMA-VI ELBO training step (float64 by default).

TEST INFRASTRUCTURE ONLY.  This module is the checker, never the product: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import it.  The product path (``viforssms_amd``) runs HIP kernels through
``libvissm.so`` and fails loudly when that library is missing.

Parity status: the reference computes in TensorFlow 1.8, which cannot be
installed here, so this restatement is pinned by
  * the reference's own data files (``dat/``) and the numpy-RNG replay produced
    by importing the reference's ``AR_dat_gen.py`` (tests/golden/make_ref_fixtures.py),
  * closed-form known answers (tests/test_oracle.py),
  * finite differences of its own autograd gradients,
and is otherwise "parity unpinned" with respect to TF1 numerics.

Every function cites the reference file:line it restates.  The tensors use the
TF layouts: dense kernels [in, out], conv1d kernels [k, C_in, C_out].
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

DT = torch.float64
LOG_2PI = math.log(2.0 * math.pi)
BN_SCALE = 1.0 / math.sqrt(1.0 + 1e-3)  # tf.layers.batch_normalization(training=False), eps 1e-3


# --------------------------------------------------------------------------------------
# elementwise helpers (TF 1.8 semantics)
# --------------------------------------------------------------------------------------
def elu(x):
    return torch.where(x > 0, x, torch.expm1(torch.clamp(x, max=0.0)))


def softplus(x):
    return torch.nn.functional.softplus(x)


def normal_logpdf(x, loc, scale):
    """tfd.Normal.log_prob: -0.5((x-mu)/s)^2 - log s - 0.5 log 2pi."""
    z = (x - loc) / scale
    return -0.5 * z * z - torch.log(torch.abs(scale) if torch.is_tensor(scale) else torch.tensor(abs(scale), dtype=x.dtype)) - 0.5 * LOG_2PI


def dense(x, w, b, act=None):
    """tf.layers.dense on the last axis (AR.py:55, :63-68)."""
    y = x @ w + b
    return act(y) if act is not None else y


def conv1d_valid(x, w, b, stride=1):
    """tf.layers.conv1d(padding='valid'): out[t] = sum_j x[s*t + j] . W[j] + b (AR.py:61-62).

    Evaluated as one [n_out, C] x [C, H] product per tap, so the memory stays O(L C) even for
    LV's kernel_ext-channel input (lotka_volterra_partial.py:78-79)."""
    k = w.shape[0]
    L = x.shape[1]
    n_out = (L - k) // stride + 1
    out = b
    for j in range(k):
        out = out + x[:, j: j + (n_out - 1) * stride + 1: stride, :] @ w[j]
    return out


# --------------------------------------------------------------------------------------
# q(theta): Chain of Invert(MaskedAutoregressiveFlow) and Permute (AR.py:377-391)
# --------------------------------------------------------------------------------------
def tf_gen_mask(num_blocks: int, n_in: int, n_out: int, exclusive: bool) -> np.ndarray:
    """Restatement of tfb masked_autoregressive._gen_slices/_gen_mask (TF 1.8): returns [n_out, n_in]."""
    mask = np.zeros([n_out, n_in], dtype=np.float64)
    d_in = n_in // num_blocks
    d_out = n_out // num_blocks
    row = d_out if exclusive else 0
    col = 0
    for _ in range(num_blocks):
        mask[row:, col:col + d_in] = 1.0
        col += d_in
        row += d_out
    return mask


def made_masks(D: int, hidden: Sequence[int]) -> List[np.ndarray]:
    """Masks (in x out) of masked_autoregressive_default_template(hidden_layers) for event size D."""
    masks = []
    n_in = D
    for i, units in enumerate(hidden):
        masks.append(tf_gen_mask(D, n_in, units, exclusive=(i == 0)).T)
        n_in = units
    masks.append(tf_gen_mask(D, n_in, 2 * D, exclusive=False).T)
    return masks


def made_shift_log_scale(x, layers, act):
    """shift_and_log_scale_fn of the default template; log_scale clipped to [-5, 3] with
    straight-through gradient (_clip_by_value_preserve_grad)."""
    h = x
    n = len(layers)
    for i, (w, b, m) in enumerate(layers):
        h = h @ (w * m) + b
        if i < n - 1:
            h = act(h)
    h = h.reshape(*x.shape, 2)
    shift, ls = h[..., 0], h[..., 1]
    ls = ls + (torch.clamp(ls, -5.0, 3.0) - ls).detach()
    return shift, ls


def qtheta_sample_logprob(x0, base_loc, base_scale, bijectors, act):
    """theta = Chain(reversed(bijectors)).forward(x0): bijectors[0] applied first (AR.py:386).

    bijectors: list of ("maf", layers) | ("perm", perm).  Invert(MAF).forward(z) =
    (z - shift(z)) * exp(-log_scale(z)), fldj = -sum log_scale(z).  log q(theta) =
    log N(x0) - sum fldj (TransformedDistribution.log_prob through the cached inverse).
    """
    logq = normal_logpdf(x0, base_loc, base_scale).sum(-1)
    z = x0
    for kind, spec in bijectors:
        if kind == "maf":
            shift, ls = made_shift_log_scale(z, spec, act)
            z = (z - shift) * torch.exp(-ls)
            logq = logq + ls.sum(-1)
        else:
            z = z[..., list(spec)]
    return z, logq


# --------------------------------------------------------------------------------------
# the IAF flow (AR.py:38-89; lotka_volterra_partial.py:55-108; SV_dense.py:37-89; fitz_nag_NVP.py:56-109)
# --------------------------------------------------------------------------------------
@dataclass
class FlowCfg:
    k: int                 # kernel_len
    H: int                 # network_dims[0]
    n_hidden: int          # len(network_dims) - 2
    n_logsig: int          # batch_dims (1-D) or 2*batch_dims (2-D)
    stride2: bool = False  # LV/FHN head stride 2 with (0,1)-interleave
    bn: bool = False       # LV/SV/FHN batch_normalization(training=False) after each hidden ELU
    feat: str = "mlp4"     # "mlp4" (AR/FHN), "sv" (SV diff-augmented mlp4), "lv" (time-mixing)


def flow_features(ts, P, cfg: FlowCfg):
    """Window-shared feature branch of one IAF: returns F [p, L-1, C_F]."""
    if cfg.feat == "mlp4":            # AR.py:53-56, fitz_nag_NVP.py:71-74
        h = ts[:, :-1, :]
        for i in range(4):
            h = dense(h, P[f"feat_w{i}"], P[f"feat_b{i}"], elu)
        return h
    if cfg.feat == "sv":              # SV_dense.py:53-56
        h = torch.cat([ts[:, 1:, :], ts[:, 1:, :-2] - ts[:, :-1, :-2]], 2)
        for i in range(4):
            h = dense(h, P[f"feat_w{i}"], P[f"feat_b{i}"], elu)
        return h
    if cfg.feat == "lv":              # lotka_volterra_partial.py:71-76
        h = ts[:, :-1, :]
        for i in range(3):
            h = dense(h, P[f"feat_w{i}"], P[f"feat_b{i}"], elu)
        h = dense(h, P["feat_w3"], P["feat_b3"], elu)   # units = feat_dims
        return h.transpose(1, 2)
    raise ValueError(cfg.feat)


def theta_term(theta, P):
    """Three linear dense layers on theta (AR.py:63-68)."""
    t = dense(theta, P["th_w0"], P["th_b0"])
    t = dense(t, P["th_w1"], P["th_b1"])
    return dense(t, P["th_w2"], P["th_b2"])


def iaf_flow(u, CF, theta, P, cfg: FlowCfg):
    """One IAF._create_flow: returns (u_next [p, L-k], sigma_log [p, n_logsig]).

    The first conv acts on concat(u[:, :-1], F) (AR.py:58-62); it is linear in its input
    channels, so it is evaluated as conv(u channel) + CF, CF = conv(F channels) + bias from
    `window_conv` (computed once per distinct window and gathered per sample)."""
    a = conv1d_valid(u[:, :-1, None], P["conv_w"][:, :1, :], 0.0) + CF + theta_term(theta, P)[:, None, :]
    h = elu(a)
    for l in range(cfg.n_hidden):
        h = elu(h @ P[f"hid_w{l}"] + P[f"hid_b{l}"])
        if cfg.bn:
            h = P[f"bn_g{l}"] * h * BN_SCALE + P[f"bn_b{l}"]
    s = 2 if cfg.stride2 else 1
    head = h[:, ::s, :] @ P["head_w"] + P["head_b"]
    mu_t, s_t = head[..., 0], head[..., 1]
    sig_t = softplus(s_t) + 1e-10
    if cfg.stride2:
        mu = torch.stack([torch.zeros_like(mu_t), mu_t], -1).reshape(u.shape[0], -1)
        sig = torch.stack([torch.ones_like(sig_t), sig_t], -1).reshape(u.shape[0], -1)
    else:
        mu, sig = mu_t, sig_t
    sigma_log = torch.log(sig[:, -cfg.n_logsig:])
    return u[:, cfg.k:] * sig + mu, sigma_log


def window_conv(F, P):
    """Feature channels of the first conv plus its bias, for each distinct window: [w, L-k, H]."""
    return conv1d_valid(F, P["conv_w"][:, 1:, :], P["conv_b"])


def swap_pairs(x):
    """Permute between 2-D flows: scatter_nd with perm list [1,0,3,2,...] (lotka_volterra_partial.py:207-213)."""
    p, L = x.shape
    return x.reshape(p, L // 2, 2).flip(-1).reshape(p, L)


def flow_stack(eps, conv_feats, theta, flows_P, cfg: FlowCfg, permute: bool):
    """Flow_Stack (AR.py:92-110; LV adds Permute between flows, last one dropped, lotka_volterra_partial.py:277-288).

    conv_feats[i] is flow i's per-sample feature-channel conv term (window_conv gathered per sample).
    Returns (sample, log q)."""
    base_lp = normal_logpdf(eps, 0.0, 1.0)[:, -cfg.n_logsig:].sum(1)   # init_dist.slp (AR.py:31-35)
    u = eps
    lq = base_lp
    n = len(flows_P)
    for i in range(n):
        u, sl = iaf_flow(u, conv_feats[i], theta, flows_P[i], cfg)
        lq = lq - sl.sum(1)
        if permute and i < n - 1:
            u = swap_pairs(u)
    return u, lq


# --------------------------------------------------------------------------------------
# ELBO per model
# --------------------------------------------------------------------------------------
def prior_logprob(theta, priors):
    mean = torch.tensor([m for m, _ in priors], dtype=theta.dtype)
    sd = torch.tensor([s for _, s in priors], dtype=theta.dtype)
    return normal_logpdf(theta, mean, sd).sum(-1)


def ar_elbo_terms(x, theta, obs_eval, obs_bin, obs_std):
    """AR.py:168-176: obs log-lik and AR(1) transition log-density; x [p, M+1]."""
    obs_lp = (normal_logpdf(x[:, 1:], obs_eval, torch.tensor(obs_std, dtype=x.dtype)) * obs_bin).sum(1)
    loc = theta[:, 1:2] * x[:, :-1] + theta[:, 0:1]
    scale = torch.exp(theta[:, 2:3])
    sde_lp = normal_logpdf(x[:, 1:], loc, scale).sum(1)
    return sde_lp, obs_lp


def lv_transform(z, mask, shift):
    """lotka_volterra_partial.py:290-297: x = softplus(z)*mask + shift; ILDJ over [:, :, 1:]."""
    p = z.shape[0]
    zz = z.reshape(p, -1, 2).transpose(1, 2)
    x = softplus(zz) * mask + shift
    ildj = (-torch.log(-torch.expm1(-x[:, :, 1:]))).sum((1, 2))
    return x, ildj


def lv_elbo_terms(x, theta, obs_eval, bin_feed, dt):
    """lotka_volterra_partial.py:234-261: obs N(.,1) and the Cholesky EM density (theta exp'd)."""
    obs_lp = (normal_logpdf(x[:, :, 1:], obs_eval, torch.tensor(1.0, dtype=x.dtype)) * bin_feed).sum((1, 2))
    th = torch.exp(theta)
    t0, t1, t2 = th[:, 0:1], th[:, 1:2], th[:, 2:3]
    x1, x2 = x[:, 0, :-1], x[:, 1, :-1]
    d1 = x[:, 0, 1:] - x1
    d2 = x[:, 1, 1:] - x2
    m1 = dt * (t0 * x1 - t1 * x1 * x2)
    m2 = dt * (t1 * x1 * x2 - t2 * x2)
    a = torch.sqrt(t0 * x1 + t1 * x1 * x2)
    b = -t1 * x1 * x2 / a
    c = torch.sqrt(t1 * x1 * x2 + t2 * x2 - b ** 2)
    # det = prod(diag(chol))^2, cov = chol chol^T with chol = sqrt(dt) [[a,0],[b,c]]
    det = (dt * a * c) ** 2
    s11 = dt * a * a
    s12 = dt * a * b
    s22 = dt * (b * b + c * c)
    q1, q2 = d1 - m1, d2 - m2
    inv_det = 1.0 / (s11 * s22 - s12 * s12)
    quad = (s22 * q1 * q1 - 2 * s12 * q1 * q2 + s11 * q2 * q2) * inv_det
    sde_lp = (-0.5 * torch.log(det) - 0.5 * quad - LOG_2PI).sum(1)
    return sde_lp, obs_lp


def sv_elbo_terms(x, theta, dt):
    """SV_dense.py:203-223: diagonal EM density; x [p, 2, M+1] = [dim_one; latent]."""
    x1, x2 = x[:, 0, :-1], x[:, 1, :-1]
    d1 = x[:, 0, 1:] - x1
    d2 = x[:, 1, 1:] - x2
    m1 = dt * (theta[:, 0:1] * x1)
    m2 = dt * (theta[:, 1:2] - torch.exp(theta[:, 2:3]) * x2)
    sq = math.sqrt(dt)
    s1 = sq * (x1 * torch.exp(0.5 * x2))
    s2 = sq * torch.exp(theta[:, 3:4]).expand_as(x1)
    sde_lp = (normal_logpdf(d1, m1, s1) + normal_logpdf(d2, m2, s2)).sum(1)
    return sde_lp


def fhn_elbo_terms(x, theta, obs_eval, bin_feed, dt, obs_sd=0.1):
    """fitz_nag_NVP.py:232-255: obs N(., 0.1) and diagonal EM density (theta raw)."""
    obs_lp = (normal_logpdf(x[:, :, 1:], obs_eval, torch.tensor(obs_sd, dtype=x.dtype)) * bin_feed).sum((1, 2))
    x1, x2 = x[:, 0, :-1], x[:, 1, :-1]
    d1 = x[:, 0, 1:] - x1
    d2 = x[:, 1, 1:] - x2
    m1 = dt * (torch.exp(theta[:, 0:1]) * (x1 - x1 ** 3 - x2 + theta[:, 1:2]))
    m2 = dt * (theta[:, 2:3] * x1 - x2 + 1.4)
    sq = math.sqrt(dt)
    s1 = (sq * torch.sqrt(torch.exp(theta[:, 3:4]))).expand_as(x1)
    s2 = (sq * torch.sqrt(torch.exp(theta[:, 4:5]))).expand_as(x1)
    sde_lp = (normal_logpdf(d1, m1, s1) + normal_logpdf(d2, m2, s2)).sum(1)
    return sde_lp, obs_lp


# --------------------------------------------------------------------------------------
# optimiser (AR.py:226-234, optimisers/adamax.py:42-58)
# --------------------------------------------------------------------------------------
def clip_by_global_norm(grads: List[torch.Tensor], clip: float):
    """tf.clip_by_global_norm: scale = clip * min(1/norm, 1/clip); inf norm -> NaN."""
    gn = torch.sqrt(sum((g.double() ** 2).sum() for g in grads))
    scale = clip * torch.minimum(1.0 / gn, torch.tensor(1.0 / clip, dtype=gn.dtype))
    if not torch.isfinite(gn):
        scale = torch.tensor(float("nan"), dtype=gn.dtype)
    return [g * scale.to(g.dtype) for g in grads], gn


def adamax_update(var, grad, v, m, lr, beta1, beta2, eps=1e-8):
    """AdamaxOptimizer._apply_dense: slot v = first moment, slot m = inf-norm, no bias correction."""
    v_new = beta1 * v + (1.0 - beta1) * grad
    m_new = torch.maximum(beta2 * m + eps, grad.abs())
    return var - lr * v_new / m_new, v_new, m_new


# --------------------------------------------------------------------------------------
# full model: parameters + ELBO for each family
# --------------------------------------------------------------------------------------
@dataclass
class ModelSpec:
    family: str            # "ar" | "lv" | "sv" | "fhn"
    p: int
    M: int                 # reference batch_dims (window length)
    k: int
    n_flows: int
    H: int
    n_layers: int          # len(network_dims)
    C_time: int            # channels of time_feats
    P_theta: int
    target: float          # T (AR) or target_dims (LV/SV/FHN), the T/M scaling numerator
    priors: list
    dt: float = 1.0
    obs_std: float = 1.0
    theta_act: str = "elu"
    base_loc: float = 0.0
    base_scale: float = 1.0
    n_maf: int = 5

    @property
    def D(self):
        return 2 if self.family in ("lv", "fhn") else 1

    @property
    def kernel_ext(self):
        return self.k * self.n_flows + self.D * self.M + self.D

    def flow_cfg(self):
        return FlowCfg(k=self.k, H=self.H, n_hidden=self.n_layers - 2, n_logsig=self.D * self.M,
                       stride2=self.D == 2, bn=self.family != "ar",
                       feat={"ar": "mlp4", "fhn": "mlp4", "sv": "sv", "lv": "lv"}[self.family])


def init_params(spec: ModelSpec, gen: torch.Generator, scale: float = 1.0, dtype=DT):
    """Random parameters in TF layouts (glorot-uniform-like; biases small random so every
    parameter's gradient path is exercised in parity tests)."""
    def glorot(shape, fan_in, fan_out):
        lim = math.sqrt(6.0 / (fan_in + fan_out)) * scale
        return (torch.rand(shape, generator=gen, dtype=dtype) * 2 - 1) * lim

    def bias(n):
        return (torch.rand(n, generator=gen, dtype=dtype) * 2 - 1) * 0.1 * scale

    H, k = spec.H, spec.k
    flows = []
    for i in range(spec.n_flows):
        P = {}
        if spec.family == "lv":
            cin = spec.C_time
            for j in range(3):
                P[f"feat_w{j}"] = glorot((cin, H), cin, H)
                P[f"feat_b{j}"] = bias(H)
                cin = H
            fd = spec.kernel_ext - 1 - i * k
            P["feat_w3"] = glorot((H, fd), H, fd)
            P["feat_b3"] = bias(fd)
            cf = spec.kernel_ext - 1
        else:
            cin = spec.C_time + (spec.C_time - 2 if spec.family == "sv" else 0)
            for j in range(4):
                P[f"feat_w{j}"] = glorot((cin, H), cin, H)
                P[f"feat_b{j}"] = bias(H)
                cin = H
            cf = H
        P["conv_w"] = glorot((k, 1 + cf, H), k * (1 + cf), k * H)
        P["conv_b"] = bias(H)
        P["th_w0"] = glorot((spec.P_theta, H), spec.P_theta, H)
        P["th_b0"] = bias(H)
        P["th_w1"] = glorot((H, H), H, H)
        P["th_b1"] = bias(H)
        P["th_w2"] = glorot((H, H), H, H)
        P["th_b2"] = bias(H)
        for l in range(spec.n_layers - 2):
            P[f"hid_w{l}"] = glorot((H, H), H, H)
            P[f"hid_b{l}"] = bias(H)
            if spec.family != "ar":
                P[f"bn_g{l}"] = 1.0 + bias(H)
                P[f"bn_b{l}"] = bias(H)
        P["head_w"] = glorot((H, 2), H, 2)
        P["head_b"] = bias(2)
        flows.append(P)
    masks = made_masks(spec.P_theta, [5, 5, 5])
    mafs = []
    for i in range(spec.n_maf):
        layers = []
        for m in masks:
            w = glorot(m.shape, m.shape[0], m.shape[1]) * torch.tensor(m, dtype=dtype)
            layers.append((w, bias(m.shape[1]) * 0.5, torch.tensor(m, dtype=dtype)))
        mafs.append(layers)
    return {"flows": flows, "mafs": mafs}


def param_leaves(params) -> List[torch.Tensor]:
    leaves = []
    for P in params["flows"]:
        leaves += [P[n] for n in sorted(P)]
    for layers in params["mafs"]:
        for w, b, _ in layers:
            leaves += [w, b]
    return leaves


def build_bijectors(params, perms):
    bij = []
    n = len(params["mafs"])
    for i in range(n):
        bij.append(("maf", params["mafs"][i]))
        if i < n - 1:
            bij.append(("perm", perms[i]))
    return bij


def elbo(spec: ModelSpec, params, perms, x0_theta, eps, time_feats, extra):
    """Per-sample ELBO [p] and diagnostics, with injected randomness.

    x0_theta: base sample of q(theta) [p, P_theta]; eps: MA base noise [p, kernel_ext];
    time_feats: [p, kernel_ext, C_time]; extra: model-specific feeds (obs_bin, mask, shift, ...).
    """
    act = torch.relu if spec.theta_act == "relu" else elu
    theta, logq_theta = qtheta_sample_logprob(x0_theta, spec.base_loc, spec.base_scale,
                                              build_bijectors(params, perms), act)
    cfg = spec.flow_cfg()
    # the feature branch and the feature channels of the first conv depend on the window only:
    # evaluate them once per distinct time_feats row and gather per sample
    uniq, inv = torch.unique(time_feats, dim=0, return_inverse=True)
    feats = []
    for i in range(spec.n_flows):
        ts = uniq if spec.family == "lv" else uniq[:, i * spec.k:, :]
        P = params["flows"][i]
        feats.append(window_conv(flow_features(ts, P, cfg), P)[inv])
    z, lq = flow_stack(eps, feats, theta, params["flows"], cfg, permute=spec.D == 2)
    scale = spec.target / spec.M
    prior = prior_logprob(theta, spec.priors)
    out = {"theta": theta, "logq_theta": logq_theta, "prior": prior}
    if spec.family == "ar":
        M = spec.M
        obs_eval = time_feats[:, -M:, 0]
        obs_bin = time_feats[:, -M:, -1]
        sde, obs = ar_elbo_terms(z, theta, obs_eval, obs_bin, spec.obs_std)
        out.update(x=z, sde=sde, obs=obs, logq=lq)
        out["elbo"] = scale * (sde - lq + obs) + prior - logq_theta
    elif spec.family == "lv":
        x, ildj = lv_transform(z, extra["mask"], extra["shift"])
        lq = lq + ildj
        p = z.shape[0]
        obs_eval = time_feats[:, -2 * spec.M:, 0].reshape(p, -1, 2).transpose(1, 2)
        sde, obs = lv_elbo_terms(x, theta, obs_eval, extra["bin"], spec.dt)
        out.update(x=x, sde=sde, obs=obs, logq=lq)
        out["elbo"] = scale * (sde - lq + obs) + prior - logq_theta
    elif spec.family == "sv":
        x2 = z * extra["mask"] + extra["shift"]
        x = torch.stack([extra["dim_one"], x2], 1)
        sde = sv_elbo_terms(x, theta, spec.dt)
        out.update(x=x, sde=sde, obs=torch.zeros_like(sde), logq=lq)
        out["elbo"] = scale * (sde - lq) + prior - logq_theta
    elif spec.family == "fhn":
        p = z.shape[0]
        x = z.reshape(p, -1, 2).transpose(1, 2)
        obs_eval = time_feats[:, -2 * spec.M:, 0].reshape(p, -1, 2).transpose(1, 2)
        sde, obs = fhn_elbo_terms(x, theta, obs_eval, extra["bin"], spec.dt)
        out.update(x=x, sde=sde, obs=obs, logq=lq)
        out["elbo"] = scale * (sde - lq + obs) + prior - logq_theta
    else:
        raise ValueError(spec.family)
    return out


def train_step(spec: ModelSpec, params, slots, perms, x0_theta, eps, time_feats, extra,
               lr, beta1=0.95, beta2=0.999, clip=2.5e8):
    """One full reference step: grad of sum(-ELBO) (AR.py:228-229), clip_by_global_norm
    (AR.py:230-232), Adamax apply (optimisers/adamax.py:42-58).  Returns (new params, new slots, info)."""
    leaves = param_leaves(params)
    for t in leaves:
        t.requires_grad_(True)
    out = elbo(spec, params, perms, x0_theta, eps, time_feats, extra)
    loss = (-out["elbo"]).sum()
    grads = torch.autograd.grad(loss, leaves, allow_unused=True)
    grads = [torch.zeros_like(t) if g is None else g for t, g in zip(leaves, grads)]
    clipped, gn = clip_by_global_norm(grads, clip)
    new_leaves, new_slots = [], []
    for t, g, (v, m) in zip(leaves, clipped, slots):
        nt, nv, nm = adamax_update(t.detach(), g, v, m, lr, beta1, beta2)
        new_leaves.append(nt)
        new_slots.append((nv, nm))
    for t in leaves:
        t.requires_grad_(False)
    return new_leaves, new_slots, {"loss": loss.detach(), "global_norm": gn, "grads": grads,
                                   "elbo": out["elbo"].detach()}


# --------------------------------------------------------------------------------------
# host-side data / feature assembly (independent restatement, used to check the product's)
# --------------------------------------------------------------------------------------
def ar_time_feats(obs, obs_bin, time_till, n_flows, k, M, fw, T, starts):
    """AR.py:135-150 + AR.py:267-283: time_feats [p, kernel_ext, fw+4]."""
    pad = n_flows * k + 1
    kext = pad + M
    obs_pad = [np.concatenate((np.zeros(pad - i), obs, np.zeros(i))) for i in range(fw)]
    time_pad = np.concatenate((np.zeros(pad), np.arange(int(T) + 1)))
    bin_feats = np.concatenate((np.ones(pad), np.zeros(int(T))))
    obs_bin_p = np.concatenate((np.zeros(pad), obs_bin))
    tt = np.concatenate((np.arange(pad + time_till[0], time_till[0], -1), time_till))
    chans = obs_pad + [bin_feats, time_pad, tt, obs_bin_p]
    out = np.zeros((len(starts), kext, fw + 4))
    for r, s in enumerate(starts):
        for c, arr in enumerate(chans):
            out[r, :, c] = arr[s:s + kext]
    return out


def _gather_rows(arr, idx, length):
    """[len(idx), length] = arr[i : i + length] for each start i (the reference's per-start slices)."""
    return np.stack([np.asarray(arr[int(i):int(i) + length]) for i in idx])


def pair_time_feats(family, obs, obs_bin, time_till, x0, dt, T, target_dims, n_flows, k, M, fw, starts):
    """LV / FHN host feeds for window starts `starts` (reference batch_select):
    LV lotka_volterra_partial.py:185-204 (arrays) + :366-386 (per-step gather);
    FHN fitz_nag_NVP.py:182-202 + :346-366.

    Returns dict(time_feats [p, kext, fw+3], mask [p,2,M+1], shift [p,2,M+1], bin [p,2,M]).
    The two families differ in bin_feats (LV zeros then ones, FHN ones then zeros) and in the
    time_till pad arange, which FHN runs down to -dt (one pair longer than the other pads)."""
    D = 2
    lead = n_flows * k + D                                 # zeros before the series in every pad
    kext = n_flows * k + D * M + 2
    series = np.asarray(obs).T.reshape(-1)                 # np.reshape(obs, -1, 'F'): t-major interleave
    lag_arrays = []
    for lag in range(0, 5 * fw, 5):
        lag_arrays.append(np.concatenate((np.zeros(lead - lag), series, np.zeros(lag))))
    times = np.concatenate((np.zeros(lead), np.repeat(np.arange(dt, T + dt, dt), D)))
    stop = 0.0 if family == "lv" else -dt
    head = np.arange(np.round(lead * (dt / D), 1), stop, -dt)
    tt_pad = np.repeat(head, D).reshape(-1, D).T          # np.reshape(np.repeat(.), (2, -1), 'F')
    till = np.concatenate((tt_pad, np.asarray(time_till)), 1).T.reshape(-1)
    if family == "lv":
        binf = np.float32(np.concatenate((np.zeros(lead), np.ones(target_dims * D))))
    else:
        binf = np.float32(np.concatenate((np.ones(lead), np.zeros(target_dims * D))))
    mask_vals = np.concatenate((np.zeros((2, 1)), np.ones((D, target_dims))), axis=1)
    shift_vals = np.concatenate((np.asarray(x0, dtype=np.float64)[:, None], np.zeros((D, target_dims))), axis=1)
    idx = D * np.asarray(starts, dtype=np.int64)
    chans = [_gather_rows(a, idx, kext) for a in lag_arrays]
    chans += [_gather_rows(binf, idx, kext), _gather_rows(times, idx, kext), _gather_rows(till, idx, kext)]
    ts = np.stack(chans, axis=2).astype(np.float64)
    st = np.asarray(starts, dtype=np.int64)
    mask = np.stack([mask_vals[:, s:s + M + 1] for s in st])
    shift = np.stack([shift_vals[:, s:s + M + 1] for s in st])
    ob = np.asarray(obs_bin, dtype=np.float64)
    binfeed = np.stack([ob[:, s:s + M] for s in st])
    return {"time_feats": ts, "mask": mask, "shift": shift, "bin": binfeed}


def sv_time_feats(obs, x0, dt, T, target_dims, n_flows, k, M, fw, starts):
    """SV host feeds (SV_dense.py:159-185 arrays, :304-328 per-step gather).

    Channels [obs lags 0,5,..,5(fw-1); time; rolling var of obs; log rolling var of the
    differences], rolling windows of kernel_len on the float32 series as loaded.
    Returns dict(time_feats [p, kext, fw+3], mask [p, M+1], shift [p, M+1], dim_one [p, M+1])."""
    obs = np.asarray(obs)
    n = obs.shape[0]
    lead = n_flows * k
    kext = n_flows * k + M + 1
    rv = np.array([np.var(obs[i:i + k]) for i in range(n - k)])
    dif = obs[1:] - obs[:-1]
    rvd = np.array([np.var(dif[i:i + k]) for i in range(dif.shape[0] - k)])
    var_pad = np.concatenate((np.zeros(lead + k), rv))
    var_diff_pad = np.concatenate((np.zeros(lead + k), np.log(rvd), np.zeros(1)))
    lag_arrays = [np.concatenate((np.zeros(lead - lag), obs, np.zeros(lag))) for lag in range(0, 5 * fw, 5)]
    times = np.concatenate((np.zeros(lead + 1), np.arange(0.1, T + dt, dt)))
    st = np.asarray(starts, dtype=np.int64)
    chans = [_gather_rows(a, st, kext) for a in lag_arrays]
    chans += [_gather_rows(times, st, kext), _gather_rows(var_pad, st, kext), _gather_rows(var_diff_pad, st, kext)]
    ts = np.stack([c.astype(np.float64) for c in chans], axis=2)
    mask_vals = np.concatenate((np.zeros(1), np.ones(target_dims)))
    shift_vals = np.concatenate((np.array([x0], dtype=np.float64), np.zeros(target_dims)))
    return {"time_feats": ts,
            "mask": np.stack([mask_vals[s:s + M + 1] for s in st]),
            "shift": np.stack([shift_vals[s:s + M + 1] for s in st]),
            "dim_one": np.stack([obs[s:s + M + 1].astype(np.float64) for s in st])}
