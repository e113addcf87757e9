"""Pins the CPU oracle (float64 restatement of the reference) with closed-form known answers,
library cross-checks and finite differences."""
import math

import numpy as np
import pytest
import torch
from scipy import stats

from oracle import nma_oracle as O

DT = O.DT


def test_adamax_first_step_known_answer():
    """m = max(1e-8, |g|), v = (1-b1) g  =>  delta = -lr (1-b1) sign(g)  (optimisers/adamax.py:51-57)."""
    g = torch.tensor([0.3, -2.0, 5e-9, 0.0], dtype=DT)
    var = torch.ones(4, dtype=DT)
    nv, v, m = O.adamax_update(var, g, torch.zeros(4, dtype=DT), torch.zeros(4, dtype=DT), 1e-3, 0.95, 0.999)
    assert torch.allclose(v, 0.05 * g)
    assert torch.allclose(m, torch.tensor([0.3, 2.0, 1e-8, 1e-8], dtype=DT))
    assert torch.allclose(nv[:2], 1 - 1e-3 * 0.05 * torch.sign(g[:2]))
    assert nv[3] == 1.0


def test_clip_identity_and_scaling():
    gs = [torch.tensor([3.0, 4.0], dtype=DT)]
    c, n = O.clip_by_global_norm(gs, 10.0)
    assert n == 5.0 and torch.equal(c[0], gs[0])
    c, n = O.clip_by_global_norm(gs, 1.0)
    assert torch.allclose(c[0], gs[0] / 5.0)
    c, n = O.clip_by_global_norm([torch.tensor([float("inf")], dtype=DT)], 1.0)
    assert torch.isnan(c[0]).all()


def test_zero_weight_flow_analytic_logq():
    """All MA weights zero => mu = head_b[0], sigma = softplus(head_b[1]) + 1e-10 everywhere."""
    cfg = O.FlowCfg(k=3, H=4, n_hidden=1, n_logsig=5)
    P = {n: torch.zeros(s, dtype=DT) for n, s in [("conv_w", (3, 5, 4)), ("conv_b", (4,)), ("th_w0", (2, 4)),
                                                  ("th_b0", (4,)), ("th_w1", (4, 4)), ("th_b1", (4,)),
                                                  ("th_w2", (4, 4)), ("th_b2", (4,)), ("hid_w0", (4, 4)),
                                                  ("hid_b0", (4,)), ("head_w", (4, 2))]}
    P["head_b"] = torch.tensor([0.7, -0.3], dtype=DT)
    u = torch.randn(2, 12, dtype=DT)
    F = torch.randn(2, 11, 4, dtype=DT)
    out, sl = O.iaf_flow(u, O.window_conv(F, P), torch.randn(2, 2, dtype=DT), P, cfg)
    sig = math.log1p(math.exp(-0.3)) + 1e-10
    assert torch.allclose(out, u[:, 3:] * sig + 0.7)
    assert torch.allclose(sl, torch.full((2, 5), math.log(sig), dtype=DT))


@pytest.mark.parametrize("stride", [1, 2])
def test_conv1d_valid_matches_torch_conv(stride):
    """The per-tap product form of tf.layers.conv1d(padding='valid') equals torch's own conv1d
    (cross-correlation, channels-last kernel [k, C_in, C_out])."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 41, 7, generator=g, dtype=DT)
    w = torch.randn(6, 7, 5, generator=g, dtype=DT)
    b = torch.randn(5, generator=g, dtype=DT)
    ref = torch.nn.functional.conv1d(x.transpose(1, 2), w.permute(2, 1, 0), b, stride=stride).transpose(1, 2)
    assert torch.allclose(O.conv1d_valid(x, w, b, stride), ref, rtol=1e-12, atol=1e-12)


def test_ar_density_known_points():
    x = torch.tensor([[10.0, 12.0, 9.0]], dtype=DT)
    th = torch.tensor([[5.0, 0.5, math.log(3.0)]], dtype=DT)
    sde, obs = O.ar_elbo_terms(x, th, torch.tensor([[11.0, 9.5]], dtype=DT), torch.tensor([[1.0, 0.0]], dtype=DT),
                               1.0)
    ref = stats.norm(0.5 * 10 + 5, 3).logpdf(12) + stats.norm(0.5 * 12 + 5, 3).logpdf(9)
    assert abs(float(sde) - ref) < 1e-12
    assert abs(float(obs) - stats.norm(11.0, 1.0).logpdf(12.0)) < 1e-12


def test_lv_density_vs_scipy():
    x = torch.tensor([[[100.0, 103.0, 98.0], [90.0, 88.0, 91.0]]], dtype=DT)
    theta = torch.log(torch.tensor([[0.5, 0.0025, 0.3]], dtype=DT))
    sde, _ = O.lv_elbo_terms(x, theta, torch.zeros(1, 2, 2, dtype=DT), torch.zeros(1, 2, 2, dtype=DT), 0.1)
    th = [0.5, 0.0025, 0.3]
    ref = 0.0
    for t in range(2):
        x1, x2 = x[0, 0, t].item(), x[0, 1, t].item()
        mu = 0.1 * np.array([th[0] * x1 - th[1] * x1 * x2, th[1] * x1 * x2 - th[2] * x2])
        A = th[0] * x1 + th[1] * x1 * x2
        B = th[1] * x1 * x2
        C = B + th[2] * x2
        cov = 0.1 * np.array([[A, -B], [-B, C]])
        d = (x[0, :, t + 1] - x[0, :, t]).numpy()
        ref += stats.multivariate_normal(mu, cov).logpdf(d)
    assert abs(float(sde) - ref) < 1e-9


def test_made_masks_autoregressive():
    """Output d of the MADE net depends only on inputs < d (Invert(MAF) is then triangular)."""
    from viforssms_amd.theta_flow import made_masks
    for D in (3, 4, 5):
        ms = made_masks(D)
        conn = np.eye(D)
        for m in ms:
            conn = (conn @ m > 0).astype(float)
        conn = conn.reshape(D, D, 2)  # input x output-dim x (shift, log_scale)
        for d in range(D):
            assert conn[d:, d, :].sum() == 0, (D, d)
        assert np.array_equal(ms[0], O.made_masks(D, [5, 5, 5])[0])


def _small_problem(family, seed=0):
    g = torch.Generator().manual_seed(seed)
    if family == "ar":
        spec = O.ModelSpec("ar", p=2, M=6, k=2, n_flows=2, H=3, n_layers=3, C_time=5, P_theta=3, target=12.0,
                           priors=[(0.0, 10.0)] * 3, base_loc=1.5, base_scale=0.5, n_maf=2)
        ts = torch.randn(2, spec.kernel_ext, 5, generator=g, dtype=DT)
        extra = {}
    else:
        spec = O.ModelSpec("lv", p=2, M=4, k=2, n_flows=2, H=3, n_layers=4, C_time=3, P_theta=3, target=4.0,
                           priors=[(-0.8, 1.0)] * 3, dt=0.1, n_maf=2)
        ts = torch.randn(2, spec.kernel_ext, 3, generator=g, dtype=DT)
        extra = {"mask": torch.ones(2, 2, 5, dtype=DT), "shift": torch.zeros(2, 2, 5, dtype=DT),
                 "bin": torch.ones(2, 2, 4, dtype=DT)}
    params = O.init_params(spec, g, scale=0.5)
    eps = torch.randn(2, spec.kernel_ext, generator=g, dtype=DT)
    x0 = torch.randn(2, 3, generator=g, dtype=DT) * 0.2
    return spec, params, eps, x0, ts, extra


@pytest.mark.parametrize("family", ["ar", "lv"])
def test_oracle_gradient_matches_finite_differences(family):
    spec, params, eps, x0, ts, extra = _small_problem(family)
    perms = [[0, 2, 1]]
    leaves = O.param_leaves(params)
    for t in leaves:
        t.requires_grad_(True)
    f = lambda: (-O.elbo(spec, params, perms, x0, eps, ts, extra)["elbo"]).sum()
    loss = f()
    grads = torch.autograd.grad(loss, leaves, allow_unused=True)
    rng = np.random.default_rng(0)
    checked = 0
    with torch.no_grad():
        for t, gr in zip(leaves, grads):
            if gr is None:
                continue
            idx = tuple(int(rng.integers(0, s)) for s in t.shape)
            h = 1e-6
            old = t[idx].item()
            t[idx] = old + h
            lp = f().item()
            t[idx] = old - h
            lm = f().item()
            t[idx] = old
            fd = (lp - lm) / (2 * h)
            assert abs(fd - gr[idx].item()) <= 1e-5 * max(1.0, abs(fd)), (t.shape, fd, gr[idx].item())
            checked += 1
    assert checked > 20
