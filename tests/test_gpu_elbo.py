"""AR(1) log-density kernels (vissm_elbo_fwd / vissm_elbo_bwd, elbo.hip ar_elbo_*_kernel) against the
float64 oracle terms (oracle/nma_oracle.py ar_elbo_terms, AR.py:168-176) and their autograd, at window
lengths around the kernel's 4-wide chunking (M < 4, M = 4..9, long odd/even M), one and several
windows, and with the obs gradient absent."""
import numpy as np
import pytest
import torch

from oracle import nma_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _case(B, M, n_win, seed):
    g = torch.Generator().manual_seed(seed)
    z = (10 + 3 * torch.randn(B, M + 1, generator=g, dtype=torch.float64))
    theta = torch.stack([5 + torch.randn(B, generator=g, dtype=torch.float64),
                         0.5 + 0.1 * torch.randn(B, generator=g, dtype=torch.float64),
                         0.3 * torch.randn(B, generator=g, dtype=torch.float64)], 1)
    obs = 10 + 3 * torch.randn(n_win, M, generator=g, dtype=torch.float64)
    obs_bin = (torch.rand(n_win, M, generator=g, dtype=torch.float64) < 0.3).double()
    win = torch.randint(0, n_win, (B,), generator=g, dtype=torch.int32)
    gs = torch.randn(B, generator=g, dtype=torch.float64)
    go = torch.randn(B, generator=g, dtype=torch.float64)
    return z, theta, obs, obs_bin, win, gs, go


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 7, 8, 9, 50, 1001, 5000])
@pytest.mark.parametrize("n_win", [1, 3])
def test_ar_elbo_kernels_match_oracle(M, n_win):
    from viforssms_amd import _lib
    from viforssms_amd.ops import ElboFeeds, elbo_terms
    B, obs_std = 37, 1.3
    z, theta, obs, obs_bin, win, gs, go = _case(B, M, n_win, seed=M * 7 + n_win)
    # oracle: float64 terms and autograd
    zr, thr = z.clone().requires_grad_(True), theta.clone().requires_grad_(True)
    wl = win.long()
    sde_r, obs_r = O.ar_elbo_terms(zr, thr, obs[wl], obs_bin[wl], obs_std)
    (sde_r * gs + obs_r * go).sum().backward()
    # HIP path
    feeds = ElboFeeds(obs=obs.float().to(DEV), obs_bin=obs_bin.float().to(DEV),
                      win=win.to(DEV) if n_win > 1 else None, n_win=n_win)
    zd = z.float().to(DEV).requires_grad_(True)
    thd = theta.float().to(DEV).requires_grad_(True)
    sde, obs_lp, _ = elbo_terms(_lib.MODEL_AR, M, 1.0, obs_std, feeds, zd, thd)
    (sde * gs.float().to(DEV) + obs_lp * go.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double()
        return float((a - b).norm() / (b.norm() + 1e-30))

    assert rel(sde, sde_r) < 1e-5
    assert rel(obs_lp, obs_r) < 1e-5
    assert rel(zd.grad, zr.grad) < 1e-5
    assert rel(thd.grad, thr.grad) < 1e-5
    # every element of dz written (no stale memory) and finite
    assert torch.isfinite(zd.grad).all()


def test_ar_elbo_bwd_without_obs_gradient():
    """g_obs absent (only the sde term is differentiated): dz has no obs contribution."""
    from viforssms_amd import _lib
    from viforssms_amd.ops import ElboFeeds, elbo_terms
    B, M, obs_std = 9, 23, 1.0
    z, theta, obs, obs_bin, win, gs, _ = _case(B, M, 1, seed=3)
    zr, thr = z.clone().requires_grad_(True), theta.clone().requires_grad_(True)
    sde_r, _ = O.ar_elbo_terms(zr, thr, obs[0:1].expand(B, -1), obs_bin[0:1].expand(B, -1), obs_std)
    (sde_r * gs).sum().backward()
    feeds = ElboFeeds(obs=obs.float().to(DEV), obs_bin=obs_bin.float().to(DEV))
    zd = z.float().to(DEV).requires_grad_(True)
    thd = theta.float().to(DEV).requires_grad_(True)
    sde, _, _ = elbo_terms(_lib.MODEL_AR, M, 1.0, obs_std, feeds, zd, thd)
    (sde * gs.float().to(DEV)).sum().backward()
    np.testing.assert_allclose(zd.grad.double().cpu().numpy(), zr.grad.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(thd.grad.double().cpu().numpy(), thr.grad.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M", [1, 3, 4, 9, 1001, 5000])
@pytest.mark.parametrize("n_win", [1, 3])
def test_ar_elbo_values_and_theta_grad_one_pass(M, n_win):
    """vissm_elbo_fwd_theta_grad (the fused training step's one pass over x): sde / obs agree with vissm_elbo_fwd
    (to fp32 rounding) and the theta gradient matches the float64 oracle's d(gs . sde)/d theta (z constant) like
    vissm_elbo_bwd's."""
    from viforssms_amd import _lib
    from viforssms_amd.ops import ElboFeeds, elbo_terms, elbo_values_and_theta_grad
    B, obs_std = 37, 1.3
    z, theta, obs, obs_bin, win, gs, go = _case(B, M, n_win, seed=M * 5 + n_win)
    thr = theta.clone().requires_grad_(True)
    wl = win.long()
    sde_r, obs_r = O.ar_elbo_terms(z, thr, obs[wl], obs_bin[wl], obs_std)
    (sde_r * gs + obs_r * go).sum().backward()
    feeds = ElboFeeds(obs=obs.float().to(DEV), obs_bin=obs_bin.float().to(DEV),
                      win=win.to(DEV) if n_win > 1 else None, n_win=n_win)
    zd, thd = z.float().to(DEV), theta.float().to(DEV)
    sde, obs_lp, dth = elbo_values_and_theta_grad(_lib.MODEL_AR, M, 1.0, obs_std, feeds, zd, thd,
                                                  gs.float().to(DEV), go.float().to(DEV))
    sde2, obs2, _ = elbo_terms(_lib.MODEL_AR, M, 1.0, obs_std, feeds, zd, thd)
    torch.cuda.synchronize()
    rel = lambda a, b: float((a.double().cpu() - b.double().cpu()).norm() / (b.double().norm() + 1e-30))
    # the same sums as vissm_elbo_fwd (the extra theta sums change the compiler's FMA contraction: an ulp or so)
    assert rel(sde, sde2) < 1e-6 and rel(obs_lp, obs2) < 1e-6
    assert rel(sde, sde_r.detach()) < 1e-5 and rel(obs_lp, obs_r.detach()) < 1e-5
    assert rel(dth, thr.grad) < 1e-5, rel(dth, thr.grad)
