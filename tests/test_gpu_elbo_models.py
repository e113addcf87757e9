"""LV / SV / FHN log-density kernels (vissm_elbo_fwd / vissm_elbo_bwd, elbo.hip stream_*_kernel<MODEL>)
against the float64 oracle terms and their autograd:
  LV  lotka_volterra_partial.py:234-261 + 290-297 (oracle lv_transform / lv_elbo_terms),
  SV  SV_dense.py:203-223 + 245-246 (sv_elbo_terms on [dim_one; z * mask + shift]),
  FHN fitz_nag_NVP.py:232-255 (fhn_elbo_terms),
at window lengths around the kernels' 4-wide chunking (M < 4, M = 4..9, the first interior chunk,
long odd / even M, the configs' own lengths), one and several windows."""
import math

import numpy as np
import pytest
import torch

from oracle import nma_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
MS = [1, 2, 3, 4, 5, 7, 8, 9, 12, 50, 1001, 1508, 2000]


def _windows_mask_shift(n_win, D, M, x0, g):
    """Reference-shaped per-window mask / shift: window 0 pins x_0 (mask 0, shift x0), later windows
    transform every entry (lotka_volterra_partial.py:381-384, SV_dense.py:322-328)."""
    mask = torch.ones(n_win, D, M + 1, dtype=torch.float64)
    shift = torch.zeros(n_win, D, M + 1, dtype=torch.float64)
    mask[0, :, 0] = 0.0
    shift[0, :, 0] = torch.as_tensor(x0, dtype=torch.float64)
    return mask, shift


def _case(model, B, M, n_win, seed):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64)
    win = torch.randint(0, n_win, (B,), generator=g, dtype=torch.int32)
    gs, go, ge = r(B), r(B), r(B)
    d = {"win": win, "gs": gs, "go": go, "ge": ge}
    if model == "lv":
        d["z"] = 100 + 10 * r(B, 2 * (M + 1))
        d["theta"] = torch.stack([math.log(0.5) + 0.1 * r(B), math.log(0.0025) + 0.1 * r(B),
                                  math.log(0.3) + 0.1 * r(B)], 1)
        d["mask"], d["shift"] = _windows_mask_shift(n_win, 2, M, [100.0, 100.0], g)
        d["obs"] = 100 + 10 * r(n_win, 2, M)
        d["bin"] = (torch.rand(n_win, 2, M, generator=g, dtype=torch.float64) < 0.2).double()
        d["dt"] = 0.1
    elif model == "sv":
        d["z"] = -8 + r(B, M + 1)
        d["theta"] = torch.stack([0.001 + 0.01 * r(B), -0.6 + 0.1 * r(B), math.log(0.08) + 0.1 * r(B),
                                  math.log(0.5) + 0.1 * r(B)], 1)
        m, s = _windows_mask_shift(n_win, 1, M, [-8.5], g)
        d["mask"], d["shift"] = m[:, 0], s[:, 0]
        d["dim_one"] = 2 + 14 * torch.rand(n_win, M + 1, generator=g, dtype=torch.float64)
        d["dt"] = 1.0
    else:
        d["z"] = r(B, 2 * (M + 1))
        d["theta"] = torch.stack([math.log(2) + 0.1 * r(B), 1 + 0.1 * r(B), 1.5 + 0.1 * r(B),
                                  math.log(0.5) + 0.1 * r(B), math.log(0.3) + 0.1 * r(B)], 1)
        d["obs"] = r(n_win, 2, M)
        d["bin"] = (torch.rand(n_win, 2, M, generator=g, dtype=torch.float64) < 0.3).double()
        d["dt"] = 0.1
    return d


def _oracle(model, d, z, theta):
    w = d["win"].long()
    B = z.shape[0]
    extra = torch.zeros(B, dtype=torch.float64)
    if model == "lv":
        x, extra = O.lv_transform(z, d["mask"][w], d["shift"][w])
        sde, obs = O.lv_elbo_terms(x, theta, d["obs"][w], d["bin"][w], d["dt"])
    elif model == "sv":
        x = torch.stack([d["dim_one"][w], z * d["mask"][w] + d["shift"][w]], 1)
        sde = O.sv_elbo_terms(x, theta, d["dt"])
        obs = torch.zeros(B, dtype=torch.float64)
    else:
        x = z.reshape(B, -1, 2).transpose(1, 2)
        sde, obs = O.fhn_elbo_terms(x, theta, d["obs"][w], d["bin"][w], d["dt"])
    return sde, obs, extra


@pytest.mark.parametrize("M", MS)
@pytest.mark.parametrize("n_win", [1, 3])
@pytest.mark.parametrize("model", ["lv", "sv", "fhn"])
def test_model_elbo_kernels_match_oracle(model, M, n_win):
    from viforssms_amd import _lib
    from viforssms_amd.ops import ElboFeeds, elbo_terms
    B = 37
    d = _case(model, B, M, n_win, seed=M * 13 + n_win + len(model))
    zr, thr = d["z"].clone().requires_grad_(True), d["theta"].clone().requires_grad_(True)
    sde_r, obs_r, ex_r = _oracle(model, d, zr, thr)
    loss = (sde_r * d["gs"]).sum()
    if model != "sv":
        loss = loss + (obs_r * d["go"]).sum()
    if model == "lv":
        loss = loss + (ex_r * d["ge"]).sum()
    loss.backward()

    f = lambda k: d[k].float().to(DEV).contiguous() if k in d else None
    feeds = ElboFeeds(obs=f("obs"), obs_bin=f("bin"), mask=f("mask"), shift=f("shift"), dim_one=f("dim_one"),
                      win=d["win"].to(DEV) if n_win > 1 else None, n_win=n_win)
    mid = {"lv": _lib.MODEL_LV, "sv": _lib.MODEL_SV, "fhn": _lib.MODEL_FHN}[model]
    zd = d["z"].float().to(DEV).requires_grad_(True)
    thd = d["theta"].float().to(DEV).requires_grad_(True)
    sde, obs, ex = elbo_terms(mid, M, d["dt"], 1.0, feeds, zd, thd)
    dl = (sde * f("gs")).sum()
    if model != "sv":
        dl = dl + (obs * f("go")).sum()
    if model == "lv":
        dl = dl + (ex * f("ge")).sum()
    dl.backward()
    torch.cuda.synchronize()

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double()
        return float((a - b).norm() / (b.norm() + 1e-30))

    tol = 2e-5
    assert rel(sde, sde_r) < tol
    if model != "sv":
        assert rel(obs, obs_r) < tol
    if model == "lv":
        # the Softplus ILDJ at x = softplus(z) is softplus(-z) ~ e^{-x}: where x is large (populations ~100)
        # the float64 oracle's -log(-expm1(-x)) rounds it to 0 (as TF's fp32 does) while the kernel keeps
        # the tiny true value, so this term is held to an absolute floor as well
        err = float((ex.detach().double().cpu() - ex_r.detach()).abs().max())
        assert err <= tol * float(ex_r.detach().abs().max()) + 1e-6, err
    assert torch.isfinite(zd.grad).all()
    assert rel(zd.grad, zr.grad) < 1e-4
    assert rel(thd.grad, thr.grad) < 1e-4


# M + 1 elements in chunks of 4 (LV: 2): no chunk, one chunk (element-wise only), the neighbour-exchange loop with a
# partial iteration, exactly one / two full iterations of 64 chunks (the deferred lane 63), one chunk past them
@pytest.mark.parametrize("M", [1, 3, 4, 5, 8, 9, 50, 128, 129, 130, 258, 259, 260, 515, 519, 1001, 2000])
@pytest.mark.parametrize("n_win", [1, 3])
@pytest.mark.parametrize("model", ["ar", "lv", "sv", "fhn"])
def test_one_pass_equals_forward_and_backward(model, M, n_win):
    """vissm_elbo_fwd_grad (values, dz and dtheta from one read of z; the training step's ELBO for every model)
    against the two launches it replaces: the values to fp32 summation order, dz to rounding (the same per-element
    formulas; the compiler contracts them into FMAs differently in the two kernels), dtheta to summation order; and against the float64 oracle's values and autograd at the
    two-launch bars (test above)."""
    from viforssms_amd import _lib
    from viforssms_amd.ops import ElboFeeds, elbo_terms, elbo_values_grad
    B = 37
    if model == "ar":
        g = torch.Generator().manual_seed(M + n_win)
        d = {"win": torch.randint(0, n_win, (B,), generator=g, dtype=torch.int32),
             "z": torch.randn(B, M + 1, generator=g, dtype=torch.float64) * 3,
             "theta": torch.stack([torch.randn(B, generator=g, dtype=torch.float64) * 0.3,
                                   0.5 + 0.1 * torch.randn(B, generator=g, dtype=torch.float64),
                                   0.2 * torch.randn(B, generator=g, dtype=torch.float64)], 1),
             "obs": torch.randn(n_win, M, generator=g, dtype=torch.float64) * 3,
             "bin": (torch.rand(n_win, M, generator=g, dtype=torch.float64) < 0.3).double(), "dt": 1.0}
        for key in ("gs", "go"):
            d[key] = torch.randn(B, generator=g, dtype=torch.float64)
        obs_std = 1.3
    else:
        d = _case(model, B, M, n_win, seed=M * 7 + n_win + len(model))
        obs_std = 1.0
    f = lambda k: d[k].float().to(DEV).contiguous() if k in d else None
    feeds = ElboFeeds(obs=f("obs"), obs_bin=f("bin"), mask=f("mask"), shift=f("shift"), dim_one=f("dim_one"),
                      win=d["win"].to(DEV) if n_win > 1 else None, n_win=n_win)
    mid = {"ar": _lib.MODEL_AR, "lv": _lib.MODEL_LV, "sv": _lib.MODEL_SV, "fhn": _lib.MODEL_FHN}[model]
    gs, go = f("gs"), (f("go") if model != "sv" else torch.zeros(B, device=DEV))
    ge = f("ge") if model == "lv" else None
    zd = d["z"].float().to(DEV).requires_grad_(True)
    thd = d["theta"].float().to(DEV).requires_grad_(True)
    sde, obs, ex = elbo_terms(mid, M, d["dt"], obs_std, feeds, zd, thd)
    dl = (sde * gs).sum() + (obs * go).sum() + ((ex * ge).sum() if ge is not None else 0.0)
    dl.backward()
    s1, o1, e1, dz1, dth1 = elbo_values_grad(mid, M, d["dt"], obs_std, feeds, zd.detach(), thd.detach(), gs, go, ge)
    torch.cuda.synchronize()

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double().cpu()
        return float((a - b).norm() / (b.norm() + 1e-30))

    assert rel(s1, sde) < 2e-6, rel(s1, sde)
    if model != "sv":
        assert rel(o1, obs) < 2e-6
    if model == "lv":
        assert float((e1 - ex.detach()).abs().max()) <= 2e-6 * float(ex.detach().abs().max()) + 1e-6
    assert rel(dz1, zd.grad) < 1e-6, rel(dz1, zd.grad)
    assert rel(dth1, thd.grad) < 1e-6
    if model != "ar":
        zr, thr = d["z"].clone().requires_grad_(True), d["theta"].clone().requires_grad_(True)
        sde_r, obs_r, ex_r = _oracle(model, d, zr, thr)
        loss = (sde_r * d["gs"]).sum()
        if model != "sv":
            loss = loss + (obs_r * d["go"]).sum()
        if model == "lv":
            loss = loss + (ex_r * d["ge"]).sum()
        loss.backward()
        assert rel(s1, sde_r) < 2e-5
        assert rel(dz1, zr.grad) < 1e-4 and rel(dth1, thr.grad) < 1e-4


@pytest.mark.parametrize("M", [9, 258, 519, 2000])
@pytest.mark.parametrize("model", ["lv", "sv"])
def test_one_pass_plain_span(model, M):
    """VissmElboData.plain_from (features.plain_from_table): windows whose mask / shift tables are dirty at element 0
    (the reference's first window), in the middle of the chunk loop, at the last element, or nowhere.  The one-pass
    kernel with the plain-span table equals the same kernel without it (the plain transform is the general one at
    mask 1, shift 0) and the two-launch path's autograd."""
    from viforssms_amd import _lib
    from viforssms_amd.features import plain_from_table
    from viforssms_amd.ops import ElboFeeds, elbo_terms, elbo_values_grad
    B, n_win = 40, 5
    d = _case(model, B, M, n_win, seed=M + len(model))
    d["win"] = torch.arange(B, dtype=torch.int32) % n_win
    D = 2 if model == "lv" else 1
    mask, shift = d["mask"].reshape(n_win, D, M + 1), d["shift"].reshape(n_win, D, M + 1)
    for w, pos in ((1, M // 2), (2, M), (3, min(4 * 65 + 1, M))):    # window 4: nowhere dirty
        mask[w, D - 1, pos] = 0.5
        shift[w, 0, max(pos - 1, 0)] = 1.5
    pf = [int(plain_from_table(mask[w].numpy(), shift[w].numpy(), M)[0]) for w in range(n_win)]
    assert pf[0] == 1 and pf[4] == 0 and pf[2] == M + 1
    f = lambda k: d[k].float().to(DEV).contiguous() if k in d else None
    kw = dict(obs=f("obs"), obs_bin=f("bin"), mask=f("mask"), shift=f("shift"), dim_one=f("dim_one"),
              win=d["win"].to(DEV), n_win=n_win)
    plain = ElboFeeds(**kw, plain_from=torch.tensor(pf, dtype=torch.int32, device=DEV))
    general = ElboFeeds(**kw)
    mid = {"lv": _lib.MODEL_LV, "sv": _lib.MODEL_SV}[model]
    gs, go = f("gs"), (f("go") if model != "sv" else torch.zeros(B, device=DEV))
    ge = f("ge") if model == "lv" else None
    zd = d["z"].float().to(DEV).requires_grad_(True)
    thd = d["theta"].float().to(DEV).requires_grad_(True)
    sde, obs, ex = elbo_terms(mid, M, d["dt"], 1.0, general, zd, thd)
    dl = (sde * gs).sum() + (obs * go).sum() + ((ex * ge).sum() if ge is not None else 0.0)
    dl.backward()
    a = elbo_values_grad(mid, M, d["dt"], 1.0, plain, zd.detach(), thd.detach(), gs, go, ge)
    b = elbo_values_grad(mid, M, d["dt"], 1.0, general, zd.detach(), thd.detach(), gs, go, ge)
    torch.cuda.synchronize()

    def rel(x, y):
        x, y = x.detach().double().cpu(), y.detach().double().cpu()
        return float((x - y).norm() / (y.norm() + 1e-30))

    for x, y in zip(a, b):
        assert rel(x, y) < 1e-6
    assert rel(a[0], sde) < 2e-6
    assert rel(a[3], zd.grad) < 1e-6 and rel(a[4], thd.grad) < 1e-6
    zr, thr = d["z"].clone().requires_grad_(True), d["theta"].clone().requires_grad_(True)
    sde_r, obs_r, ex_r = _oracle(model, d, zr, thr)
    loss = (sde_r * d["gs"]).sum() + ((obs_r * d["go"]).sum() if model != "sv" else 0.0)
    if model == "lv":
        loss = loss + (ex_r * d["ge"]).sum()
    loss.backward()
    assert rel(a[0], sde_r) < 2e-5
    assert rel(a[3], zr.grad) < 1e-4 and rel(a[4], thr.grad) < 1e-4


# the observation list (VissmElboData.obs_list): sparse bins (the reference's every 100th / 10th step), dense bins, a
# window with none; M around the chunk edges, the tail and full iterations
@pytest.mark.parametrize("M", [1, 3, 5, 9, 130, 259, 519, 2000])
@pytest.mark.parametrize("model", ["lv", "fhn"])
def test_one_pass_obs_list(model, M):
    """vissm_elbo_fwd_grad with the per-window list of observed elements (the observation term evaluated after the
    chunk loop at those elements only, its dz added to the stored one) equals the same kernel reading the obs rows
    at every element: values to summation order, dz to rounding, dtheta exactly; and the float64 oracle at the
    two-launch bars.  The training step takes the list from features.obs_list_table (DeviceTable)."""
    from viforssms_amd import _lib
    from viforssms_amd.features import obs_list_table
    from viforssms_amd.ops import ElboFeeds, elbo_values_grad
    B, n_win = 40, 4
    d = _case(model, B, M, n_win, seed=3 * M + len(model))
    d["win"] = torch.arange(B, dtype=torch.int32) % n_win
    every = 100 if model == "lv" else 10
    bins = torch.zeros(n_win, 2, M, dtype=torch.float64)
    bins[0, :, every - 1::every] = 1.0                       # the reference's spacing (x_every, x_2every, ...)
    bins[1] = d["bin"][1]                                    # dense random
    bins[2, 0, M - 1] = 1.0                                  # the last element only, one coordinate
    d["bin"] = bins                                          # window 3: none observed
    lists = [obs_list_table(bins[w].numpy(), M)[0] for w in range(n_win)]
    stride = max(len(x) for x in lists)
    ol = torch.full((n_win, stride), -1, dtype=torch.int32)
    for w, x in enumerate(lists):
        ol[w, :len(x)] = torch.as_tensor(x)
    assert (ol[3] == -1).all() and (ol[2][ol[2] >= 0] == M).all()
    f = lambda k: d[k].float().to(DEV).contiguous() if k in d else None
    kw = dict(obs=f("obs"), obs_bin=f("bin"), mask=f("mask"), shift=f("shift"), win=d["win"].to(DEV), n_win=n_win)
    listed = ElboFeeds(**kw, obs_list=ol.to(DEV))
    every_elem = ElboFeeds(**kw)
    mid = {"lv": _lib.MODEL_LV, "fhn": _lib.MODEL_FHN}[model]
    gs, go = f("gs"), f("go")
    ge = f("ge") if model == "lv" else None
    zd, thd = d["z"].float().to(DEV), d["theta"].float().to(DEV)
    a = elbo_values_grad(mid, M, d["dt"], 1.0, listed, zd, thd, gs, go, ge)
    b = elbo_values_grad(mid, M, d["dt"], 1.0, every_elem, zd, thd, gs, go, ge)
    torch.cuda.synchronize()

    def rel(x, y):
        x, y = x.detach().double().cpu(), y.detach().double().cpu()
        return float((x - y).norm() / (y.norm() + 1e-30))

    assert rel(a[0], b[0]) < 2e-6 and rel(a[1], b[1]) < 2e-6, (rel(a[0], b[0]), rel(a[1], b[1]))
    if model == "lv":
        assert rel(a[2], b[2]) < 2e-6
    assert rel(a[3], b[3]) < 1e-6, rel(a[3], b[3])
    assert torch.equal(a[4], b[4])
    zr, thr = d["z"].clone().requires_grad_(True), d["theta"].clone().requires_grad_(True)
    sde_r, obs_r, ex_r = _oracle(model, d, zr, thr)
    loss = (sde_r * d["gs"]).sum() + (obs_r * d["go"]).sum()
    if model == "lv":
        loss = loss + (ex_r * d["ge"]).sum()
    loss.backward()
    assert rel(a[0], sde_r) < 2e-5 and rel(a[1], obs_r.detach()) < 2e-5
    assert rel(a[3], zr.grad) < 1e-4 and rel(a[4], thr.grad) < 1e-4
