"""The fused window-shared feature branch + first-conv feature channels (vissm_feat_fwd / _bwd, ops.feat_conv)
against the torch fp32 form of the same layers (nma.IAF.features + conv_shared: four dense + ELU layers,
AR.py:53-62 / SV_dense.py:53-62 / fitz_nag_NVP.py:71-79, then the valid conv over the features): C and the
gradients of every dense layer, the conv kernel and bias for a random dC, at the configs' shapes (AR-cfg, the AR
paper shape's windows, FHN's stride-2 conv, SV's feature construction) and small edge shapes.  fp32 FMAs in a
different order than the library GEMMs: relative L2 error within 2e-6, every element within 1e-4 relative to
the tensor's scale; bitwise reproducible run to run."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from viforssms_amd.ops import feat_conv  # noqa: E402
from viforssms_amd.linalg import linear  # noqa: E402

DEV = "cuda:0"


def _torch_ref(h0, s, Lh, ws):
    W = list(ws)
    h = h0
    for j in range(4):
        h = torch.nn.functional.elu(linear(h, W[2 * j], W[2 * j + 1]))
    cw, cb = W[8], W[9]
    k, H = cw.shape[0], cw.shape[2]
    out = cb.expand(h.shape[0], Lh, H).clone()
    for j in range(k):
        out = out + h[:, j:j + s * (Lh - 1) + 1:s, :] @ cw[j, 1:, :]
    return out


def _case(n_win, Lf, Cin, H, k, s, seed, sv=False):
    g = torch.Generator(device=DEV).manual_seed(seed)
    r = lambda *sh, sc=1.0: (torch.randn(*sh, generator=g, device=DEV) * sc)
    Lh = (Lf - k) // s + 1
    if sv:   # SV: the feature rows are built from the window's channels (nma.IAF.window_conv)
        ts = r(n_win, Lf + 1, Cin)
        h0 = torch.cat([ts[:, 1:, :], ts[:, 1:, :-2] - ts[:, :-1, :-2]], 2)
    else:    # a strided view like the AR / FHN windows (ts[:, i k:, :][:, :-1, :]) with windows further apart
        big = r(n_win, Lf + 7, Cin)
        h0 = big[:, 3:3 + Lf, :]
    cin = h0.shape[2]
    ws = [r(cin, H, sc=1 / np.sqrt(cin)), r(H, sc=0.1)]
    for _ in range(3):
        ws += [r(H, H, sc=1 / np.sqrt(H)), r(H, sc=0.1)]
    ws += [r(k, 1 + H, H, sc=1 / np.sqrt(k * H)), r(H, sc=0.1)]
    ws = [w.requires_grad_() for w in ws]
    dC = r(n_win, Lh, H)
    return h0, s, Lh, ws, dC


def _rel(a, b):
    a, b = a.detach(), b.detach()
    return float((a - b).double().norm() / b.double().norm().clamp_min(1e-30))


SHAPES = {  # name -> (n_win, Lf, Cin, H, k, s, sv)
    "ar_cfg": (1, 5024, 14, 50, 8, 1, False),         # AR-cfg flow 0 (kernel_ext 5025)
    "ar_paper": (50, 199, 14, 50, 50, 1, False),      # hyperparameters.txt: 50 windows, k = 50
    "fhn_cfg": (1, 4061, 14, 50, 20, 2, False),       # FHN: interleaved 2-D, stride-2 conv, k = 20
    "sv_cfg": (1, 1657, 8, 50, 50, 1, True),          # SV: k = 50, the differenced feature channels
    "edge_small": (3, 9, 3, 7, 9, 1, False),          # one output position (Lf = k)
    "edge_s2": (2, 40, 5, 33, 5, 2, False),
    "edge_h64": (1, 70, 63, 64, 3, 1, False),
}


@pytest.mark.parametrize("name", list(SHAPES))
def test_feat_conv_matches_torch(name):
    n_win, Lf, Cin, H, k, s, sv = SHAPES[name]
    h0, s, Lh, ws, dC = _case(n_win, Lf, Cin, H, k, s, seed=Lf + k, sv=sv)
    C = feat_conv(h0, s, Lh, *ws)
    g = torch.autograd.grad(C, ws, dC)
    Cr = _torch_ref(h0, s, Lh, ws)
    gr = torch.autograd.grad(Cr, ws, dC)
    assert C.shape == Cr.shape == (n_win, Lh, H)
    errs = {"C": _rel(C, Cr)}
    names = ["W0", "b0", "W1", "b1", "W2", "b2", "W3", "b3", "conv_w", "conv_b"]
    for nm, a, b in zip(names, g, gr):
        if nm == "conv_w":      # the sample channel is the flow kernel's: zero here
            assert torch.count_nonzero(a[:, 0, :]) == 0
            a, b = a[:, 1:, :], b[:, 1:, :]
        errs[nm] = _rel(a, b)
        assert (a - b).abs().max() <= 1e-4 * b.abs().max() + 1e-12, (nm, float((a - b).abs().max()))
    print(name, {kk: f"{v:.1e}" for kk, v in errs.items()})
    assert max(errs.values()) < 2e-6, errs
    # deterministic: a second run is bitwise equal
    C2 = feat_conv(h0, s, Lh, *ws)
    g2 = torch.autograd.grad(C2, ws, dC)
    assert torch.equal(C, C2) and all(torch.equal(a, b) for a, b in zip(g, g2))


@pytest.mark.parametrize("prec,etol,gtol", [("fp32", 1e-6, 1e-5), ("bf16", 1e-4, 1e-2)])
def test_feat_conv_in_the_ar_step_matches_torch_form(prec, etol, gtol):
    """The AR-cfg training step's per-sample ELBO and gradient with the fused feature branch against the torch
    form's (VISSM_FEAT_TORCH=1): fp32 to rounding; bf16 (the benchmark's step, its last flow fused) within the
    bf16 products' rounding of the slightly different C."""
    import os
    from tests.parity_util import build_model
    from viforssms_amd._lib import TRAIN_PRECISIONS
    res = {}
    for mode in ("hip", "torch"):
        os.environ["VISSM_FEAT_TORCH"] = "1" if mode == "torch" else "0"
        try:
            model = build_model("ar", 20, 5000, 8, 3, 50, 3, 10, DEV, T=5000, precision=TRAIN_PRECISIONS[prec],
                                impute=5, condition=True)
            np.random.seed(3)
            batch = model.engine.make_batch(model.select_windows())
            g = torch.Generator().manual_seed(5)
            md = model.mdef
            eps = torch.randn(20, md.kernel_ext, generator=g).to(DEV)
            x0 = (torch.randn(20, md.P_theta, generator=g) * md.theta_base[1] + md.theta_base[0]).to(DEV)
            out = model.elbo_step(batch, 0, eps=eps, x0_theta=x0, apply=False)
            res[mode] = (out["elbo"].double().cpu(), model.store.grad.double().cpu().clone())
        finally:
            os.environ.pop("VISSM_FEAT_TORCH", None)
    e_h, g_h = res["hip"]
    e_t, g_t = res["torch"]
    de, dg = float(((e_h - e_t).abs() / e_t.abs()).max()), float((g_h - g_t).norm() / g_t.norm())
    print(prec, "elbo", de, "grad", dg)
    assert de < etol and dg < gtol
