"""The last AR(1) flow fused with its ELBO terms (vissm_flow_ar_elbo_fused; the training step's path
at bf16 / bf16x3): the training step's per-sample ELBO and gradient against the float64 oracle
(AR.py:50-89 + 168-187, tolerances of tests/test_gpu_parity.py), and against the unfused path
(flow forward + ELBO kernels + flow backward) on the same draw.  Shapes cover the fused kernel's
15-position tiles (M around 15 / 30, partial last tiles), several t-chunks (chunk starts recompute
the previous position), one and several windows, k = 1 and k = 32, and the BASELINE configs[1]
length (M = T = 5000, kernel_len 8)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from tests.parity_util import build_model, run_parity_case  # noqa: E402
from viforssms_amd import _lib  # noqa: E402

DEV = "cuda:0"
X2F = _lib.VISSM_PREC_BF16X2F
X2 = _lib.VISSM_PREC_BF16X2
# bf16x2f (the fused kernel's recompute on split weights, backward products bf16): the north-star ELBO bar at the
# configs' lengths, the gradient at bf16 accuracy; bf16x2 (every weight product split, backward chain included): the
# fp32 bar on both at the configs' lengths
TOL = {2: dict(elbo=1e-4, grad=1e-3, param=2e-2), 1: dict(elbo=5e-3, grad=5e-2, param=2e-1),
       X2F: dict(elbo=1e-4, grad=5e-2, param=2e-1), X2: dict(elbo=1e-4, grad=1e-3, param=2e-2)}
CASES = [  # B, M, k, n_flows, H, n_layers, fw, T, starts
    (4, 14, 4, 2, 16, 3, 3, None, None),
    (5, 15, 4, 2, 16, 3, 3, None, None),
    (17, 16, 8, 3, 50, 3, 10, None, None),
    (3, 31, 1, 2, 20, 3, 3, None, None),
    (20, 300, 8, 3, 50, 3, 10, None, None),
    (2, 40, 32, 2, 24, 3, 4, None, None),
    (6, 30, 5, 2, 20, 3, 4, 150, [0, 30, 60, 60, 120, 0]),
    (5, 40, 4, 1, 16, 3, 3, None, None),   # one flow: the fused flow's input is the base noise itself
]


def _check(res, t):
    print({k: v for k, v in res.items() if k != "per_param"})
    assert res["fused"], "the step did not take the fused path"
    assert res["finite"]
    assert res["elbo_rel_err"] < t["elbo"], res["elbo_rel_err"]
    assert res["grad_rel_err"] < t["grad"], res["grad_rel_err"]
    assert res["grad_max_param_err"] < t["param"], (res["worst_param"], res["grad_max_param_err"])


@pytest.mark.parametrize("prec", [2, 1])
@pytest.mark.parametrize("B,M,k,nf,H,nl,fw,T,starts", CASES)
def test_fused_step_matches_oracle(B, M, k, nf, H, nl, fw, T, starts, prec):
    res = run_parity_case("ar", B, M, k, nf, H, nl, fw, device=DEV, T=T, starts=starts, precision=prec,
                          step_path=True)
    _check(res, TOL[prec])


@pytest.mark.parametrize("prec", [2, 1, X2F, X2])
def test_fused_step_ar_cfg_length(prec):
    """BASELINE configs[1] (AR(1) T = 5000, impute 5, kernel_len 8): two sample groups, many t-chunks."""
    res = run_parity_case("ar", 20, 5000, 8, 3, 50, 3, 10, device=DEV, precision=prec, impute=5, condition=True,
                          step_path=True)
    _check(res, TOL[prec])


@pytest.mark.parametrize("prec", [2, 1, X2F, X2])
def test_fused_step_ar_cfg_bench_geometry(prec):
    """The fused kernel as the B = 65536 benchmark launches it (SURVEY configs[1]): there each 16-sample
    group's 334 fused tiles (15 outputs each) split into 2 t-chunks of 167; VissmFlowDesc.chunk_tiles = 167
    runs that geometry at B = 20, so the per-sample carries (transposed-conv overhang, the previous x) and
    the dW / d theta / log sigma accumulations cross ~160 real tiles inside one work item on the k = 8 kernels
    the benchmark uses (the automatic geometry at B = 20 cuts every chunk to one tile)."""
    res = run_parity_case("ar", 20, 5000, 8, 3, 50, 3, 10, device=DEV, precision=prec, impute=5, condition=True,
                          step_path=True, chunk_tiles=167)
    _check(res, TOL[prec])


@pytest.mark.parametrize("prec", [2, 1, X2F, X2])
def test_fused_equals_unfused(prec):
    """Same model, same draw: the fused step's ELBO and gradient against forward + ELBO kernels + backward."""
    B, M, k = 33, 500, 8
    model = build_model("ar", B, M, k, 3, 50, 3, 10, DEV, precision=prec, impute=5, condition=True)
    batch = model.engine.make_batch(np.zeros(B, dtype=np.int64))
    g = torch.Generator().manual_seed(9)
    eps = torch.randn(B, model.mdef.kernel_ext, generator=g).to(DEV)
    x0 = (torch.randn(B, 3, generator=g) * 0.5 + 1.5).to(DEV)
    outs, grads = [], []
    for fuse in (True, False):
        model.engine.fuse_last = fuse
        o = model.elbo_step(batch, 0, eps=eps, x0_theta=x0, apply=False)
        torch.cuda.synchronize()
        outs.append(o["elbo"].double().cpu())
        grads.append(model.store.grad.double().cpu().clone())
    tol = {2: 1e-5, 1: 2e-3, X2F: 1e-4, X2: 1e-4}[prec]
    assert float(((outs[0] - outs[1]).abs() / outs[1].abs()).max()) < tol
    assert float((grads[0] - grads[1]).norm() / grads[1].norm()) < {2: 1e-4, X2: 1e-3}.get(prec, 2e-2)


@pytest.mark.parametrize("fuse", [True, False])
@pytest.mark.parametrize("chunk_tiles", [0, 167])
def test_theta_fold_equals_theta_term(fuse, chunk_tiles, monkeypatch):
    """The theta fold (VissmFlowParams.theta_rank: the two-sample AR kernels form theta_term = theta w_theta +
    b_theta inside their layer-0 product from split-bf16 theta / w_theta, AR.py:63-72) against the same kernels
    reading the fp32 theta_term rows: same model and draw, bf16, an odd sample count (a ghost partner in the last
    pair), the automatic and the benchmark's chunk geometry, fused and unfused last flow.  The fold's products
    carry ~2^-16 relative error, far inside the bf16 activations' rounding, so ELBO and gradient agree to the
    run-to-run scale of that rounding."""
    B, M, k = 33, 5000 if chunk_tiles else 500, 8
    model = build_model("ar", B, M, k, 3, 50, 3, 10, DEV, precision=1, impute=5, condition=True)
    model.engine.fuse_last = fuse
    model.engine.chunk_tiles = chunk_tiles
    batch = model.engine.make_batch(np.zeros(B, dtype=np.int64))
    g = torch.Generator().manual_seed(11)
    eps = torch.randn(B, model.mdef.kernel_ext, generator=g).to(DEV)
    x0 = (torch.randn(B, 3, generator=g) * 0.5 + 1.5).to(DEV)
    outs, grads = [], []
    for fold in ("1", "0"):
        monkeypatch.setenv("VISSM_THETA_FOLD", fold)
        o = model.elbo_step(batch, 0, eps=eps, x0_theta=x0, apply=False)
        torch.cuda.synchronize()
        outs.append(o["elbo"].double().cpu())
        grads.append(model.store.grad.double().cpu().clone())
    assert torch.isfinite(outs[0]).all() and torch.isfinite(grads[0]).all()
    assert float(((outs[0] - outs[1]).abs() / outs[1].abs()).max()) < 2e-4
    assert float((grads[0] - grads[1]).norm() / grads[1].norm()) < 1e-2
