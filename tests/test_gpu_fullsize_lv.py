"""The Lotka-Volterra benchmark launch itself (bench.py --model lv: BASELINE configs[3]'s per-GPU shape, B = 16384
trajectories per GPU = 131072 over 8, M = T = 5000, kernel_len 20, 3 flows, [50]*5, bf16), through the training
step's gradient (lotka_volterra_partial.py:68-104 flows, 235-297 ELBO, 402-405 the step):

* per-sample ELBO of 16+ trajectories spread over the batch (first / last sample groups, both halves of a
  group, every t-chunk boundary region of the 8 chunks x 40 tiles the bwd2n / fwd2 kernels run at this batch)
  against the float64 oracle on the same injected eps and q(theta) base draws, at the bf16 tolerance of
  test_gpu_config_parity.py;
* the whole-batch gradient against the sum of the four quarter-batch gradients (B = 4096 each: 256 groups x 32
  chunks of 10 tiles instead of 1024 x 8 of 40, other slab row counts): the fixed-order partial slabs, the halo
  join, the cross-tile transposed-conv carries and the window-shared GEMMs' backward on summed dC must give the
  same sum up to fp32 re-association;
* a second evaluation of the full batch reproduces ELBO and gradient bit for bit.
test_gpu_config_parity.test_family_cfg_bench_geometry holds the oracle gradient at this launch geometry (B = 3)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from tests.parity_util import build_model, oracle_elbo_rows  # noqa: E402
from viforssms_amd import _lib  # noqa: E402

DEV = "cuda:0"
B, M, K = 16384, 5000, 20


@pytest.fixture(scope="module")
def full():
    torch.cuda.set_device(torch.device(DEV))
    model = build_model("lv", B, M, K, 3, 50, 5, 10, DEV, precision=_lib.VISSM_PREC_BF16, condition=True)
    # the window-shared GEMMs over the 10,061 time-mixing features at split-bf16 (fp32-class): at bf16 their input
    # gradient rounds the batch's summed dC to bf16, so the sum of four quarter-batch gradients would differ from
    # the full batch's by bf16 rounding of those GEMM operands, not by anything in the flow kernels under test
    model.engine.feature_gemm_override = "x3"
    g = torch.Generator(device=DEV).manual_seed(2025)
    eps = torch.randn(B, model.mdef.kernel_ext, generator=g, device=DEV)
    x0 = torch.randn(B, model.mdef.P_theta, generator=g, device=DEV) * model.mdef.theta_base[1] + model.mdef.theta_base[0]
    batch = model.engine.make_batch(np.zeros(B, dtype=np.int64))
    out = model.elbo_step(batch, 0, eps=eps, x0_theta=x0, apply=False)
    model.store.sync_grads()
    torch.cuda.synchronize()
    yield model, eps, x0, out["elbo"].detach().clone(), model.store.grad.detach().clone()
    del model
    torch.cuda.empty_cache()


def test_lv_full_batch_elbo_rows_match_oracle(full):
    model, eps, x0, elbo, _ = full
    rng = np.random.default_rng(11)
    rows = np.unique(np.concatenate([[0, 1, 14, 15, 16, 8191, 8192, B - 17, B - 16, B - 2, B - 1],
                                     rng.choice(B, 9, replace=False)]))
    e = eps[rows].double().cpu()
    x = x0[rows].double().cpu()
    ref = oracle_elbo_rows(model, np.zeros(len(rows), dtype=np.int64), e, x)
    got = elbo[rows].double().cpu().numpy()
    err = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-6)
    print({"rows": rows.tolist(), "max_rel_err": float(err.max()), "elbo_ref_mean": float(ref.mean())})
    assert len(rows) >= 16
    assert np.isfinite(got).all()
    assert float(err.max()) < 5e-3, err   # bf16 tolerance (test_gpu_config_parity.TOL["bf16"])


def test_lv_full_batch_gradient_equals_quarter_sum(full):
    model, eps, x0, _, grad_full = full
    q = B // 4
    acc = torch.zeros_like(grad_full, dtype=torch.float64)
    batch_q = model.engine.make_batch(np.zeros(q, dtype=np.int64))
    for i in range(4):
        sl = slice(i * q, (i + 1) * q)
        model.elbo_step(batch_q, 0, eps=eps[sl].contiguous(), x0_theta=x0[sl].contiguous(), apply=False)
        model.store.sync_grads()
        acc += model.store.grad.double()
    torch.cuda.synchronize()
    gf = grad_full.double()
    rel = float((gf - acc).norm() / gf.norm())
    print({"grad_rel_diff_full_vs_quarters": rel, "grad_norm": float(gf.norm())})
    assert torch.isfinite(gf).all()
    assert rel < 1e-4, rel


def test_lv_full_batch_deterministic(full):
    model, eps, x0, elbo, grad_full = full
    batch = model.engine.make_batch(np.zeros(B, dtype=np.int64))
    out = model.elbo_step(batch, 0, eps=eps, x0_theta=x0, apply=False)
    model.store.sync_grads()
    torch.cuda.synchronize()
    assert torch.equal(out["elbo"], elbo)
    assert torch.equal(model.store.grad, grad_full)
