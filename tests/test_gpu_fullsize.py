"""The benchmark's own launch, not a scaled-down stand-in: AR(1) B = 65536 trajectories, M = T = 5000,
impute 5, kernel_len 8, 3 flows, [50]*3, bf16 (BASELINE.json configs[1]; bench.py's workload), through the
training step's path (AR.py:168-187 + 226-229: flows, the last one fused with the ELBO terms, and the
gradient of sum(-ELBO)).

* per-sample ELBO of 24 trajectories spread over the batch (first / last sample groups, a partial
  position in every group, both t-chunks) against the float64 oracle on the same injected eps and q(theta)
  base draws, at the bf16 tolerance of test_gpu_config_parity.py;
* the whole-batch gradient against the sum of the four quarter-batch gradients (B = 16384 each: a
  different launch geometry -- 1024 groups x 8 t-chunks instead of 4096 x 2 -- and other slab row
  counts): the fixed-order partial slabs, the halo join and the 4096-row bf16 dC reduction must give the
  same sum up to fp32 re-association;
* the run is deterministic (a second evaluation of the full batch reproduces ELBO and gradient bit for
  bit).
The oracle cannot evaluate 65536 x 5000 transitions (the gradient of the full batch is checked by the
decomposition above; tests/test_gpu_fused.py and test_gpu_config_parity.py hold the oracle gradient at the
same launch geometry via VissmFlowDesc.chunk_tiles)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from tests.parity_util import build_model, oracle_elbo_rows  # noqa: E402
from viforssms_amd import _lib  # noqa: E402

DEV = "cuda:0"
B, M, K = 65536, 5000, 8


@pytest.fixture(scope="module")
def full():
    torch.cuda.set_device(torch.device(DEV))
    model = build_model("ar", B, M, K, 3, 50, 3, 10, DEV, precision=_lib.VISSM_PREC_BF16, impute=5, condition=True)
    g = torch.Generator(device=DEV).manual_seed(2024)
    eps = torch.randn(B, model.mdef.kernel_ext, generator=g, device=DEV)
    x0 = torch.randn(B, model.mdef.P_theta, generator=g, device=DEV) * model.mdef.theta_base[1] + model.mdef.theta_base[0]
    batch = model.engine.make_batch(np.zeros(B, dtype=np.int64))
    assert model.engine.fused_ok(batch, B)
    out = model.elbo_step(batch, 0, eps=eps, x0_theta=x0, apply=False)
    model.store.sync_grads()
    torch.cuda.synchronize()
    return model, eps, x0, out["elbo"].detach().clone(), model.store.grad.detach().clone()


def test_full_batch_elbo_rows_match_oracle(full):
    model, eps, x0, elbo, _ = full
    rng = np.random.default_rng(7)
    rows = np.unique(np.concatenate([[0, 1, 15, 16, 31, 32767, 32768, B - 17, B - 16, B - 1],
                                     rng.choice(B, 14, replace=False)]))
    e = eps[rows].double().cpu()
    x = x0[rows].double().cpu()
    ref = oracle_elbo_rows(model, np.zeros(len(rows), dtype=np.int64), e, x)
    got = elbo[rows].double().cpu().numpy()
    err = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-6)
    print({"rows": rows.tolist(), "max_rel_err": float(err.max()), "elbo_ref_mean": float(ref.mean())})
    assert np.isfinite(got).all()
    assert float(err.max()) < 5e-3, err   # bf16 tolerance (test_gpu_config_parity.TOL["bf16"])


def test_full_batch_gradient_equals_quarter_sum(full):
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


def test_full_batch_deterministic(full):
    model, eps, x0, elbo, grad_full = full
    batch = model.engine.make_batch(np.zeros(B, dtype=np.int64))
    out = model.elbo_step(batch, 0, eps=eps, x0_theta=x0, apply=False)
    model.store.sync_grads()
    torch.cuda.synchronize()
    assert torch.equal(out["elbo"], elbo)
    assert torch.equal(model.store.grad, grad_full)
