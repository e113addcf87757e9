"""The training loop's adjacent pieces on the HIP path, each against the
float64 oracle or an exact invariant:

* pre-training: each family's pre-training loss (AR: -obs_loss, AR.py:201-202; LV: (x - 75)^2,
  lotka_volterra_partial.py:301-302; SV: (x + 7)^2 and (theta - init)^2, SV_dense.py:251-254; FHN: x^2
  and (theta - init)^2, fitz_nag_NVP.py:288-292) and its gradient vs the oracle's, then one
  pretrain_step: Adamax(1e-3, beta1 = 0.9) from zero slots moves every variable by
  -lr * 0.1 * sign(g) per optimiser (two optimisers for SV / FHN);
* save_paths (AR.py:323-362, lotka_volterra_partial.py:423-462, SV_dense.py:361-395,
  fitz_nag_NVP.py:409-450): the written posterior paths for
  every window start vs the oracle's flow stack on the same Philox draws;
* checkpoint: save -> perturb -> load restores params, both slot sets, the step and the numpy RNG
  (the next window draw after load equals the one after save);
* logging: the scalar names of AR.py:205-238 and the theta histograms of AR.py:218-224;
* the non-finite guard: a step with an infinite gradient norm is skipped on the device and counted,
  while the unguarded kernel keeps the reference's NaN behaviour (AR.py:230-232)."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import nma_oracle as O  # noqa: E402
from oracle import bridge  # noqa: E402
from tests.parity_util import build_model, oracle_inputs  # noqa: E402

DEV = "cuda:0"
SHAPES = {  # family -> (B, M, k, n_flows, H, n_layers, fw, T)
    "ar": (6, 30, 5, 2, 20, 3, 4, 90),
    "lv": (5, 24, 4, 2, 16, 5, 3, 48),
    "sv": (5, 24, 6, 2, 16, 5, 3, 48),
    "fhn": (5, 24, 4, 2, 16, 5, 3, 48),
}


def _model(family, **kw):
    B, M, k, nf, H, nl, fw, T = SHAPES[family]
    return build_model(family, B, M, k, nf, H, nl, fw, DEV, T=T, **kw)


def _draws(model, step):
    eps, _, x0 = model.engine.draw(step, model.p_local, 0, model.p)
    return eps, x0


def _oracle(model, starts, eps, x0):
    spec = bridge.spec_from_mdef(model.mdef, eps.shape[0])
    params = bridge.oracle_params(model.store.state_numpy(), spec, model.engine.theta_dist.masks_np)
    ts, ex = oracle_inputs(model, starts)
    leaves = O.param_leaves(params)
    for t in leaves:
        t.requires_grad_(True)
    out = O.elbo(spec, params, model.engine.perms, x0.double().cpu(), eps.double().cpu(), ts, ex)
    return spec, params, leaves, out


def _pretrain_losses(family, x, theta, obs):
    if family == "ar":
        return [(-obs).sum()]
    if family == "lv":
        return [((x - 75.0) ** 2).sum()]
    if family == "sv":
        from viforssms_amd.sv import PARAM_INIT
        init = torch.tensor(PARAM_INIT, dtype=theta.dtype, device=theta.device)
        return [((x + 7.0) ** 2).sum(), ((theta - init) ** 2).sum()]
    from viforssms_amd.fhn import THETA_INIT
    init = torch.tensor(THETA_INIT, dtype=theta.dtype, device=theta.device)
    return [(x ** 2).sum(), ((theta - init) ** 2).sum()]


def _oracle_grad_vec(model, spec, params, leaves, loss):
    g = torch.autograd.grad(loss, leaves, retain_graph=True, allow_unused=True)
    g = [torch.zeros_like(t) if x is None else x for t, x in zip(leaves, g)]
    by = bridge.oracle_grads_by_name(params, g, spec)
    return np.concatenate([by[n].ravel() for n in model.store.names()])


@pytest.mark.parametrize("family", ["ar", "lv", "sv", "fhn"])
def test_pretrain_loss_gradient_and_step_match_oracle(family):
    model = _model(family)
    model.pre_train = True
    starts = np.zeros(model.p, dtype=np.int64)
    batch = model.engine.make_batch(starts)
    step = model.global_step
    eps, x0 = _draws(model, step)
    spec, params, leaves, o = _oracle(model, starts, eps, x0)
    o_losses = _pretrain_losses(family, o["x"], o["theta"], o["obs"])
    o_grads = [_oracle_grad_vec(model, spec, params, leaves, L) for L in o_losses]

    # product: the same losses through the HIP forward, gradients through the HIP backward
    st = model.store
    p_grads = []
    for i in range(len(o_losses)):
        st.zero_grad()
        out = model.forward(batch, step)
        x = model.engine.lf_sample(out["z"], batch)
        L = _pretrain_losses(family, x, out["theta"], out["obs"])[i]
        lp, lo = float(L.detach()), float(o_losses[i].detach())
        assert abs(lp / lo - 1.0) < 1e-4, (i, lp, lo)
        L.backward()
        st.sync_grads()
        p_grads.append(st.grad.double().cpu().numpy().copy())
    for g_ref, g in zip(o_grads, p_grads):
        assert np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref) < 1e-3

    # one pretrain_step from zero pre-training slots: -lr * (1 - beta1) * sign(g) per optimiser
    before = st.flat.double().cpu().numpy().copy()
    model.pretrain_step(batch, 0)
    torch.cuda.synchronize()
    delta = st.flat.double().cpu().numpy() - before
    want = sum(-1e-3 * 0.1 * np.sign(g) for g in o_grads)
    # compare where every optimiser's reference gradient is clearly signed or exactly zero (a variable a
    # loss does not depend on: zero gradient, no move); a ~0 gradient's sign is decided by rounding
    gmax = [np.abs(g).max() for g in o_grads]
    keep = np.all([(np.abs(g) > 1e-4 * m) | (g == 0) for g, m in zip(o_grads, gmax)], axis=0)
    assert keep.sum() > 100
    assert np.abs(delta - want)[keep].max() < 2e-6


@pytest.mark.parametrize("family", ["ar", "lv", "sv", "fhn"])
def test_save_paths_match_oracle(family, tmp_path):
    """save_paths (AR.py:323-362, lotka_volterra_partial.py:423-462, SV_dense.py:361-395 -- the observed
    coordinate stacked with the transformed latent one --, fitz_nag_NVP.py:409-450) vs the oracle's paths."""
    model = _model(family)
    path = str(tmp_path / "paths.txt")
    model.save_paths(path)
    got = np.loadtxt(path, ndmin=2)
    eps, x0 = _draws(model, model.global_step)
    parts = []
    for idx in np.arange(0, model.target_len(), model.batch_dims):
        _, _, _, o = _oracle(model, np.full(model.p, idx), eps, x0)
        x = o["x"].detach()
        x = x.unsqueeze(1) if x.dim() == 2 else x
        parts.append(x[:, :, 1:].numpy())
    ref = np.concatenate(parts, axis=2)
    ref = ref[:, 0, :] if ref.shape[1] == 1 else ref.reshape(ref.shape[0], -1)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-5


def test_checkpoint_round_trip_restores_values(tmp_path):
    model = _model("ar")
    model.pre_train = False
    model.train(None, None, max_runs=3, verbose=False)
    model._opt_pre[0].v.normal_()
    model._opt_pre[0].m.uniform_()
    ck = str(tmp_path / "ck.pt")
    np.random.seed(123)
    model.save(ck)
    snap = {"flat": model.store.flat.clone(), "v": model._opt_main.v.clone(), "m": model._opt_main.m.clone(),
            "pv": model._opt_pre[0].v.clone(), "pm": model._opt_pre[0].m.clone()}
    step = model.global_step
    next_draw = model.select_windows()
    # perturb everything the checkpoint holds
    model.train(None, None, max_runs=2, verbose=False)
    model._opt_pre[0].v.zero_()
    np.random.seed(7)
    assert not torch.equal(model.store.flat, snap["flat"])
    model.load(ck)
    assert torch.equal(model.store.flat, snap["flat"])
    assert torch.equal(model._opt_main.v, snap["v"]) and torch.equal(model._opt_main.m, snap["m"])
    assert torch.equal(model._opt_pre[0].v, snap["pv"]) and torch.equal(model._opt_pre[0].m, snap["pm"])
    assert model.global_step == step and not model.pre_train
    assert np.array_equal(model.select_windows(), next_draw)


def test_training_log_has_reference_scalars_and_theta_histograms(tmp_path):
    model = _model("ar")
    model.pre_train = False
    model.train(str(tmp_path / "train"), None, max_runs=3, verbose=False)
    runs = [os.path.join(r, f) for r, _, fs in os.walk(tmp_path / "train") for f in fs]
    assert len(runs) == 1
    recs = [json.loads(line) for line in open(runs[0])]
    assert [r["step"] for r in recs] == [0, 1, 2]
    names = {"loss/ELBO", "loss/SDE_log_prob", "loss/theta_log_prob", "loss/obs_log_prob", "loss/path_log_prob",
             "optimize/global_norm", "optimize/skipped_steps"}
    assert names <= set(recs[-1])
    h = recs[-1]["histograms"]
    assert set(h) == {"parameters/0", "parameters/1", "parameters/2"}
    for i, v in enumerate(h.values()):
        assert sum(v["counts"]) == model.p and v["count"] == model.p
        assert v["min"] <= v["mean"] <= v["max"]
    assert h["parameters/2"]["min"] > 0   # theta_2 is a log-parameter: exponentiated (AR.py:218-221)


def test_nonfinite_gradient_guard():
    from viforssms_amd.ops import AdamaxKernel
    n = 4099
    g = torch.randn(n, device=DEV)
    g[17] = float("inf")
    for guard in (True, False):
        p = torch.randn(n, device=DEV)
        v, m = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
        p0 = p.clone()
        k = AdamaxKernel(n, DEV)
        k.step(p, g, v, m, 1e-3, 0.95, 0.999, 1e-8, 2.5e8, guard=guard)
        torch.cuda.synchronize()
        if guard:
            assert torch.equal(p, p0) and int(k.skipped) == 1
            assert not v.any() and not m.any()
            g2 = torch.randn(n, device=DEV)
            k.step(p, g2, v, m, 1e-3, 0.95, 0.999, 1e-8, 2.5e8, guard=True)  # a finite step still applies
            torch.cuda.synchronize()
            assert int(k.skipped) == 1 and not torch.equal(p, p0)
        else:
            assert torch.isnan(p).all()   # tf.clip_by_global_norm with an infinite norm: NaN everywhere


def test_training_loop_skips_nonfinite_step():
    model = _model("ar")
    model.pre_train = False
    model.build_flow()
    batch = model.engine.make_batch(np.zeros(model.p, dtype=np.int64))
    before = model.store.flat.clone()
    out = model.elbo_step(batch, 0, apply=False)
    model.store.grad[3] = float("nan")
    o = model._opt_main
    o.kernel.step(model.store.flat, model.store.grad, o.v, o.m, 1e-3, 0.95, 0.999, 1e-8, model.clip_norm(),
                  guard=model.skip_nonfinite)
    torch.cuda.synchronize()
    assert torch.equal(model.store.flat, before) and int(o.kernel.skipped) == 1
    assert np.isfinite(out["elbo"].cpu().numpy()).all()
