"""The captured-graph training step (viforssms_amd.graph) against eager execution.

1. Replays vs the same step run eagerly on the same all-windows batch from the same parameters:
   the same ELBO, gradient and global norm — the capture loses or reorders nothing.
2. The all-windows batch vs the usual distinct-windows batch (one eager step): same ELBO and
   gradient up to the summation order of the window-shared GEMMs (unused windows add zeros).
   (Parameter trajectories are not compared across the two: Adamax normalises every gradient
   by its own running max, so a near-zero gradient that flips sign moves its parameter by
   ~lr/20 either way.)"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from tests.parity_util import build_model  # noqa: E402

DEV = "cuda:0"
CASES = [
    ("ar", 8, 30, 5, 2, 20, 3, 4, 150, 0),    # five windows, fp32 kernels
    ("ar", 6, 40, 8, 3, 50, 3, 10, 40, 1),    # M = T (one window), bf16 matrix cores
    ("lv", 6, 40, 4, 2, 24, 5, 3, 160, 0),    # 2-D, stride-2 head, BN hidden layers
]


def _pair(family, B, M, k, nf, H, nl, fw, T, prec):
    ms = [build_model(family, B, M, k, nf, H, nl, fw, DEV, T=T, precision=prec) for _ in range(2)]
    for m in ms:
        m.build_flow()
        m.pre_train = False
    assert torch.equal(ms[0].store.flat, ms[1].store.flat)
    return ms


@pytest.mark.parametrize("family,B,M,k,nf,H,nl,fw,T,prec", CASES)
def test_graph_replay_equals_eager_step(family, B, M, k, nf, H, nl, fw, T, prec):
    """Each step starts both models from the graph model's parameters and Adamax slots; the
    replayed step's ELBO, gradient and global norm equal the eager step's (library GEMMs may pick
    other algorithms under capture: rounding-level differences only)."""
    from viforssms_amd.graph import GraphedStep
    eager, graph = _pair(family, B, M, k, nf, H, nl, fw, T, prec)
    ref = GraphedStep(eager)  # its all-windows batch and device inputs, run eagerly
    rng = np.random.default_rng(5)
    universe = np.arange(0, eager.target_len(), M)
    for step in range(6):  # two warm-ups, the capture, three replays
        with torch.no_grad():
            eager.store.flat.copy_(graph.store.flat)
            eager._opt_main.v.copy_(graph._opt_main.v)
            eager._opt_main.m.copy_(graph._opt_main.m)
        starts = rng.choice(universe, size=B, replace=True)
        ref._inputs(starts, step)
        oe = eager.elbo_step(ref.batch, step, row0_dev=ref.row0)
        og = graph.graphed_step(starts, step)
        torch.cuda.synchronize()
        ee, eg = oe["elbo"].detach().double(), og["elbo"].detach().double()
        assert float((ee - eg).abs().max() / ee.abs().max()) < 1e-6, step
        ge, gg = eager.store.grad.double(), graph.store.grad.double()
        assert float((ge - gg).norm() / ge.norm()) < 1e-5, step
        assert abs(float(og["global_norm"]) / float(oe["global_norm"]) - 1.0) < 1e-5, step
    assert graph._graphed.graph is not None


@pytest.mark.parametrize("family,B,M,k,nf,H,nl,fw,T,prec", CASES[:1] + CASES[2:])
def test_all_windows_batch_matches_distinct_windows(family, B, M, k, nf, H, nl, fw, T, prec):
    from viforssms_amd.graph import GraphedStep
    a, b = _pair(family, B, M, k, nf, H, nl, fw, T, prec)
    gs = GraphedStep(b)
    starts = np.random.default_rng(7).choice(np.arange(0, a.target_len(), M), size=B, replace=True)
    gs._inputs(starts, 0)
    oa = a.elbo_step(a.batch_for(starts), 0, apply=False)
    ob = b.elbo_step(gs.batch, 0, apply=False, row0_dev=gs.row0)
    torch.cuda.synchronize()
    ea, eb = oa["elbo"].detach(), ob["elbo"].detach()
    assert torch.allclose(eb, ea, rtol=1e-5, atol=1e-5 * float(ea.abs().mean()))
    ga, gb = a.store.grad.double(), b.store.grad.double()
    assert float((ga - gb).norm() / ga.norm()) < 1e-5


def test_graph_steps_without_synchronize_match_synchronized_steps():
    """Replays issued back to back (the host runs ahead of the GPU, as bench.py --graph and main.py
    --graph do) give bitwise the same ELBOs and parameters as replays with a synchronize after every
    step: each step's window map reaches the GPU before the host stages the next one."""
    family, B, M, k, nf, H, nl, fw, T, prec = CASES[0]
    a, b = _pair(family, B, M, k, nf, H, nl, fw, T, prec)
    rng = np.random.default_rng(11)
    universe = np.arange(0, a.target_len(), M)
    draws = [rng.choice(universe, size=B, replace=True) for _ in range(10)]
    ea, eb = [], []
    for step, starts in enumerate(draws):
        ea.append(a.graphed_step(starts, step)["elbo"].clone())   # stream-ordered copy, no host sync
    for step, starts in enumerate(draws):
        eb.append(b.graphed_step(starts, step)["elbo"].clone())
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    for step, (x, y) in enumerate(zip(ea, eb)):
        assert torch.equal(x, y), step
    assert torch.equal(a.store.flat, b.store.flat)
