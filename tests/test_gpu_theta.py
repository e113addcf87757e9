"""q(theta) on the HIP kernels (vissm_theta_fwd / vissm_theta_bwd, csrc/theta.hip) against the tensor-op
restatement ThetaFlow.sample_and_log_prob_torch (itself pinned to the float64 oracle's
qtheta_sample_logprob, AR.py:376-391, by the end-to-end parity tests): theta, log q and every MAF
variable's gradient, for the families' shapes (P = 3 elu, 4 relu, 5 elu), partial waves and blocks,
log-scales beyond the [-5, 3] clip (straight-through gradient), and bitwise determinism."""
import numpy as np
import pytest
import torch

from viforssms_amd.params import ParamStore
from viforssms_amd.theta_flow import ThetaFlow

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _flow(P, n, act, scale=1.0, seed=0):
    rng = np.random.default_rng(seed)
    st = ParamStore()
    perms = [list(rng.permutation(P)) for _ in range(n - 1)]
    tf = ThetaFlow(st, P, n, perms, 0.5, 1.5, act, rng=rng)
    st.finalize(DEV)
    with torch.no_grad():
        # non-zero biases and larger weights so every term (and the clip) is exercised
        g = torch.Generator().manual_seed(seed)
        for name, t in st.tensors.items():
            t.add_((torch.randn(t.shape, generator=g) * (0.3 * scale)).to(DEV) * (1.0 if "bias" in name else 0.0))
            if "kernel" in name:
                t.mul_(scale)
    return st, tf


def _run(st, tf, x0, gth, glq, hip):
    st.zero_grad()
    f = tf.sample_and_log_prob if hip else tf.sample_and_log_prob_torch
    th, lq = f(x0)
    loss = (th * gth).sum() + (lq * glq).sum()
    loss.backward()
    st.sync_grads()
    torch.cuda.synchronize()
    return th.detach().clone(), lq.detach().clone(), st.grad.clone()


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("P,n,act,B", [(3, 5, "elu", 1000), (4, 5, "relu", 65), (5, 4, "elu", 64), (3, 2, "elu", 1),
                                       (3, 5, "elu", 65536), (2, 1, "relu", 130), (1, 3, "elu", 257)])
def test_theta_kernels_match_tensor_ops(P, n, act, B):
    st, tf = _flow(P, n, act, seed=P + n)
    g = torch.Generator().manual_seed(7)
    x0 = (torch.randn(B, P, generator=g) * 1.5 + 0.5).to(DEV)
    gth = torch.randn(B, P, generator=g).to(DEV)
    glq = torch.randn(B, generator=g).to(DEV)
    th_t, lq_t, g_t = _run(st, tf, x0, gth, glq, hip=False)
    th_h, lq_h, g_h = _run(st, tf, x0, gth, glq, hip=True)
    assert _rel(th_h, th_t) < 1e-5, _rel(th_h, th_t)
    assert _rel(lq_h, lq_t) < 1e-5, _rel(lq_h, lq_t)
    assert _rel(g_h, g_t) < 1e-4, _rel(g_h, g_t)
    # per variable
    for name, (a, sz) in st.offsets.items():
        ref = g_t[a:a + sz]
        if ref.norm() > 0:
            assert _rel(g_h[a:a + sz], ref) < 1e-3, name


def test_theta_clip_is_straight_through():
    st, tf = _flow(3, 3, "elu", scale=3.0, seed=4)
    with torch.no_grad():  # log-scale biases near and beyond the clip bounds [-5, 3]
        for i in range(3):
            st.tensors[f"theta/maf{i}/dense3/bias"][1::2] = torch.tensor([3.5, -5.2, 2.8], device=DEV)
    g = torch.Generator().manual_seed(3)
    x0 = (torch.randn(500, 3, generator=g) * 3).to(DEV)
    gth = torch.randn(500, 3, generator=g).to(DEV)
    glq = torch.ones(500).to(DEV)
    # the clip is active for some samples
    with torch.no_grad():
        _, ls = tf._shift_log_scale(0, x0)
    assert bool(((ls <= -5) | (ls >= 3)).any())  # (the returned log-scale is the clipped value)
    th_t, lq_t, g_t = _run(st, tf, x0, gth, glq, hip=False)
    th_h, lq_h, g_h = _run(st, tf, x0, gth, glq, hip=True)
    assert _rel(th_h, th_t) < 1e-5 and _rel(lq_h, lq_t) < 1e-5
    assert _rel(g_h, g_t) < 1e-4, _rel(g_h, g_t)


def test_theta_backward_deterministic_and_accumulates():
    st, tf = _flow(3, 5, "elu", seed=1)
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(3000, 3, generator=g).to(DEV)
    gth = torch.randn(3000, 3, generator=g).to(DEV)
    glq = torch.randn(3000, generator=g).to(DEV)
    _, _, g1 = _run(st, tf, x0, gth, glq, hip=True)
    _, _, g2 = _run(st, tf, x0, gth, glq, hip=True)
    assert torch.equal(g1, g2)
    # the backward adds into the gradient buffer (two backwards without zeroing = twice the gradient)
    st.zero_grad()
    for _ in range(2):
        th, lq = tf.sample_and_log_prob(x0)
        ((th * gth).sum() + (lq * glq).sum()).backward()
    torch.cuda.synchronize()
    assert torch.allclose(st.grad, 2 * g1, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("B,P", [(1, 3), (63, 3), (64, 3), (65, 4), (1000, 3), (65536, 3), (4097, 8)])
def test_theta_branch_backward_kernel(B, P):
    """vissm_theta_branch_bwd (the flows' theta branch, nma._ThetaBranch: ((theta W0 + b0) W1 + b1) W2 + b2,
    AR.py:63-68) against float64 autograd of the three layers, every output to fp32 summation order, and bitwise
    reproducible."""
    from viforssms_amd.ops import theta_branch_bwd
    g = torch.Generator().manual_seed(B + P)
    r = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64)
    H = 50
    theta, d = r(B, P), r(B, H)
    W0, b0, W1, b1, W2, b2 = r(P, 50) * 0.3, r(50) * 0.1, r(50, 50) * 0.14, r(50) * 0.1, r(50, H) * 0.14, r(H) * 0.1
    leaves = [t.clone().requires_grad_(True) for t in (theta, W0, b0, W1, b1, W2, b2)]
    th, w0, c0, w1, c1, w2, c2 = leaves
    (((th @ w0 + c0) @ w1 + c1) @ w2 + c2).backward(d)
    ref = [t.grad for t in leaves]
    dev = lambda t: t.float().cuda()
    got = theta_branch_bwd(*(dev(t) for t in (theta, d, W0, b0, W1, b1, W2)))
    again = theta_branch_bwd(*(dev(t) for t in (theta, d, W0, b0, W1, b1, W2)))
    torch.cuda.synchronize()
    for name, a, b, c in zip(("dtheta", "dW0", "db0", "dW1", "db1", "dW2", "db2"), got, again, ref):
        assert torch.equal(a, b), name
        err = float((a.double().cpu() - c).norm() / (c.norm() + 1e-30))
        assert err < 1e-5, (name, err)


@pytest.mark.parametrize("B,P", [(0, 3), (1, 3), (1000, 3), (65536, 3), (77, 8)])
def test_theta_branch_forward_kernel(B, P):
    """vissm_theta_branch_fwd: the collapsed weights Wc = W0 W1 W2, bc = (b0 W1 + b1) W2 + b2 and theta_term =
    theta Wc + bc against float64 (AR.py:63-68's three dense layers)."""
    from viforssms_amd.ops import theta_branch_fwd
    g = torch.Generator().manual_seed(B + 7 * P)
    r = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64)
    theta = r(B, P)
    W0, b0, W1, b1, W2, b2 = r(P, 50) * 0.3, r(50) * 0.1, r(50, 50) * 0.14, r(50) * 0.1, r(50, 50) * 0.14, r(50) * 0.1
    ref = ((theta @ W0 + b0) @ W1 + b1) @ W2 + b2
    Wc_ref, bc_ref = W0 @ W1 @ W2, (b0 @ W1 + b1) @ W2 + b2
    tt, Wc, bc = theta_branch_fwd(*(t.float().cuda() for t in (theta, W0, b0, W1, b1, W2, b2)))
    torch.cuda.synchronize()
    rel = lambda a, b: float((a.double().cpu() - b).norm() / (b.norm() + 1e-30))
    assert rel(Wc, Wc_ref) < 1e-6 and rel(bc, bc_ref) < 1e-6
    assert tt.shape == (B, 50)
    if B:
        assert rel(tt, ref) < 1e-6
