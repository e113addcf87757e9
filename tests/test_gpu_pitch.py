"""Row pitches of the flow ABI (VissmFlowDesc.u_pitch / out_pitch): a flow whose u, du, u_next and du_next rows
lie a pitch > L (L - k) floats apart gives bitwise the results of the dense layout, on every flow implementation
(fp32, bf16, bf16x3; one and three hidden layers; stride 2 with the pair swap; the fused last AR(1) flow), with
several t-chunks (the halo join at the pitch) and pitches that are not multiples of 16.  The engine pads the rows
of every flow output that feeds another flow (Engine.pad_rows); its training-step gradient is bitwise that of
dense rows."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from viforssms_amd import _lib  # noqa: E402
from viforssms_amd.ops import FlowShape, MAFlowFn, ar_last_flow_fused  # noqa: E402

DEV = torch.device("cuda", 0)
P = {"fp32": _lib.VISSM_PREC_FP32, "bf16": _lib.VISSM_PREC_BF16, "bf16x3": _lib.VISSM_PREC_BF16X3}


def _padded(x: torch.Tensor, extra: int) -> torch.Tensor:
    buf = torch.full((x.shape[0], x.shape[1] + extra), float("nan"), device=x.device)
    buf[:, :x.shape[1]] = x
    return buf[:, :x.shape[1]]


def _run(sh, u, C, tt, ws, gnext, gls, tf, extra_u, extra_g):
    ins = [t.clone().requires_grad_(True) for t in (u, C, tt, *ws)]
    ui = _padded(ins[0].detach(), extra_u).requires_grad_(True) if extra_u else ins[0]
    bn = (ins[8], ins[9]) if sh.bn else (None, None)
    un, ls = MAFlowFn.apply(sh, None, ui, ins[1], ins[2], ins[3], ins[4], ins[5], bn[0], bn[1], ins[6], ins[7], tf)
    g = _padded(gnext, extra_g) if extra_g else gnext
    torch.autograd.backward([un, ls], [g, gls])
    return [un.detach().contiguous(), ls.detach(), ui.grad.contiguous()] + [t.grad for t in ins[1:]]


@pytest.mark.parametrize("prec", ["fp32", "bf16", "bf16x3"])
@pytest.mark.parametrize("nh,stride2,k", [(1, False, 8), (3, True, 20), (3, False, 50)])
def test_flow_pitch_bitwise(prec, nh, stride2, k):
    g = torch.Generator(device=DEV).manual_seed(3)
    r = lambda *s, sc=1.0: (torch.randn(*s, generator=g, device=DEV) * sc).contiguous()
    B, T, H = 5, 700, 50
    D = 2 if stride2 else 1
    L = 3 * k + D * T + D
    base = FlowShape(B=B, L=L, k=k, H=H, n_hidden=nh, bn=nh > 1, stride2=stride2, swap_out=stride2,
                     n_logsig=D * T, n_win=1, precision=P[prec], chunk_tiles=2)
    u, C, tt = r(B, L), r(1, base.Lh, H, sc=0.3), r(B, H, sc=0.2)
    ws = [r(k, H, sc=0.3), r(nh, H, H, sc=0.15), r(nh, H, sc=0.1), r(H, 2, sc=0.2), r(2, sc=0.1)]
    if nh > 1:
        ws += [1 + r(nh, H, sc=0.1), r(nh, H, sc=0.1)]
    gnext, gls = r(B, base.Lout), r(B)
    ref = _run(base, u, C, tt, ws, gnext, gls, None, 0, 0)
    for pad_out, eu, eg in [(True, 7, 3), (False, 16 - L % 16, 0), (True, 0, 16 - base.Lout % 16)]:
        sh = FlowShape(**{**base.__dict__, "pad_out": pad_out})
        out = _run(sh, u, C, tt, ws, gnext, gls, None, eu, eg)
        names = ["u_next", "logsig", "du", "dC", "dtheta", "dw_eps", "dw_hid", "db_hid", "dw_head", "db_head"]
        for name, a, b in zip(names + (["dbn_g", "dbn_b"] if nh > 1 else []), out, ref):
            assert torch.equal(a, b), (name, pad_out, eu, eg, float((a - b).abs().max()))


@pytest.mark.parametrize("prec", ["bf16", "bf16x3"])
def test_fused_flow_pitch_bitwise(prec):
    g = torch.Generator(device=DEV).manual_seed(5)
    r = lambda *s, sc=1.0: (torch.randn(*s, generator=g, device=DEV) * sc).contiguous()
    B, M, k, H = 6, 400, 8, 50
    L = M + 1 + k
    sh = FlowShape(B=B, L=L, k=k, H=H, n_hidden=1, bn=False, stride2=False, swap_out=False, n_logsig=M, n_win=1,
                   precision=P[prec], chunk_tiles=4)
    u, C, tt = r(B, L), r(1, sh.Lh, H, sc=0.3), r(B, H, sc=0.2)
    theta = torch.stack([r(B, sc=0.3) + 1.0, torch.rand(B, generator=g, device=DEV) * 0.8,
                         r(B, sc=0.2).abs() + 0.5], 1).contiguous()
    obs, obs_bin = r(1, M), (torch.rand(1, M, generator=g, device=DEV) < 0.3).float()
    ws = [r(k, H, sc=0.3), r(1, H, H, sc=0.15), r(1, H, sc=0.1), r(H, 2, sc=0.2), r(2, sc=0.1)]
    ref = ar_last_flow_fused(sh, None, u, C, tt, theta, obs, obs_bin, 1.0, 5000 / M, *ws)
    out = ar_last_flow_fused(sh, None, _padded(u, 16 - L % 16), C, tt, theta, obs, obs_bin, 1.0, 5000 / M, *ws)
    for i, (a, b) in enumerate(zip(out[:5], ref[:5])):
        assert torch.equal(a.contiguous(), b.contiguous()), i
    for a, b in zip(out[5], ref[5]):
        assert torch.equal(a, b)


def _step(family, prec, pad, step_path):
    from tests.parity_util import build_model
    B, M, k, nf, H, nl, fw = {"ar": (6, 300, 8, 3, 50, 3, 10), "lv": (4, 200, 20, 3, 50, 5, 10),
                              "fhn": (4, 200, 20, 3, 50, 5, 10), "sv": (3, 52, 50, 5, 50, 5, 5)}[family]
    model = build_model(family, B, M, k, nf, H, nl, fw, str(DEV), precision=prec, seed=3)
    model.engine.pad_rows = pad
    model.engine.chunk_tiles = 3
    md = model.mdef
    batch = model.engine.make_batch(np.zeros(B, dtype=np.int64))
    g = torch.Generator().manual_seed(14)
    eps = torch.randn(B, md.kernel_ext, generator=g).to(DEV)
    x0 = (torch.randn(B, md.P_theta, generator=g) * md.theta_base[1] + md.theta_base[0]).to(DEV)
    st = model.store
    if step_path:
        out = model.elbo_step(batch, 0, eps=eps, x0_theta=x0, apply=False)
    else:
        st.zero_grad()
        out = model.forward(batch, 0, eps=eps, x0_theta=x0)
        (-out["elbo"]).sum().backward()
    st.sync_grads()
    torch.cuda.synchronize()
    return out["elbo"].detach().clone(), st.grad.detach().clone()


@pytest.mark.parametrize("family,prec,step_path", [("ar", 1, True), ("ar", 1, False), ("ar", 0, False),
                                                   ("lv", 1, False), ("fhn", 1, False), ("sv", 1, False)])
def test_engine_padded_rows_bitwise(family, prec, step_path):
    """The ELBO and flat gradient (training step: AR's last flow fused) with padded flow rows equal dense rows'."""
    e0, g0 = _step(family, prec, False, step_path)
    e1, g1 = _step(family, prec, True, step_path)
    assert torch.equal(e0, e1)
    assert torch.equal(g0, g1), float((g0 - g1).abs().max())
