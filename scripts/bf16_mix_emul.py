"""Which flow products need the split (bf16x3) operands for the ELBO to meet 1e-4?  CPU emulation on the
float64 oracle: the operands of each product class of the IAF flow (layer 0 = the sample channel's
taps u x w_eps, hidden = ELU output x W + bias, head = ELU output x W_head + bias) are rounded to bf16
(round to nearest even) or kept exact (bf16x3 is exact to ~2^-16), accumulation exact; C (feature
channels + bias) and the theta term enter in full precision, as in the kernels (the MFMA C operand).
Case: the AR-cfg shape at its own length (parity_util.build_model, conditioned draw), several seeds.
usage: python scripts/bf16_mix_emul.py [B] [seeds]"""
import itertools
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import nma_oracle as O  # noqa: E402
from tests.parity_util import build_model, oracle_inputs  # noqa: E402
from oracle import bridge  # noqa: E402


def rb(x):
    """round to bf16 (RNE) and back, float64 in / out"""
    return x.float().bfloat16().double()


MODE = {"l0": False, "hid": False, "head": False}   # True: bf16 operands
WEIGHTS_EXACT = False   # True: only the activation operands are rounded (bf16x2: W_hi x + W_lo x)


def q(x, cls, weight=False):
    if weight and WEIGHTS_EXACT:
        return x
    return rb(x) if MODE[cls] else x


def iaf_flow_emul(u, CF, theta, P, cfg):
    w = P["conv_w"][:, :1, :]
    k = w.shape[0]
    x = u[:, :-1, None]
    n_out = x.shape[1] - k + 1
    a = CF + O.theta_term(theta, P)[:, None, :]
    for j in range(k):
        a = a + q(x[:, j:j + n_out, :], "l0") @ q(w[j], "l0", True)
    h = O.elu(a)
    for l in range(cfg.n_hidden):
        h = O.elu(q(h, "hid") @ q(P[f"hid_w{l}"], "hid", True) + q(P[f"hid_b{l}"], "hid", True))
    head = q(h, "head") @ q(P["head_w"], "head", True) + q(P["head_b"], "head", True)
    mu, sig = head[..., 0], O.softplus(head[..., 1]) + 1e-10
    return u[:, cfg.k:] * sig + mu, torch.log(sig[:, -cfg.n_logsig:])


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    global WEIGHTS_EXACT
    modes = [(w,) + m for w in (False, True) for m in itertools.product([False, True], repeat=3)]
    errs = {m: [] for m in modes}
    for seed in range(3, 3 + seeds):
        model = build_model("ar", B, 5000, 8, 3, 50, 3, 10, "cpu", seed=seed, impute=5, condition=True)
        md = model.mdef
        spec = bridge.spec_from_mdef(md, B)
        params = bridge.oracle_params(model.store.state_numpy(), spec, model.engine.theta_dist.masks_np)
        starts = np.zeros(B, dtype=np.int64)
        ts, ex = oracle_inputs(model, starts)
        g = torch.Generator().manual_seed(seed + 11)
        eps = torch.randn(B, md.kernel_ext, generator=g, dtype=torch.float64)
        x0 = torch.randn(B, md.P_theta, generator=g, dtype=torch.float64) * md.theta_base[1] + md.theta_base[0]
        with torch.no_grad():
            ref = O.elbo(spec, params, model.engine.perms, x0, eps, ts, ex)["elbo"].numpy()
            orig = O.iaf_flow
            O.iaf_flow = iaf_flow_emul
            try:
                for m in modes:
                    WEIGHTS_EXACT = m[0]
                    MODE.update(l0=m[1], hid=m[2], head=m[3])
                    e = O.elbo(spec, params, model.engine.perms, x0, eps, ts, ex)["elbo"].numpy()
                    errs[m].append(float(np.max(np.abs(e - ref) / np.abs(ref))))
            finally:
                O.iaf_flow = orig
    print("(weights exact, bf16 operands in layer0, hidden, head) -> max per-sample ELBO rel err over seeds")
    for m in modes:
        print(m, ["%.2e" % v for v in errs[m]], "max %.2e" % max(errs[m]))


if __name__ == "__main__":
    main()
