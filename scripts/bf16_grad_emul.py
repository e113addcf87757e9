"""Which rounding limits the GRADIENT of the bf16 training modes?  CPU emulation on the float64 oracle at the AR-cfg
shape (conditioned draw, as tests/test_gpu_config_parity.py): every flow product runs through a custom autograd
function that rounds (bf16, round to nearest even) exactly the operands the HIP kernels round --

  forward / recompute:  activations (u taps, ELU outputs) and weights (w_eps, hidden, head) of each MFMA;
  backward chain:       dI = W dZ, dcon = w_eps dA0, the head backward W_head (g_mu, g_r): weight and gradient;
  weight gradients:     dW = I dZ^T, dW_eps = U dA0^T, dW_head = I1 G^T: activation and gradient operands;
  window-shared / theta: dC and d theta_term sum the bf16-rounded dA0 image --

each switch on or off, accumulation exact.  Split-weight modes keep the weight operand exact (w_hi x + w_lo x is
exact to ~2^-16).  Reports the per-sample ELBO and the whole-gradient relative L2 error against the exact float64
oracle gradient.  usage: python scripts/bf16_grad_emul.py [B] [seeds] [M]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import nma_oracle as O  # noqa: E402
from oracle import bridge  # noqa: E402
from tests.parity_util import build_model, oracle_inputs  # noqa: E402

from oracle.precision_model import MODE, iaf_flow_emul  # noqa: E402  (the rounding model, shared with the tests)


MODES = {
    "bf16 (headline)": dict(fwd_x=1, fwd_w=1, bwd_g=1, bwd_w=1, wg_x=1),
    "bf16x2f (split fwd/recompute weights)": dict(fwd_x=1, fwd_w=0, bwd_g=1, bwd_w=1, wg_x=1),
    "bf16x2 (split weights everywhere)": dict(fwd_x=1, fwd_w=0, bwd_g=1, bwd_w=0, wg_x=1),
    "bf16x2, gradient operands exact": dict(fwd_x=1, fwd_w=0, bwd_g=0, bwd_w=0, wg_x=1),
    "bf16 fwd, split backward chain weights": dict(fwd_x=1, fwd_w=1, bwd_g=1, bwd_w=0, wg_x=1),
    "bf16x3 (~exact)": dict(),
}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
    errs = {m: ([], []) for m in MODES}
    orig = O.iaf_flow
    for seed in range(3, 3 + seeds):
        model = build_model("ar", B, M, 8, 3, 50, 3, 10, "cpu", seed=seed, impute=5, condition=True)
        md = model.mdef
        spec = bridge.spec_from_mdef(md, B)
        params = bridge.oracle_params(model.store.state_numpy(), spec, model.engine.theta_dist.masks_np)
        ts, ex = oracle_inputs(model, np.zeros(B, dtype=np.int64))
        g = torch.Generator().manual_seed(seed + 11)
        eps = torch.randn(B, md.kernel_ext, generator=g, dtype=torch.float64)
        x0 = torch.randn(B, md.P_theta, generator=g, dtype=torch.float64) * md.theta_base[1] + md.theta_base[0]
        leaves = O.param_leaves(params)

        def run():
            for t in leaves:
                t.grad = None
                t.requires_grad_(True)
            o = O.elbo(spec, params, model.engine.perms, x0, eps, ts, ex)
            (-o["elbo"]).sum().backward()
            return o["elbo"].detach().numpy(), torch.cat([t.grad.reshape(-1) for t in leaves]).clone()

        e_ref, g_ref = run()
        O.iaf_flow = iaf_flow_emul
        try:
            for m, flags in MODES.items():
                MODE.clear()
                MODE.update({k: bool(v) for k, v in flags.items()})
                e, gg = run()
                errs[m][0].append(float(np.max(np.abs(e - e_ref) / np.abs(e_ref))))
                errs[m][1].append(float((gg - g_ref).norm() / g_ref.norm()))
        finally:
            O.iaf_flow = orig
        print(f"seed {seed} done", flush=True)
    print(f"AR-cfg flows, M = {M}, B = {B}, {seeds} seeds: max per-sample ELBO rel err / gradient rel L2 err")
    for m, (e, gq) in errs.items():
        print(f"  {m:42s} ELBO {max(e):.2e}   grad {max(gq):.2e}")


if __name__ == "__main__":
    main()
