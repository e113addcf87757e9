"""The three-hidden-layer kernels that ship from flow_v5n.hip (LV / FHN, kernel_len <= 24) are built with
-mllvm -amdgpu-mfma-vgpr-form=1 and inline-asm AGPR accumulators; the same flag miscompiled SV's k = 50 du variant
(profiles/r06/svflag: deterministic, not a wait-state hazard -- padding every instruction reproduces it bit for bit;
DESIGN.md §8).  Here every shipped shape runs through that build and through the same source built without the flag
(flow_v5s.hip, VISSM_NH3_DEFAULT_FORM=1): the per-sample ELBO and every variable's gradient must agree to fp32
rounding, at the benchmark's launch geometry (the t-chunks its items walk) and at small edge shapes, for the first
flow's no-du variant and the du variant of the others, LV's stride-2 head with the pair swap and FHN's."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from tests.parity_util import bench_geometry, build_model  # noqa: E402
from viforssms_amd._lib import TRAIN_PRECISIONS as PREC  # noqa: E402

DEV = "cuda:0"


def _elbo_and_grad(model, batch, eps, x0):
    st = model.store
    st.zero_grad()
    out = model.forward(batch, 0, eps=eps, x0_theta=x0)
    (-out["elbo"]).sum().backward()
    st.sync_grads()
    torch.cuda.synchronize()
    return out["elbo"].detach().double().cpu().numpy(), st.grad.detach().double().cpu().numpy().copy()


@pytest.mark.parametrize("family,B,M,k,nf,H,fw,bench_B", [
    ("lv", 3, 5000, 20, 3, 50, 10, 16384),   # LV-cfg at the bench geometry
    ("fhn", 3, 2000, 20, 3, 50, 10, 8192),   # FHN-cfg at the bench geometry
    ("lv", 5, 40, 24, 2, 32, 3, 0),          # k = 24 (two layer-0 K blocks), partial group
    ("fhn", 4, 24, 4, 2, 16, 3, 0),          # small k and H
])
def test_vgpr_form_build_matches_default_form(family, B, M, k, nf, H, fw, bench_B):
    prec = PREC["bf16"]
    model = build_model(family, B, M, k, nf, H, 5, fw, DEV, precision=prec, seed=7, condition=M > 1000)
    if bench_B:
        model.engine.chunk_tiles = bench_geometry(family, prec, bench_B, M, k, nf, H)[0]["chunk_tiles"]
    md = model.mdef
    batch = model.engine.make_batch(np.zeros(B, dtype=np.int64))
    g = torch.Generator().manual_seed(11)
    eps = torch.randn(B, md.kernel_ext, generator=g).to(DEV)
    x0 = (torch.randn(B, md.P_theta, generator=g) * md.theta_base[1] + md.theta_base[0]).to(DEV)
    old = os.environ.pop("VISSM_NH3_DEFAULT_FORM", None)
    try:
        e_v, g_v = _elbo_and_grad(model, batch, eps, x0)        # flow_v5n.hip: VGPR form + asm accumulators
        os.environ["VISSM_NH3_DEFAULT_FORM"] = "1"
        e_d, g_d = _elbo_and_grad(model, batch, eps, x0)        # flow_v5s.hip: the compiler's default form
    finally:
        os.environ.pop("VISSM_NH3_DEFAULT_FORM", None)
        if old is not None:
            os.environ["VISSM_NH3_DEFAULT_FORM"] = old
    assert np.isfinite(e_v).all() and np.isfinite(g_v).all()
    de = float(np.max(np.abs(e_v - e_d) / np.maximum(np.abs(e_d), 1e-6)))
    st = model.store
    worst = max((float(np.linalg.norm(g_v[a:a + n] - g_d[a:a + n]) / (np.linalg.norm(g_d[a:a + n]) + 1e-30)), name)
                for name, (a, n) in st.offsets.items() if np.linalg.norm(g_d[a:a + n]) > 0)
    print(family, M, k, "ELBO", de, "worst variable", worst, "bitwise", bool(np.array_equal(g_v, g_d)))
    assert de < 1e-6, de
    assert worst[0] < 1e-5, worst
