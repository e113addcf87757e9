"""Host-side model construction for the four families (no GPU compute): variable inventory,
window selection and the FHN train_paths freeze mask."""
import numpy as np
import pytest

from tests.parity_util import build_model


def _flow_vars(model, i):
    return {n: model.store.tensors[n].shape for n in model.store.names() if n.startswith(f"flow{i}/")}


@pytest.mark.parametrize("family,k", [("ar", 4), ("lv", 4), ("sv", 6), ("fhn", 4)])
def test_variable_inventory(family, k):
    """Per flow: 4 feature dense layers, the [k, 1 + CF, H] conv, 3 theta dense, n_hidden 1x1
    layers (+ BN gamma/beta for LV/SV/FHN) and the [H, 2] head (AR.py:38-89 and variants)."""
    nl = 3 if family == "ar" else 5
    m = build_model(family, 4, 24, k, 2, 16, nl, 3, "cpu")
    md = m.mdef
    for i in range(md.n_flows):
        v = _flow_vars(m, i)
        nh = nl - 2
        assert len(v) == 8 + 2 + 6 + nh * (2 if family == "ar" else 4) + 2
        CF = md.kernel_ext - 1 if family == "lv" else 16
        assert v[f"flow{i}/conv/kernel"] == (k, 1 + CF, 16)
        assert v[f"flow{i}/head/kernel"] == (16, 2)
        if family == "lv":   # last feature layer is as wide as the flow's input
            assert v[f"flow{i}/feat3/kernel"] == (16, md.kernel_ext - 1 - i * k)
    assert md.kernel_ext == k * 2 + md.D * 24 + md.D
    n_maf = {"ar": 5, "lv": 4, "sv": 5, "fhn": 4}[family]
    assert sum(1 for n in m.store.names() if n.startswith("theta/")) == n_maf * 8


def test_lv_window_selection_uses_target_dims():
    m = build_model("lv", 6, 40, 4, 2, 16, 5, 3, "cpu", T=160)
    np.random.seed(0)
    s = m.select_windows()
    assert set(s.tolist()) <= {0, 40, 80, 120} and len(s) == 6


def test_fhn_train_paths_false_freezes_path_variables():
    from viforssms_amd.fhn import VI_SSM
    from viforssms_amd.data import fhn_data_gen
    from viforssms_amd.vi_ssm import ThetaSpec
    obs, ob, tt, _ = fhn_data_gen(40, obs_every=10, seed=0)
    spec = ThetaSpec(4, [[0, 1, 2, 3, 4]] * 3, 0.0, 1.0, "elu")
    m = VI_SSM(obs, ob, tt, np.array([2.0, 3.0]), spec, [(0.0, 10.0)] * 5, 0.1, 4.0, 2, 4, 40, [16] * 5, 40, 2, 3,
               train_paths=False, device="cpu")
    mask = m.grad_mask().numpy()
    for name, (a, n) in m.store.offsets.items():
        frozen = name.startswith("flow") and "/feat" not in name and "/bn" not in name  # BN, features stay trainable
        assert (mask[a:a + n] == (0.0 if frozen else 1.0)).all(), name


def test_drop_in_scripts_expose_reference_names():
    import importlib
    for mod in ("lotka_volterra_partial", "SV_dense", "fitz_nag_NVP", "AR"):
        m = importlib.import_module(mod)
        assert hasattr(m, "VI_SSM")
