"""The device window gather (vissm_gather_windows via features.DeviceTable, the product's per-step
feed assembly on the GPU) against the host restatement of the reference's gather
(features.FeatureTable.windows / feeds: AR.py:267-288, lotka_volterra_partial.py:366-386,
SV_dense.py:304-328): bit-identical time_feats and ELBO feeds for every family, with repeated,
unsorted and edge window starts (first and last start of arange(0, T, M))."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from tests.parity_util import build_model  # noqa: E402

DEV = "cuda:0"
CASES = [  # family, B, M, k, n_flows, H, n_layers, fw, T
    ("ar", 9, 30, 5, 2, 16, 3, 4, 150),
    ("ar", 50, 50, 50, 3, 16, 3, 10, 5000),  # hyperparameters.txt window geometry
    ("lv", 7, 40, 4, 2, 16, 5, 3, 160),
    ("fhn", 7, 40, 4, 2, 16, 5, 3, 160),
    ("sv", 7, 40, 8, 2, 16, 5, 3, 160),
]


@pytest.mark.parametrize("family,B,M,k,nf,H,nl,fw,T", CASES)
def test_device_gather_equals_host_gather(family, B, M, k, nf, H, nl, fw, T):
    model = build_model(family, B, M, k, nf, H, nl, fw, DEV, T=T)
    universe = np.arange(0, model.target_len(), M)
    rng = np.random.default_rng(1)
    starts = rng.choice(universe, size=B, replace=True)
    starts[0], starts[-1] = universe[0], universe[-1]
    batch = model.engine.make_batch(starts)
    torch.cuda.synchronize()
    tab = model.engine.table
    uniq, inv = np.unique(starts, return_inverse=True)
    ts_h = tab.windows(uniq).astype(np.float32)
    assert np.array_equal(batch.uniq, uniq)
    assert np.array_equal(batch.ts.cpu().numpy(), ts_h)
    assert np.array_equal(batch.win.cpu().numpy(), inv.astype(np.int32))
    feeds_h = tab.feeds(uniq, tab.windows(uniq))
    for key, want in feeds_h.items():
        got = getattr(batch.feeds, key)
        assert got is not None, key
        assert np.array_equal(got.cpu().numpy(), np.asarray(want, dtype=np.float32)), key


def test_single_window_batch_has_no_map():
    model = build_model("ar", 6, 40, 8, 3, 16, 3, 10, DEV, T=40)
    batch = model.engine.make_batch(np.zeros(6, dtype=np.int64))
    assert batch.win is None and batch.n_win == 1
    assert np.array_equal(batch.ts.cpu().numpy()[0], model.engine.table.windows([0])[0].astype(np.float32))
