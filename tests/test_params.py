"""ParamStore's gradient hand-off (params.py; the flat gradient buffer Adamax reads, AR.py:228-234): the default
accumulation into zeroed .grad views and the released-view path (release_grads before the backward, sync_grads
after) give the same flat gradient, including a variable used twice (two contributions), one that receives none
(its slice stays zero) and stacked variables (views of one gradient), and the views are restored afterwards."""
import numpy as np
import torch

from viforssms_amd.params import ParamStore


def _store():
    rng = np.random.default_rng(3)
    st = ParamStore()
    for name, shape in (("a/kernel", (4, 3)), ("a/bias", (3,)), ("b/kernel", (3, 3)), ("c/kernel", (3, 3)),
                        ("unused", (5,))):
        st.add(name, rng.standard_normal(shape))
    return st.finalize("cpu")


def _loss(st, x):
    h = torch.tanh(x @ st["a/kernel"] + st["a/bias"])
    w = torch.stack([st["b/kernel"], st["c/kernel"]])          # stacked: the backward hands out views
    y = (h @ w[0]) * (h @ w[1]) + h @ st["b/kernel"]            # b/kernel used twice
    return (y ** 2).sum()


def _step(st, x, release):
    st.zero_grad()
    if release:
        st.release_grads()
    _loss(st, x).backward()
    st.sync_grads()
    return st.grad.clone()


def test_released_views_give_the_same_flat_gradient():
    x = torch.randn(6, 4, generator=torch.Generator().manual_seed(1))
    st = _store()
    g_views = _step(st, x, release=False)
    g_rel = _step(st, x, release=True)
    assert torch.allclose(g_rel, g_views, rtol=1e-6, atol=1e-6)
    a, sz = st.offsets["unused"]
    assert float(g_rel[a:a + sz].abs().max()) == 0.0
    for name, t in st.tensors.items():     # .grad points at the flat buffer again
        a, sz = st.offsets[name]
        assert t.grad.data_ptr() == st.grad[a:a + sz].data_ptr()
    # a second released step starts from zero (no carry-over into the flat buffer)
    assert torch.allclose(_step(st, x, release=True), g_views, rtol=1e-6, atol=1e-6)
