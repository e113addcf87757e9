"""optimisers.adamax.AdamaxOptimizer (the drop-in facade of optimisers/adamax.py:11-61) on the HIP kernels,
against the oracle's clip_by_global_norm + adamax_update (AR.py:230-234, optimisers/adamax.py:42-58)
over several steps: contiguous, non-contiguous (a transposed view) and fp16 variables in one call,
with and without the global-norm clip, and the in-place path for consecutive views of one buffer."""
import pytest
import torch

from oracle import nma_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _oracle_steps(vals, grads_seq, lr, b1, b2, clip, eps):
    vals = [v.double().clone() for v in vals]
    slots = [(torch.zeros_like(v), torch.zeros_like(v)) for v in vals]
    for grads in grads_seq:
        gs = [g.double() for g in grads]
        if clip > 0:
            gs, _ = O.clip_by_global_norm(gs, clip)
        out = []
        for i, (v, g, (sv, sm)) in enumerate(zip(vals, gs, slots)):
            nv, nsv, nsm = O.adamax_update(v, g, sv, sm, lr, b1, b2, eps[i])
            out.append(nv)
            slots[i] = (nsv, nsm)
        vals = out
    return vals, slots


@pytest.mark.parametrize("clip", [0.0, 5.0])
def test_facade_mixed_layouts_and_dtypes(clip):
    from optimisers.adamax import AdamaxOptimizer
    g = torch.Generator().manual_seed(1)
    a = torch.randn(37, generator=g)
    base = torch.randn(6, 9, generator=g)
    h = torch.randn(11, generator=g).half()
    vars_ = [a.to(DEV), base.to(DEV).t(), h.to(DEV)]          # the second is a non-contiguous view
    assert not vars_[1].is_contiguous()
    init = [v.detach().float().cpu().clone() for v in vars_]
    opt = AdamaxOptimizer(learning_rate=1e-2, beta1=0.95)
    grads_seq = []
    for _ in range(3):
        grads = [torch.randn(v.shape, generator=g) * 3 for v in vars_]
        grads_seq.append(grads)
        opt.apply_gradients([(gr.to(DEV).to(v.dtype), v) for gr, v in zip(grads, vars_)], clip_norm=clip)
    torch.cuda.synchronize()
    grads_in = [[gr.to(v.dtype).float() for gr, v in zip(grads, vars_)] for grads in grads_seq]
    ref, slots = _oracle_steps(init, grads_in, 1e-2, 0.95, 0.999, clip, [1e-8, 1e-8, 1e-7])
    for i, (v, r) in enumerate(zip(vars_, ref)):
        tol = 2e-3 if v.dtype == torch.float16 else 1e-5
        assert torch.allclose(v.double().cpu(), r, rtol=tol, atol=tol), i
    for i, v in enumerate(vars_[:2]):
        assert torch.allclose(opt.get_slot(v, "v").double().cpu(), slots[i][0], rtol=1e-5, atol=1e-6)
        assert torch.allclose(opt.get_slot(v, "m").double().cpu(), slots[i][1], rtol=1e-5, atol=1e-6)


def test_facade_consecutive_views_update_in_place():
    from optimisers.adamax import AdamaxOptimizer
    flat = torch.randn(100, device=DEV)
    views = [flat[0:30].view(5, 6), flat[30:100]]
    copies = [v.clone() for v in views]
    g = [torch.randn_like(v) for v in views]
    o1, o2 = AdamaxOptimizer(1e-3, 0.9), AdamaxOptimizer(1e-3, 0.9)
    assert o1._group_for(views).flat_view is not None
    o1.apply_gradients(list(zip(g, views)), clip_norm=2.0)
    o2.apply_gradients(list(zip(g, copies)), clip_norm=2.0)
    torch.cuda.synchronize()
    assert o2._group_for(copies).flat_view is None
    for v, c in zip(views, copies):
        assert torch.equal(v, c)


def test_facade_slots_follow_changing_groupings():
    """var lists [a, b] -> [a] (b's gradient None) -> [a, b] again: the cached group of the first call must pick up
    a's slots from the second call (one slot pair per variable, optimisers/adamax.py:36-40) and get_slot must keep
    returning the live values; checked against a per-variable oracle Adamax."""
    from optimisers.adamax import AdamaxOptimizer
    g = torch.Generator().manual_seed(5)
    a0, b0 = torch.randn(13, generator=g), torch.randn(7, generator=g)
    a, b = a0.to(DEV), b0.to(DEV)
    opt = AdamaxOptimizer(learning_rate=1e-2, beta1=0.9)
    seq = [("ab", torch.randn(13, generator=g), torch.randn(7, generator=g)),
           ("a", torch.randn(13, generator=g), None),
           ("ab", torch.randn(13, generator=g), torch.randn(7, generator=g)),
           ("a", torch.randn(13, generator=g), None),
           ("ab", torch.randn(13, generator=g), torch.randn(7, generator=g))]
    for _, ga, gb in seq:
        opt.apply_gradients([(ga.to(DEV), a), (None if gb is None else gb.to(DEV), b)])
    torch.cuda.synchronize()
    ra, sa = _oracle_steps([a0], [[ga] for _, ga, _ in seq], 1e-2, 0.9, 0.999, 0.0, [1e-8])
    rb, sb = _oracle_steps([b0], [[gb] for _, _, gb in seq if gb is not None], 1e-2, 0.9, 0.999, 0.0, [1e-8])
    assert torch.allclose(a.double().cpu(), ra[0], rtol=1e-5, atol=1e-6)
    assert torch.allclose(b.double().cpu(), rb[0], rtol=1e-5, atol=1e-6)
    for var, slots in ((a, sa[0]), (b, sb[0])):
        assert torch.allclose(opt.get_slot(var, "v").double().cpu(), slots[0], rtol=1e-5, atol=1e-6)
        assert torch.allclose(opt.get_slot(var, "m").double().cpu(), slots[1], rtol=1e-5, atol=1e-6)
