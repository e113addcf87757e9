"""Data-parallel path on CPU (gloo, world_size 2): every rank draws the same window starts,
owns samples [r*p_local, (r+1)*p_local), and the SUM all-reduce of the per-rank gradients of
sum(-ELBO) equals the full-batch gradient (the reference's single-process step, AR.py:228-234).
The per-rank gradients come from the oracle (the GPU kernels are covered by tests/test_gpu_parity.py);
what is tested here is the sharding, the window agreement and the collective."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nma_oracle as O
from oracle import bridge

P, M, T, SEED = 4, 50, 300, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _model():
    from tests.parity_util import build_model
    return build_model("ar", P, M, 6, 2, 12, 3, 3, "cpu", T=T, seed=3)


def _oracle_grad(model, starts, rows):
    md = model.mdef
    g = torch.Generator().manual_seed(11)
    eps = torch.randn(P, md.kernel_ext, generator=g, dtype=torch.float64)[rows]
    x0 = (torch.randn(P, md.P_theta, generator=g, dtype=torch.float64) * md.theta_base[1] + md.theta_base[0])[rows]
    batch = model.engine.make_batch(np.asarray(starts)[rows])
    inv = np.unique(np.asarray(starts)[rows], return_inverse=True)[1]
    ts = torch.tensor(batch.ts.double().numpy()[inv], dtype=O.DT)
    spec = bridge.spec_from_mdef(md, len(rows))
    params = bridge.oracle_params(model.store.state_numpy(), spec, model.engine.theta_dist.masks_np)
    leaves = O.param_leaves(params)
    for t in leaves:
        t.requires_grad_(True)
    out = O.elbo(spec, params, model.engine.perms, x0, eps, ts, {})
    grads = torch.autograd.grad((-out["elbo"]).sum(), leaves, allow_unused=True)
    grads = [torch.zeros_like(t) if g is None else g for t, g in zip(leaves, grads)]
    byname = bridge.oracle_grads_by_name(params, grads, spec)
    return np.concatenate([byname[n].ravel() for n in model.store.names()])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from viforssms_amd.vi_ssm import DistCtx
    model = _model()
    model.dist = DistCtx(rank, world)
    model.p_local = P // world
    np.random.seed(SEED)
    starts = model.select_windows()
    # every rank must draw the same global window starts
    gathered = [torch.zeros(P, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gathered, torch.as_tensor(starts))
    same = all(torch.equal(gathered[0], x) for x in gathered)
    local = model.batch_for(starts)
    rows = np.arange(rank * model.p_local, (rank + 1) * model.p_local)
    assert np.array_equal(local.starts, starts[rows])
    grad = torch.tensor(_oracle_grad(model, starts, rows))
    model.dist.all_reduce_(grad)
    if rank == 0:
        out.put((same, starts, grad.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gradient_equals_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time
    deadline = time.time() + 240
    while True:
        try:
            same, starts, reduced = q.get(timeout=1)
            break
        except queue.Empty:
            assert not any(p.exitcode not in (None, 0) for p in procs), "a rank failed"
            assert time.time() < deadline, "timed out"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert same
    full = _oracle_grad(_model(), starts, np.arange(P))
    assert np.allclose(reduced, full, rtol=1e-10, atol=1e-10 * np.abs(full).max())


def _overlap_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from viforssms_amd.vi_ssm import DistCtx
    model = _model()
    model.build_flow()
    model.dist = DistCtx(rank, world)
    st = model.store
    buckets = model._grad_buckets()
    res = []
    for overlap in (True, False):
        model.overlap_allreduce = overlap
        st.zero_grad()
        g = torch.Generator().manual_seed(100 + rank)
        # a loss touching every variable, differently per rank; flows' terms enter in reverse order
        loss = sum((st[n] * torch.randn(st[n].shape, generator=g, dtype=st[n].dtype)).sum() for n in st.names())
        model._arm_overlap()
        loss.backward()
        launched = len(model._ov["handles"]) if model._ov is not None else 0
        model._reduce_grads()
        res.append((launched, st.grad.clone().numpy()))
    if rank == 0:
        out.put(([b[0] for b in buckets], res))
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_overlapped_allreduce_equals_blocking_allreduce():
    """The per-flow gradient buckets (launched asynchronously from the accumulate hooks during the
    backward) reduce to exactly the single blocking all-reduce of the flat gradient, on 2 gloo ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time
    deadline = time.time() + 240
    while True:
        try:
            keys, res = q.get(timeout=1)
            break
        except queue.Empty:
            assert not any(p.exitcode not in (None, 0) for p in procs), "a rank failed"
            assert time.time() < deadline, "timed out"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert keys == ["flow1", "flow0", "rest"]       # backward completion order, q(theta) last
    (n_ov, g_ov), (n_blk, g_blk) = res
    assert n_ov == 2 and n_blk == 0                 # both flow buckets went out during the backward
    assert np.array_equal(g_ov, g_blk)
