"""Data parallelism on the HIP path: 2 ranks share cuda:0 over gloo (RCCL needs one
GPU per rank; the driver's 8-GPU run uses RCCL with the same code).  Each rank draws the same window
starts, its own Philox rows (keyed by the global sample index), runs the HIP forward/backward on its
half of the samples and SUM-all-reduces the flat gradient -- per-flow buckets launched from the
backward's accumulate hooks, overlapping the remaining flows' kernels.  Checked against one process
running the full batch: the all-reduced gradient equals the full-batch HIP gradient (to fp32 summation
order), the parameters after clip + Adamax are bitwise identical on both ranks, and the bucketed
overlapped reduce equals the single blocking all-reduce bitwise.  AR at fp32 (two windows) and LV at bf16 (one
window: the two-sample three-layer backward and the split-bf16 window-shared GEMMs, whose dC inputs are the
rank-local sums)."""
import os
import queue
import socket
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

P, SEED = 16, 5
# family -> (B, M, k, n_flows, H, n_layers, fw), T, precision, gradient tolerance
CASES = {"ar": ((P, 30, 5, 2, 20, 3, 4), 150, 0, 1e-5),
         "lv": ((P, 24, 4, 2, 16, 5, 3), 24, 1, 1e-4)}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _model(family="ar"):
    from tests.parity_util import build_model
    (B, M, k, nf, H, nl, fw), T, prec, _ = CASES[family]
    return build_model(family, B, M, k, nf, H, nl, fw, "cuda:0", T=T, precision=prec, seed=3)


def _worker(rank, world, port, overlap, family, out, shared=True):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from viforssms_amd.vi_ssm import DistCtx
    model = _model(family)
    model.dist = DistCtx(rank, world)
    model.p_local = P // world
    model.overlap_allreduce = overlap
    model.shared_dc_allreduce = shared
    np.random.seed(SEED)
    starts = model.select_windows()
    o = model.elbo_step(model.batch_for(starts), 0)
    torch.cuda.synchronize()
    out.put((rank, overlap, starts, model.store.grad.cpu().numpy(), model.store.flat.cpu().numpy(),
             o["elbo"].cpu().numpy(), float(o["global_norm"][0]), model.last_allreduce_bytes))
    dist.barrier()
    dist.destroy_process_group()


def _run(overlap, family, shared=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, overlap, family, q, shared)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.time() + 240
    while len(res) < 2:
        try:
            r = q.get(timeout=1)
            res[r[0]] = r
        except queue.Empty:
            assert not any(p.exitcode not in (None, 0) for p in procs), "a rank failed"
            assert time.time() < deadline, "timed out"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("family", ["ar", "lv"])
def test_two_rank_hip_gradient_equals_full_batch_and_params_agree(family):
    gtol = CASES[family][3]
    ov = _run(True, family)
    blk = _run(False, family)
    # full batch, one process
    model = _model(family)
    np.random.seed(SEED)
    starts = model.select_windows()
    o = model.elbo_step(model.batch_for(starts), 0)
    torch.cuda.synchronize()
    full_g = model.store.grad.double().cpu().numpy()
    full_p = model.store.flat.double().cpu().numpy()
    full_e = o["elbo"].cpu().numpy()
    for res in (ov, blk):
        (_, _, s0, g0, p0, e0, n0, _), (_, _, s1, g1, p1, e1, n1, _) = res[0], res[1]
        assert np.array_equal(s0, starts) and np.array_equal(s1, starts)
        # the ranks' ELBOs are the two halves of the full batch (same Philox rows)
        assert np.allclose(np.concatenate([e0, e1]), full_e, rtol=1e-5, atol=1e-5 * np.abs(full_e).max())
        assert np.array_equal(g0, g1) and n0 == n1
        assert np.array_equal(p0, p1)                        # replicated update: bitwise identical
        assert np.linalg.norm(g0 - full_g) / np.linalg.norm(full_g) < gtol
        assert abs(n0 / float(o["global_norm"][0]) - 1) < gtol
        # Adamax's first step moves by lr*0.05*sign(g): compare where the gradient is clearly signed
        keep = np.abs(full_g) > 1e-4 * np.abs(full_g).max()
        assert np.abs(p0 - full_p)[keep].max() < 2e-6
    assert np.array_equal(ov[0][3], blk[0][3])              # bucketed + overlapped == one blocking reduce


def test_lv_window_shared_gradients_summed_through_dC():
    """LV, one window on both ranks: each flow's dC (and w_eps gradient) is SUM-all-reduced inside the backward and
    the window-shared backward (feature MLP, conv over the time-mixing features: lotka_volterra_partial.py:71-82)
    runs replicated on it, so those variables leave the gradient all-reduce (VISSMBase._shared_grad_plan).  Same
    gradient as all-reducing every variable (linear in dC), fewer bytes, ranks bitwise equal."""
    via_dc = _run(True, "lv", shared=True)
    full = _run(True, "lv", shared=False)
    g_dc, g_full = via_dc[0][3], full[0][3]
    assert np.array_equal(via_dc[0][3], via_dc[1][3]) and np.array_equal(via_dc[0][4], via_dc[1][4])
    assert np.linalg.norm(g_dc - g_full) / np.linalg.norm(g_full) < 1e-4
    b_dc, b_full = via_dc[0][7], full[0][7]
    print({"allreduce_bytes_via_dC": b_dc, "allreduce_bytes_all_variables": b_full})
    assert 0 < b_dc < b_full
