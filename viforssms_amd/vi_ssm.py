"""VI_SSM: the reference's model + training-loop class, shared by the four families.

Mirrors VI_SSM (AR.py:113-362 and the LV/SV/FHN variants): build_flow(), train(tensorboard_path,
save_path), save(PATH), load(PATH), save_paths(PATH_obs).  One training step is
  window pick (np.random.choice, AR.py:263-265) -> feature gather -> ELBO on the GPU (libvissm)
  -> grad of sum(-ELBO) -> [RCCL all-reduce SUM over ranks] -> fused global-norm clip + Adamax.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .nma import Engine, ModelDef, Batch, AdamaxSlots, ScalarLog


@dataclass
class ThetaSpec:
    """What the reference passes as ``theta_dist``: the q(theta) flow architecture
    (Chain of Invert(MAF) with these permutations, base N(loc, scale), activation)."""
    n_bijectors: int
    perms: List[List[int]]
    base_loc: float
    base_scale: float
    activation: str = "elu"

    @staticmethod
    def build(P_theta: int, n_bijectors: int, base_loc: float, base_scale: float, activation: str = "elu"):
        """Draws the permutations with the global numpy RNG exactly as the reference
        (np.random.permutation per Permute, AR.py:383-385)."""
        perms = [list(map(int, np.random.permutation(np.arange(0, P_theta)))) for _ in range(n_bijectors - 1)]
        return ThetaSpec(n_bijectors, perms, base_loc, base_scale, activation)


class DistCtx:
    """Data parallelism over samples: rank r owns samples [r*p_local, (r+1)*p_local) of every step."""

    def __init__(self, rank: int = 0, world: int = 1, group=None):
        self.rank, self.world, self.group = rank, world, group

    @staticmethod
    def from_env():
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return DistCtx(dist.get_rank(), dist.get_world_size())
        return DistCtx()

    def all_reduce_(self, t: torch.Tensor):
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t


class VISSMBase:
    """Engine + optimisers + reference training loop."""

    def __init__(self, mdef: ModelDef, table, theta_spec: ThetaSpec, p: int, pre_train: bool,
                 early_stopping: float, learn_rate: float, grad_clip: float, device=None, seed: int = 1,
                 precision: int = _lib.VISSM_PREC_FP32, dist: Optional[DistCtx] = None, log_every: int = 1,
                 init_seed: int = 1, skip_nonfinite: bool = True):
        mdef.n_maf = theta_spec.n_bijectors
        mdef.theta_base = (theta_spec.base_loc, theta_spec.base_scale)
        mdef.theta_act = theta_spec.activation
        self.mdef = mdef
        self.p = int(p)
        self.dist = dist or DistCtx()
        if self.p % self.dist.world:
            raise ValueError(f"p={p} must divide evenly over {self.dist.world} ranks")
        self.p_local = self.p // self.dist.world
        self.engine = Engine(mdef, table, device=device, seed=seed, precision=precision, perms=theta_spec.perms,
                             init_seed=init_seed)
        self.store = self.engine.store
        self.pre_train = pre_train
        self.early_stopping = early_stopping
        self.learn_rate = learn_rate
        self.grad_clip = grad_clip
        self.log_every = max(1, int(log_every))
        # SURVEY.md §5 failure detection: a step whose all-reduced global norm is not finite is skipped on
        # the device (params and slots untouched) and counted in optimize/skipped_steps; False restores the
        # reference's clip_by_global_norm behaviour (NaN written into every variable, AR.py:230-232)
        self.skip_nonfinite = bool(skip_nonfinite)
        # >1 ranks: all-reduce each flow's gradient bucket as soon as its backward completes (overlap)
        self.overlap_allreduce = True
        # >1 ranks on the same windows: all-reduce each flow's dC instead of its window-shared variables' gradients
        # where that is fewer bytes (_shared_grad_plan; LV)
        self.shared_dc_allreduce = True
        self.last_allreduce_bytes = 0
        self.T = mdef.scale_num
        self.batch_dims = mdef.M
        self._batch_cache: Dict[tuple, Batch] = {}
        self._opt_main: Optional[AdamaxSlots] = None
        self._opt_pre: List[AdamaxSlots] = []
        self.last: Dict[str, float] = {}
        self.global_step = 0

    # ------------------------------------------------------------------ graph
    def build_flow(self):
        """Allocates the optimiser slots (main Adamax beta1=0.95 with global-norm clip; pre-training
        Adamax beta1=0.9 with its own slots), as build_flow does in the reference."""
        n = self.store.numel
        dev = self.engine.device
        self._opt_main = AdamaxSlots(n, dev)
        self._opt_pre = [AdamaxSlots(n, dev) for _ in range(self.n_pretrain_opts())]
        return self

    def n_pretrain_opts(self) -> int:
        return 1

    # ------------------------------------------------------------------ windows
    def select_windows(self) -> np.ndarray:
        """AR.py:257-265: batch_select = np.random.choice(arange(0, T, M), p, replace = M p >= T)."""
        T = int(self.target_len())
        M = self.batch_dims
        replace = (M * self.p) >= T
        return np.random.choice(np.arange(0, T, M), size=self.p, replace=replace)

    def target_len(self) -> int:
        return int(self.T)

    def batch_for(self, starts_global: np.ndarray) -> Batch:
        """This rank's batch of the step's window starts (all ranks' draws).  Also records whether every rank
        holds the same distinct windows (each rank replays the same draw, so this needs no communication): then
        the window-shared gradients can be summed through dC (_shared_grad_plan)."""
        r = self.dist.rank
        starts_global = np.asarray(starts_global, dtype=np.int64)
        local = starts_global[r * self.p_local:(r + 1) * self.p_local]
        uniq = np.unique(local)
        same = all(np.array_equal(np.unique(starts_global[q * self.p_local:(q + 1) * self.p_local]), uniq)
                   for q in range(self.dist.world))
        key = (tuple(uniq.tolist()) if len(uniq) == 1 else None)
        if key is not None and key in self._batch_cache and self._batch_cache[key].B == len(local):
            b = self._batch_cache[key]
        else:
            b = self.engine.make_batch(local)
            if key is not None:
                self._batch_cache = {key: b}
        b.ranks_same_windows = same
        return b

    # ------------------------------------------------------------------ window-shared gradients over ranks
    def _shared_grad_plan(self, batch: Batch, fused: bool) -> bool:
        """Sum the window-shared gradients through dC (Engine.grad_sum) on this step?  Needs >1 ranks holding the
        same windows (batch_for) and the unfused step, and pays when the flows' dC ([n_win, Lh, H] each) is
        smaller than the variables it replaces in the all-reduce: LV (31.8 M parameters, 127 MB, vs 3 x 1 MB of
        dC at the LV-cfg shape), not AR (its window-shared variables are smaller than its dC).  A captured step
        keeps the single blocking all-reduce of every gradient."""
        if (self.dist.world <= 1 or fused or not getattr(batch, "ranks_same_windows", False)
                or not self.shared_dc_allreduce
                or (self.store.grad.is_cuda and torch.cuda.is_current_stream_capturing())):
            return False
        md = self.mdef
        s = 2 if md.D == 2 else 1
        n_dc = sum(batch.n_win * ((md.kernel_ext - (i + 1) * md.k) // s) * fl.spec.H + fl.spec.k * fl.spec.H
                   for i, fl in enumerate(self.engine.flows))
        n_shared = sum(self.store.offsets[n][1] for fl in self.engine.flows for n in fl.shared_grad_names())
        self._plan_dc_numel = n_dc   # dC and w_eps gradients all-reduced inside the backward
        return n_dc < n_shared

    def _shared_names(self):
        return {n for fl in self.engine.flows for n in fl.shared_grad_names()}

    # ------------------------------------------------------------------ one step
    def _draws(self, batch: Batch, step: int, eps=None, x0_theta=None, row0_dev=None):
        """(eps, base log-prob or None, q(theta) base draw): injected (parity tests) or drawn from the Philox
        streams keyed by the global sample index (row0_dev: that index's step base on the device, for a
        captured step)."""
        base_lp = None
        if eps is None or x0_theta is None:
            e, blp, x0 = self.engine.draw(step, batch.B, self.dist.rank * self.p_local, self.p, row0_dev)
            if eps is None:
                eps, base_lp = e, blp
            if x0_theta is None:
                x0_theta = x0
        return eps, base_lp, x0_theta

    def forward(self, batch: Batch, step: int, eps=None, x0_theta=None, row0_dev=None):
        """One ELBO evaluation (randomness as in _draws)."""
        eps, base_lp, x0_theta = self._draws(batch, step, eps, x0_theta, row0_dev)
        return self.engine.forward(batch, eps, base_lp, x0_theta)

    def elbo_step(self, batch: Batch, step: int, eps=None, x0_theta=None, apply: bool = True, row0_dev=None):
        """grad of sum(-ELBO) (AR.py:228-229) -> all-reduce -> clip_by_global_norm -> Adamax (AR.py:230-234)."""
        st = self.store
        st.zero_grad()
        fused = self.engine.fused_ok(batch, batch.B)
        shared = self._shared_grad_plan(batch, fused)
        if fused:
            # the last flow fused with the AR(1) ELBO terms (one kernel instead of the flow's forward and
            # backward and the ELBO's dz); the multi-root backward carries the same gradient of sum(-ELBO)
            e, bl, x0 = self._draws(batch, step, eps, x0_theta, row0_dev)
            out, (roots, grads) = self.engine.forward_fused(batch, e, bl, x0)
            self._arm_overlap()
            torch.autograd.backward(roots, grads)
            del roots, grads
        elif self.engine.onepass_ok():
            # the log-densities' values, dz and dtheta from one pass over the path (vissm_elbo_fwd_grad: the loss's
            # upstream gradients are constants), the rest of the gradient through autograd (multi-root backward)
            e, bl, x0 = self._draws(batch, step, eps, x0_theta, row0_dev)
            self.engine.grad_sum = self.dist if shared else None
            try:
                out, (roots, grads) = self.engine.forward_onepass(batch, e, bl, x0)
            finally:
                self.engine.grad_sum = None
            self._arm_overlap(shared)
            torch.autograd.backward(roots, grads)
            del roots, grads
        else:
            self.engine.grad_sum = self.dist if shared else None
            try:
                out = self.forward(batch, step, eps, x0_theta, row0_dev)
            finally:
                self.engine.grad_sum = None
            loss = (-out["elbo"]).sum()
            self._arm_overlap(shared)
            loss.backward()
            del loss
        # drop the autograd graph now: its parameter-accumulation nodes would otherwise live on into
        # the next step (and, under graph capture, run on the stream they were created on)
        out = {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
        self._reduce_grads(shared)
        if apply:
            o = self._opt_main
            gn = o.kernel.step(st.flat, st.grad, o.v, o.m, self.learn_rate, 0.95, 0.999, 1e-8, self.clip_norm(),
                               guard=self.skip_nonfinite)
            out["global_norm"] = gn
        return out

    def graphed_step(self, starts: np.ndarray, step: int):
        """elbo_step for the windows `starts` (all ranks' draws) through the captured graph."""
        if getattr(self, "_graphed", None) is None:
            from .graph import GraphedStep
            self._graphed = GraphedStep(self)
        return self._graphed.step(starts, step)

    def clip_norm(self) -> float:
        return float(self.grad_clip)

    def grad_mask(self):
        """Optional 0/1 mask over the flat gradient (frozen variables); None = all trainable."""
        return None

    # ------------------------------------------------------------------ gradient all-reduce
    def _grad_buckets(self, exclude=()):
        """Per-flow buckets of the flat gradient (each flow's variables are contiguous: flow{i}/...), in the
        order the backward completes them (last flow first), then the rest (q(theta)'s MAF, complete only
        at the end).  A flow's bucket is final once every one of its variables has accumulated.  exclude:
        variables left out (the window-shared ones when their gradient was summed through dC; they are a
        prefix of each flow's range, so the buckets stay contiguous)."""
        st = self.store
        groups: Dict[str, List[str]] = {}
        for n in st.names():
            if n in exclude:
                continue
            key = n.split("/")[0] if n.startswith("flow") else "rest"
            groups.setdefault(key, []).append(n)
        out = []
        for key, names in groups.items():
            a = st.offsets[names[0]][0]
            b = st.offsets[names[-1]][0] + st.offsets[names[-1]][1]
            if b - a != sum(st.offsets[n][1] for n in names):
                raise RuntimeError(f"gradient bucket {key} is not contiguous")
            out.append((key, a, b, names))
        flows = sorted((x for x in out if x[0] != "rest"), key=lambda x: -int(x[0][4:]))
        return flows + [x for x in out if x[0] == "rest"]

    def _bucket_cfg(self, shared: bool):
        """(buckets, owner) for the step's mode: every variable, or without the window-shared ones (shared)."""
        cache = self.__dict__.setdefault("_ov_cfg", {})
        if shared not in cache:
            buckets = self._grad_buckets(self._shared_names() if shared else ())
            owner = {n: bi for bi, (_, _, _, names) in enumerate(buckets[:-1]) for n in names}
            cache[shared] = (buckets, owner)
        return cache[shared]

    def _arm_overlap(self, shared: bool = False):
        """Before a backward on >1 ranks: each flow bucket's SUM all-reduce is launched (async) from the
        post-accumulate hook of its last variable, so it runs over xGMI while the earlier flows' backward
        kernels still execute; _reduce_grads waits for them.  shared: the step sums the
        window-shared gradients through dC, so their variables are in no bucket."""
        capturing = self.store.grad.is_cuda and torch.cuda.is_current_stream_capturing()
        if self.dist.world <= 1 or not self.overlap_allreduce or capturing:
            self._ov = None   # (a captured step keeps the single blocking all-reduce)
            if not capturing and os.environ.get("VISSM_GRAD_RELEASE", "1") != "0":
                # no hook reads a .grad before _reduce_grads' sync_grads: let autograd keep the gradient tensors
                # instead of adding each into its zeroed flat view (params.ParamStore.release_grads)
                self.store.release_grads()
            return
        st = self.store
        if not getattr(self, "_ov_hooked", False):
            for n in st.names():
                if n.startswith("flow"):
                    st.tensors[n].register_post_accumulate_grad_hook(self._make_hook(n))
            self._ov_hooked = True
        buckets, owner = self._bucket_cfg(shared)
        self._ov = {"left": [len(x[3]) for x in buckets], "handles": {}, "bad": set(), "buckets": buckets,
                    "owner": owner}

    def _make_hook(self, name):
        def hook(t):
            ov = getattr(self, "_ov", None)
            if ov is None or name not in ov["owner"]:
                return
            bi = ov["owner"][name]
            a, sz = self.store.offsets[name]
            if t.grad is None or t.grad.data_ptr() != self.store.grad[a:a + sz].data_ptr():
                ov["bad"].add(bi)   # autograd re-allocated this .grad: reduce the bucket after sync_grads
            ov["left"][bi] -= 1
            if ov["left"][bi] == 0 and bi not in ov["bad"]:
                import torch.distributed as dist
                _, lo, hi, _ = ov["buckets"][bi]
                ov["handles"][bi] = dist.all_reduce(self.store.grad[lo:hi], op=dist.ReduceOp.SUM,
                                                    group=self.dist.group, async_op=True)
        return hook

    def _reduce_grads(self, shared: bool = False):
        """SUM the flat gradient over the ranks (the buckets the backward hooks launched, then the rest).
        shared: the window-shared variables' gradients are already full-batch sums on every rank (summed
        through dC inside the backward) and are left out.  Records last_allreduce_bytes."""
        st = self.store
        ov, self._ov = getattr(self, "_ov", None), None
        st.sync_grads()
        if self.dist.world <= 1:
            self.last_allreduce_bytes = 0
        elif ov is None and not shared:
            self.dist.all_reduce_(st.grad)
            self.last_allreduce_bytes = 4 * st.grad.numel()
        else:
            buckets = ov["buckets"] if ov is not None else self._bucket_cfg(shared)[0]
            handles = ov["handles"] if ov is not None else {}
            for h in handles.values():
                h.wait()
            for bi, (_, lo, hi, _) in enumerate(buckets):
                if bi not in handles:
                    self.dist.all_reduce_(st.grad[lo:hi])
            self.last_allreduce_bytes = 4 * sum(hi - lo for _, lo, hi, _ in buckets)
            if shared:
                self.last_allreduce_bytes += 4 * self._plan_dc_numel
        m = self.grad_mask()
        if m is not None:   # elementwise: commutes with the SUM over ranks
            st.grad.mul_(m)

    def minimize_pair(self, loss1: torch.Tensor, loss2: torch.Tensor, beta1: float = 0.9, lr: float = 1e-3):
        """Two AdamaxOptimizer(lr, beta1).minimize ops run in one session step (gradients from the same
        forward values, each with its own slots): SV pre_train_step + param_init, FHN t1 + t2."""
        st = self.store
        st.zero_grad()
        loss1.backward(retain_graph=True)
        self._reduce_grads()
        g1 = st.grad.clone()
        st.zero_grad()
        loss2.backward()
        self._reduce_grads()
        s1, s2 = self._opt_pre[0], self._opt_pre[1]
        s1.kernel.step(st.flat, g1, s1.v, s1.m, lr, beta1, 0.999, 1e-8, 0.0)
        s2.kernel.step(st.flat, st.grad, s2.v, s2.m, lr, beta1, 0.999, 1e-8, 0.0)

    def minimize(self, loss: torch.Tensor, slots: AdamaxSlots, beta1: float = 0.9, lr: float = 1e-3):
        """AdamaxOptimizer(learning_rate=lr, beta1).minimize(loss) for a pre-training loss (no clip)."""
        st = self.store
        st.zero_grad()
        loss.backward()
        self._reduce_grads()
        slots.kernel.step(st.flat, st.grad, slots.v, slots.m, lr, beta1, 0.999, 1e-8, 0.0)

    # model-specific pre-training step; returns True when pre-training is finished
    def pretrain_step(self, batch: Batch, run: int) -> bool:
        raise NotImplementedError

    # ------------------------------------------------------------------ loop
    def summaries(self, out) -> Dict[str, float]:
        s = self.mdef.scale_num / self.mdef.M
        vals = {
            "loss/ELBO": out["elbo"].mean(),
            "loss/SDE_log_prob": s * out["sde"].mean(),
            "loss/theta_log_prob": out["logq_theta"].mean(),
            "loss/obs_log_prob": s * out["obs"].mean(),
            "loss/path_log_prob": s * out["logq"].mean(),
        }
        if "global_norm" in out:
            vals["optimize/global_norm"] = out["global_norm"][0]
            if self.skip_nonfinite and self._opt_main is not None:
                vals["optimize/skipped_steps"] = self._opt_main.kernel.skipped[0]
        keys = list(vals)
        stacked = torch.stack([v.detach().float().reshape(()) for v in vals.values()])
        if self.dist.world > 1:
            stacked = stacked.clone()
            self.dist.all_reduce_(stacked)
            stacked = stacked / self.dist.world
        host = stacked.cpu().numpy()
        res = {k: float(v) for k, v in zip(keys, host)}
        if "optimize/skipped_steps" in res and self.dist.world > 1:
            res["optimize/skipped_steps"] *= self.dist.world   # identical on every rank: undo the mean
        return res

    def histograms(self, out, bins: int = 30) -> Dict[str, Dict]:
        """The reference's theta histograms (AR.py:218-224: tf.summary.histogram per theta component,
        exponentiated where the component is a log-parameter, family 'parameters'), over all ranks'
        samples: min, max, mean, std and `bins` equal-width counts."""
        theta = out["theta"].detach().float()
        pos = list(self.mdef.theta_pos) or [False] * theta.shape[1]
        res = {}
        for i in range(theta.shape[1]):
            x = theta[:, i].exp() if pos[i] else theta[:, i]
            # finite entries only: a non-finite draw (a skipped step's theta, an exp overflow) must not end the
            # loop in torch.histc; "nonfinite" counts the rest
            ok = torch.isfinite(x)
            xf = torch.where(ok, x, torch.zeros_like(x))
            big = torch.finfo(x.dtype).max
            stats = torch.stack([torch.where(ok, x, torch.full_like(x, big)).min(),
                                 -torch.where(ok, x, torch.full_like(x, -big)).max(), xf.sum(), (xf * xf).sum(),
                                 ok.sum().to(x.dtype), (~ok).sum().to(x.dtype)])
            if self.dist.world > 1:
                import torch.distributed as dist
                mm = stats[:2].clone()
                dist.all_reduce(mm, op=dist.ReduceOp.MIN, group=self.dist.group)
                ss = stats[2:].clone()
                self.dist.all_reduce_(ss)
                stats = torch.cat([mm, ss])
            lo, hi, s1, s2, n, nbad = stats.double().cpu().tolist()
            hi = -hi
            if n > 0:
                counts = torch.histc(x[ok], bins=bins, min=lo, max=hi if hi > lo else lo + 1.0)
            else:
                counts = torch.zeros(bins, device=x.device)
                lo = hi = float("nan")
            self.dist.all_reduce_(counts)
            mean = s1 / n if n > 0 else float("nan")
            std = max(s2 / n - mean * mean, 0.0) ** 0.5 if n > 0 else float("nan")
            res[f"parameters/{i}"] = {"min": lo, "max": hi, "mean": mean, "std": std, "count": int(n),
                                      "nonfinite": int(nbad), "edges": [lo, hi], "counts": counts.cpu().tolist()}
        return res

    def train(self, tensorboard_path: Optional[str], save_path: Optional[str], max_runs: Optional[int] = None,
              verbose: bool = True, graph: bool = False):
        """VI_SSM.train (AR.py:240-310): endless unless early_stopping / max_runs.  graph: the ELBO
        steps after pre-training run as a captured HIP graph (viforssms_amd.graph)."""
        if self._opt_main is None:
            self.build_flow()
        if tensorboard_path:
            os.makedirs(tensorboard_path, exist_ok=True)
        writer = ScalarLog(tensorboard_path if self.dist.rank == 0 else None)
        run = 0
        total = 0
        if verbose and self.dist.rank == 0:
            print("Training model...")
        converged = False
        while not converged:
            starts = self.select_windows()
            if self.pre_train:
                batch = self.batch_for(starts)
                if run == 0 and verbose and self.dist.rank == 0:
                    print("Pre-training...")
                if self.pretrain_step(batch, run):
                    self.pre_train = False
                    if verbose and self.dist.rank == 0:
                        print("Finished pre-training")
                    run = 0
            else:
                if graph:
                    out = self.graphed_step(starts, self.global_step)
                else:
                    out = self.elbo_step(self.batch_for(starts), self.global_step)
                if run % self.log_every == 0:
                    self.last = self.summaries(out)
                    # histograms only for an active writer: they cost a host sync per theta component (and
                    # collectives over ranks), which a run without a log file would pay for nothing
                    # (decided by tensorboard_path, the same on every rank, so the ranks' collectives match)
                    hist = self.histograms(out) if tensorboard_path else None
                    writer.write(run, self.last, hist)
            self.global_step += 1
            if run == self.early_stopping:
                converged = True
            if save_path and run % 1000 == 0 and self.dist.rank == 0:
                self.save(save_path)
            run += 1
            total += 1
            if max_runs is not None and total >= max_runs:
                break
        writer.close()
        return self

    # ------------------------------------------------------------------ persistence
    def save(self, PATH: str):
        """Own checkpoint format (torch.save of tensors only, loadable with weights_only=True): flat params,
        the main and pre-training Adamax slot sets, the global step, the skipped-step count and the numpy
        global RNG state that draws the windows (AR.py:263-265) -- so a resumed run draws the same windows."""
        d = os.path.dirname(PATH)
        if d:
            os.makedirs(d, exist_ok=True)
        st = self.store
        blob = {
            "params": st.flat.detach().cpu(),
            "names": "\n".join(st.names()),
            "global_step": torch.tensor(self.global_step),
            "main_v": self._opt_main.v.cpu() if self._opt_main else torch.zeros(0),
            "main_m": self._opt_main.m.cpu() if self._opt_main else torch.zeros(0),
        }
        for i, o in enumerate(self._opt_pre):
            blob[f"pre{i}_v"] = o.v.cpu()
            blob[f"pre{i}_m"] = o.m.cpu()
        if self._opt_main is not None:
            blob["skipped_steps"] = self._opt_main.kernel.skipped.cpu()
        name, key, pos, has_gauss, gauss = np.random.get_state()
        blob["np_rng_key"] = torch.from_numpy(np.asarray(key, dtype=np.int64))
        blob["np_rng_meta"] = torch.tensor([int(pos), int(has_gauss)], dtype=torch.int64)
        blob["np_rng_gauss"] = torch.tensor([float(gauss)], dtype=torch.float64)
        blob["pre_train"] = torch.tensor(int(bool(self.pre_train)))
        torch.save(blob, PATH)
        print("Model saved")

    def load(self, PATH: str):
        self.pre_train = False
        blob = torch.load(PATH, weights_only=True)
        if blob["names"] != "\n".join(self.store.names()):
            raise ValueError("checkpoint variables do not match this model")
        if self._opt_main is None:
            self.build_flow()
        with torch.no_grad():
            self.store.flat.copy_(blob["params"].to(self.store.flat.device))
            if blob["main_v"].numel():
                self._opt_main.v.copy_(blob["main_v"])
                self._opt_main.m.copy_(blob["main_m"])
            for i, o in enumerate(self._opt_pre):
                if f"pre{i}_v" in blob:
                    o.v.copy_(blob[f"pre{i}_v"])
                    o.m.copy_(blob[f"pre{i}_m"])
            if "skipped_steps" in blob:
                self._opt_main.kernel.skipped.copy_(blob["skipped_steps"])
        self.global_step = int(blob["global_step"])
        if "np_rng_key" in blob:
            pos, has_gauss = (int(x) for x in blob["np_rng_meta"].tolist())
            np.random.set_state(("MT19937", blob["np_rng_key"].numpy().astype(np.uint32), pos, has_gauss,
                                 float(blob["np_rng_gauss"][0])))
        print("Model restored")

    @torch.no_grad()
    def sample_paths(self, starts: np.ndarray, step: int = 0):
        batch = self.engine.make_batch(np.asarray(starts))
        out = self.forward(batch, step)
        return self.engine.lf_sample(out["z"], batch)

    def save_paths(self, PATH_obs: str):
        """Posterior path samples for every window start (AR.py:323-362; the reference's AR version
        feeds a non-existent placeholder and crashes, AR.py:355 -- this one runs)."""
        M = self.batch_dims
        stack = []
        for idx in np.arange(0, self.target_len(), M):
            print(idx, "/", self.target_len())
            x = self.sample_paths(np.tile(idx, self.p_local), step=self.global_step)
            stack.append(x[:, :, 1:].cpu().numpy())
        paths = np.concatenate(stack, axis=2)
        d = os.path.dirname(PATH_obs)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(PATH_obs, "w") as f:
            np.savetxt(f, np.reshape(paths, (paths.shape[0], -1)) if paths.shape[1] > 1 else paths[:, 0, :])
