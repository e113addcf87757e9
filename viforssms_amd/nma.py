"""Neural moving-average (NMA) flow stack and the shared VI_SSM engine.

Reference classes (AR.py:24-110; lotka_volterra_partial.py:25-159; SV_dense.py:23-136;
fitz_nag_NVP.py:26-156): ``init_dist`` (base noise), ``IAF`` (one locally-variant IAF
with feature injection), ``Permute`` (pair swap between 2-D flows), ``Flow_Stack``.

Split of each IAF:
  * window-shared, per step: feature MLP on time_feats, the feature part of the first
    conv (a conv over features, written as k shifted GEMMs) + conv bias -> C[win, m, H],
    and the theta branch (three linear layers) -> theta_term[b, H].  Small; torch GEMMs.
  * per transition (the hot path): the sample-channel conv, hidden 1x1 layers, head,
    affine transform and log-sigma sum -> libvissm ``vissm_flow_fwd/bwd``.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field
from datetime import datetime
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .ops import (FlowShape, kernel_precision, ma_flow, feat_conv, lv_feat_conv, sv_feat_conv, normal_base, normal_base_dev, base_logprob, elbo_terms,
                  ElboFeeds, AdamaxKernel, ar_fused_supported, ar_last_flow_fused, elbo_values_and_theta_grad,
                  elbo_values_grad, theta_branch_bwd, theta_branch_fwd)
from .params import ParamStore, glorot_uniform
from .theta_flow import ThetaFlow
from .linalg import linear, linear_bf16, linear_x3, tn_split_k

LOG_2PI = math.log(2 * math.pi)


def elu(x):
    return torch.nn.functional.elu(x)


class _ThetaBranch(torch.autograd.Function):
    """theta_term = ((theta W0 + b0) W1 + b1) W2 + b2 — the reference's three linear dense layers
    (AR.py:63-68) — evaluated as one [B, P] x [P, H] product with the collapsed weights.  Every
    gradient follows from S = theta^T d and s = sum_b d (d = d theta_term), so the backward has
    no [B, H] intermediates and no K = B weight GEMMs besides S."""

    @staticmethod
    def forward(ctx, theta, W0, b0, W1, b1, W2, b2):
        W12 = W1 @ W2
        ctx.save_for_backward(theta, W0, b0, W1, b1, W2, W12)
        if os.environ.get("VISSM_THETA_BRANCH_ASSOC") == "1":   # diagnostic: the same products, other rounding order
            return torch.addmm((b0 @ W1 + b1) @ W2 + b2, theta, (W0 @ W1) @ W2)
        return torch.addmm(b0 @ W12 + b1 @ W2 + b2, theta, W0 @ W12)

    @staticmethod
    def backward(ctx, d):
        theta, W0, b0, W1, b1, W2, W12 = ctx.saved_tensors
        d = d.contiguous()
        if (d.is_cuda and theta.shape[1] <= 8 and max(W0.shape[1], W1.shape[1], W2.shape[1]) <= 64
                and _theta_branch_kernels("bwd")):
            # one pass over d for S, s and dtheta, then the [<= 64]^2 algebra in one block (vissm_theta_branch_bwd:
            # three launches for the ~14 small library kernels below)
            return theta_branch_bwd(theta, d, W0, b0, W1, b1, W2)
        S = tn_split_k(theta.contiguous(), d)      # theta^T d      [P, H]
        s = d.sum(0)                                # sum_b d        [H]
        SW2, sW2 = S @ W2.t(), s @ W2.t()           # through layer 2: theta^T dh1, sum dh1
        dW2 = (W0 @ W1).t() @ S + torch.outer(b0 @ W1 + b1, s)   # h1^T d, h1 = theta W0 W1 + b0 W1 + b1
        dW1 = W0.t() @ SW2 + torch.outer(b0, sW2)               # h0^T dh1, h0 = theta W0 + b0
        dW0 = SW2 @ W1.t()                                      # theta^T dh0, dh0 = dh1 W1^T
        dtheta = d @ (W0 @ W12).t()
        return dtheta, dW0, sW2 @ W1.t(), dW1, sW2, dW2, s


def _theta_branch_kernels(which: str) -> bool:
    """The theta-branch HIP kernels (vissm_theta_branch_fwd / _bwd) run by default; VISSM_THETA_BRANCH_KERNEL=0
    selects the library-GEMM form (_ThetaBranch), "fwd" / "bwd" one direction only (the forward kernel also runs the
    backward kernel).  Each matches float64 to 1e-5 (tests/test_gpu_theta.py).  Round 5 kept them opt-in because the
    fp32 recovery run ended outside its sd bound with them; round 6 found that departure in the float64 oracle's own
    run of the reference schedule (profiles/r06/recovery/: the posterior reaches the generating values, then wanders
    off along the theta0 / (1 - theta1) ridge, at a step that depends on the rounding and the draws, for every form),
    and the recovery test now asks every seed to reach the posterior (tests/test_gpu_posterior.py)."""
    v = os.environ.get("VISSM_THETA_BRANCH_KERNEL", "1")
    return v == "1" or v == which or (which == "bwd" and v == "fwd")


class _ThetaBranchK(torch.autograd.Function):
    """_ThetaBranch on the GPU in two launches each way (vissm_theta_branch_fwd / _bwd): returns theta_term and the
    collapsed weights (Wc, bc) it was formed with, which the two-sample AR kernels' theta fold takes as constants
    (IAF.theta_factors reuses them: no second evaluation)."""

    @staticmethod
    def forward(ctx, theta, W0, b0, W1, b1, W2, b2):
        ctx.save_for_backward(theta, W0, b0, W1, b1, W2)
        tt, Wc, bc = theta_branch_fwd(theta, W0, b0, W1, b1, W2, b2)
        ctx.mark_non_differentiable(Wc, bc)
        return tt, Wc, bc

    @staticmethod
    def backward(ctx, d, _dWc, _dbc):
        theta, W0, b0, W1, b1, W2 = ctx.saved_tensors
        return theta_branch_bwd(theta, d.contiguous(), W0, b0, W1, b1, W2)


class _SumGradOverRanks(torch.autograd.Function):
    """Identity forward; the backward SUM-all-reduces the incoming gradient over the data-parallel ranks.  Placed
    on the window-shared conv output C (and the sample-channel slice of the same conv kernel) when every rank
    holds the same windows: the window-shared backward (feature MLP, conv over features -- LV's 31.8 M
    parameters) is linear in dC, so running it replicated on the summed dC gives every rank the full-batch
    gradient of those parameters with a [n_win, Lh, H] all-reduce per flow instead of theirs (vi_ssm.py).

    Ordering invariant (RCCL needs the same collective sequence on every rank): these blocking all-reduces run
    inside the autograd backward, interleaved with the per-flow bucket all-reduces VISSMBase launches from
    post-accumulate hooks.  Both are issued in the order autograd visits the nodes, which is a function of the graph
    alone; every rank builds the same graph (same model, same window plan -- the plan is only taken when all ranks
    hold the same windows -- and the same per-rank batch shape), so the sequence agrees.  A rank-dependent graph
    (e.g. a different flow count or a branch on local data) would break it."""

    @staticmethod
    def forward(ctx, x, dist_ctx):
        ctx.dist = dist_ctx
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        ctx.dist.all_reduce_(g)
        return g, None


class _DiagSum(torch.autograd.Function):
    """C[w, m, :] = sum_j G[w, s m + j, j, :] (the valid conv's diagonal gather).  The backward
    writes dC into the (non-overlapping) diagonal of a zero dG with one strided copy instead of
    as_strided's generic accumulate-scatter (an index sort + atomics)."""

    @staticmethod
    def forward(ctx, G, Lh, s):
        nw, Lf, k, H = G.shape
        ctx.meta = (G.shape, Lh, s)
        return G.as_strided((nw, Lh, k, H), (Lf * k * H, s * k * H, k * H + H, 1)).sum(2)

    @staticmethod
    def backward(ctx, dC):
        (nw, Lf, k, H), Lh, s = ctx.meta
        dG = torch.zeros((nw, Lf, k, H), dtype=dC.dtype, device=dC.device)
        dG.as_strided((nw, Lh, k, H), (Lf * k * H, s * k * H, k * H + H, 1)).copy_(
            dC.unsqueeze(2).expand(nw, Lh, k, H))
        return dG, None, None


# ---------------------------------------------------------------------------------------
# building blocks (names mirror the reference classes)
# ---------------------------------------------------------------------------------------
class init_dist:
    """N(0, 1)^kernel_ext base; slp(p) -> (sample, log-prob over the last batch_dims entries) (AR.py:24-35).
    Draws come from a counter-based Philox stream keyed by (seed, global sample index)."""

    def __init__(self, kernel_ext: int, batch_dims: int, device):
        self.kernel_ext = kernel_ext
        self.batch_dims = batch_dims
        self.device = device

    def slp(self, p: int, seed: int = 0, offset: int = 0, eps: Optional[torch.Tensor] = None):
        if eps is not None:
            return eps, base_logprob(eps, self.batch_dims)
        return normal_base(seed, offset, p, self.kernel_ext, self.batch_dims, self.device)


class Permute:
    """Adjacent-pair swap between the flows of the 2-D models (lotka_volterra_partial.py:137-159).
    Fused into the preceding flow's output store (VissmFlowDesc.swap_out)."""

    @staticmethod
    def apply(x: torch.Tensor) -> torch.Tensor:
        p, L = x.shape
        return x.view(p, L // 2, 2).flip(-1).reshape(p, L)


@dataclass
class IAFSpec:
    k: int
    H: int
    n_hidden: int
    bn: bool
    stride2: bool
    feat: str          # "mlp4" | "sv" | "lv"
    C_time: int
    P_theta: int
    CF: int            # feature channels entering the conv
    feat_dims: int = 0  # LV: units of the time-mixing dense layer


class IAF:
    """One IAF flow (AR.py:38-89 and variants)."""

    def __init__(self, store: ParamStore, idx: int, spec: IAFSpec, rng: np.random.Generator):
        self.idx = idx
        self.spec = spec
        self.store = store
        s, H, k = spec, spec.H, spec.k
        pre = f"flow{idx}"
        self.pre = pre
        # feature branch (tf.layers.dense, glorot-uniform kernels, zero biases)
        if s.feat == "lv":
            dims = [s.C_time, H, H, H, s.feat_dims]
        else:
            cin = s.C_time + (s.C_time - 2 if s.feat == "sv" else 0)
            dims = [cin, H, H, H, H]
        for j in range(4):
            store.add(f"{pre}/feat{j}/kernel", glorot_uniform((dims[j], dims[j + 1]), dims[j], dims[j + 1], rng))
            store.add(f"{pre}/feat{j}/bias", np.zeros(dims[j + 1]))
        # first conv: kernel [k, 1 + CF, H]
        store.add(f"{pre}/conv/kernel", glorot_uniform((k, 1 + s.CF, H), k * (1 + s.CF), k * H, rng))
        store.add(f"{pre}/conv/bias", np.zeros(H))
        # theta branch: three linear dense layers
        tdims = [s.P_theta, H, H, H]
        for j in range(3):
            store.add(f"{pre}/theta{j}/kernel", glorot_uniform((tdims[j], tdims[j + 1]), tdims[j], tdims[j + 1], rng))
            store.add(f"{pre}/theta{j}/bias", np.zeros(tdims[j + 1]))
        # hidden 1x1 convs (+ BN affine)
        for l in range(s.n_hidden):
            store.add(f"{pre}/hidden{l}/kernel", glorot_uniform((H, H), H, H, rng))
            store.add(f"{pre}/hidden{l}/bias", np.zeros(H))
            if s.bn:
                store.add(f"{pre}/bn{l}/gamma", np.ones(H))
                store.add(f"{pre}/bn{l}/beta", np.zeros(H))
        store.add(f"{pre}/head/kernel", glorot_uniform((H, 2), H, 2, rng))
        store.add(f"{pre}/head/bias", np.zeros(2))

    def _p(self, name):
        return self.store[f"{self.pre}/{name}"]

    # ---- window-shared parts (torch) ----
    def features(self, ts: torch.Tensor) -> torch.Tensor:
        """Feature branch on the time_feats of this flow -> F [n_win, L-1, CF]."""
        f = self.spec.feat
        if f == "sv":                                              # SV_dense.py:53
            h = torch.cat([ts[:, 1:, :], ts[:, 1:, :-2] - ts[:, :-1, :-2]], 2)
        else:
            h = ts[:, :-1, :]
        for j in range(4):
            h = elu(linear(h, self._p(f"feat{j}/kernel"), self._p(f"feat{j}/bias")))
        if f == "lv":                                              # lotka_volterra_partial.py:75-76
            h = h.transpose(1, 2)
        return h

    def conv_shared(self, F: torch.Tensor, Lh: int, s: int, gemm: Optional[str] = None) -> torch.Tensor:
        """C[w, m, :] = conv_b + sum_j F[w, s m + j, :] @ conv_w[j, 1:, :]  (valid conv over the features).

        One GEMM against all k taps at once, G = F @ [W_0 | ... | W_{k-1}]  ([.., Lf, k H]), then the
        diagonal gather C[m] = sum_j G[s m + j, j] as a strided view (LV's F is 10061 x 10061: a loop of
        k sliced matmuls copied a 400 MB strided slice per tap)."""
        W = self._p("conv/kernel")
        k, H = self.spec.k, self.spec.H
        nw, Lf, CF = F.shape
        Wcat = W[:, 1:, :].permute(1, 0, 2).reshape(CF, k * H)
        # (gemm "x3": the three-product split-bf16 form, fp32-class, for the bf16 training precisions -- LV's
        #  [10061 x 10061] feature matrix makes this the step's largest GEMM; "bf16": single bf16 products)
        lin = {"x3": linear_x3, "bf16": linear_bf16}.get(gemm, linear)
        G = lin(F, Wcat).view(nw, Lf, k, H)  # F may be a transposed view (LV)
        return (_DiagSum.apply(G.contiguous(), Lh, s) + self._p("conv/bias")).contiguous()

    def window_conv(self, ts: torch.Tensor, Lh: int, s: int, gemm: Optional[str] = None) -> torch.Tensor:
        """C = conv_shared(features(ts)): the first conv's window-shared part.  On the GPU, at kernel_len <= 24 (the AR
        configurations and FHN's k = 20, stride 2), the feature branch (a few thousand rows of [C] -> 50 -> 50 -> 50 ->
        50, then the k-tap conv) runs as one HIP launch each way (ops.feat_conv, vissm_feat_fwd / _bwd) instead of ~40
        torch launches per flow: AR-cfg step -0.25 ms; FHN-cfg 14.08 -> 13.88 ms at 8 positions per block (round 6;
        at 32 per block, round 4, it had lost to the torch form by 1 ms).  SV's k = 50 (its diff-augmented input goes
        through the same kernels) measured 43.6 -> 44.8 ms and keeps the library GEMMs, as does LV's time-mixing
        feature layer ([kernel_ext - 1] channels).  VISSM_FEAT_TORCH=1 selects the torch form everywhere,
        VISSM_FEAT_MAX_K moves the kernel_len bound (A/B timing)."""
        f = self.spec.feat
        kmax = int(os.environ.get("VISSM_FEAT_MAX_K", "24"))
        if (ts.is_cuda and f in ("mlp4", "sv") and s <= self.spec.k <= kmax
                and os.environ.get("VISSM_FEAT_TORCH") != "1"):   # vissm_feat_* need kernel_len >= stride
            p = self._p
            # SV's MLP input is the features with their first differences (SV_dense.py:53): formed here, data only
            h0 = ts[:, :-1, :] if f == "mlp4" else torch.cat([ts[:, 1:, :], ts[:, 1:, :-2] - ts[:, :-1, :-2]], 2)
            return feat_conv(h0, s, Lh, p("feat0/kernel"), p("feat0/bias"), p("feat1/kernel"), p("feat1/bias"),
                             p("feat2/kernel"), p("feat2/bias"), p("feat3/kernel"), p("feat3/bias"),
                             p("conv/kernel"), p("conv/bias"))
        # LV: the hand-written branch (ops.lv_feat_conv: vissm_lv_* + vissm_gemm_bf16) at the bf16 precision, LV-cfg
        # step 64.0 -> 62.1 ms against the torch form (profiles/r06/lvfeat/; VISSM_LV_FEAT=torch selects the latter).
        # At the parity precisions its split-bf16 form (vissm_gemm_bf16x3, hi / lo planes) measured 191.4 against the
        # torch form's 190.5 ms per bf16x2f step (profiles/r06/lv_x3/), so there it runs on VISSM_LV_FEAT=hip only
        lvf = os.environ.get("VISSM_LV_FEAT", "")
        if f == "lv" and ts.is_cuda and ((gemm == "bf16" and lvf != "torch") or (gemm == "x3" and lvf == "hip")):
            p = self._p
            return lv_feat_conv(ts[:, :-1, :], s, Lh, p("feat0/kernel"), p("feat0/bias"), p("feat1/kernel"),
                                p("feat1/bias"), p("feat2/kernel"), p("feat2/bias"), p("feat3/kernel"),
                                p("feat3/bias"), p("conv/kernel"), p("conv/bias"), x3=gemm == "x3")
        # SV (k = 50) at the non-fp32 precisions: the hand-written branch (ops.sv_feat_conv: vissm_lv_mlp_* with the
        # first-difference input, the conv as one split-bf16 matrix-core GEMM each way); VISSM_SV_FEAT=torch selects
        # the torch form (fp32 layers, linear_x3 conv)
        if f == "sv" and ts.is_cuda and gemm == "x3" and os.environ.get("VISSM_SV_FEAT", "hip") != "torch":
            p = self._p
            return sv_feat_conv(ts, s, Lh, p("feat0/kernel"), p("feat0/bias"), p("feat1/kernel"), p("feat1/bias"),
                                p("feat2/kernel"), p("feat2/bias"), p("feat3/kernel"), p("feat3/bias"),
                                p("conv/kernel"), p("conv/bias"))
        return self.conv_shared(self.features(ts), Lh, s, gemm=gemm)

    def theta_factors(self, theta: torch.Tensor):
        """(theta, w_theta, b_theta) with theta_term = theta w_theta + b_theta: the collapsed weights _ThetaBranch
        forms (the same fp32 products), passed to the flow kernels as constants (VissmFlowParams.theta_rank) so
        the two-sample AR kernels form the theta term inside their layer-0 product; the gradient still flows
        through theta_term."""
        st, self._fold = getattr(self, "_fold", None), None   # consumed here: no graph or weights kept past the step
        if st is not None and st[0] is theta:   # the collapsed weights theta_term was just formed with
            return theta.detach().contiguous(), st[1], st[2]
        p = self._p
        with torch.no_grad():
            W1, W2 = p("theta1/kernel"), p("theta2/kernel")
            W12 = W1 @ W2
            return (theta.detach().contiguous(), (p("theta0/kernel") @ W12).contiguous(),
                    (p("theta0/bias") @ W12 + p("theta1/bias") @ W2 + p("theta2/bias")).contiguous())

    def theta_term(self, theta: torch.Tensor) -> torch.Tensor:
        p = self._p
        args = (theta, p("theta0/kernel"), p("theta0/bias"), p("theta1/kernel"), p("theta1/bias"), p("theta2/kernel"),
                p("theta2/bias"))
        self._fold = None
        if (theta.is_cuda and theta.shape[1] <= 8 and max(a.shape[-1] for a in args[1:]) <= 64
                and _theta_branch_kernels("fwd")):
            tt, Wc, bc = _ThetaBranchK.apply(*args)
            self._fold = (theta, Wc, bc)
            return tt
        return _ThetaBranch.apply(*args).contiguous()

    # ---- per-transition part (HIP) ----
    def weights(self):
        """The flow kernel's weight tensors (autograd expressions of the variables): w_eps = the sample
        channel of the first conv, stacked hidden kernels / biases / BN, head."""
        s = self.spec
        w_eps = self._p("conv/kernel")[:, 0, :].contiguous()
        if s.n_hidden > 0:
            w_hid = torch.stack([self._p(f"hidden{l}/kernel") for l in range(s.n_hidden)])
            b_hid = torch.stack([self._p(f"hidden{l}/bias") for l in range(s.n_hidden)])
        else:
            w_hid = b_hid = None
        if s.bn and s.n_hidden > 0:
            bn_g = torch.stack([self._p(f"bn{l}/gamma") for l in range(s.n_hidden)])
            bn_b = torch.stack([self._p(f"bn{l}/beta") for l in range(s.n_hidden)])
        else:
            bn_g = bn_b = None
        return w_eps, w_hid, b_hid, bn_g, bn_b, self._p("head/kernel"), self._p("head/bias")

    def shared_grad_names(self) -> List[str]:
        """Variables whose gradient reaches them only through the window-shared conv output C and the sample
        channel of the first conv kernel: the feature MLP and the first conv (its kernel's channel 0 is w_eps)."""
        return [f"{self.pre}/feat{j}/{t}" for j in range(4) for t in ("kernel", "bias")] + \
            [f"{self.pre}/conv/kernel", f"{self.pre}/conv/bias"]

    def flow(self, shape: FlowShape, win, u, C, theta_term, tf=None, grad_sum=None):
        """grad_sum (a DistCtx): C and w_eps enter through _SumGradOverRanks (their gradients summed over the
        ranks inside the backward, see Engine.grad_sum)."""
        s = self.spec
        w_eps = self._p("conv/kernel")[:, 0, :].contiguous()
        if grad_sum is not None:
            C = _SumGradOverRanks.apply(C, grad_sum)
            w_eps = _SumGradOverRanks.apply(w_eps, grad_sum)
        if s.n_hidden > 0:
            w_hid = torch.stack([self._p(f"hidden{l}/kernel") for l in range(s.n_hidden)])
            b_hid = torch.stack([self._p(f"hidden{l}/bias") for l in range(s.n_hidden)])
        else:
            w_hid = b_hid = None
        if s.bn and s.n_hidden > 0:
            bn_g = torch.stack([self._p(f"bn{l}/gamma") for l in range(s.n_hidden)])
            bn_b = torch.stack([self._p(f"bn{l}/beta") for l in range(s.n_hidden)])
        else:
            bn_g = bn_b = None
        return ma_flow(shape, win, u, C, theta_term, w_eps, w_hid, b_hid, bn_g, bn_b,
                       self._p("head/kernel"), self._p("head/bias"), tf)


# ---------------------------------------------------------------------------------------
# per-step batch
# ---------------------------------------------------------------------------------------
@dataclass
class Batch:
    starts: np.ndarray                # reference batch_select for this rank's samples
    uniq: np.ndarray                  # distinct window starts
    ts: torch.Tensor                  # time_feats of the distinct windows [n_win, kext, C]
    win: Optional[torch.Tensor]       # int32 [B] sample -> window (None when n_win == 1)
    feeds: ElboFeeds
    host_feeds: Dict[str, np.ndarray] = field(default_factory=dict)

    @property
    def B(self):
        return len(self.starts)

    @property
    def n_win(self):
        return len(self.uniq)


@dataclass
class ModelDef:
    family: str
    model_id: int
    D: int
    M: int
    k: int
    n_flows: int
    network_dims: Sequence[int]
    C_time: int
    P_theta: int
    scale_num: float        # T (AR) or target_dims: ELBO scale = scale_num / M
    priors: Sequence
    dt: float = 1.0
    obs_std: float = 1.0
    theta_base: tuple = (0.0, 1.0)
    theta_act: str = "elu"
    n_maf: int = 5
    clip: float = 2.5e8
    theta_pos: Sequence[bool] = ()

    @property
    def kernel_ext(self):
        return self.k * self.n_flows + self.D * self.M + self.D

    @property
    def n_logsig(self):
        return self.D * self.M


class Engine:
    """Parameters + one differentiable ELBO evaluation on the GPU."""

    def __init__(self, mdef: ModelDef, table, device=None, seed: int = 1, precision: int = _lib.VISSM_PREC_FP32,
                 perms: Optional[Sequence[Sequence[int]]] = None, init_seed: int = 1):
        _lib.load()   # fail loudly, before any work, if the HIP library is missing
        self.mdef = mdef
        self.table = table
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.seed = int(seed)
        self.precision = precision
        self.fuse_last = True   # AR, bf16 / bf16x3: last flow fused with the ELBO in the training step
        # tiles per t-chunk forced on every flow launch (VissmFlowDesc.chunk_tiles; 0 = automatic): parity tests
        # run a large batch's launch geometry at a small batch
        self.chunk_tiles = 0
        # a flow output that feeds another flow is allocated with rows padded to 16 floats (FlowShape.pad_out), so
        # that flow's du t-chunk stores are 64-byte aligned; VISSM_ROW_PAD=0 keeps dense rows (A/B)
        self.pad_rows = os.environ.get("VISSM_ROW_PAD", "1") != "0"
        # data parallelism: a DistCtx here makes forward() route each flow's C and w_eps through
        # _SumGradOverRanks (set per step by VISSMBase when every rank holds the same windows)
        self.grad_sum = None
        H = mdef.network_dims[0]
        if any(h != H for h in mdef.network_dims):
            raise ValueError("all network_dims must be equal (the reference adds layer outputs of width network_dims[0])")
        rng = np.random.default_rng(init_seed)
        self.store = ParamStore()
        kext = mdef.kernel_ext
        self.flows: List[IAF] = []
        for i in range(mdef.n_flows):
            if mdef.family == "lv":
                spec = IAFSpec(mdef.k, H, len(mdef.network_dims) - 2, True, True, "lv", mdef.C_time, mdef.P_theta,
                               CF=kext - 1, feat_dims=kext - 1 - i * mdef.k)
            else:
                spec = IAFSpec(mdef.k, H, len(mdef.network_dims) - 2, mdef.family != "ar", mdef.D == 2,
                               "sv" if mdef.family == "sv" else "mlp4", mdef.C_time, mdef.P_theta, CF=H)
            self.flows.append(IAF(self.store, i, spec, rng))
        if perms is None:
            perms = [list(np.random.permutation(np.arange(0, mdef.P_theta))) for _ in range(mdef.n_maf - 1)]
        self.perms = [list(map(int, p)) for p in perms]
        self.theta_dist = ThetaFlow(self.store, mdef.P_theta, mdef.n_maf, self.perms, mdef.theta_base[0],
                                    mdef.theta_base[1], mdef.theta_act, rng)
        self.store.finalize(self.device)
        self._check_precision()

    def _check_precision(self):
        """bf16x2 is the split-weight mode of the one-hidden-layer matrix-core kernels (k <= 32: the AR
        configurations), forward and backward.  Elsewhere every flow call would fall back to the exact-fp32 kernels
        and the mode's name would misstate what ran, so the engine refuses it up front (vissm_flow_kernel_precision).
        bf16x2f (a host mode: forward at VISSM_PREC_BF16X2, backward bf16) stays available on every shape: where the
        split-weight forward does not cover it (the three-hidden-layer families) the forward runs the exact-fp32
        kernels -- never less precise than asked -- and the backward the bf16 kernels."""
        if self.precision != _lib.VISSM_PREC_BF16X2:
            return
        md = self.mdef
        s = 2 if md.D == 2 else 1
        L = md.kernel_ext
        for i, fl in enumerate(self.flows):
            shape = FlowShape(B=1, L=L, k=md.k, H=fl.spec.H, n_hidden=fl.spec.n_hidden, bn=fl.spec.bn,
                              stride2=(s == 2), swap_out=(md.D == 2 and i < md.n_flows - 1), n_logsig=md.n_logsig,
                              n_win=1, precision=_lib.VISSM_PREC_BF16X2)
            if kernel_precision(shape) != _lib.VISSM_PREC_BF16X2:
                raise ValueError(
                    f"precision bf16x2 runs on the split-weight matrix-core kernels only (one hidden layer, "
                    f"kernel_len <= 32); {md.family} with {fl.spec.n_hidden} hidden layers and kernel_len {md.k} "
                    "is not covered: use fp32, bf16, bf16x3 or bf16x2f")
            L -= md.k

    # ---- batches ----
    def make_batch(self, starts: np.ndarray) -> Batch:
        """The step's batch for reference window starts `starts` (batch_select): on the GPU the windows
        are gathered from the device-resident tables (features.DeviceTable, vissm_gather_windows) and
        only the int32 starts are uploaded; on a CPU device (host-side tests) the host gather runs."""
        starts = np.asarray(starts, dtype=np.int64)
        uniq, inv = np.unique(starts, return_inverse=True)
        if self.device.type == "cuda":
            return self._make_batch_device(starts, uniq, inv)
        ts_np = self.table.windows(uniq)
        feeds_np = self.table.feeds(uniq, ts_np)
        dev = self.device
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=dev)
        win = None if len(uniq) == 1 else torch.as_tensor(inv.astype(np.int32), device=dev)
        feeds = ElboFeeds(obs=t(feeds_np["obs"]) if "obs" in feeds_np else None,
                          obs_bin=t(feeds_np["obs_bin"]) if "obs_bin" in feeds_np else None,
                          mask=t(feeds_np["mask"]) if "mask" in feeds_np else None,
                          shift=t(feeds_np["shift"]) if "shift" in feeds_np else None,
                          dim_one=t(feeds_np["dim_one"]) if "dim_one" in feeds_np else None,
                          win=win, n_win=len(uniq))
        return Batch(starts, uniq, t(ts_np), win, feeds, feeds_np)

    def _make_batch_device(self, starts, uniq, inv) -> Batch:
        if getattr(self, "_dtab", None) is None:
            from .features import DeviceTable
            self._dtab = DeviceTable(self.table, self.device)
        n = len(uniq)
        idx = np.concatenate([uniq, inv]).astype(np.int32) if n > 1 else uniq.astype(np.int32)
        idx_dev = torch.from_numpy(idx).to(self.device)
        ts, f = self._dtab.batch(idx_dev[:n], n)
        win = idx_dev[n:] if n > 1 else None
        feeds = ElboFeeds(obs=f.get("obs"), obs_bin=f.get("obs_bin"), mask=f.get("mask"), shift=f.get("shift"),
                          dim_one=f.get("dim_one"), win=win, n_win=n, plain_from=f.get("plain_from"),
                          obs_list=f.get("obs_list"))
        return Batch(starts, uniq, ts, win, feeds, {})

    # ---- random inputs (Philox; keyed by global sample index so sharding is exact) ----
    def draw(self, step: int, B: int, global_offset: int, B_total: int, row0_dev: Optional[torch.Tensor] = None):
        """eps [B, kernel_ext] + base log-prob and the q(theta) base draw, Philox rows row0 + b with
        row0 = step * B_total + global_offset (or read from row0_dev, a device counter a captured
        graph advances)."""
        md = self.mdef
        if row0_dev is not None:
            eps, base_lp = normal_base_dev(self.seed, row0_dev, B, md.kernel_ext, md.n_logsig)
            n, _ = normal_base_dev(self.seed ^ 0x5DEECE66D, row0_dev, B, md.P_theta, 0)
        else:
            row0 = step * B_total + global_offset
            eps, base_lp = normal_base(self.seed, row0, B, md.kernel_ext, md.n_logsig, self.device)
            n, _ = normal_base(self.seed ^ 0x5DEECE66D, row0, B, md.P_theta, 0, self.device)
        x0 = n * md.theta_base[1] + md.theta_base[0]
        return eps, base_lp, x0

    # ---- forward ----
    def forward(self, batch: Batch, eps: torch.Tensor, base_lp: Optional[torch.Tensor], x0_theta: torch.Tensor):
        md = self.mdef
        z, lq, theta, logq_theta = self._flows_forward(batch, eps, base_lp, x0_theta)
        sde, obs, extra = elbo_terms(md.model_id, md.M, md.dt, md.obs_std, batch.feeds, z, theta)
        if md.family == "lv":
            lq = lq + extra
        prior = self.prior_logprob(theta)
        scale = md.scale_num / md.M
        if md.family == "sv":
            elbo = scale * (sde - lq) + prior - logq_theta
        else:
            elbo = scale * (sde - lq + obs) + prior - logq_theta
        return {"elbo": elbo, "sde": sde, "obs": obs, "logq": lq, "theta": theta, "logq_theta": logq_theta,
                "prior": prior, "z": z}

    def onepass_ok(self) -> bool:
        """The training step can take the ELBO's values and gradients from one pass over z (vissm_elbo_fwd_grad);
        VISSM_ELBO_ONEPASS=0 keeps the forward + backward launches (A/B)."""
        return os.environ.get("VISSM_ELBO_ONEPASS", "1") != "0"

    def forward_onepass(self, batch: Batch, eps: torch.Tensor, base_lp: Optional[torch.Tensor],
                        x0_theta: torch.Tensor):
        """The training step's ELBO with the log-density terms in one pass over the path (vissm_elbo_fwd_grad): the
        loss is -sum_b ELBO_b, so the upstream gradients of (sde, obs, extra) are the constants (-scale, -scale or 0
        for SV, +scale for LV's ILDJ term, which enters log q) before the forward runs.  Returns (out, (roots,
        grads)) as forward_fused: autograd from the scalar root for the terms outside the log-densities (flows' log
        sigma, prior, q(theta)), dz and dtheta fed in at z and theta."""
        md = self.mdef
        z, lq, theta, logq_theta = self._flows_forward(batch, eps, base_lp, x0_theta)
        B = z.shape[0]
        scale = md.scale_num / md.M
        dev = z.device
        gs = torch.full((B,), -scale, dtype=torch.float32, device=dev)
        go = gs if md.family != "sv" else torch.zeros_like(gs)
        ge = torch.full((B,), scale, dtype=torch.float32, device=dev) if md.family == "lv" else None
        th = theta.detach().contiguous()
        sde, obs, extra, dz, dth = elbo_values_grad(md.model_id, md.M, md.dt, md.obs_std, batch.feeds, z.detach(),
                                                    th, gs, go, ge)
        prior = self.prior_logprob(theta)
        rest = scale * (-lq) + prior - logq_theta            # ELBO terms outside the log-densities (autograd)
        roots = [(-rest).sum(), z, theta]
        grads = [None, dz.view_as(z), dth]
        keep = [i for i, r in enumerate(roots) if r.requires_grad]
        roots, grads = [roots[i] for i in keep], [grads[i] for i in keep]
        lq_out = lq.detach() + (extra if md.family == "lv" else 0.0)
        if md.family == "sv":
            elbo = scale * (sde - lq_out) + prior.detach() - logq_theta.detach()
        else:
            elbo = scale * (sde - lq_out + obs) + prior.detach() - logq_theta.detach()
        out = {"elbo": elbo, "sde": sde, "obs": obs, "logq": lq_out, "theta": th, "logq_theta": logq_theta.detach(),
               "prior": prior.detach(), "z": z.detach()}
        return out, (roots, grads)

    def _flows_forward(self, batch: Batch, eps: torch.Tensor, base_lp: Optional[torch.Tensor],
                       x0_theta: torch.Tensor):
        """q(theta) and the flow stack: the path z, log q of the flows (base log-prob minus the log sigma sums),
        theta and log q(theta), all in the autograd graph."""
        md = self.mdef
        if base_lp is None:
            base_lp = base_logprob(eps, md.n_logsig)
        theta, logq_theta = self.theta_dist.sample_and_log_prob(x0_theta)
        s = 2 if md.D == 2 else 1
        u, lq = eps, base_lp
        B = eps.shape[0]
        L = md.kernel_ext
        for i, fl in enumerate(self.flows):
            ts = batch.ts if md.family == "lv" else batch.ts[:, i * md.k:, :]
            Lh = (L - md.k) // s
            C = fl.window_conv(ts, Lh, s, gemm=self.feature_gemm())
            tt = fl.theta_term(theta)
            pf, pb = self.flow_precisions()
            shape = FlowShape(B=B, L=L, k=md.k, H=fl.spec.H, n_hidden=fl.spec.n_hidden, bn=fl.spec.bn,
                              stride2=(s == 2), swap_out=(md.D == 2 and i < md.n_flows - 1),
                              n_logsig=md.n_logsig, n_win=batch.n_win, precision=pf, bwd_precision=pb,
                              chunk_tiles=self.chunk_tiles, pad_out=self.pad_rows and i < md.n_flows - 1)
            u, ls = fl.flow(shape, batch.win, u, C, tt, self.theta_fold(fl, theta), grad_sum=self.grad_sum)
            lq = lq - ls
            L -= md.k
        return u, lq, theta, logq_theta

    # ---- the last AR(1) flow fused with its ELBO terms (training step) ----
    def _last_shape(self, batch: Batch, B: int) -> FlowShape:
        md = self.mdef
        fl = self.flows[-1]
        L = md.kernel_ext - (md.n_flows - 1) * md.k
        # bf16x2f: the fused kernel recomputes the flow on split weights (the bf16x2 forward's products: x and log
        # sigma at that precision) and runs its backward products at bf16 (VISSM_PREC_BF16X2_BF16); bf16x2 runs
        # every weight product split (VISSM_PREC_BF16X2)
        prec = _lib.VISSM_PREC_BF16X2_BF16 if self.precision == _lib.VISSM_PREC_BF16X2F else self.precision
        return FlowShape(B=B, L=L, k=md.k, H=fl.spec.H, n_hidden=fl.spec.n_hidden, bn=fl.spec.bn, stride2=False,
                         swap_out=False, n_logsig=md.n_logsig, n_win=batch.n_win, precision=prec,
                         chunk_tiles=self.chunk_tiles)

    def theta_fold(self, fl: IAF, theta: torch.Tensor):
        """The theta branch's factors for the flow kernels (IAF.theta_factors) at the bf16 products of the AR
        family, whose two-sample kernels fold them into the layer-0 product; None elsewhere (the kernels read
        theta_term).  VISSM_THETA_FOLD=0 turns it off (A/B)."""
        if (self.mdef.family != "ar" or self.precision == _lib.VISSM_PREC_FP32 or theta.shape[1] > 5
                or os.environ.get("VISSM_THETA_FOLD", "1") == "0"):
            fl._fold = None   # the theta-branch kernel's collapsed weights go unused: drop them (and theta's graph)
            return None
        return fl.theta_factors(theta)

    def feature_gemm(self) -> Optional[str]:
        """How the window-shared conv over features runs where that GEMM is large (LV: the time-mixing features have
        kernel_ext - 1 channels): single bf16 products with fp32 accumulation at the bf16 precision (the mode's own
        arithmetic; LV-cfg step 76.5 -> 71.5 ms, the LV bf16 parity cases unchanged), split-bf16 products ("x3",
        fp32-class) at the parity precisions bf16x3 / bf16x3f / bf16x2f, fp32 otherwise (None).  For LV at a
        non-fp32 precision only, Engine.feature_gemm_override or VISSM_FEATURE_GEMM = bf16 | x3 | fp32 replaces the
        choice (A/B timing; tests that isolate the flow kernels from the bf16 rounding of these GEMMs); fp32 runs
        and the other families never change arithmetic.  SV (k = 50, a [L x 50] by [50 x 2500] conv product) runs its
        conv in the split-bf16 form at every non-fp32 precision ("x3": the hand-written branch, window_conv;
        VISSM_FEATURE_GEMM=fp32 restores the torch fp32 form for it too)."""
        if self.precision == _lib.VISSM_PREC_FP32 or self.mdef.family not in ("lv", "sv"):
            return None
        if self.mdef.family == "sv":
            mode = getattr(self, "feature_gemm_override", None) or os.environ.get("VISSM_FEATURE_GEMM")
            return None if mode == "fp32" else "x3"
        mode = getattr(self, "feature_gemm_override", None) or os.environ.get("VISSM_FEATURE_GEMM")
        if mode:
            if mode not in ("bf16", "x3", "fp32"):
                raise ValueError(f"feature GEMM mode {mode!r} is not bf16 / x3 / fp32")
            return None if mode == "fp32" else mode
        return "bf16" if self.precision == _lib.VISSM_PREC_BF16 else "x3"

    def flow_precisions(self):
        """(forward, backward) flow-kernel precisions of the engine's mode (host modes _lib.HOST_MODES:
        bf16x3f / bf16x2f = bf16x3 / bf16x2 forward products, bf16 backward products)."""
        if self.precision in _lib.HOST_MODES:
            return _lib.HOST_MODES[self.precision]
        return self.precision, None

    def fused_ok(self, batch: Batch, B: int) -> bool:
        """The step can run the last flow fused with the AR(1) ELBO (bf16 / bf16x3 matrix-core kernels)."""
        if (self.mdef.family != "ar" or self.precision == _lib.VISSM_PREC_FP32 or not self.fuse_last
                or (self.precision in _lib.HOST_MODES and self.precision != _lib.VISSM_PREC_BF16X2F)):
            return False
        return ar_fused_supported(self._last_shape(batch, B))

    def forward_fused(self, batch: Batch, eps: torch.Tensor, base_lp: Optional[torch.Tensor], x0_theta: torch.Tensor):
        """The training step's ELBO with the last flow fused with its AR(1) ELBO terms: returns (out, (roots,
        grads)) where out holds the per-sample ELBO and its terms (values) and
        torch.autograd.backward(roots, grads) accumulates the gradient of -sum_b ELBO_b (AR.py:228-229): the
        fused kernel's gradients w.r.t. its inputs (u, C, theta term, theta via sde / obs, the flow's weights)
        enter at those tensors, the rest (earlier flows, q(theta), prior) from the scalar root."""
        md = self.mdef
        if base_lp is None:
            base_lp = base_logprob(eps, md.n_logsig)
        theta, logq_theta = self.theta_dist.sample_and_log_prob(x0_theta)
        u, lq = eps, base_lp
        B = eps.shape[0]
        L = md.kernel_ext
        for i, fl in enumerate(self.flows[:-1]):
            Lh = L - md.k
            C = fl.window_conv(batch.ts[:, i * md.k:, :], Lh, 1)
            tt = fl.theta_term(theta)
            pf, pb = self.flow_precisions()
            shape = FlowShape(B=B, L=L, k=md.k, H=fl.spec.H, n_hidden=fl.spec.n_hidden, bn=fl.spec.bn, stride2=False,
                              swap_out=False, n_logsig=md.n_logsig, n_win=batch.n_win, precision=pf, bwd_precision=pb,
                              chunk_tiles=self.chunk_tiles, pad_out=self.pad_rows)
            u, ls = fl.flow(shape, batch.win, u, C, tt, self.theta_fold(fl, theta))
            lq = lq - ls
            L -= md.k
        fl = self.flows[-1]
        i = md.n_flows - 1
        C = fl.window_conv(batch.ts[:, i * md.k:, :], L - md.k, 1)
        tt = fl.theta_term(theta)
        shape = self._last_shape(batch, B)
        w_eps, w_hid, b_hid, _, _, w_head, b_head = fl.weights()
        scale = md.scale_num / md.M
        f = batch.feeds
        x, logsig, du, dC, dtt, gw = ar_last_flow_fused(
            shape, batch.win, u.detach(), C.detach(), tt.detach(), theta.detach().contiguous(), f.obs,
            f.obs_bin, md.obs_std, scale, w_eps.detach(), w_hid.detach(), b_hid.detach(), w_head.detach(),
            b_head.detach(), self.theta_fold(fl, theta))
        # sde / obs from the written path and their theta gradient (x is a constant here: the fused kernel
        # differentiated through it)
        th = theta.detach().contiguous()
        g = torch.full((B,), -scale, dtype=torch.float32, device=eps.device)
        sde, obs, dth = elbo_values_and_theta_grad(md.model_id, md.M, md.dt, md.obs_std, f, x, th, g, g)
        prior = self.prior_logprob(theta)
        rest = scale * (-lq) + prior - logq_theta            # ELBO terms outside the fused flow (autograd)
        # the gradient of -sum ELBO: autograd from the scalar root, the fused kernel's input gradients fed in
        # at their tensors (a multi-root backward: no surrogate products)
        roots = [(-rest).sum(), u, C, tt, theta, w_eps, w_hid, b_hid, w_head, b_head]
        grads = [None, du, dC, dtt, dth] + list(gw)
        # only the roots that carry a gradient (a one-flow stack's u is the base noise eps: no graph behind it)
        keep = [i for i, r in enumerate(roots) if r.requires_grad]
        roots, grads = [roots[i] for i in keep], [grads[i] for i in keep]
        elbo = scale * (sde + obs + logsig) + rest.detach()
        out = {"elbo": elbo, "sde": sde, "obs": obs, "logq": (lq.detach() - logsig), "theta": th,
               "logq_theta": logq_theta.detach(), "prior": prior.detach(), "z": x}
        return out, (roots, grads)

    def prior_logprob(self, theta):
        md = self.mdef
        key = (theta.device, theta.dtype)
        cache = self.__dict__.setdefault("_prior_t", {})
        if key not in cache:  # device constants made once (no host->device copy inside a captured step)
            cache[key] = (torch.tensor([m for m, _ in md.priors], dtype=theta.dtype, device=theta.device),
                          torch.tensor([s for _, s in md.priors], dtype=theta.dtype, device=theta.device))
        mean, sd = cache[key]
        zz = (theta - mean) / sd
        return (-0.5 * zz * zz - torch.log(sd) - 0.5 * LOG_2PI).sum(-1)

    def lf_sample(self, z: torch.Tensor, batch: Batch) -> torch.Tensor:
        """The latent path x [B, D, M+1] (torch; used by pre-training losses and save_paths)."""
        md = self.mdef
        B = z.shape[0]
        f = batch.feeds
        w = batch.win.long() if batch.win is not None else torch.zeros(B, dtype=torch.long, device=z.device)
        if md.family == "ar":
            return z.view(B, 1, -1)
        if md.family == "lv":
            zz = z.view(B, -1, 2).transpose(1, 2)
            return torch.nn.functional.softplus(zz) * f.mask[w] + f.shift[w]
        if md.family == "sv":
            return torch.stack([f.dim_one[w], z * f.mask[w] + f.shift[w]], 1)
        return z.view(B, -1, 2).transpose(1, 2)


# ---------------------------------------------------------------------------------------
# optimiser slots + scalar logging
# ---------------------------------------------------------------------------------------
class AdamaxSlots:
    """Slot pair (v = first moment, m = inf-norm) for one AdamaxOptimizer instance over the flat buffer."""

    def __init__(self, n: int, device):
        self.v = torch.zeros(n, dtype=torch.float32, device=device)
        self.m = torch.zeros(n, dtype=torch.float32, device=device)
        self.kernel = AdamaxKernel(n, device)


class ScalarLog:
    """TensorBoard-scalar replacement: JSON lines under <tensorboard_path>/<dd:mm:yy-HH:MM:SS>/scalars.jsonl
    with the reference's summary names (AR.py:205-238)."""

    def __init__(self, tensorboard_path: Optional[str], enabled: bool = True):
        self.f = None
        if tensorboard_path and enabled:
            d = os.path.join(tensorboard_path, datetime.now().strftime("%d:%m:%y-%H:%M:%S"))
            os.makedirs(d, exist_ok=True)
            self.f = open(os.path.join(d, "scalars.jsonl"), "a")

    def write(self, run: int, values: Dict[str, float], histograms: Optional[Dict[str, Dict]] = None):
        if self.f is None:
            return
        import json
        rec = {"step": run, **{k: float(v) for k, v in values.items()}}
        if histograms:
            rec["histograms"] = histograms
        self.f.write(json.dumps(rec) + "\n")
        self.f.flush()

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None
