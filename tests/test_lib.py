"""The C-ABI library: it loads without a GPU, exports every symbol include/vissm.h declares, and the
hand-derived ELBO transition gradients (compiled for the host from the same header the kernels use)
match the oracle's autograd.  No GPU compute here."""
import ctypes
import math
import os
import re

import numpy as np
import pytest
import torch

from oracle import nma_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vissm.h")
HOSTCHECK = os.path.join(ROOT, "viforssms_amd", "libvissm_hostcheck.so")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(vissm_[a-z_0-9]+)\s*\(", src)))


def test_library_loads_and_exports_all_symbols():
    from viforssms_amd import _lib
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} not bound in _lib.SIGNATURES"
    assert lib.vissm_version() >= 1


def test_library_built_from_this_tree():
    """The pushed binary is the built one: the source hash compiled into libvissm.so equals the hash of csrc/ +
    include/vissm.h + the Makefile as they are now (fails when the .so is older than, or other than, the sources)."""
    from viforssms_amd import _lib, srchash
    lib = _lib.load()
    assert lib.vissm_source_hash().decode() == srchash.source_hash()
    assert lib.vissm_build_flags() == b"", "an A/B variant build is installed as the production library"
    assert "viforssms_amd/csrc/flow_v5.hip" in srchash.source_files()


def test_loader_refuses_foreign_library(monkeypatch):
    from viforssms_amd import _lib, srchash
    lib = _lib.load()
    monkeypatch.setattr(srchash, "source_hash", lambda root=None: "0" * 64)
    with pytest.raises(_lib.VissmError, match="built from other sources"):
        _lib.check_source_hash(lib)


def test_library_rejects_bad_shapes_without_gpu():
    from viforssms_amd import _lib
    lib = _lib.load()
    d = _lib.FlowDesc(4, 10, 99, 16, 1, 0, 0, 0, 5, 1, 0, 0)  # k > 64
    assert lib.vissm_flow_workspace_size(ctypes.byref(d), 0) == 0
    rc = lib.vissm_normal_base(1, 0, None, None, 2, 0, 0, None)
    assert rc < 0 and b"bad shape" in lib.vissm_last_error()


def test_feature_kernels_refuse_kernel_shorter_than_stride():
    """vissm_feat_*: a forward block writes s (kT - 1) + k rows and the backward reads s kT, so k < stride would leave
    rows the backward reads unwritten; the shape check refuses it (host arithmetic only, no GPU)."""
    from viforssms_amd import _lib
    lib = _lib.load()

    def ws(k, s, Lh=10):
        d = _lib.FeatDesc(n_win=1, Lf=s * (Lh - 1) + k + 5, Cin=3, H=50, k=k, stride=s, Lh=Lh, in_win_stride=0)
        return lib.vissm_feat_workspace_size(ctypes.byref(d))

    assert ws(2, 2) > 0 and ws(1, 1) > 0 and ws(20, 2) > 0
    assert ws(1, 2) == 0
    assert b"kernel_len 1 < stride 2" in lib.vissm_last_error()


def test_elbo_fwd_grad_checks_without_gpu():
    """vissm_elbo_fwd_grad (the training step's one-pass log-density call): a null z / dz is refused and B = 0 is a
    no-op, before any device work; VissmElboData carries the observation list as its last fields (include/vissm.h)."""
    from viforssms_amd import _lib
    lib = _lib.load()
    assert [f[0] for f in _lib.ElboData._fields_][-2:] == ["obs_list", "obs_stride"]
    fake = ctypes.c_void_p(16)   # never dereferenced: the checks run first
    d = _lib.ElboDesc(_lib.MODEL_FHN, 4, 10, 1, 0.1, 1.0)
    data = _lib.ElboData(None, fake, fake, None, None, None, None, None, 0)
    rc = lib.vissm_elbo_fwd_grad(ctypes.byref(d), ctypes.byref(data), None, fake, fake, fake, None, fake, fake,
                                 None, fake, fake, None)
    assert rc < 0 and b"null pointer" in lib.vissm_last_error()
    d0 = _lib.ElboDesc(_lib.MODEL_FHN, 0, 10, 1, 0.1, 1.0)
    assert lib.vissm_elbo_fwd_grad(ctypes.byref(d0), ctypes.byref(data), fake, fake, fake, fake, None, fake, fake,
                                   None, fake, fake, None) == 0
    # an observation list without its stride is refused before any launch
    bad = _lib.ElboData(None, fake, fake, None, None, None, None, fake, 0)
    rc = lib.vissm_elbo_fwd_grad(ctypes.byref(d), ctypes.byref(bad), fake, fake, fake, fake, None, fake, fake,
                                 None, fake, fake, None)
    assert rc < 0 and b"obs_stride" in lib.vissm_last_error()


def test_bf16x2_precisions_without_gpu():
    """VISSM_PREC_BF16X2 (split weights, bf16 activations) is a forward and backward precision with workspace on
    both sides; VISSM_PREC_BF16X2_BF16 belongs to the fused last AR flow only and the other entry points refuse it
    before touching the device (include/vissm.h)."""
    from viforssms_amd import _lib
    lib = _lib.load()
    d = _lib.FlowDesc(4, 40, 8, 50, 1, 0, 0, 0, 32, 1, _lib.VISSM_PREC_BF16X2, 0)
    assert lib.vissm_flow_workspace_size(ctypes.byref(d), 0) > 0
    assert lib.vissm_flow_workspace_size(ctypes.byref(d), 1) > 0
    assert lib.vissm_flow_ar_elbo_fused_supported(ctypes.byref(d)) == 1
    buf = (ctypes.c_float * 64)()
    p = ctypes.cast(buf, ctypes.c_void_p).value
    w = _lib.FlowParams(*([p] * len(_lib.FlowParams._fields_)))
    gr = _lib.FlowGrads(*([p] * len(_lib.FlowGrads._fields_)))
    dx = _lib.FlowDesc(4, 40, 8, 50, 1, 0, 0, 0, 32, 1, _lib.VISSM_PREC_BF16X2_BF16, 0)
    rc = lib.vissm_flow_bwd(ctypes.byref(dx), ctypes.byref(w), p, p, None, p, p, p, p, p, p, ctypes.byref(gr), p, 64,
                            None)
    assert rc < 0 and b"vissm_flow_ar_elbo_fused only" in lib.vissm_last_error()
    rc = lib.vissm_flow_fwd(ctypes.byref(dx), ctypes.byref(w), p, p, None, p, p, p, p, 64, None)
    assert rc < 0 and b"vissm_flow_ar_elbo_fused only" in lib.vissm_last_error()
    # the fused last AR flow takes both at the two-sample kernel's shape (k <= 8, one window)
    assert lib.vissm_flow_ar_elbo_fused_supported(ctypes.byref(dx)) == 1
    assert lib.vissm_flow_ar_elbo_fused_workspace_size(ctypes.byref(dx)) > 0
    d33 = _lib.FlowDesc(4, 60, 20, 50, 1, 0, 0, 0, 32, 1, _lib.VISSM_PREC_BF16X2, 0)   # k = 20: not that shape
    assert lib.vissm_flow_ar_elbo_fused_supported(ctypes.byref(d33)) == 0
    assert set(_lib.HOST_MODES) <= set(_lib.TRAIN_PRECISIONS.values())


@pytest.mark.parametrize("family,B,M,k,nf,prec,want", [
    # the benchmark launches (bench.py MODEL_DEFAULTS, BASELINE configs[1-4]): tiles per t-chunk of flow 0's backward
    ("ar", 65536, 5000, 8, 3, "bf16", 157),
    ("lv", 16384, 5000, 20, 3, "bf16", 40), ("fhn", 8192, 2000, 20, 3, "bf16", 8), ("sv", 16384, 1508, 50, 5, "bf16", 14),
    ("lv", 16384, 5000, 20, 3, "fp32", 79), ("fhn", 8192, 2000, 20, 3, "fp32", 16), ("sv", 16384, 1508, 50, 5, "fp32", 27),
    # the parity batches without chunk_tiles: LV / FHN one tile per chunk on the bf16 kernels, SV 5
    ("lv", 3, 5000, 20, 3, "bf16", 1), ("fhn", 20, 2000, 20, 3, "bf16", 1), ("sv", 20, 1508, 50, 5, "bf16", 5)])
def test_flow_geometry_without_gpu(family, B, M, k, nf, prec, want):
    """vissm_flow_geometry (host arithmetic) gives the chunk geometry the parity tests force through chunk_tiles
    (tests/test_gpu_config_parity.py: the benchmark's launch geometry at a small batch)."""
    from tests.parity_util import bench_geometry
    from viforssms_amd import _lib
    geo = bench_geometry(family, _lib.TRAIN_PRECISIONS[prec], B, M, k, nf)
    assert geo[0]["chunk_tiles"] == want, geo
    assert geo[0]["tile"] == (16 if prec != "fp32" else 32)
    for g in geo:
        assert g["n_groups"] == (B + 15) // 16 and g["n_chunks"] >= 1


def test_flow_geometry_forced_chunk_tiles():
    from viforssms_amd import _lib
    d = _lib.FlowDesc(3, 10062, 20, 50, 3, 1, 1, 1, 10000, 1, _lib.VISSM_PREC_BF16, 40)
    g = _lib.flow_geometry(d, 1)
    assert g == {"tile": 16, "chunk_tiles": 40, "n_chunks": 8, "n_groups": 1}
    d.k = 99
    with pytest.raises(_lib.VissmError):
        _lib.flow_geometry(d, 1)


def test_flow_row_pitch_validates_without_gpu():
    """VissmFlowDesc.u_pitch / out_pitch (0 = dense) must cover the row: a pitch below L (L - k) is rejected before
    any launch; the fused last flow writes x dense (out_pitch 0 or L - k only)."""
    from viforssms_amd import _lib
    from viforssms_amd.ops import FlowShape
    lib = _lib.load()
    sh = FlowShape(B=4, L=5017, k=8, H=50, n_hidden=1, bn=False, stride2=False, swap_out=False, n_logsig=5000, n_win=1,
                   precision=_lib.VISSM_PREC_BF16)
    for up, op, ok in [(0, 0, True), (5024, 5024, True), (5017, 5009, True), (5016, 0, False), (0, 5008, False)]:
        d = sh.desc(up, op)
        assert (lib.vissm_flow_workspace_size(ctypes.byref(d), 1) > 0) == ok, (up, op)
    assert lib.vissm_flow_ar_elbo_fused_workspace_size(ctypes.byref(sh.desc(5024, 0))) > 0


def _host():
    lib = ctypes.CDLL(HOSTCHECK)
    f = lib.vissm_host_trans
    f.restype = None
    f.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_float)] * 3 + [ctypes.c_float, ctypes.POINTER(ctypes.c_float)]
    return lib


def _arr(v):
    a = (ctypes.c_float * len(v))(*[float(x) for x in v])
    return a


def _oracle_trans(model, xh, xt, th, dt):
    """lp and gradients of one transition from the oracle's density functions (float64 autograd)."""
    xh_t = torch.tensor(xh, dtype=O.DT, requires_grad=True)
    xt_t = torch.tensor(xt, dtype=O.DT, requires_grad=True)
    th_t = torch.tensor(th, dtype=O.DT, requires_grad=True)
    if model == 0:
        x = torch.stack([xh_t[0], xt_t[0]]).view(1, 2)
        lp, _ = O.ar_elbo_terms(x, th_t.view(1, -1), torch.zeros(1, 1, dtype=O.DT), torch.zeros(1, 1, dtype=O.DT), 1.0)
    else:
        x = torch.stack([xh_t, xt_t], 1).view(1, 2, 2)
        if model == 1:
            lp, _ = O.lv_elbo_terms(x, th_t.view(1, -1), torch.zeros(1, 2, 1, dtype=O.DT),
                                    torch.zeros(1, 2, 1, dtype=O.DT), dt)
        elif model == 2:
            lp = O.sv_elbo_terms(x, th_t.view(1, -1), dt)
        else:
            lp, _ = O.fhn_elbo_terms(x, th_t.view(1, -1), torch.zeros(1, 2, 1, dtype=O.DT),
                                     torch.zeros(1, 2, 1, dtype=O.DT), dt)
    lp = lp.sum()
    gh, gt, gth = torch.autograd.grad(lp, [xh_t, xt_t, th_t])
    return lp.item(), gh.numpy(), gt.numpy(), gth.numpy()


CASES = [
    (0, [10.3], [12.1], [5.0, 0.5, math.log(3.0)], 1.0),
    (0, [-2.0], [0.7], [0.3, -0.9, -0.4], 1.0),
    (1, [100.0, 90.0], [103.0, 88.5], [math.log(0.5), math.log(0.0025), math.log(0.3)], 0.1),
    (1, [20.0, 300.0], [19.0, 305.0], [math.log(0.44), math.log(0.003), math.log(0.29)], 0.1),
    (2, [3.1, -8.0], [3.3, -7.7], [0.01, -0.6, math.log(0.08), math.log(0.5)], 1.0),
    (3, [0.4, 1.2], [0.45, 1.3], [math.log(2.0), 1.0, 1.5, math.log(0.5), math.log(0.3)], 0.1),
    (3, [-1.5, 0.2], [-1.4, 0.1], [0.2, -0.5, 0.7, -1.0, 0.3], 0.1),
]


@pytest.mark.parametrize("case", CASES)
def test_transition_gradients_match_oracle(case):
    model, xh, xt, th, dt = case
    lib = _host()
    out = (ctypes.c_float * 10)()
    xh2 = list(xh) + [0.0] * (2 - len(xh))
    xt2 = list(xt) + [0.0] * (2 - len(xt))
    lib.vissm_host_trans(model, _arr(xh2), _arr(xt2), _arr(list(th) + [0.0] * (5 - len(th))), dt, out)
    lp, gh, gt, gth = _oracle_trans(model, xh, xt, th, dt)
    D = len(xh)
    got = np.array(out[:])
    scale = max(1.0, abs(lp))
    assert abs(got[0] - lp) <= 2e-6 * scale
    gscale = max(1.0, np.abs(np.concatenate([gh, gt, gth])).max())
    assert np.allclose(got[1:1 + D], gh, atol=3e-5 * gscale, rtol=1e-4)
    assert np.allclose(got[3:3 + D], gt, atol=3e-5 * gscale, rtol=1e-4)
    assert np.allclose(got[5:5 + len(th)], gth, atol=3e-5 * gscale, rtol=1e-4)


def test_softplus_ildj_matches_oracle():
    lib = ctypes.CDLL(HOSTCHECK)
    f = lib.vissm_host_sp_ildj
    f.restype = ctypes.c_float
    f.argtypes = [ctypes.c_float, ctypes.POINTER(ctypes.c_float)]
    for y in (0.05, 0.7, 3.0, 40.0):
        g = ctypes.c_float()
        v = f(y, ctypes.byref(g))
        yt = torch.tensor(y, dtype=O.DT, requires_grad=True)
        ref = -torch.log(-torch.expm1(-yt))
        (gr,) = torch.autograd.grad(ref, [yt])
        assert abs(v - ref.item()) <= 1e-5 * max(1, abs(ref.item()))
        assert abs(g.value - gr.item()) <= 1e-4 * max(1, abs(gr.item()))


def test_hostcheck_sanitized():
    """The host build of elbo_math.hpp (hostcheck.cpp) under -fsanitize=address,undefined (SURVEY.md §5 race /
    memory checking on host code; GPU sanitizers are unavailable on the pool): every model's transition gradient
    against central finite differences over 200 states each, the softplus ILDJ, the observation term and the ABI
    layout query, with any sanitizer report fatal."""
    import subprocess
    csrc = os.path.join(ROOT, "viforssms_amd", "csrc")
    subprocess.run(["make", "-C", csrc, "build/hostcheck_san"], check=True, capture_output=True)
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(csrc, "build", "hostcheck_san")], capture_output=True, text=True, env=env,
                       timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


def test_abi_struct_layouts_match_ctypes():
    """The ctypes mirrors of VissmFlowDesc / VissmFlowParams / VissmFlowGrads (viforssms_amd/_lib.py) have the C
    compiler's sizes and last-field offsets (include/vissm.h; round 3 appended the theta-fold fields)."""
    from viforssms_amd import _lib
    lib = ctypes.CDLL(HOSTCHECK)
    f = lib.vissm_host_abi_layout
    f.restype = None
    f.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]
    for which, (cls, last) in enumerate([(_lib.FlowDesc, "out_pitch"), (_lib.FlowParams, "theta_rank"),
                                         (_lib.FlowGrads, "b_head"), (_lib.ElboData, "obs_stride")]):
        out = (ctypes.c_size_t * 2)()
        f(which, out)
        assert out[0] == ctypes.sizeof(cls), (cls.__name__, out[0], ctypes.sizeof(cls))
        assert out[1] == getattr(cls, last).offset, (cls.__name__, last)


def test_feat_workspace_size_validates_without_gpu():
    """vissm_feat_workspace_size (host arithmetic): the fused feature branch's shape limits (Cin <= 63, H <= 64,
    k <= 64, stride 1 | 2, s (Lh - 1) + k <= Lf) are checked before any launch; 0 = rejected."""
    from viforssms_amd import _lib
    lib = _lib.load()
    ok = _lib.FeatDesc(1, 5024, 14, 50, 8, 1, 5017, 5024 * 14)
    assert lib.vissm_feat_workspace_size(ctypes.byref(ok)) > 0
    for bad in [(1, 5024, 14, 65, 8, 1, 5017, 0), (1, 5024, 64, 50, 8, 1, 5017, 0), (1, 5024, 14, 50, 65, 1, 4960, 0),
                (1, 5024, 14, 50, 8, 3, 1000, 0), (1, 5024, 14, 50, 8, 1, 5018, 0), (2, 100, 14, 50, 8, 1, 93, 99 * 14)]:
        assert lib.vissm_feat_workspace_size(ctypes.byref(_lib.FeatDesc(*bad))) == 0, bad


def test_asm_mfma_accumulators_hazard_free():
    """The three-layer backward's weight-gradient accumulators live in AGPRs through inline-asm MFMAs (hipcc pads no
    hazard for an asm statement): in the device assembly of flow_v5n.hip no compiler instruction touches an AGPR that
    an asm MFMA wrote fewer than 12 wait states earlier on any path (scripts/check_agpr_asm.py; ~1 min of hipcc)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_agpr_asm.py")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "bwd2n_kernel" in r.stdout


def test_agpr_audit_detects_unpadded_reads(tmp_path):
    """scripts/check_agpr_asm.py is not vacuous: on a synthetic kernel it flags a compiler read of an AGPR an asm MFMA
    just wrote, across a fall-through and a branch edge, and passes once a drain statement sits in between."""
    import subprocess
    import sys

    def kernel(between):
        return "\n".join(["_Z4testv:", "; %bb.0:", ";;#ASMSTART", "s_nop 1",
                          "v_mfma_f32_16x16x32_bf16 a[0:3], v[0:3], v[4:7], a[0:3]", ";;#ASMEND", *between,
                          "s_cbranch_scc1 .LBB0_2", "; %bb.1:", "v_add_f32_e32 v9, v9, v9", ".LBB0_2:",
                          "v_accvgpr_read_b32 v8, a1", "s_endpgm", ".Lfunc_end0:", ""])
    bad = tmp_path / "bad.s"
    bad.write_text(kernel([]))
    good = tmp_path / "good.s"
    good.write_text(kernel([";;#ASMSTART", "s_nop 7", "s_nop 3", ";;#ASMEND"]))
    far = tmp_path / "far.s"
    far.write_text(kernel(["v_add_f32_e32 v9, v9, v9"] * 12))
    script = os.path.join(ROOT, "scripts", "check_agpr_asm.py")
    assert subprocess.run([sys.executable, script, str(bad)], capture_output=True).returncode == 1
    assert subprocess.run([sys.executable, script, str(good)], capture_output=True).returncode == 0
    assert subprocess.run([sys.executable, script, str(far)], capture_output=True).returncode == 0


def test_flow_kernel_precision_query():
    """vissm_flow_kernel_precision: bf16 / bf16x3 / bf16x2 run as asked on the shapes flow5 covers and fall back to
    the exact-fp32 kernels elsewhere (k > 32 at one hidden layer; bf16x2 / bf16x3 at three hidden layers)."""
    from viforssms_amd import _lib
    from viforssms_amd.ops import FlowShape, kernel_precision
    ar = dict(B=4, L=40, k=8, H=50, n_hidden=1, bn=False, stride2=False, swap_out=False, n_logsig=24, n_win=1)
    lv = dict(B=4, L=40, k=4, H=50, n_hidden=3, bn=True, stride2=True, swap_out=True, n_logsig=24, n_win=1)
    for prec in (_lib.VISSM_PREC_FP32, _lib.VISSM_PREC_BF16, _lib.VISSM_PREC_BF16X3, _lib.VISSM_PREC_BF16X2):
        assert kernel_precision(FlowShape(**ar, precision=prec)) == prec
    k50 = dict(ar, k=50, L=80)
    assert kernel_precision(FlowShape(**k50, precision=_lib.VISSM_PREC_BF16X2)) == _lib.VISSM_PREC_FP32
    assert kernel_precision(FlowShape(**k50, precision=_lib.VISSM_PREC_BF16)) == _lib.VISSM_PREC_BF16
    assert kernel_precision(FlowShape(**lv, precision=_lib.VISSM_PREC_BF16)) == _lib.VISSM_PREC_BF16
    assert kernel_precision(FlowShape(**lv, precision=_lib.VISSM_PREC_BF16X2)) == _lib.VISSM_PREC_FP32
    with pytest.raises(_lib.VissmError):
        kernel_precision(FlowShape(**ar, precision=_lib.VISSM_PREC_BF16X2_BF16))


@pytest.mark.parametrize("family,k", [("lv", 4), ("ar", 50)])
def test_engine_refuses_bf16x2_beyond_split_kernels(family, k):
    """bf16x2 on LV / SV / FHN or AR with k > 32 used to run an fp32 forward under the bf16x2 label and
    then stop in the first backward (du = NULL on the fp32 kernels); the engine now refuses it up front.  bf16x2f
    (forward split weights or exact fp32, backward bf16) stays valid there."""
    from tests.parity_util import build_model
    from viforssms_amd import _lib
    nl = 5 if family == "lv" else 3
    with pytest.raises(ValueError, match="bf16x2"):
        build_model(family, 4, 24, k, 2, 16, nl, 3, "cpu", precision=_lib.TRAIN_PRECISIONS["bf16x2"])
    build_model(family, 4, 24, k, 2, 16, nl, 3, "cpu", precision=_lib.TRAIN_PRECISIONS["bf16x2f"])
