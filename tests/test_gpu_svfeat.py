"""The split-bf16 matrix-core GEMM (vissm_gemm_bf16x3) and stochastic volatility's feature branch built on it
(ops.SvFeatConvFn: vissm_lv_mlp_* at four layers with the first-difference input, SV_dense.py:50-62).

* x3 GEMM: every operand layout and split-K against the float64 product of the fp32 operands the hi / lo planes
  split (fp32-class: relative error within 3e-5, where one bf16 product is ~3e-3), at shapes off the 128 x 128 x 32
  tile.
* SV branch: C and every variable's gradient against the float64 torch form (nma.IAF.features + conv_shared); the
  HIP form's arithmetic is fp32 layers and fp32-class conv products, held to 3x the fp32 torch form's error + 2e-5."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from viforssms_amd.ops import gemm_bf16x3, sv_feat_conv  # noqa: E402
from viforssms_amd.linalg import linear  # noqa: E402

DEV = "cuda:0"


def _r8(n):
    return (n + 7) // 8 * 8


def _split(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def _mat(rows, cols, ld, g):
    """fp32 [rows][ld] random in the first cols columns, NaN padding (never read), and its hi / lo planes"""
    x = torch.full((rows, ld), float("nan"), device=DEV)
    x[:, :cols] = torch.randn(rows, cols, generator=g, device=DEV)
    hi, lo = _split(x)
    return x, hi, lo


@pytest.mark.parametrize("a_kmajor", [False, True])
@pytest.mark.parametrize("b_kmajor", [False, True])
@pytest.mark.parametrize("M,N,K", [(37, 45, 70), (130, 257, 50), (1508, 50, 2500), (50, 2500, 1508)])
def test_gemm_x3_layouts(a_kmajor, b_kmajor, M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M * 5 + N * 3 + K + 2 * a_kmajor + b_kmajor)
    A, Ah, Al = _mat(K, M, _r8(M), g) if a_kmajor else _mat(M, K, _r8(K), g)
    B, Bh, Bl = _mat(K, N, _r8(N), g) if b_kmajor else _mat(N, K, _r8(K), g)
    Am = (A[:, :M].t() if a_kmajor else A[:, :K]).double()
    Bm = (B[:, :N] if b_kmajor else B[:, :K].t()).double()
    ref = Am @ Bm
    for split in (1, 4):
        C = torch.full((M, N), float("nan"), device=DEV)
        gemm_bf16x3(M, N, K, Ah, Al, A.shape[1], a_kmajor, Bh, Bl, B.shape[1], b_kmajor, C, N, split_k=split)
        torch.cuda.synchronize()
        err = float((C.double() - ref).norm() / ref.norm())
        assert err < 3e-5, (split, err)


@pytest.mark.parametrize("a_kmajor,b_kmajor", [(False, True), (True, False)])
@pytest.mark.parametrize("M,N,K", [(37, 45, 70), (300, 257, 96)])
def test_gemm_x3_bf16_epilogues(a_kmajor, b_kmajor, M, N, K):
    """x3 ELU / elu' epilogues: the output as a hi / lo plane pair (lo at C + M ldc), aux read the same way; the
    pair's sum within 2^-15 of the float64 value (one bf16 plane alone is 2^-8)"""
    from viforssms_amd import _lib
    g = torch.Generator(device=DEV).manual_seed(M + N + K + a_kmajor)
    A, Ah, Al = _mat(K, M, _r8(M), g) if a_kmajor else _mat(M, K, _r8(K), g)
    B, Bh, Bl = _mat(K, N, _r8(N), g) if b_kmajor else _mat(N, K, _r8(K), g)
    Am = (A[:, :M].t() if a_kmajor else A[:, :K]).double()
    Bm = (B[:, :N] if b_kmajor else B[:, :K].t()).double()
    ref = Am @ Bm
    ldc = _r8(N) + 8
    Y = torch.full((2, M, ldc), float("nan"), device=DEV, dtype=torch.bfloat16)
    gemm_bf16x3(M, N, K, Ah, Al, A.shape[1], a_kmajor, Bh, Bl, B.shape[1], b_kmajor, Y, ldc, _lib.GEMM_ELU_BF16)
    torch.cuda.synchronize()
    elu = torch.where(ref > 0, ref, torch.expm1(ref))
    y = Y[0, :, :N].double() + Y[1, :, :N].double()
    assert float((y - elu).abs().max()) <= 2 ** -15 * float(elu.abs().max())
    assert torch.isnan(Y[:, :, N:].float()).all()
    Z = torch.empty(2, M, ldc, device=DEV, dtype=torch.bfloat16)
    gemm_bf16x3(M, N, K, Ah, Al, A.shape[1], a_kmajor, Bh, Bl, B.shape[1], b_kmajor, Z, ldc, _lib.GEMM_DELU_BF16,
                aux=Y)
    torch.cuda.synchronize()
    dref = ref * torch.where(y < 0, y + 1, torch.ones_like(y))
    z = Z[0, :, :N].double() + Z[1, :, :N].double()
    assert float((z - dref).abs().max()) <= 2 ** -15 * float(dref.abs().max())


def _sv_case(L, Cr, k, H=50, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    r = lambda *sh, sc=1.0: (torch.randn(*sh, generator=g, device=DEV) * sc).requires_grad_(True)
    Cin = 2 * Cr - 2
    ws = [r(Cin, H, sc=0.3), r(H, sc=0.1), r(H, H, sc=0.15), r(H, sc=0.1), r(H, H, sc=0.15), r(H, sc=0.1),
          r(H, H, sc=0.15), r(H, sc=0.1), r(k, 1 + H, H, sc=0.03), r(H, sc=0.1)]
    ts = torch.randn(2, L, Cr, generator=g, device=DEV)
    return ts, ws


def _torch_form(ts, ws, s, Lh):
    """nma.IAF.features + conv_shared for SV (SV_dense.py:50-62)"""
    h = torch.cat([ts[:, 1:, :], ts[:, 1:, :-2] - ts[:, :-1, :-2]], 2)
    for j in range(4):
        h = torch.nn.functional.elu(linear(h, ws[2 * j], ws[2 * j + 1]))
    W = ws[8]
    k, H = W.shape[0], W.shape[2]
    nw, Lf, _ = h.shape
    G = linear(h, W[:, 1:, :].permute(1, 0, 2).reshape(-1, k * H)).view(nw, Lf, k, H)
    idx = torch.arange(Lh, device=DEV)[:, None] * s + torch.arange(k, device=DEV)[None, :]
    C = G[:, idx, torch.arange(k, device=DEV)[None, :]].sum(2) + ws[9]
    return C


@pytest.mark.parametrize("L,Cr,k,s", [(1509, 8, 50, 1), (302, 8, 50, 2), (90, 5, 9, 1)])
def test_sv_feature_branch_matches_torch_form(L, Cr, k, s):
    ts, ws = _sv_case(L, Cr, k, seed=L + k)
    Lh = (L - 1 - k) // s + 1
    dC = torch.randn(2, Lh, ws[0].shape[1], device=DEV, generator=torch.Generator(device=DEV).manual_seed(7))

    def grads(fn):
        for w in ws:
            w.grad = None
        C = fn()
        (C * dC).sum().backward()
        return C.detach(), [w.grad.detach().clone() for w in ws]

    wd = [w.detach().double().requires_grad_(True) for w in ws]
    C64 = _torch_form(ts.double(), wd, s, Lh)
    (C64 * dC.double()).sum().backward()
    g64 = [w.grad for w in wd]
    Ch, gh = grads(lambda: sv_feat_conv(ts, s, Lh, *ws))
    Cf, gf = grads(lambda: _torch_form(ts, ws, s, Lh))
    rel = lambda a, b: float((a.double() - b).norm() / (b.norm() + 1e-30))
    eC_h, eC_f = rel(Ch, C64.detach()), rel(Cf, C64.detach())
    assert eC_h < 3 * eC_f + 2e-5, (eC_h, eC_f)
    for i, (a, b, ref) in enumerate(zip(gh, gf, g64)):
        if i == 8:   # the conv kernel: its sample channel 0 is the flow kernel's (zero here, in both forms)
            assert float(a[:, 0, :].abs().max()) == 0.0
        e_h, e_f = rel(a, ref), rel(b, ref)
        assert e_h < 3 * e_f + 2e-5, (i, e_h, e_f)
