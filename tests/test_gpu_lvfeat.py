"""The bf16 matrix-core GEMM (vissm_gemm_bf16) and Lotka-Volterra's feature branch built on it (vissm_lv_*,
ops.LvFeatConvFn; lotka_volterra_partial.py:71-82).

* GEMM: every operand layout, the three epilogues and split-K against a float64 product of the same bf16-rounded
  operands (fp32 accumulation: relative error within 1e-5), at shapes that are not multiples of the 128 x 128 x 32
  tile (edge chunks, partial K steps).
* LV feature branch: C and the gradient of every variable against the float64 torch form of the same layers
  (nma.IAF.features + conv_shared in fp32 arithmetic): the HIP form rounds the time-mixing layer's and the conv's
  operands to bf16, as the bf16 training precision's torch form (linear_bf16) rounds the conv's, so both are held
  to the same bound, and the HIP form's error must stay within 3x the torch bf16 form's + a floor."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from viforssms_amd import _lib  # noqa: E402
from viforssms_amd.ops import gemm_bf16, lv_feat_conv  # noqa: E402
from viforssms_amd.linalg import linear, linear_bf16  # noqa: E402

DEV = "cuda:0"


def _r8(n):
    return (n + 7) // 8 * 8


def _mat(rows, cols, ld, g, scale=1.0):
    """bf16 [rows][ld] with random entries in the first cols columns (NaN in the padding: it must never be read)"""
    x = torch.full((rows, ld), float("nan"), device=DEV, dtype=torch.bfloat16)
    x[:, :cols] = (torch.randn(rows, cols, generator=g, device=DEV) * scale).to(torch.bfloat16)
    return x


@pytest.mark.parametrize("a_kmajor", [False, True])
@pytest.mark.parametrize("b_kmajor", [False, True])
@pytest.mark.parametrize("M,N,K", [(37, 45, 70), (130, 257, 96), (300, 64, 1000), (64, 333, 1201)])
def test_gemm_layouts(a_kmajor, b_kmajor, M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N * 3 + K + 2 * a_kmajor + b_kmajor)
    A = _mat(K, M, _r8(M), g) if a_kmajor else _mat(M, K, _r8(K), g)
    B = _mat(K, N, _r8(N), g) if b_kmajor else _mat(N, K, _r8(K), g)
    Am = (A[:, :M].t() if a_kmajor else A[:, :K]).double()          # [M][K]
    Bm = (B[:, :N] if b_kmajor else B[:, :K].t()).double()          # [K][N]
    ref = Am @ Bm
    for split in (1, 3):
        C = torch.full((M, N), float("nan"), device=DEV)
        gemm_bf16(M, N, K, A, A.shape[1], a_kmajor, B, B.shape[1], b_kmajor, C, N, _lib.GEMM_F32, split_k=split)
        torch.cuda.synchronize()
        err = float((C.double() - ref).norm() / ref.norm())
        assert err < 1e-5, (split, err)
    # ELU epilogue into a padded bf16 C, then the elu' epilogue against it
    ldc = _r8(N) + 8
    Y = torch.full((M, ldc), float("nan"), device=DEV, dtype=torch.bfloat16)
    gemm_bf16(M, N, K, A, A.shape[1], a_kmajor, B, B.shape[1], b_kmajor, Y, ldc, _lib.GEMM_ELU_BF16)
    torch.cuda.synchronize()
    elu = torch.where(ref > 0, ref, torch.expm1(ref))
    yv = Y[:, :N].double()
    assert float((yv - elu).abs().max()) <= 2 ** -7 * float(elu.abs().max()) + 1e-6
    assert torch.isnan(Y[:, N:].float()).all()      # the padding is left alone
    Z = torch.empty(M, ldc, device=DEV, dtype=torch.bfloat16)
    gemm_bf16(M, N, K, A, A.shape[1], a_kmajor, B, B.shape[1], b_kmajor, Z, ldc, _lib.GEMM_DELU_BF16, aux=Y)
    torch.cuda.synchronize()
    dref = ref * torch.where(yv < 0, yv + 1, torch.ones_like(yv))
    assert float((Z[:, :N].double() - dref).abs().max()) <= 2 ** -7 * float(dref.abs().max()) + 1e-6


def test_gemm_rejects_unaligned_leading_dimension():
    A = torch.zeros(16, 20, device=DEV, dtype=torch.bfloat16)
    B = torch.zeros(16, 24, device=DEV, dtype=torch.bfloat16)
    C = torch.zeros(16, 16, device=DEV)
    with pytest.raises(_lib.VissmError):
        gemm_bf16(16, 16, 20, A, 20, False, B, 24, False, C, 16)


def _lv_case(R, U, k, s, Cin=13, H=50, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    r = lambda *sh, sc=1.0: (torch.randn(*sh, generator=g, device=DEV) * sc).requires_grad_(True)
    ws = [r(Cin, H, sc=0.3), r(H, sc=0.1), r(H, H, sc=0.15), r(H, sc=0.1), r(H, H, sc=0.15), r(H, sc=0.1),
          r(H, U, sc=0.15), r(U, sc=0.1), r(k, 1 + R, H, sc=0.02), r(H, sc=0.1)]
    h0 = torch.randn(1, R, Cin, generator=g, device=DEV)
    Lh = (U - k) // s + 1
    return h0, ws, Lh


def _torch_form(h0, ws, s, Lh, lin):
    """nma.IAF.features + conv_shared for LV (lotka_volterra_partial.py:71-82), the conv's products by `lin`"""
    h = h0
    for j in range(4):
        h = torch.nn.functional.elu(linear(h, ws[2 * j], ws[2 * j + 1]))
    F = h.transpose(1, 2)                                    # [1, U, R]
    W = ws[8]
    k, H = W.shape[0], W.shape[2]
    G = lin(F, W[:, 1:, :].permute(1, 0, 2).reshape(-1, k * H)).view(1, F.shape[1], k, H)
    idx = torch.arange(Lh, device=DEV)[:, None] * s + torch.arange(k, device=DEV)[None, :]
    C = G[0][idx, torch.arange(k, device=DEV)[None, :]].sum(1) + ws[9]
    return C[None]


@pytest.mark.parametrize("R,U,k,s", [(301, 283, 20, 2), (257, 250, 9, 1), (1031, 1001, 20, 2)])
def test_lv_feature_branch_x3_matches_fp32_torch_form(R, U, k, s):
    """The parity precisions' form (every product split-bf16, D and dP as hi / lo planes): within 3x the fp32 torch
    form's error against float64 + 2e-5, at C and every variable's gradient"""
    h0, ws, Lh = _lv_case(R, U, k, s, seed=R + U + 1)
    dC = torch.randn(1, Lh, ws[0].shape[1], device=DEV, generator=torch.Generator(device=DEV).manual_seed(6))

    def grads(fn):
        for w in ws:
            w.grad = None
        C = fn()
        (C * dC).sum().backward()
        return C.detach(), [w.grad.detach().clone() for w in ws]

    wd = [w.detach().double().requires_grad_(True) for w in ws]
    C64 = _torch_form(h0.double(), wd, s, Lh, linear)
    (C64 * dC.double()).sum().backward()
    g64 = [w.grad for w in wd]
    Ch, gh = grads(lambda: lv_feat_conv(h0, s, Lh, *ws, x3=True))
    Cf, gf = grads(lambda: _torch_form(h0, ws, s, Lh, linear))
    rel = lambda a, b: float((a.double() - b).norm() / (b.norm() + 1e-30))
    eC_h, eC_f = rel(Ch, C64.detach()), rel(Cf, C64.detach())
    assert eC_h < 3 * eC_f + 2e-5, (eC_h, eC_f)
    for i, (a, b, ref) in enumerate(zip(gh, gf, g64)):
        if i == 8:
            assert float(a[:, 0, :].abs().max()) == 0.0
        e_h, e_f = rel(a, ref), rel(b, ref)
        assert e_h < 3 * e_f + 2e-5, (i, e_h, e_f)


@pytest.mark.parametrize("R,U,k,s", [(301, 283, 20, 2), (257, 250, 9, 1), (1031, 1001, 20, 2)])
def test_lv_feature_branch_matches_torch_form(R, U, k, s):
    h0, ws, Lh = _lv_case(R, U, k, s, seed=R + U)
    dC = torch.randn(1, Lh, ws[0].shape[1], device=DEV, generator=torch.Generator(device=DEV).manual_seed(5))

    def grads(fn):
        for w in ws:
            w.grad = None
        C = fn()
        (C * dC).sum().backward()
        return C.detach(), [w.grad.detach().clone() for w in ws]

    wd = [w.detach().double().requires_grad_(True) for w in ws]
    C64 = _torch_form(h0.double(), wd, s, Lh, linear)
    (C64 * dC.double()).sum().backward()
    g64 = [w.grad for w in wd]
    Ch, gh = grads(lambda: lv_feat_conv(h0, s, Lh, *ws))
    Cb, gb = grads(lambda: _torch_form(h0, ws, s, Lh, linear_bf16))
    rel = lambda a, b: float((a.double() - b).norm() / (b.norm() + 1e-30))
    eC_h, eC_b = rel(Ch, C64), rel(Cb, C64)
    assert eC_h < 3 * eC_b + 1e-3, (eC_h, eC_b)
    for i, (a, b, ref) in enumerate(zip(gh, gb, g64)):
        if i == 8:   # the conv kernel: its sample channel 0 is the flow kernel's (zero here, in both forms)
            assert float(a[:, 0, :].abs().max()) == 0.0
        e_h, e_b = rel(a, ref), rel(b, ref)
        assert e_h < 3 * e_b + 2e-3, (i, e_h, e_b)
