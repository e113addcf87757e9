"""Fixed-order slab reductions (vissm_reduce_rows / vissm_reduce_rows_bf16) at the sizes the B = 65536
benchmark launch reduces: the flow backward's window-shared dC partials are one bf16 row per 16-sample
group, 4096 rows x Lh * H = 5017 * 50 columns (flow5, one window), and the fp32 slabs (d theta, weight
partials) are reduced by vissm_reduce_rows.  The sums run row by row in fp32 (r = 0 .. R-1), so the
result must equal a float32 sequential sum bit for bit and stay within the fp32 rounding bound of the
float64 sum."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from viforssms_amd import _lib  # noqa: E402

DEV = "cuda:0"


def _seq_sum_f32(rows: np.ndarray) -> np.ndarray:
    acc = np.zeros(rows.shape[1], dtype=np.float32)
    for r in range(rows.shape[0]):
        acc = acc + rows[r]          # float32 + float32 -> float32, row order
    return acc


@pytest.mark.parametrize("R,N", [(4096, 5017 * 50), (4096, 5009 * 50 + 1), (7, 33), (1, 2)])
def test_reduce_rows_bf16_matches_sequential_fp32(R, N):
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(R * 31 + N)
    x = (torch.randn(R, N, generator=g, device=DEV) * torch.rand(R, 1, generator=g, device=DEV) * 10).to(torch.bfloat16)
    out = torch.empty(N, dtype=torch.float32, device=DEV)
    _lib.check(lib.vissm_reduce_rows_bf16(x.data_ptr(), out.data_ptr(), R, N, _lib.stream_handle(torch.device(DEV))),
               "vissm_reduce_rows_bf16")
    torch.cuda.synchronize()
    rows = x.float().cpu().numpy()
    got = out.cpu().numpy()
    ref32 = _seq_sum_f32(rows)
    assert np.array_equal(got, ref32), int((got != ref32).sum())
    ref64 = rows.astype(np.float64).sum(0)
    bound = R * 2.0 ** -24 * np.abs(rows).astype(np.float64).sum(0) + 1e-30
    assert (np.abs(got - ref64) <= bound).all()


@pytest.mark.parametrize("R,N", [(4096, 50 * 4096 // 64), (8192, 2551), (3, 5)])
def test_reduce_rows_fp32_matches_sequential(R, N):
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(R + N)
    x = torch.randn(R, N, generator=g, device=DEV)
    out = torch.empty(N, dtype=torch.float32, device=DEV)
    _lib.check(lib.vissm_reduce_rows(x.data_ptr(), out.data_ptr(), R, N, _lib.stream_handle(torch.device(DEV))),
               "vissm_reduce_rows")
    torch.cuda.synchronize()
    rows = x.cpu().numpy()
    assert np.array_equal(out.cpu().numpy(), _seq_sum_f32(rows))
