"""Timing of the LV feature GEMM shapes: fp32 torch.mm vs the split-bf16 (bf16x3) form, and the error of the
latter against a float64 product on a sample."""
import time, torch
from viforssms_amd.linalg import mm_bf16x3

def t(f, n=5):
    f(); torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - s) / n * 1e3

N, K = 10061, 1000
F = torch.randn(N, N, device="cuda")
W = torch.randn(N, K, device="cuda") * 0.01
Ft = F.t()
print("fwd fp32 %.3f ms  x3 %.3f ms" % (t(lambda: F @ W), t(lambda: mm_bf16x3(F, W))))
print("fwd(transposed view) fp32 %.3f ms  x3 %.3f ms" % (t(lambda: Ft @ W), t(lambda: mm_bf16x3(Ft, W))))
a = F.to(torch.bfloat16)
print("bf16 mm out fp32 %.3f ms" % t(lambda: torch.mm(a, W.to(torch.bfloat16), out_dtype=torch.float32)))
print("split cost %.3f ms" % t(lambda: (F.to(torch.bfloat16), (F - F.to(torch.bfloat16).float()).to(torch.bfloat16))))
ref = (F[:256].double() @ W.double())
e = ((mm_bf16x3(F, W)[:256].double() - ref).norm() / ref.norm()).item()
e32 = (((F @ W)[:256].double() - ref).norm() / ref.norm()).item()
print("rel err x3 %.2e fp32 %.2e" % (e, e32))
