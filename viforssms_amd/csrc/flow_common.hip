// Epilogue kernels shared by the flow implementations (flow_v2 / flow_v4 / flow_v5):
// the t-chunk halo join of du, the per-window dC reduce, and the scatter of the reduced
// weight-gradient vector into the caller's VissmFlowGrads (no BN folding: flow_v2 / flow_v4
// accumulate d gamma directly; flow_v5 has its own BN-unfolding scatter).
#include "common.hpp"

namespace vissm {

namespace {

// du[b][s*(c+1)*CH + q] += halo[b][c][q]: the transposed-conv overhang of t-chunk c into c + 1 (rows pL apart)
__global__ void halo_fixup_kernel(float* __restrict__ du, const float* __restrict__ halo, int B, int L, int pL, int k,
                                  int n_chunks, int s, int CH) {
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < (n_chunks - 1) * k; i += blockDim.x) {
    const int c = i / k, q = i % k;
    const int pos = s * (c + 1) * CH + q;
    if (pos < L) du[static_cast<size_t>(b) * pL + pos] += halo[(static_cast<size_t>(b) * n_chunks + c) * k + q];
  }
}

// out[w][c] = sum over samples b with win[b] == w of slab[b][c], in sample order (deterministic)
__global__ void reduce_by_window_kernel(const float* __restrict__ slab, const int32_t* __restrict__ win,
                                        float* __restrict__ out, int B, int N) {
  const int wv = blockIdx.y;
  const int cidx = blockIdx.x * blockDim.x + threadIdx.x;
  if (cidx >= N) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b)
    if (win[b] == wv) s += slab[static_cast<size_t>(b) * N + cidx];
  out[static_cast<size_t>(wv) * N + cidx] = s;
}

// red = [w_eps (kH) | w_hid (nh H^2) | b_hid (nh H) | bn_g (nh H) | bn_b (nh H) | w_head (2H) | b_head (2)]
__global__ void scatter_wgrad_kernel(const float* __restrict__ red, VissmFlowGrads g, int k, int H, int nh, int bn) {
  const int nW = k * H + nh * H * H + 3 * nh * H + 2 * H + 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nW; i += gridDim.x * blockDim.x) {
    const float v = red[i];
    int off = 0;
    if (i < (off += k * H)) { g.w_eps[i] = v; continue; }
    if (i < off + nh * H * H) { g.w_hid[i - off] = v; continue; }
    off += nh * H * H;
    if (i < off + nh * H) { g.b_hid[i - off] = v; continue; }
    off += nh * H;
    if (i < off + nh * H) { if (bn && g.bn_g) g.bn_g[i - off] = v * kBnScale; continue; }
    off += nh * H;
    if (i < off + nh * H) { if (bn && g.bn_b) g.bn_b[i - off] = v; continue; }
    off += nh * H;
    if (i < off + 2 * H) { g.w_head[i - off] = v; continue; }
    off += 2 * H;
    g.b_head[i - off] = v;
  }
}

}  // namespace

int launch_halo_fixup(float* du, const float* halo, int B, int L, int pL, int k, int n_chunks, int s, int CH,
                      hipStream_t st) {
  if (n_chunks <= 1) return VISSM_OK;
  hipLaunchKernelGGL(halo_fixup_kernel, dim3(B), dim3(256), 0, st, du, halo, B, L, pL, k, n_chunks, s, CH);
  VISSM_CHECK_LAUNCH("flow_halo");
  return VISSM_OK;
}

int launch_reduce_by_window(const float* slab, const int32_t* win, float* out, int B, int n_win, int64_t N,
                            hipStream_t st) {
  dim3 rg(static_cast<unsigned>((N + 255) / 256), n_win);
  hipLaunchKernelGGL(reduce_by_window_kernel, rg, dim3(256), 0, st, slab, win, out, B, static_cast<int>(N));
  VISSM_CHECK_LAUNCH("flow_reduce_window");
  return VISSM_OK;
}

int launch_scatter_wgrad(const float* red, const VissmFlowGrads* g, int k, int H, int nh, int bn, hipStream_t st) {
  const int nW = k * H + nh * H * H + 3 * nh * H + 2 * H + 2;
  hipLaunchKernelGGL(scatter_wgrad_kernel, dim3((nW + 255) / 256), dim3(256), 0, st, red, *g, k, H, nh, bn);
  VISSM_CHECK_LAUNCH("flow_scatter");
  return VISSM_OK;
}

}  // namespace vissm
