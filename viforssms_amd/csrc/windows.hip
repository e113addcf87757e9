// Window gather (include/vissm.h vissm_gather_windows): the per-step time_feats / ELBO-feed
// assembly of the reference's train loop (AR.py:267-288; lotka_volterra_partial.py:366-386;
// SV_dense.py:304-328) as one device gather from padded channel tables that stay resident in HBM.
// The step uploads only its window starts; no host gather, no feed upload.
#include "common.hpp"

namespace vissm {
namespace {

// one thread per output element, the output's fastest dimension across adjacent lanes
__global__ __launch_bounds__(256) void gather_windows_kernel(VissmGatherDesc d, const float* __restrict__ src,
                                                             const int32_t* __restrict__ starts,
                                                             float* __restrict__ out) {
  const int64_t total = static_cast<int64_t>(d.n) * d.len * d.C;
  // decompose in the order of the smallest output stride first, so stores coalesce
  const bool c_fast = d.os_c <= d.os_j;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int64_t r, j, c;
    if (c_fast) {
      c = i % d.C;
      const int64_t q = i / d.C;
      j = q % d.len;
      r = q / d.len;
    } else {
      j = i % d.len;
      const int64_t q = i / d.len;
      c = q % d.C;
      r = q / d.C;
    }
    const int64_t s = static_cast<int64_t>(d.stride) * starts[r] + d.offset + j * d.j_step + c * d.c_pitch;
    out[r * d.os_r + j * d.os_j + c * d.os_c] = src[s];
  }
}

}  // namespace
}  // namespace vissm

using namespace vissm;

extern "C" int vissm_gather_windows(const VissmGatherDesc* d, const float* src, const int32_t* starts, float* out,
                                    void* stream) {
  VISSM_CHECK_ARG(d && src && starts && out, "gather_windows: null pointer");
  VISSM_CHECK_ARG(d->n >= 0 && d->len >= 0 && d->C >= 1 && d->stride >= 1 && d->j_step >= 1,
                  "gather_windows: bad shape (n=%d len=%d C=%d stride=%d)", d->n, d->len, d->C, d->stride);
  const int64_t total = static_cast<int64_t>(d->n) * d->len * d->C;
  if (total == 0) return VISSM_OK;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 1 << 16);
  hipLaunchKernelGGL(gather_windows_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, as_stream(stream), *d,
                     src, starts, out);
  VISSM_CHECK_LAUNCH("gather_windows");
  return VISSM_OK;
}
