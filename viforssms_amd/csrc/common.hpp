// Shared helpers of libvissm: error state, launch checking, Philox RNG,
// wave/block reductions.  gfx950 only (wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <cstdio>

#include "../../include/vissm.h"

namespace vissm {

void set_error(const char* fmt, ...);

#define VISSM_CHECK_ARG(cond, ...)        \
  do {                                    \
    if (!(cond)) {                        \
      ::vissm::set_error(__VA_ARGS__);    \
      return VISSM_EINVAL;                \
    }                                     \
  } while (0)

#define VISSM_CHECK_LAUNCH(what)                                               \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess) {                                                    \
      ::vissm::set_error("%s: %s", what, hipGetErrorString(e_));               \
      return VISSM_ELAUNCH;                                                    \
    }                                                                          \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. 2011), counter = (lo(ctr), hi(ctr), lo(sub), hi(sub)),
// key = seed.  Box-Muller on the 4 outputs gives 4 N(0,1) values.
// ---------------------------------------------------------------------------
struct u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32 -> 64-bit product per word (v_mad_u64_u32) instead of separate hi / lo multiplies
    const uint64_t p0 = static_cast<uint64_t>(M0) * c.x, p1 = static_cast<uint64_t>(M1) * c.z;
    const uint32_t hi0 = static_cast<uint32_t>(p0 >> 32), lo0 = static_cast<uint32_t>(p0);
    const uint32_t hi1 = static_cast<uint32_t>(p1 >> 32), lo1 = static_cast<uint32_t>(p1);
    u4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

__device__ __forceinline__ float u01(uint32_t x) {
  // (0, 1]: never 0 so log() is finite
  return (static_cast<float>(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------------------
// reductions (wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Fixed-order block sum; all threads get the result.  `red` must hold blockDim/64 entries.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  T s = 0;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }
// derivative of ELU expressed through its output (TF EluGrad: y < 0 ? dy*(y+1) : dy)
__device__ __forceinline__ float elu_grad_from_out(float y) { return y < 0.f ? y + 1.f : 1.f; }
__device__ __forceinline__ float softplus_f(float x) {
  // log(1 + e^x), stable
  return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
}
__device__ __forceinline__ float sigmoid_f(float x) {
  return x >= 0.f ? 1.f / (1.f + expf(-x)) : expf(x) / (1.f + expf(x));
}

constexpr float kLog2Pi = 1.8378770664093453f;
constexpr float kBnScale = 0.99950037468777f;  // 1/sqrt(1 + 1e-3)

int launch_reduce_rows(const float* slab, float* out, int64_t R, int64_t N, hipStream_t st);
// same result, two passes for few columns / many rows; uses the slab's part-head rows as scratch
int launch_reduce_rows_inplace(float* slab, float* out, int64_t R, int64_t N, hipStream_t st);
// the same sum over a slab of bf16 partials (R rows of N bf16 at `slab`), fp32 accumulation, fixed order
int launch_reduce_rows_bf16(const void* slab, float* out, int64_t R, int64_t N, hipStream_t st);

// flow epilogues shared by the flow implementations (flow_common.hip)
int launch_halo_fixup(float* du, const float* halo, int B, int L, int pL, int k, int n_chunks, int s, int CH,
                      hipStream_t st);
int launch_reduce_by_window(const float* slab, const int32_t* win, float* out, int B, int n_win, int64_t N,
                            hipStream_t st);
int launch_scatter_wgrad(const float* red, const VissmFlowGrads* g, int k, int H, int nh, int bn, hipStream_t st);

// opt-in event timing of main kernels (vissm_profile_*)
bool prof_on();
void prof_begin(int kind, hipStream_t st);
void prof_end(int kind, hipStream_t st, double bytes = 0.0);

}  // namespace vissm
