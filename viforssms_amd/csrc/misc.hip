// libvissm: error state, base noise (init_dist), deterministic row reduction,
// global-norm clip + Adamax (optimisers/adamax.py:42-58, AR.py:230-232).
#include "common.hpp"

#include <cstdarg>
#include <cmath>
#include <algorithm>
#include <mutex>
#include <vector>

#ifndef VISSM_SRC_HASH
#error "build through the Makefile: it defines VISSM_SRC_HASH (the source hash _lib.load() checks)"
#endif
#ifndef VISSM_BUILD_FLAGS
#define VISSM_BUILD_FLAGS ""
#endif

namespace vissm {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ---------------------------------------------------------------------------
// base noise + base log-prob.  One block per sample row; Philox counter =
// (column group, row + offset) so the stream is independent of the launch
// geometry and of how rows are sharded across ranks.
// ---------------------------------------------------------------------------
// Box-Muller on the hardware transcendentals: r = sqrt(-2 ln u1) from v_log_f32 (log2) and
// v_sqrt_f32, the angle 2 pi u2 through v_sin_f32 / v_cos_f32, whose argument is in revolutions
// (u2 itself, in (0, 1]) -- no range reduction.  Every kernel that draws the stream uses this.
__device__ __forceinline__ void box_muller4(u4 r, float (&v)[4]) {
  constexpr float kM2Ln2 = -1.3862943611198906f;  // -2 ln 2
  const float r1 = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(r.x)));
  const float r2 = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(r.z)));
  const float t1 = u01(r.y), t2 = u01(r.w);
  v[0] = r1 * __builtin_amdgcn_cosf(t1);
  v[1] = r1 * __builtin_amdgcn_sinf(t1);
  v[2] = r2 * __builtin_amdgcn_cosf(t2);
  v[3] = r2 * __builtin_amdgcn_sinf(t2);
}

// One wave per row (kNbW rows per 256-thread block): the base log-prob is a wave reduction, no
// block barrier.
// (offset_dev: the row offset read from device memory instead, so a captured graph can advance it)
constexpr int kNbW = 4;
__global__ __launch_bounds__(256) void normal_base_kernel(uint64_t seed, uint64_t offset,
                                                          const uint64_t* __restrict__ offset_dev,
                                                          float* __restrict__ eps, float* __restrict__ base_lp,
                                                          int B, int L, int n_last) {
  const int lane = threadIdx.x & 63;
  const int b = __builtin_amdgcn_readfirstlane(blockIdx.x * kNbW + (threadIdx.x >> 6));
  if (b >= B) return;  // wave-uniform
  const uint64_t row = (offset_dev ? *offset_dev : offset) + static_cast<uint64_t>(b);
  const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
  float* out = eps + static_cast<size_t>(b) * L;
  double acc = 0.0;
  for (int g = lane; g * 4 < L; g += 64) {
    u4 c{static_cast<uint32_t>(g), 0u, static_cast<uint32_t>(row), static_cast<uint32_t>(row >> 32)};
    u4 r = philox4x32_10(c, k0, k1);
    float v[4];
    box_muller4(r, v);
    const int j0 = g * 4;
    if (j0 + 3 < L) {
      // one 16-byte store (rows are only dword-aligned: L is odd in general)
      typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
      *reinterpret_cast<f4u*>(out + j0) = f4u{v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (j0 + q < L) out[j0 + q] = v[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (j0 + q < L && j0 + q >= L - n_last) acc += -0.5 * static_cast<double>(v[q]) * v[q];
  }
  const double s = wave_sum(acc);
  if (lane == 0) base_lp[b] = static_cast<float>(s - 0.5 * kLog2Pi * n_last);
}

// Short rows (the q(theta) base draws, L = P_theta): one thread per row, the same Philox stream
// (counter (group, row)) and the same fixed-order sum, without a 256-thread block per row.
constexpr int kShortRow = 64;
__global__ __launch_bounds__(256) void normal_base_short_kernel(uint64_t seed, uint64_t offset,
                                                                const uint64_t* __restrict__ offset_dev,
                                                                float* __restrict__ eps, float* __restrict__ base_lp,
                                                                int B, int L, int n_last) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t row = (offset_dev ? *offset_dev : offset) + static_cast<uint64_t>(b);
  const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
  float* out = eps + static_cast<size_t>(b) * L;
  double acc = 0.0;
  for (int g = 0; g * 4 < L; ++g) {
    u4 c{static_cast<uint32_t>(g), 0u, static_cast<uint32_t>(row), static_cast<uint32_t>(row >> 32)};
    u4 r = philox4x32_10(c, k0, k1);
    float v[4];
    box_muller4(r, v);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = g * 4 + q;
      if (j < L) {
        out[j] = v[q];
        if (j >= L - n_last) acc += -0.5 * static_cast<double>(v[q]) * v[q];
      }
    }
  }
  base_lp[b] = static_cast<float>(acc - 0.5 * kLog2Pi * n_last);
}

static void launch_normal(uint64_t seed, uint64_t offset, const uint64_t* offset_dev, float* eps, float* base_lp,
                          int B, int L, int n_last, hipStream_t st) {
  if (L <= kShortRow)
    hipLaunchKernelGGL(normal_base_short_kernel, dim3((B + 255) / 256), dim3(256), 0, st, seed, offset, offset_dev, eps,
                       base_lp, B, L, n_last);
  else
    hipLaunchKernelGGL(normal_base_kernel, dim3((B + kNbW - 1) / kNbW), dim3(256), 0, st, seed, offset, offset_dev, eps,
                       base_lp, B, L, n_last);
}

__global__ __launch_bounds__(256) void base_logprob_kernel(const float* __restrict__ eps, float* __restrict__ base_lp,
                                                           int L, int n_last) {
  __shared__ double red[4];
  const int b = blockIdx.x;
  const float* row = eps + static_cast<size_t>(b) * L;
  double acc = 0.0;
  for (int j = L - n_last + threadIdx.x; j < L; j += blockDim.x) acc += -0.5 * static_cast<double>(row[j]) * row[j];
  double s = block_sum(acc, red);
  if (threadIdx.x == 0) base_lp[b] = static_cast<float>(s - 0.5 * kLog2Pi * n_last);
}

// ---------------------------------------------------------------------------
// out[c] = sum_r slab[r][c], fixed order.  Columns across threads (coalesced),
// rows split in chunks of RCH across blockIdx.y then summed in order by a second pass.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void reduce_rows_strided_kernel(const float* __restrict__ slab,
                                                                  float* __restrict__ out, int64_t R, int64_t N,
                                                                  int64_t row_stride) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= N) return;
  float s = 0.f;
  for (int64_t r = 0; r < R; ++r) s += slab[r * row_stride + c];
  out[c] = s;
}

__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                          int64_t R, int64_t N, int64_t rows_per_part,
                                                          int64_t out_stride) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= N) return;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * rows_per_part;
  const int64_t r1 = min(R, r0 + rows_per_part);
  // fixed order: r0, r0+1, ... (four loads in flight, summed in row order)
  float s = 0.f;
  int64_t r = r0;
  for (; r + 4 <= r1; r += 4) {
    const float a0 = slab[r * N + c], a1 = slab[(r + 1) * N + c], a2 = slab[(r + 2) * N + c],
                a3 = slab[(r + 3) * N + c];
    s += a0;
    s += a1;
    s += a2;
    s += a3;
  }
  for (; r < r1; ++r) s += slab[r * N + c];
  out[static_cast<int64_t>(blockIdx.y) * out_stride + c] = s;
}

// two columns per thread (one 4-byte load of a bf16 pair per row), eight rows in flight, row order
// rows in flight per thread of the bf16 slab reduction: 32 (AR-cfg dC reduce 0.389 -> 0.360 ms per launch against 8,
// profiles/r06/ab_r06m.log; the sums stay in row order, bit-exact with the sequential fp32 sum)
#ifndef VISSM_REDUCE_DEPTH
#define VISSM_REDUCE_DEPTH 32
#endif
constexpr int kRedDepth = VISSM_REDUCE_DEPTH;
__global__ __launch_bounds__(256) void reduce_rows_bf16_kernel(const __bf16* __restrict__ slab, float* __restrict__ out,
                                                               int64_t R, int64_t N) {
  const int64_t c = 2 * (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x);
  if (c >= N) return;
  float s0 = 0.f, s1 = 0.f;
  if (c + 1 < N && (N % 2) == 0) {
    typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
    const bf2v* p = reinterpret_cast<const bf2v*>(slab + c);
    const int64_t st = N / 2;
    int64_t r = 0;
    // VISSM_REDUCE_DEPTH rows in flight per thread (the launch has only ~8 waves per CU); the sums stay in row order
    for (; r + kRedDepth <= R; r += kRedDepth) {
      bf2v v[kRedDepth];
#pragma unroll
      for (int i = 0; i < kRedDepth; ++i) v[i] = p[(r + i) * st];
#pragma unroll
      for (int i = 0; i < kRedDepth; ++i) {
        s0 += static_cast<float>(v[i][0]);
        s1 += static_cast<float>(v[i][1]);
      }
    }
    for (; r + 8 <= R; r += 8) {
      bf2v v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = p[(r + i) * st];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s0 += static_cast<float>(v[i][0]);
        s1 += static_cast<float>(v[i][1]);
      }
    }
    for (; r < R; ++r) {
      const bf2v v = p[r * st];
      s0 += static_cast<float>(v[0]);
      s1 += static_cast<float>(v[1]);
    }
    out[c] = s0;
    out[c + 1] = s1;
  } else {
    for (int64_t r = 0; r < R; ++r) s0 += static_cast<float>(slab[r * N + c]);
    out[c] = s0;
    if (c + 1 < N) {
      for (int64_t r = 0; r < R; ++r) s1 += static_cast<float>(slab[r * N + c + 1]);
      out[c + 1] = s1;
    }
  }
}

int launch_reduce_rows_bf16(const void* slab, float* out, int64_t R, int64_t N, hipStream_t st) {
  if (R <= 0 || N <= 0) return VISSM_OK;
  const int64_t threads = (N + 1) / 2;
  dim3 grid(static_cast<unsigned>((threads + 255) / 256), 1);
  hipLaunchKernelGGL(reduce_rows_bf16_kernel, grid, dim3(256), 0, st, static_cast<const __bf16*>(slab), out, R, N);
  VISSM_CHECK_LAUNCH("reduce_rows_bf16");
  return VISSM_OK;
}

// x = hi + lo with hi = bf16(x), lo = bf16(x - hi), both round-to-nearest-even (the operands of the split-bf16
// library GEMMs): one read of x, one write of each plane; four elements per thread, grid-stride
__global__ __launch_bounds__(256) void split_bf16_kernel(const float* __restrict__ x, __bf16* __restrict__ hi,
                                                         __bf16* __restrict__ lo, int64_t n) {
  typedef __bf16 bf4v __attribute__((ext_vector_type(4)));
  const int64_t n4 = n / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    const float e[4] = {v.x, v.y, v.z, v.w};
    bf4v h, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      h[j] = static_cast<__bf16>(e[j]);
      l[j] = static_cast<__bf16>(e[j] - static_cast<float>(h[j]));
    }
    reinterpret_cast<bf4v*>(hi)[i] = h;
    reinterpret_cast<bf4v*>(lo)[i] = l;
  }
  if (blockIdx.x == 0 && threadIdx.x < n - 4 * n4) {
    const int64_t j = 4 * n4 + threadIdx.x;
    const __bf16 h = static_cast<__bf16>(x[j]);
    hi[j] = h;
    lo[j] = static_cast<__bf16>(x[j] - static_cast<float>(h));
  }
}

int launch_reduce_rows(const float* slab, float* out, int64_t R, int64_t N, hipStream_t st) {
  if (R <= 0 || N <= 0) return VISSM_OK;
  // single pass: rows summed sequentially per column (deterministic)
  dim3 grid(static_cast<unsigned>((N + 255) / 256), 1);
  hipLaunchKernelGGL(reduce_rows_kernel, grid, dim3(256), 0, st, slab, out, R, N, R, N);
  VISSM_CHECK_LAUNCH("reduce_rows");
  return VISSM_OK;
}

int launch_reduce_rows_inplace(float* slab, float* out, int64_t R, int64_t N, hipStream_t st) {
  if (R <= 0 || N <= 0) return VISSM_OK;
  // two deterministic passes when there are few columns: parts of rpp rows each are summed in
  // order into the part's first row (in place: no other part reads it), then the parts in order
  const int64_t want_threads = 1 << 17;
  int64_t parts = (want_threads + N - 1) / N;
  parts = std::min<int64_t>(parts, R / 8);
  if (parts <= 1) return launch_reduce_rows(slab, out, R, N, st);
  const int64_t rpp = (R + parts - 1) / parts;
  parts = (R + rpp - 1) / rpp;
  dim3 g1(static_cast<unsigned>((N + 255) / 256), static_cast<unsigned>(parts));
  hipLaunchKernelGGL(reduce_rows_kernel, g1, dim3(256), 0, st, slab, slab, R, N, rpp, rpp * N);
  VISSM_CHECK_LAUNCH("reduce_rows_p1");
  // pass 2 over the part heads: rows 0, rpp, 2 rpp, ... == a slab of `parts` rows with stride rpp*N
  dim3 g2(static_cast<unsigned>((N + 255) / 256), 1);
  hipLaunchKernelGGL(reduce_rows_strided_kernel, g2, dim3(256), 0, st, slab, out, parts, N, rpp * N);
  VISSM_CHECK_LAUNCH("reduce_rows_p2");
  return VISSM_OK;
}

// ---------------------------------------------------------------------------
// global norm + clip + Adamax
// ---------------------------------------------------------------------------
constexpr int kNormBlocks = 1024;

__global__ __launch_bounds__(256) void sqnorm_partial_kernel(const float* __restrict__ x, int64_t n,
                                                             double* __restrict__ part) {
  __shared__ double red[4];
  double acc = 0.0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * 4;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n && ((reinterpret_cast<uintptr_t>(x + i) & 15) == 0)) {
      float4 v = *reinterpret_cast<const float4*>(x + i);
      acc += static_cast<double>(v.x) * v.x + static_cast<double>(v.y) * v.y + static_cast<double>(v.z) * v.z +
             static_cast<double>(v.w) * v.w;
    } else {
      for (int64_t j = i; j < min(n, i + 4); ++j) acc += static_cast<double>(x[j]) * x[j];
    }
  }
  double s = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// skip (guarded step only, may be NULL): set to 1 when the norm is not finite, else 0; *skipped counts
// the skipped steps
__global__ __launch_bounds__(1024) void sqnorm_final_kernel(const double* __restrict__ part, int np,
                                                            float* __restrict__ sq_out, float* __restrict__ norm_out,
                                                            float* __restrict__ scale_out, float clip,
                                                            int32_t* __restrict__ skip, int32_t* __restrict__ skipped) {
  __shared__ double red[16];
  double v = threadIdx.x < np ? part[threadIdx.x] : 0.0;
  double s = block_sum(v, red);
  if (threadIdx.x == 0) {
    double nrm = sqrt(s);
    if (sq_out) *sq_out = static_cast<float>(s);
    if (norm_out) *norm_out = static_cast<float>(nrm);
    if (scale_out) {
      // tf.clip_by_global_norm: clip * min(1/norm, 1/clip); non-finite norm -> NaN
      float sc;
      if (clip <= 0.f) sc = 1.f;
      else if (!isfinite(nrm)) sc = NAN;
      else sc = static_cast<float>(static_cast<double>(clip) * fmin(1.0 / nrm, 1.0 / static_cast<double>(clip)));
      *scale_out = sc;
    }
    if (skip) {
      const int bad = isfinite(nrm) ? 0 : 1;
      skip[0] = bad;
      if (skipped) skipped[0] += bad;
    }
  }
}

__global__ __launch_bounds__(256) void adamax_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                     float* __restrict__ v, float* __restrict__ m, int64_t n,
                                                     const float* __restrict__ scale_ptr, float lr, float b1,
                                                     float b2, float eps, const int32_t* __restrict__ skip) {
  if (skip && skip[0]) return;  // guarded step with a non-finite norm: params and slots untouched
  const float sc = *scale_ptr;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gi = g[i] * sc;
    float vi = b1 * v[i] + (1.f - b1) * gi;
    float mi = fmaxf(b2 * m[i] + eps, fabsf(gi));
    v[i] = vi;
    m[i] = mi;
    p[i] = p[i] - lr * (vi / mi);
  }
}

// ---------------------------------------------------------------------------
// opt-in event timing
// ---------------------------------------------------------------------------
struct ProfRec {
  int kind;
  hipEvent_t a, b;
  double bytes;  // algorithmic HBM bytes of the launch (streaming kernels; 0 when not stated)
};
static bool g_prof = false;
static std::mutex g_prof_mu;
static std::vector<ProfRec> g_prof_recs;
constexpr int kProfKinds = 8;
static thread_local hipEvent_t g_open[kProfKinds] = {};

bool prof_on() { return g_prof; }

void prof_begin(int kind, hipStream_t st) {
  if (!g_prof || kind < 0 || kind >= kProfKinds) return;
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return;
  (void)hipEventRecord(e, st);
  g_open[kind] = e;
}

void prof_end(int kind, hipStream_t st, double bytes) {
  if (!g_prof || kind < 0 || kind >= kProfKinds || !g_open[kind]) return;
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return;
  (void)hipEventRecord(e, st);
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof_recs.push_back({kind, g_open[kind], e, bytes});
  g_open[kind] = nullptr;
}

}  // namespace vissm

using namespace vissm;

extern "C" {

const char* vissm_last_error(void) { return vissm::g_err; }
int vissm_version(void) { return 1; }
const char* vissm_source_hash(void) { return VISSM_SRC_HASH; }
const char* vissm_build_flags(void) { return VISSM_BUILD_FLAGS; }

int vissm_normal_base(uint64_t seed, uint64_t offset, float* eps, float* base_lp, int32_t B, int32_t L,
                      int32_t n_last, void* stream) {
  VISSM_CHECK_ARG(B >= 0 && L > 0 && n_last >= 0 && n_last <= L, "normal_base: bad shape B=%d L=%d n_last=%d", B,
                  L, n_last);
  VISSM_CHECK_ARG(eps && base_lp, "normal_base: null pointer");
  if (B == 0) return VISSM_OK;
  prof_begin(VISSM_PROF_NORMAL, as_stream(stream));
  launch_normal(seed, offset, nullptr, eps, base_lp, B, L, n_last, as_stream(stream));
  VISSM_CHECK_LAUNCH("normal_base");
  prof_end(VISSM_PROF_NORMAL, as_stream(stream), 4.0 * B * (static_cast<double>(L) + 1));
  return VISSM_OK;
}

int vissm_normal_base_dev(uint64_t seed, const uint64_t* offset_dev, float* eps, float* base_lp, int32_t B,
                          int32_t L, int32_t n_last, void* stream) {
  VISSM_CHECK_ARG(B >= 0 && L > 0 && n_last >= 0 && n_last <= L, "normal_base_dev: bad shape B=%d L=%d n_last=%d",
                  B, L, n_last);
  VISSM_CHECK_ARG(eps && base_lp && offset_dev, "normal_base_dev: null pointer");
  if (B == 0) return VISSM_OK;
  prof_begin(VISSM_PROF_NORMAL, as_stream(stream));
  launch_normal(seed, 0, offset_dev, eps, base_lp, B, L, n_last, as_stream(stream));
  VISSM_CHECK_LAUNCH("normal_base_dev");
  prof_end(VISSM_PROF_NORMAL, as_stream(stream), 4.0 * B * (static_cast<double>(L) + 1));
  return VISSM_OK;
}

int vissm_base_logprob(const float* eps, float* base_lp, int32_t B, int32_t L, int32_t n_last, void* stream) {
  VISSM_CHECK_ARG(B >= 0 && L > 0 && n_last >= 0 && n_last <= L, "base_logprob: bad shape");
  VISSM_CHECK_ARG(eps && base_lp, "base_logprob: null pointer");
  if (B == 0) return VISSM_OK;
  hipLaunchKernelGGL(base_logprob_kernel, dim3(B), dim3(256), 0, as_stream(stream), eps, base_lp, L, n_last);
  VISSM_CHECK_LAUNCH("base_logprob");
  return VISSM_OK;
}

int vissm_reduce_rows(const float* slab, float* out, int64_t R, int64_t N, void* stream) {
  VISSM_CHECK_ARG(slab && out && R >= 0 && N >= 0, "reduce_rows: bad args");
  return launch_reduce_rows(slab, out, R, N, as_stream(stream));
}

int vissm_reduce_rows_bf16(const void* slab, float* out, int64_t R, int64_t N, void* stream) {
  VISSM_CHECK_ARG(slab && out && R >= 0 && N >= 0, "reduce_rows_bf16: bad args");
  return launch_reduce_rows_bf16(slab, out, R, N, as_stream(stream));
}

int vissm_split_bf16(const float* x, void* hi, void* lo, int64_t n, void* stream) {
  VISSM_CHECK_ARG(n >= 0, "split_bf16: bad size");
  if (n == 0) return VISSM_OK;
  VISSM_CHECK_ARG(x && hi && lo, "split_bf16: null pointer");
  VISSM_CHECK_ARG((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(hi) & 7) == 0 &&
                      (reinterpret_cast<uintptr_t>(lo) & 7) == 0,
                  "split_bf16: x must be 16-byte and hi / lo 8-byte aligned");
  const int64_t n4 = std::max<int64_t>(1, n / 4);
  const unsigned blocks = static_cast<unsigned>(std::min<int64_t>((n4 + 255) / 256, 8192));
  hipLaunchKernelGGL(split_bf16_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), x, static_cast<__bf16*>(hi),
                     static_cast<__bf16*>(lo), n);
  VISSM_CHECK_LAUNCH("split_bf16");
  return VISSM_OK;
}

size_t vissm_adamax_workspace_size(int64_t n) {
  (void)n;
  return align_up(kNormBlocks * sizeof(double)) + align_up(4 * sizeof(float));
}

static int sqnorm_impl(const float* x, int64_t n, float* sq_out, float* norm_out, float* scale_out, float clip,
                       void* ws, size_t ws_bytes, hipStream_t st, int32_t* skip = nullptr,
                       int32_t* skipped = nullptr) {
  VISSM_CHECK_ARG(ws && ws_bytes >= vissm_adamax_workspace_size(n), "workspace too small");
  double* part = reinterpret_cast<double*>(ws);
  int nb = static_cast<int>(std::min<int64_t>(kNormBlocks, std::max<int64_t>(1, (n + 1023) / 1024)));
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(nb), dim3(256), 0, st, x, n, part);
  VISSM_CHECK_LAUNCH("sqnorm_partial");
  hipLaunchKernelGGL(sqnorm_final_kernel, dim3(1), dim3(1024), 0, st, part, nb, sq_out, norm_out, scale_out, clip,
                     skip, skipped);
  VISSM_CHECK_LAUNCH("sqnorm_final");
  return VISSM_OK;
}

int vissm_sqnorm(const float* x, int64_t n, float* out, void* workspace, size_t ws_bytes, void* stream) {
  VISSM_CHECK_ARG(x && out && n >= 0, "sqnorm: bad args");
  return sqnorm_impl(x, n, out, nullptr, nullptr, 0.f, workspace, ws_bytes, as_stream(stream));
}

static int adamax_impl(float* params, const float* grads, float* v, float* m, int64_t n, float lr, float beta1,
                       float beta2, float eps, float clip, float* gnorm_out, bool guard, int32_t* skipped,
                       void* workspace, size_t ws_bytes, hipStream_t st) {
  VISSM_CHECK_ARG(params && grads && v && m && n >= 0, "adamax_step: bad args");
  // workspace: [norm partials (doubles)] [scale, norm scratch, skip flag]
  float* scratch = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + align_up(kNormBlocks * sizeof(double)));
  int32_t* skip = guard ? reinterpret_cast<int32_t*>(scratch + 2) : nullptr;
  int rc = sqnorm_impl(grads, n, nullptr, gnorm_out ? gnorm_out : scratch + 1, scratch, clip, workspace, ws_bytes, st,
                       skip, skipped);
  if (rc) return rc;
  int nb = static_cast<int>(std::min<int64_t>(2048, std::max<int64_t>(1, (n + 255) / 256)));
  hipLaunchKernelGGL(adamax_kernel, dim3(nb), dim3(256), 0, st, params, grads, v, m, n, scratch, lr, beta1, beta2,
                     eps, skip);
  VISSM_CHECK_LAUNCH("adamax");
  return VISSM_OK;
}

int vissm_adamax_step(float* params, const float* grads, float* v, float* m, int64_t n, float lr, float beta1,
                      float beta2, float eps, float clip, float* gnorm_out, void* workspace, size_t ws_bytes,
                      void* stream) {
  return adamax_impl(params, grads, v, m, n, lr, beta1, beta2, eps, clip, gnorm_out, false, nullptr, workspace,
                     ws_bytes, as_stream(stream));
}

int vissm_adamax_step_guarded(float* params, const float* grads, float* v, float* m, int64_t n, float lr,
                              float beta1, float beta2, float eps, float clip, float* gnorm_out, int32_t* skipped,
                              void* workspace, size_t ws_bytes, void* stream) {
  return adamax_impl(params, grads, v, m, n, lr, beta1, beta2, eps, clip, gnorm_out, true, skipped, workspace,
                     ws_bytes, as_stream(stream));
}


void vissm_profile_enable(int32_t on) { vissm::g_prof = on != 0; }

void vissm_profile_reset(void) {
  std::lock_guard<std::mutex> lk(vissm::g_prof_mu);
  for (auto& r : vissm::g_prof_recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  vissm::g_prof_recs.clear();
}

int vissm_profile_read(int32_t kind, double* total_ms, int64_t* count) {
  VISSM_CHECK_ARG(total_ms && count, "profile_read: null pointer");
  std::lock_guard<std::mutex> lk(vissm::g_prof_mu);
  double tot = 0.0;
  int64_t n = 0;
  for (auto& r : vissm::g_prof_recs) {
    if (r.kind != kind) continue;
    if (hipEventSynchronize(r.b) != hipSuccess) {
      set_error("profile_read: event sync failed");
      return VISSM_ELAUNCH;
    }
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, r.a, r.b);
    tot += ms;
    ++n;
  }
  *total_ms = tot;
  *count = n;
  return VISSM_OK;
}

int vissm_profile_bytes(int32_t kind, double* total_bytes) {
  VISSM_CHECK_ARG(total_bytes, "profile_bytes: null pointer");
  std::lock_guard<std::mutex> lk(vissm::g_prof_mu);
  double tot = 0.0;
  for (auto& r : vissm::g_prof_recs)
    if (r.kind == kind) tot += r.bytes;
  *total_bytes = tot;
  return VISSM_OK;
}

}  // extern "C"
