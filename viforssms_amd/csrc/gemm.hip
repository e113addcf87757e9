// Bf16 matrix-core GEMM with fused epilogues (vissm_gemm_bf16): C[m][n] = sum_k A[m][k] B[k][n], bf16 operands, fp32
// accumulation, for the window-shared products of the Lotka-Volterra feature branch (lotka_volterra_partial.py:71-82:
// the 50 -> kernel_ext - 1 time-mixing dense layer and the first conv over its 10,061 output channels, forward and
// backward; lvfeat.hip), where the operands come in both orientations.
//
// Operand layouts (VissmGemmDesc): A row-major (a_kmajor = 0: A[m][k] at a[m lda + k], k contiguous) or K-major
// (a_kmajor = 1: at a[k lda + m]); B "column-major" (b_kmajor = 0: B[k][n] at b[n ldb + k]) or K-major (b_kmajor = 1:
// at b[k ldb + n]).  Rows are read in 16-byte chunks of 8 bf16 (leading dimensions multiples of 8, 16-byte aligned
// pointers; chunks past the matrix edge read as zeros).
//
// Design: a 128 x 128 output tile per 256-thread block, 64 x 64 per wave (4 x 4 v_mfma_f32_16x16x32_bf16 blocks,
// 64 accumulator registers); K in steps of 32 through two LDS buffers (global loads of step k + 1 in flight while step
// k computes; one barrier per step).  An operand whose contiguous dimension is k sits in LDS as [row][k] with 80-byte
// rows (fragment reads: two ds_read_b64 per lane, k = 4g..4g+3 and 16+4g..16+4g+3, conflict-free: the row stride is
// 20 banks); a K-major one as [k][row] with 288-byte rows, read with ds_read_b64_tr_b16 (the same k order; row stride
// 8 banks mod 64).  Epilogues: fp32 store, ELU -> bf16, x elu'(y) of a bf16 ELU output -> bf16.  Split-K
// (gridDim.z > 1) writes per-split fp32 partials that a fixed-order pass sums (deterministic).
//
// Split-bf16 form (vissm_gemm_bf16x3; SV's window-shared conv, SV_dense.py:56-62, and LV's branch at the parity
// precisions, at fp32-class accuracy): the K loop runs over three passes of the K range, (A_hi, B_hi), (A_hi, B_lo),
// (A_lo, B_hi), into the same accumulators; each pass is padded to a whole number of K steps, so a step never
// straddles two passes and split-K divides the 3 K range like any other.  Its bf16 epilogues write the output as a
// hi / lo plane pair (the lo plane M ldc elements after C) and read aux the same way.
#include "common.hpp"

namespace vissm {
namespace gemm {

typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) bf4 lds_bf4;

// K step: 32 (64 halves the barriers but takes 180 VGPRs and 72 KB of LDS, two blocks per CU instead of three: LV-cfg
// step 61.75 -> 62.75 ms, profiles/r06/lvfeat/ab_bk64.log)
#ifndef VISSM_GEMM_BK
#define VISSM_GEMM_BK 32
#endif
// register prefetch depth: 1 = the global loads of step k + 1 are issued while step k computes; 2 = step k + 2 (two
// register sets, +16 VGPRs) measured slower: LV-cfg GEMM time 15.3 -> 16.8 ms per 54 launches, 15.7 at <= 168 VGPRs
// (three blocks per CU) -- the loads' latency is not what holds these tiles (profiles/r06/gemm_pf/)
#ifndef VISSM_GEMM_PF
#define VISSM_GEMM_PF 1
#endif
// blocks per CU the register allocation is held to (3: <= 168 VGPRs)
#ifndef VISSM_GEMM_MINB
#define VISSM_GEMM_MINB 2
#endif
constexpr int BM = 128, BN = 128, BK = VISSM_GEMM_BK, NT = 256;
constexpr int KS = BK / 32;    // MFMA k-steps per K-step
constexpr int CPR = BK / 8;    // 16-byte chunks per [row][k] image row
constexpr int NCH = 128 * BK / 8 / NT;   // staged chunks per thread per operand
constexpr int RP = BK + 8;     // [row][k] image pitch (elements): 80- or 144-byte rows (20 / 36 banks: conflict-free)
constexpr int CP = 128 + 16;   // [k][row] image pitch: 288-byte rows
constexpr int IMG = 128 * RP > BK * CP ? 128 * RP : BK * CP;   // elements per operand image

struct KArgs {
  int64_t M, N, K, lda, ldb, ldc;
  int64_t Kp;        // one pass's K range padded to a multiple of BK (the loop runs over npass Kp)
  int64_t kper;      // range per split of the npass Kp loop (multiple of BK)
  int64_t slab;      // elements between split partials (split-K)
};

__device__ __forceinline__ f4 mfma32(bf8 a, bf8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ bf8 cat8(bf4 a, bf4 b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7); }

// 16-byte chunk (8 bf16) of a matrix whose rows of `ld` elements are contiguous: row r, columns c .. c + 7 (zeros past
// the edge: r >= nr or c >= nc; nc is a multiple of 8 or the chunk is read element-wise)
__device__ __forceinline__ u4v ld_chunk(const __bf16* __restrict__ p, int64_t ld, int64_t r, int64_t c, int64_t nr,
                                        int64_t nc) {
  if (r >= nr || c >= nc) return u4v{0u, 0u, 0u, 0u};
  const __bf16* q = p + r * ld + c;
  if (c + 8 <= nc) return *reinterpret_cast<const u4v*>(q);
  bf8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = c + j < nc ? q[j] : static_cast<__bf16>(0.f);
  return __builtin_bit_cast(u4v, v);
}

// the staging of one operand: two 16-byte chunks per thread per K-step
//   KM = false: rows r0 .. r0 + 127 of a [rows][k] matrix (k contiguous): chunk q -> row q >> 2, k (q & 3) 8
//   KM = true:  a [k][rows] matrix (rows contiguous): chunk q -> k q >> 4, row (q & 15) 8
template <bool KM>
struct Stage {
  u4v v[NCH];
  __device__ __forceinline__ void load(const __bf16* __restrict__ p, int64_t ld, int64_t r0, int64_t k0, int64_t nrows,
                                       int64_t kend) {
    if (r0 + 128 <= nrows && k0 + BK <= kend) {   // interior tile (block-uniform): no edge checks
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int q = threadIdx.x + NT * i;
        if constexpr (!KM) v[i] = *reinterpret_cast<const u4v*>(p + (r0 + q / CPR) * ld + k0 + (q % CPR) * 8);
        else v[i] = *reinterpret_cast<const u4v*>(p + (k0 + (q >> 4)) * ld + r0 + (q & 15) * 8);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int q = threadIdx.x + NT * i;
      if constexpr (!KM) v[i] = ld_chunk(p, ld, r0 + q / CPR, k0 + (q % CPR) * 8, nrows, kend);
      else v[i] = ld_chunk(p, ld, k0 + (q >> 4), r0 + (q & 15) * 8, kend, nrows);
    }
  }
  __device__ __forceinline__ void store(__bf16* img) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int q = threadIdx.x + NT * i;
      if constexpr (!KM) *reinterpret_cast<u4v*>(img + (q / CPR) * RP + (q % CPR) * 8) = v[i];
      else *reinterpret_cast<u4v*>(img + (q >> 4) * CP + (q & 15) * 8) = v[i];
    }
  }
};

// K = 32 fragment of rows rb .. rb + 15 of the tile: lane (g, c) gets row rb + c, k = 4g + jj and 16 + 4g + jj
template <bool KM>
__device__ __forceinline__ bf8 frag(const __bf16* img, int rb, int g, int c, int ks = 0) {
  if constexpr (!KM) {
    const __bf16* p = img + (rb + c) * RP + 32 * ks + 4 * g;
    return cat8(*reinterpret_cast<const bf4*>(p), *reinterpret_cast<const bf4*>(p + 16));
  } else {
    const __bf16* p = img + (32 * ks + 4 * g + (c >> 2)) * CP + rb + 4 * (c & 3);
    return cat8(__builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf4*)p),
                __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf4*)(p + 16 * CP)));
  }
}

__device__ __forceinline__ float elu_acc(float x) { return x > 0.f ? x : expm1f(x); }

// EPI: 0 fp32 store (split-K: partial z at C + z slab), 1 ELU -> bf16, 2 x elu'(aux) -> bf16 (aux: bf16 ELU output,
// same layout as C)
// X3: the split-bf16 form (A2 / B2 the lo planes; passes above)
template <bool AKM, bool BKM, int EPI, bool X3 = false>
__global__ __launch_bounds__(NT, VISSM_GEMM_MINB) void gemm_kernel(KArgs a, const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                     void* __restrict__ Cv, const __bf16* __restrict__ aux,
                                                     const __bf16* __restrict__ A2 = nullptr,
                                                     const __bf16* __restrict__ B2 = nullptr) {
  // the two operands' double buffers in one array (the bf16 epilogue stages its 4 x 8.5 KB through all of it)
  __shared__ __attribute__((aligned(16))) __bf16 smem[4][IMG];
  __bf16(*sa)[IMG] = smem;
  __bf16(*sb)[IMG] = smem + 2;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int wm = w >> 1, wn = w & 1;
  // XCD-aware tile order: the dispatcher deals a grid's blocks round-robin over the 8 XCDs (each with its own L2), so
  // consecutive block ids land on different L2s; renumbering them so that each XCD runs a contiguous run of tiles (all
  // n-tiles of an m-tile together) lets the n-tiles sharing an A tile read it through one L2 instead of eight
  int mt, nt;
  {
    const int nbx = gridDim.x, total = gridDim.x * gridDim.y;
    const int b = blockIdx.y * nbx + blockIdx.x, x = b & 7, i = b >> 3;
    const int per = total >> 3, rem = total & 7;
    const int t = x * per + min(x, rem) + i;
    mt = t / nbx;
    nt = t - mt * nbx;
  }
  const int64_t m0 = static_cast<int64_t>(mt) * BM, n0 = static_cast<int64_t>(nt) * BN;
  const int64_t kb = static_cast<int64_t>(blockIdx.z) * a.kper;
  const int64_t ke = min(X3 ? 3 * a.Kp : a.K, kb + a.kper);
  // K step at loop position kk: its pass's operands and its k within the pass (X3; block-uniform)
  auto load = [&](Stage<AKM>& la, Stage<BKM>& lb, int64_t kk) {
    if constexpr (X3) {
      const int pass = static_cast<int>(kk / a.Kp);
      const int64_t k0 = kk - pass * a.Kp;
      la.load(pass == 2 ? A2 : A, a.lda, m0, k0, a.M, a.K);
      lb.load(pass == 1 ? B2 : B, a.ldb, n0, k0, a.N, a.K);
    } else {
      la.load(A, a.lda, m0, kk, a.M, ke);
      lb.load(B, a.ldb, n0, kk, a.N, ke);
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int nk = static_cast<int>((ke - kb + BK - 1) / BK);
  auto compute = [&](int cur) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<AKM>(sa[cur], wm * 64 + 16 * i, g, c, ks);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BKM>(sb[cur], wn * 64 + 16 * j, g, c, ks);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma32(af[i], bfr[j], acc[i][j]);
    }
  };
  Stage<AKM> la;
  Stage<BKM> lb;
  if (nk > 0) {
    load(la, lb, kb);
    la.store(sa[0]);
    lb.store(sb[0]);
  }
#if VISSM_GEMM_PF >= 2
  Stage<AKM> la1;
  Stage<BKM> lb1;
  if (nk > 1) load(la1, lb1, kb + BK);
  __syncthreads();
  // step kt: (ra, rb) held step kt (in LDS by now) and take the loads of step kt + 2; (qa, qb) hold step kt + 1,
  // stored into the other LDS buffer after the compute; the two register sets swap roles every step
  auto step = [&](int kt, Stage<AKM>& ra, Stage<BKM>& rb, Stage<AKM>& qa, Stage<BKM>& qb) {
    const int cur = kt & 1;
    if (kt + 2 < nk) load(ra, rb, kb + static_cast<int64_t>(kt + 2) * BK);
    compute(cur);
    if (kt + 1 < nk) {
      qa.store(sa[cur ^ 1]);
      qb.store(sb[cur ^ 1]);
    }
    __syncthreads();
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, la, lb, la1, lb1);
    step(kt + 1, la1, lb1, la, lb);
  }
  if (kt < nk) step(kt, la, lb, la1, lb1);
#else
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) load(la, lb, kb + static_cast<int64_t>(kt + 1) * BK);
    compute(cur);
    if (more) {
      la.store(sa[cur ^ 1]);
      lb.store(sb[cur ^ 1]);
    }
    __syncthreads();
  }
#endif
  // epilogue: lane (g, c) of block (i, j) holds C[m = base_m + 16 i + 4 g + r][n = base_n + 16 j + c]
  if constexpr (EPI != 0) {
    // bf16 outputs through LDS (the operand buffers are free after the loop's last barrier): each wave writes its
    // 64 x 64 fp32 tile in two 32-row halves into its own [32][64 + 4] region, then stores 8 consecutive columns per
    // lane (16-byte stores; the elu' epilogue reads its aux chunk the same way) instead of scattered 2-byte stores
    static_assert(4 * 32 * 68 * 4 <= 4 * IMG * 2, "epilogue staging exceeds the operand buffers");
    float* stg = reinterpret_cast<float*>(&smem[0][0]) + w * (32 * 68);   // 4 waves x 8.5 KB
    const int64_t bm = m0 + wm * 64, bn = n0 + wn * 64;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) stg[(16 * ii + 4 * g + r) * 68 + 16 * j + c] = acc[2 * half + ii][j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // lane l: rows (l >> 3) + 8 t (t = 0..3) of the half, columns 8 (l & 7) .. + 7
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int rr = (lane >> 3) + 8 * t, cc = 8 * (lane & 7);
        const int64_t m = bm + 32 * half + rr, n = bn + cc;
        if (m >= a.M || n >= a.N) continue;
        float x[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = stg[rr * 68 + cc + e];
        __bf16* dst = reinterpret_cast<__bf16*>(Cv) + m * a.ldc + n;
        const bool full = n + 8 <= a.N && ((m * a.ldc + n) & 7) == 0;
        // X3: the output and aux are hi / lo plane pairs, the lo plane M ldc elements after the hi one
        const int64_t plane = a.M * a.ldc;
        auto ld8 = [&](const __bf16* src) {
          bf8 y;
          if (full) y = *reinterpret_cast<const bf8*>(src);
          else
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = n + e < a.N ? src[e] : static_cast<__bf16>(0.f);
          return y;
        };
        auto st8 = [&](__bf16* q, bf8 o) {
          if (full) *reinterpret_cast<bf8*>(q) = o;
          else
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (n + e < a.N) q[e] = o[e];
        };
        float v[8];
        if constexpr (EPI == 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = elu_acc(x[e]);
        } else {
          const __bf16* src = aux + m * a.ldc + n;
          const bf8 y = ld8(src);
          bf8 yl;
          if constexpr (X3) yl = ld8(src + plane);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float yv = static_cast<float>(y[e]);
            if constexpr (X3) yv += static_cast<float>(yl[e]);
            v[e] = yv < 0.f ? x[e] * (yv + 1.f) : x[e];
          }
        }
        bf8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = static_cast<__bf16>(v[e]);
        st8(dst, o);
        if constexpr (X3) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = static_cast<__bf16>(v[e] - static_cast<float>(o[e]));
          st8(dst + plane, o);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + 16 * j + c;
      if (n >= a.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 64 + 16 * i + 4 * g + r;
        if (m >= a.M) continue;
        const float x = acc[i][j][r];
        if constexpr (EPI == 0) {
          reinterpret_cast<float*>(Cv)[static_cast<int64_t>(blockIdx.z) * a.slab + m * a.ldc + n] = x;
        } else if constexpr (EPI == 1) {
          reinterpret_cast<__bf16*>(Cv)[m * a.ldc + n] = static_cast<__bf16>(elu_acc(x));
        } else {
          const float y = static_cast<float>(aux[m * a.ldc + n]);
          reinterpret_cast<__bf16*>(Cv)[m * a.ldc + n] = static_cast<__bf16>(y < 0.f ? x * (y + 1.f) : x);
        }
      }
    }
}

}  // namespace gemm
}  // namespace vissm

using namespace vissm;
using namespace vissm::gemm;

// shared argument checks and launch of both entry points (x3: the split-bf16 form, fp32 epilogue)
static int gemm_launch(const VissmGemmDesc* d, const void* A, const void* A2, const void* B, const void* B2, void* C,
                       const void* aux, void* workspace, size_t ws_bytes, void* stream, bool x3) {
  const char* nm = x3 ? "gemm_bf16x3" : "gemm_bf16";
  VISSM_CHECK_ARG(d && A && B && C && (!x3 || (A2 && B2)), "%s: null argument", nm);
  VISSM_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0, "%s: negative size", nm);
  if (d->M == 0 || d->N == 0) return VISSM_OK;
  VISSM_CHECK_ARG(d->lda % 8 == 0 && d->ldb % 8 == 0, "%s: leading dimensions must be multiples of 8", nm);
  VISSM_CHECK_ARG(((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B) | reinterpret_cast<uintptr_t>(A2) |
                    reinterpret_cast<uintptr_t>(B2)) & 15) == 0,
                  "%s: operands must be 16-byte aligned", nm);
  VISSM_CHECK_ARG(d->lda >= (d->a_kmajor ? d->M : d->K) && d->ldb >= (d->b_kmajor ? d->N : d->K),
                  "%s: leading dimension below the row length", nm);
  VISSM_CHECK_ARG(d->ldc >= d->N, "%s: ldc < N", nm);
  VISSM_CHECK_ARG(d->epilogue >= VISSM_GEMM_F32 && d->epilogue <= VISSM_GEMM_DELU_BF16, "%s: epilogue", nm);
  VISSM_CHECK_ARG(d->epilogue != VISSM_GEMM_DELU_BF16 || aux, "%s: the elu' epilogue needs aux", nm);
  const int split = d->split_k > 1 ? d->split_k : 1;
  VISSM_CHECK_ARG(split == 1 || (d->epilogue == VISSM_GEMM_F32 && d->ldc == d->N),
                  "%s: split-K needs the fp32 epilogue and ldc == N", nm);
  VISSM_CHECK_ARG(split == 1 || (workspace && ws_bytes >= vissm_gemm_workspace_size(d)), "%s: workspace too small", nm);
  hipStream_t st = as_stream(stream);
  KArgs a;
  a.M = d->M; a.N = d->N; a.K = d->K; a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.Kp = (d->K + BK - 1) / BK * BK;
  const int64_t krange = x3 ? 3 * a.Kp : d->K;
  a.kper = ((krange + split - 1) / split + BK - 1) / BK * BK;
  if (a.kper <= 0) a.kper = BK;
  a.slab = d->M * d->N;
  const int nz = static_cast<int>((krange + a.kper - 1) / a.kper) > 0 ? static_cast<int>((krange + a.kper - 1) / a.kper) : 1;
  dim3 grid(static_cast<unsigned>((d->N + BN - 1) / BN), static_cast<unsigned>((d->M + BM - 1) / BM),
            static_cast<unsigned>(split == 1 ? 1 : nz));
  void* out = split == 1 ? C : workspace;
  const __bf16* pa = static_cast<const __bf16*>(A);
  const __bf16* pb = static_cast<const __bf16*>(B);
  const __bf16* pa2 = static_cast<const __bf16*>(A2);
  const __bf16* pb2 = static_cast<const __bf16*>(B2);
  const __bf16* px = static_cast<const __bf16*>(aux);
#define GEMM_EPI(AK, BKk)                                                                                      \
  do {                                                                                                       \
    if (x3 && d->epilogue == VISSM_GEMM_F32) hipLaunchKernelGGL((gemm_kernel<AK, BKk, 0, true>), grid, dim3(NT), 0, st, a, pa, pb, out, px, pa2, pb2); \
    else if (x3 && d->epilogue == VISSM_GEMM_ELU_BF16) hipLaunchKernelGGL((gemm_kernel<AK, BKk, 1, true>), grid, dim3(NT), 0, st, a, pa, pb, out, px, pa2, pb2); \
    else if (x3) hipLaunchKernelGGL((gemm_kernel<AK, BKk, 2, true>), grid, dim3(NT), 0, st, a, pa, pb, out, px, pa2, pb2); \
    else if (d->epilogue == VISSM_GEMM_F32) hipLaunchKernelGGL((gemm_kernel<AK, BKk, 0>), grid, dim3(NT), 0, st, a, pa, pb, out, px, pa2, pb2); \
    else if (d->epilogue == VISSM_GEMM_ELU_BF16) hipLaunchKernelGGL((gemm_kernel<AK, BKk, 1>), grid, dim3(NT), 0, st, a, pa, pb, out, px, pa2, pb2); \
    else hipLaunchKernelGGL((gemm_kernel<AK, BKk, 2>), grid, dim3(NT), 0, st, a, pa, pb, out, px, pa2, pb2);   \
  } while (0)
  if (d->a_kmajor) {
    if (d->b_kmajor) GEMM_EPI(true, true);
    else GEMM_EPI(true, false);
  } else {
    if (d->b_kmajor) GEMM_EPI(false, true);
    else GEMM_EPI(false, false);
  }
#undef GEMM_EPI
  VISSM_CHECK_LAUNCH(nm);
  if (split > 1) return launch_reduce_rows(static_cast<const float*>(workspace), static_cast<float*>(C), grid.z, d->M * d->N, st);
  return VISSM_OK;
}

extern "C" {

size_t vissm_gemm_workspace_size(const VissmGemmDesc* d) {
  if (!d || d->split_k <= 1) return 0;
  return align_up(static_cast<size_t>(d->split_k) * d->M * d->N * sizeof(float));
}

int vissm_gemm_bf16(const VissmGemmDesc* d, const void* A, const void* B, void* C, const void* aux, void* workspace,
                    size_t ws_bytes, void* stream) {
  return gemm_launch(d, A, nullptr, B, nullptr, C, aux, workspace, ws_bytes, stream, false);
}

size_t vissm_gemm_bf16x3_workspace_size(const VissmGemmDesc* d) { return vissm_gemm_workspace_size(d); }

int vissm_gemm_bf16x3(const VissmGemmDesc* d, const void* A_hi, const void* A_lo, const void* B_hi, const void* B_lo,
                      void* C, const void* aux, void* workspace, size_t ws_bytes, void* stream) {
  return gemm_launch(d, A_hi, A_lo, B_hi, B_lo, C, aux, workspace, ws_bytes, stream, true);
}

}  // extern "C"
