// IAF flow of the neural-MA sampler on the bf16 matrix cores
// (v_mfma_f32_16x16x32_bf16, fp32 accumulation): forward and backward.
//
// Precision: VISSM_PREC_BF16 (one product per MFMA: bf16 operands) or
// VISSM_PREC_BF16X3 (split operands a = a_hi + a_lo, three products
// a_hi b_hi + a_hi b_lo + a_lo b_hi: ~2^-16 relative per product).
//
// Reference: IAF._create_flow / IAF.slp (AR.py:50-89), stride-2 head
// (lotka_volterra_partial.py:97-104), Permute fused into the store (swap_out).
//
// Design (wave-centric, no block barriers on the step path):
//   * a work unit = one (sample, tile of P = 32 head positions) is processed by
//     ONE wave; a block's 4 waves run independent work items and share only the
//     weight fragments staged in LDS once per block;
//   * activations are MFMA accumulators X[rb][cb] (lane (g, c) holds rows
//     h = 16 rb + 4 g + r, column p = 16 cb + c).  Products that contract over h
//     (forward layers, head, dX = W dZ, dcon = w_eps dA0) take the accumulators
//     directly as the B operand: k-step ks packs rows 32 ks + 16 (j >> 2) + 4 g
//     + (j & 3) of the lane's own registers, and the weight fragments in LDS are
//     pre-permuted to the same k order (hperm below) -- no LDS round trip, no
//     lane movement;
//   * products that contract over positions (dW = X dZ^T, dW_eps = U dA0^T,
//     d theta = dA0 1) need h on the lane: the wave writes the bf16 tile into a
//     private swizzled [p][h] LDS image (8-byte stores) and reads it back
//     transposed with ds_read_b64_tr_b16;
//   * bias gradients come free from a row of ones in the padded activations
//     (row 63 of X_l: W is zero there, so the forward is unchanged and
//     dW[63][:] accumulates sum_p dZ);
//   * grid decomposition, carries, halo and fixed-order partial slabs are those
//     of flow_v4.hip (sample groups x t-chunks; backward walks tiles outer /
//     samples inner so the window-shared dC tile is summed over the group in
//     registers).
// Supported here: n_hidden <= 1 without BN, H <= 63, k <= 64 (the AR
// configurations); other shapes are served by flow_v4 (fp32).
#include "common.hpp"

namespace vissm {
namespace flow5 {

constexpr int P = 32;
constexpr int HP = 64;
constexpr int S = 16;
constexpr int NW = 4;
constexpr int NT = 64 * NW;

typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf4 lds_bf4;

template <int NP>
struct Fr {
  bf8 h, l;  // l used only when NP == 3
};

__device__ __forceinline__ f4 mfma(bf8 a, bf8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int NP>
__device__ __forceinline__ f4 mm(const Fr<NP>& a, const Fr<NP>& b, f4 c) {
  if constexpr (NP == 3) {
    c = mfma(a.l, b.h, c);
    c = mfma(a.h, b.l, c);
  }
  return mfma(a.h, b.h, c);
}

// b exact in bf16 (ones)
template <int NP>
__device__ __forceinline__ f4 mm_bexact(const Fr<NP>& a, bf8 b, f4 c) {
  if constexpr (NP == 3) c = mfma(a.l, b, c);
  return mfma(a.h, b, c);
}

template <int NP>
__device__ __forceinline__ Fr<NP> split8(const float (&v)[8]) {
  Fr<NP> f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)v[j];
    f.h[j] = h;
    if constexpr (NP == 3) f.l[j] = (__bf16)(v[j] - (float)h);
  }
  return f;
}

// chain B fragment: k-step ks of activations X (rows 32ks .. 32ks+31), column block cb
template <int NP>
__device__ __forceinline__ Fr<NP> chain_frag(const f4 (&X)[4][2], int ks, int cb) {
  float v[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = X[2 * ks][cb][j];
    v[4 + j] = X[2 * ks + 1][cb][j];
  }
  return split8<NP>(v);
}

// hidden row of element j of k-step ks in lane group g (the chain k order)
__host__ __device__ __forceinline__ int hperm(int ks, int g, int j) {
  return 32 * ks + 16 * (j >> 2) + 4 * g + (j & 3);
}

// ---------------------------------------------------------------------------
// weight fragments: [frag][plane (hi, lo)][lane] of 8 bf16, index layout
//   WF(l, ob, ks)  l*8 + ob*2 + ks             forward hidden   A[h_out][h_in perm]
//   WB(l, ib, ks)  8*NH + l*8 + ib*2 + ks      dX = W dZ        A[h_in][h_out perm]
//   WE(kb, ob)     16*NH + kb*4 + ob           layer 0          A[h][j]
//   WC(jb, ks)     16*NH + 4*KB + jb*2 + ks    dcon             A[j][h perm]
//   WH(ks)         16*NH + 4*KB + 2*JB + ks    head             A[o][h perm]
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int n_frags(int NH, int KB, int JB) { return 16 * NH + 4 * KB + 2 * JB + 2; }

struct KArgs {
  int B, L, k, H, s, swap_out, n_logsig, Lout, Lh, CH, n_chunks, S, n_groups, n_items;
};

__global__ void prep_kernel(VissmFlowParams w, int H, int k, int nh, int NP, int KB, int JB, bf8* __restrict__ img,
                            float* __restrict__ cst) {
  const int f = blockIdx.x, lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const int NPL = NP == 3 ? 2 : 1;
  float v[8];
  for (int j = 0; j < 8; ++j) {
    float x = 0.f;
    int r = f;
    if (r < 8 * nh) {  // WF
      const int l = r >> 3, ob = (r >> 1) & 3, ks = r & 1;
      const int hin = hperm(ks, g, j), hout = 16 * ob + c;
      if (hin < H && hout < H) x = w.w_hid[(static_cast<size_t>(l) * H + hin) * H + hout];
    } else if ((r -= 8 * nh) < 8 * nh) {  // WB
      const int l = r >> 3, ib = (r >> 1) & 3, ks = r & 1;
      const int hin = 16 * ib + c, hout = hperm(ks, g, j);
      if (hin < H && hout < H) x = w.w_hid[(static_cast<size_t>(l) * H + hin) * H + hout];
    } else if ((r -= 8 * nh) < 4 * KB) {  // WE
      const int kb = r >> 2, ob = r & 3;
      const int jt = 32 * kb + 8 * g + j, h = 16 * ob + c;
      if (jt < k && h < H) x = w.w_eps[jt * H + h];
    } else if ((r -= 4 * KB) < 2 * JB) {  // WC
      const int jb = r >> 1, ks = r & 1;
      const int jt = 16 * jb + c, h = hperm(ks, g, j);
      if (jt < k && h < H) x = w.w_eps[jt * H + h];
    } else {  // WH
      const int ks = r - 2 * JB;
      const int h = hperm(ks, g, j);
      if (c < 2 && h < H) x = w.w_head[h * 2 + c];
    }
    v[j] = x;
  }
  bf8 hi, lo;
  for (int j = 0; j < 8; ++j) {
    hi[j] = (__bf16)v[j];
    lo[j] = (__bf16)(v[j] - (float)hi[j]);
  }
  img[(f * NPL + 0) * 64 + lane] = hi;
  if (NPL == 2) img[(f * NPL + 1) * 64 + lane] = lo;
  if (f == 0) {
    // constants: bias[nh][64], w_head[2][64], b_head[2]
    for (int l = 0; l < nh; ++l) cst[l * HP + lane] = lane < H ? w.b_hid[l * H + lane] : 0.f;
    cst[nh * HP + lane] = lane < H ? w.w_head[lane * 2 + 0] : 0.f;
    cst[nh * HP + HP + lane] = lane < H ? w.w_head[lane * 2 + 1] : 0.f;
    if (lane < 2) cst[nh * HP + 2 * HP + lane] = w.b_head[lane];
  }
}

// ---------------------------------------------------------------------------
// per-block LDS
// ---------------------------------------------------------------------------
template <int NH, int KB, int JB, int NP>
struct Shared {
  static constexpr int NFR = n_frags(NH, KB, JB);
  static constexpr int NPL = NP == 3 ? 2 : 1;
  bf8 img[NFR][NPL][64];
  float cst[(NH + 2) * HP + 4];
};

// transposed-image addressing: [p][h] bf16, 16 chunks of 4 per 128-byte row, chunk XOR (row & 15)
__device__ __forceinline__ int timg_off(int p, int ch) { return p * HP + 4 * (ch ^ (p & 15)); }

template <int NP>
struct Img {
  __bf16* plane[NP == 3 ? 2 : 1];
};

// store a [64 h][32 p] activation tile (normal accumulator layout) into a transposed image
template <int NP>
__device__ __forceinline__ void put_image(__bf16* hi, __bf16* lo, const f4 (&X)[4][2], int g, int c) {
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      bf4 h4, l4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const __bf16 hh = (__bf16)X[rb][cb][r];
        h4[r] = hh;
        if constexpr (NP == 3) l4[r] = (__bf16)(X[rb][cb][r] - (float)hh);
      }
      const int off = timg_off(16 * cb + c, 4 * rb + g);
      *reinterpret_cast<bf4*>(hi + off) = h4;
      if constexpr (NP == 3) *reinterpret_cast<bf4*>(lo + off) = l4;
    }
}

// a lane's own entries of an image it wrote (normal layout), as fp32 (hi + lo)
template <int NP>
__device__ __forceinline__ f4 get_own(const __bf16* hi, const __bf16* lo, int rb, int cb, int g, int c) {
  const int off = timg_off(16 * cb + c, 4 * rb + g);
  const bf4 h4 = *reinterpret_cast<const bf4*>(hi + off);
  f4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = (float)h4[i];
  if constexpr (NP == 3) {
    const bf4 l4 = *reinterpret_cast<const bf4*>(lo + off);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] += (float)l4[i];
  }
  return r;
}

__device__ __forceinline__ bf8 tr_read(const __bf16* img, int hb, int g, int c) {
  const int q = c >> 2, pp = c & 3;
  const int r0 = 8 * g + q, r1 = 8 * g + 4 + q;
  const int ch = 4 * hb + pp;
  bf4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf4*)(img + timg_off(r0, ch)));
  bf4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf4*)(img + timg_off(r1, ch)));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int NP>
__device__ __forceinline__ Fr<NP> tr_frag(const __bf16* hi, const __bf16* lo, int hb, int g, int c) {
  Fr<NP> f;
  f.h = tr_read(hi, hb, g, c);
  if constexpr (NP == 3) f.l = tr_read(lo, hb, g, c);
  return f;
}

// Compiler-only fence: the weight fragments are loop-invariant LDS loads; without it the
// compiler hoists all of them out of the unit loop and keeps ~100-200 VGPRs live.
__device__ __forceinline__ void fence() { asm volatile("" ::: "memory"); }

template <int NH, int KB, int JB, int NP>
__device__ __forceinline__ Fr<NP> wfrag(const Shared<NH, KB, JB, NP>& sh, int f, int lane) {
  Fr<NP> r;
  r.h = sh.img[f][0][lane];
  if constexpr (NP == 3) r.l = sh.img[f][1][lane];
  return r;
}

template <int NH, int KB, int JB, int NP>
__device__ __forceinline__ void load_shared(Shared<NH, KB, JB, NP>& sh, const bf8* __restrict__ img,
                                            const float* __restrict__ cst) {
  constexpr int N = Shared<NH, KB, JB, NP>::NFR * Shared<NH, KB, JB, NP>::NPL * 64;
  for (int i = threadIdx.x; i < N; i += NT) (&sh.img[0][0][0])[i] = img[i];
  for (int i = threadIdx.x; i < (NH + 2) * HP + 4; i += NT) sh.cst[i] = cst[i];
}

__device__ __forceinline__ float ld_guard(const float* __restrict__ p, int i, int n) { return i < n ? p[i] : 0.f; }

// layer-0 B fragment: U[j = 32 kb + 8 g + jj][p = 16 cb + c] = u[t0 + s p + j]
template <int NP>
__device__ __forceinline__ Fr<NP> u_frag(const float* __restrict__ ub, int L, int k, int t0, int s, int kb, int cb,
                                         int g, int c) {
  float v[8];
  const int j0 = 32 * kb + 8 * g;
  const int base = t0 + s * (16 * cb + c) + j0;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) v[jj] = (j0 + jj < k) ? ld_guard(ub, base + jj, L) : 0.f;
  return split8<NP>(v);
}

// dW_eps A fragment: U[j = 16 jb + c][p = 8 g + jj] = u[t0 + s p + j]
template <int NP>
__device__ __forceinline__ Fr<NP> ua_frag(const float* __restrict__ ub, int L, int k, int t0, int s, int jb, int nP,
                                          int g, int c) {
  float v[8];
  const int j = 16 * jb + c;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int p = 8 * g + jj;
    v[jj] = (j < k && p < nP) ? ld_guard(ub, t0 + s * p + j, L) : 0.f;
  }
  return split8<NP>(v);
}

// forward of one unit; on return X[l] (l = 0..NH) hold the layer outputs (row 63 of X[l < NH]
// set to 1 for the bias-gradient trick) and mu/r the head outputs of this lane's columns.
template <int NH, int KB, int JB, int NP>
__device__ __forceinline__ void unit_forward(const KArgs& a, const Shared<NH, KB, JB, NP>& sh,
                                             const float* __restrict__ ub, const float* __restrict__ Cw,
                                             const float* __restrict__ thb, int m0, int nP, int t0,
                                             f4 (&X)[NH + 1][4][2], float (&mu)[2], float (&rr)[2]) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  // accumulator init: C^T + theta term
  float th[4][4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 16 * rb + 4 * g + r;
      th[rb][r] = h < a.H ? thb[h] : 0.f;
    }
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int p = 16 * cb + c;
    const bool pv = p < nP;
    const float* crow = Cw + static_cast<size_t>(m0 + p) * a.H;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * rb + 4 * g + r;
        X[0][rb][cb][r] = (pv && h < a.H) ? crow[h] + th[rb][r] : 0.f;
      }
  }
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const Fr<NP> uf = u_frag<NP>(ub, a.L, a.k, t0, a.s, kb, cb, g, c);
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) X[0][ob][cb] = mm<NP>(wfrag(sh, 16 * NH + kb * 4 + ob, lane), uf, X[0][ob][cb]);
    }
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) X[0][rb][cb][r] = elu_f(X[0][rb][cb][r]);
#pragma unroll
  for (int l = 0; l < NH; ++l) {
    fence();
    f4 Z[4][2];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) {
      const f4 bv = *reinterpret_cast<const f4*>(&sh.cst[l * HP + 16 * ob + 4 * g]);
      Z[ob][0] = bv;
      Z[ob][1] = bv;
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const Fr<NP> xf = chain_frag<NP>(X[l], ks, cb);
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) Z[ob][cb] = mm<NP>(wfrag(sh, l * 8 + ob * 2 + ks, lane), xf, Z[ob][cb]);
      }
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) X[l + 1][rb][cb][r] = elu_f(Z[rb][cb][r]);
  }
  // head (16 output rows, o = 0: mu, o = 1: sigma pre-softplus)
  fence();
  const int fh = 16 * NH + 4 * KB + 2 * JB;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    f4 d = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) d = mm<NP>(wfrag(sh, fh + ks, lane), chain_frag<NP>(X[NH], ks, cb), d);
    mu[cb] = __shfl(d[0], c, 64) + sh.cst[NH * HP + 2 * HP + 0];
    rr[cb] = __shfl(d[1], c, 64) + sh.cst[NH * HP + 2 * HP + 1];
  }
}

// ---------------------------------------------------------------------------
// forward kernel: one work item (sample group x t-chunk) per wave; samples outer
// ---------------------------------------------------------------------------
template <int NH, int KB, int JB, int NP>
__global__ __launch_bounds__(NT, 2) void fwd_kernel(KArgs a, const float* __restrict__ u, const float* __restrict__ C,
                                                    const int32_t* __restrict__ win, const float* __restrict__ tht,
                                                    const bf8* __restrict__ img, const float* __restrict__ cst,
                                                    float* __restrict__ u_next, float* __restrict__ ls_slab) {
  __shared__ Shared<NH, KB, JB, NP> sh;
  load_shared(sh, img, cst);
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int item = blockIdx.x * NW + w;
  if (item >= a.n_items) return;
  const int grp = item / a.n_chunks, ch = item % a.n_chunks;
  const int m_lo = ch * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int b_lo = grp * a.S, nb = min(a.S, a.B - b_lo);
  for (int bl = 0; bl < nb; ++bl) {
    const int b = b_lo + bl;
    const float* ub = u + static_cast<size_t>(b) * a.L;
    float* ob = u_next + static_cast<size_t>(b) * a.Lout;
    const int wi = win ? win[b] : 0;
    const float* Cw = C + static_cast<size_t>(wi) * a.Lh * a.H;
    float ls = 0.f;
    for (int m0 = m_lo; m0 < m_hi; m0 += P) {
      fence();
      const int nP = min(P, m_hi - m0), t0 = a.s * m0;
      f4 X[NH + 1][4][2];
      float mu[2], rr[2];
      unit_forward<NH, KB, JB, NP>(a, sh, ub, Cw, tht + static_cast<size_t>(b) * a.H, m0, nP, t0, X, mu, rr);
      if (g == 0) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const int p = 16 * cb + c;
          if (p < nP) {
            const float sg = softplus_f(rr[cb]) + 1e-10f;
            const int o = t0 + a.s * p + (a.s - 1);
            ob[a.swap_out ? (o ^ 1) : o] = ub[o + a.k] * sg + mu[cb];
            if (a.s == 2) {
              const int oe = t0 + 2 * p;
              ob[a.swap_out ? (oe ^ 1) : oe] = ub[oe + a.k];
            }
            if (o >= a.Lout - a.n_logsig) ls += logf(sg);
          }
        }
      }
    }
    const float v = wave_sum(ls);
    if (lane == 0) ls_slab[static_cast<size_t>(ch) * a.B + b] = v;
  }
}

// ---------------------------------------------------------------------------
// backward kernel: one work item per wave; tiles outer, samples inner
// ---------------------------------------------------------------------------
template <int NH, int KB, int JB, int NP>
__global__ __launch_bounds__(NT, 1) void bwd_kernel(KArgs a, const float* __restrict__ u, const float* __restrict__ C,
                                                    const int32_t* __restrict__ win, const float* __restrict__ tht,
                                                    const float* __restrict__ gout, const float* __restrict__ dls,
                                                    const bf8* __restrict__ img, const float* __restrict__ cst,
                                                    float* __restrict__ du, float* __restrict__ dC_slab,
                                                    float* __restrict__ dth_slab, float* __restrict__ dW_slab,
                                                    float* __restrict__ halo) {
  static_assert(NH == 1, "flow5 backward: one hidden layer");
  constexpr int NPL = NP == 3 ? 2 : 1;
  constexpr int KP = 16 * JB;  // carry slots (k <= KP)
  __shared__ Shared<NH, KB, JB, NP> sh;
  __shared__ __bf16 timg[NW][2][NPL][P * HP];  // [wave][slot][plane][p][h]
  __shared__ float dthl[NW][S][HP];
  __shared__ float carry[NW][S][KP];
  __shared__ float gsc[NW][4][P];              // go (= d mu), sigma, go (even, stride 2), d r
  load_shared(sh, img, cst);
  for (int i = threadIdx.x; i < NW * S * HP; i += NT) (&dthl[0][0][0])[i] = 0.f;
  for (int i = threadIdx.x; i < NW * S * KP; i += NT) (&carry[0][0][0])[i] = 0.f;
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int item = blockIdx.x * NW + w;
  if (item >= a.n_items) return;  // no block-level synchronisation below this point
  const int grp = item / a.n_chunks, chn = item % a.n_chunks;
  const int m_lo = chn * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int b_lo = grp * a.S, nb = min(a.S, a.B - b_lo);
  __bf16* xi_h = timg[w][0][0];
  __bf16* xi_l = timg[w][0][NPL - 1];
  __bf16* dz_h = timg[w][1][0];
  __bf16* dz_l = timg[w][1][NPL - 1];
  float* dsc = reinterpret_cast<float*>(&timg[w][0][0][0]);  // dcon [j][p] fp32, aliases slot 0 (after its reads)
  float* mycarry = &carry[w][0][0];
  const float* whmu = &sh.cst[NH * HP];
  const float* whr = &sh.cst[NH * HP + HP];

  f4 dW[4][4], dWe[JB][4], dWh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int o = 0; o < 4; ++o) dW[i][o] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < JB; ++i)
#pragma unroll
    for (int o = 0; o < 4; ++o) dWe[i][o] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) dWh[i] = f4{0.f, 0.f, 0.f, 0.f};
  bf8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;

  for (int m0 = m_lo; m0 < m_hi; m0 += P) {
    const int nP = min(P, m_hi - m0), t0 = a.s * m0, fin = a.s * nP;
    f4 dCa[4][2];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) dCa[rb][0] = dCa[rb][1] = f4{0.f, 0.f, 0.f, 0.f};
    for (int bl = 0; bl < nb; ++bl) {
      fence();
      const int b = b_lo + bl;
      const float* ub = u + static_cast<size_t>(b) * a.L;
      const int wi = win ? win[b] : 0;
      const float* Cw = C + static_cast<size_t>(wi) * a.Lh * a.H;
      f4 X[NH + 1][4][2];
      float mu[2], rr[2];
      unit_forward<NH, KB, JB, NP>(a, sh, ub, Cw, tht + static_cast<size_t>(b) * a.H, m0, nP, t0, X, mu, rr);
      // X0 with its ones row -> transposed image (slot 0) for dW
      if (a.H < 64 && g == 3) X[0][3][0][3] = X[0][3][1][3] = 1.f;
      put_image<NP>(xi_h, xi_l, X[0], g, c);

      // ---- head backward ----
      const float* gb = gout + static_cast<size_t>(b) * a.Lout;
      const float dl = dls[b];
      float gmu[2], gr[2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int p = 16 * cb + c;
        const int oq = a.s * p + (a.s - 1);
        const bool pv = p < nP;
        const int o = t0 + oq;
        const float sig = softplus_f(rr[cb]) + 1e-10f;
        const float gv = pv ? gb[a.swap_out ? (o ^ 1) : o] : 0.f;
        float dsig = pv ? gv * ub[o + a.k] : 0.f;
        if (pv && o >= a.Lout - a.n_logsig) dsig += dl / sig;
        gmu[cb] = gv;
        gr[cb] = dsig * sigmoid_f(rr[cb]);
        if (g == 0) {
          gsc[w][0][p] = gv;
          gsc[w][1][p] = sig;
          gsc[w][3][p] = gr[cb];
          if (a.s == 2) {
            const int oe = t0 + 2 * p;
            gsc[w][2][p] = pv ? gb[a.swap_out ? (oe ^ 1) : oe] : 0.f;
          }
        }
      }
      // head weight gradient dW_head[h][o] += sum_p X1[h][p] G[o][p] (G = (d mu, d r)); the ones
      // row of X1 gives the head bias gradient
      if (a.H < 64 && g == 3) X[1][3][0][3] = X[1][3][1][3] = 1.f;
      put_image<NP>(dz_h, dz_l, X[1], g, c);
      fence();
      {
        float gvv[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) gvv[jj] = c < 2 ? gsc[w][c == 0 ? 0 : 3][8 * g + jj] : 0.f;
        const Fr<NP> gf = split8<NP>(gvv);
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) dWh[hb] = mm<NP>(tr_frag<NP>(dz_h, dz_l, hb, g, c), gf, dWh[hb]);
      }
      // dX1 = w_mu gmu + w_r gr; dz1 = dX1 * elu'(E1)
      f4 D[4][2];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const f4 wm = *reinterpret_cast<const f4*>(&whmu[16 * rb + 4 * g]);
        const f4 wr = *reinterpret_cast<const f4*>(&whr[16 * rb + 4 * g]);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            D[rb][cb][r] = (wm[r] * gmu[cb] + wr[r] * gr[cb]) * elu_grad_from_out(X[1][rb][cb][r]);
      }
      put_image<NP>(dz_h, dz_l, D, g, c);
      // dX0 = W dz1 (chain)
      fence();
      f4 dX[4][2];
#pragma unroll
      for (int ib = 0; ib < 4; ++ib) dX[ib][0] = dX[ib][1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const Fr<NP> df = chain_frag<NP>(D, ks, cb);
#pragma unroll
          for (int ib = 0; ib < 4; ++ib) dX[ib][cb] = mm<NP>(wfrag(sh, 8 * NH + ib * 2 + ks, lane), df, dX[ib][cb]);
        }
      // dW1 += X0 dz1^T (transposed images)
      fence();
#pragma unroll
      for (int ib = 0; ib < 4; ++ib) {
        const Fr<NP> xa = tr_frag<NP>(xi_h, xi_l, ib, g, c);
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) dW[ib][ob] = mm<NP>(xa, tr_frag<NP>(dz_h, dz_l, ob, g, c), dW[ib][ob]);
      }
      // first layer: dA0 = dX0 * elu'(X0), X0 read back from its image (hi + lo; row 63 held 1:
      // dX0 is 0 there)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const f4 x0 = get_own<NP>(xi_h, xi_l, rb, cb, g, c);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = dX[rb][cb][r] * elu_grad_from_out(x0[r]);
            D[rb][cb][r] = v;
            dCa[rb][cb][r] += v;
          }
        }
      // dcon[j][p] = sum_h w_eps[j][h] dA0[h][p]
      fence();
      f4 dcn[JB][2];
#pragma unroll
      for (int jb = 0; jb < JB; ++jb) dcn[jb][0] = dcn[jb][1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const Fr<NP> df = chain_frag<NP>(D, ks, cb);
#pragma unroll
          for (int jb = 0; jb < JB; ++jb)
            dcn[jb][cb] = mm<NP>(wfrag(sh, 16 * NH + 4 * KB + jb * 2 + ks, lane), df, dcn[jb][cb]);
        }
      // dA0 -> slot 1 image; dW_eps and d theta from its transposed fragments
      put_image<NP>(dz_h, dz_l, D, g, c);
      fence();
      f4 dth4[4];
#pragma unroll
      for (int hb = 0; hb < 4; ++hb) {
        const Fr<NP> ta = tr_frag<NP>(dz_h, dz_l, hb, g, c);
        dth4[hb] = mm_bexact<NP>(ta, ones, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int jb = 0; jb < JB; ++jb) {
          const Fr<NP> uf = ua_frag<NP>(ub, a.L, a.k, t0, a.s, jb, nP, g, c);
          dWe[jb][hb] = mm<NP>(uf, ta, dWe[jb][hb]);
        }
      }
      if (c == 0) {
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) {
          f4* dp = reinterpret_cast<f4*>(&dthl[w][bl][16 * hb + 4 * g]);
          *dp = *dp + dth4[hb];
        }
      }
      // dcon -> fp32 scratch [j][p] (slot 0: its transposed reads are done)
#pragma unroll
      for (int jb = 0; jb < JB; ++jb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r) dsc[(16 * jb + 4 * g + r) * P + 16 * cb + c] = dcn[jb][cb][r];
      // du over local positions q in [0, fin + k): transposed conv + pass-through + carry
      {
        float* db = du + static_cast<size_t>(b) * a.L;
        float vq[2];
        int qq[2];
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int q = lane + 64 * it;
          qq[it] = q;
          float v = 0.f;
          if (q < fin + a.k) {
            for (int j = 0; j < a.k; ++j) {
              const int t = q - j;
              if (t >= 0) {
                if (a.s == 1) {
                  if (t < nP) v += dsc[j * P + t];
                } else if (!(t & 1) && (t >> 1) < nP) {
                  v += dsc[j * P + (t >> 1)];
                }
              }
            }
            const int oq = q - a.k;
            if (oq >= 0 && oq < fin) {
              if (a.s == 1) v += gsc[w][0][oq] * gsc[w][1][oq];
              else v += (oq & 1) ? gsc[w][0][oq >> 1] * gsc[w][1][oq >> 1] : gsc[w][2][oq >> 1];
            }
            if (q < a.k) v += mycarry[bl * KP + q];
          }
          vq[it] = v;
        }
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int q = qq[it];
          if (q < fin) db[t0 + q] = vq[it];
          else if (q < fin + a.k) mycarry[bl * KP + q - fin] = vq[it];
        }
      }
    }
    // tile done: its dC over the group
    float* dcs = dC_slab + (static_cast<size_t>(grp) * a.Lh + m0) * a.H;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int p = 16 * cb + c;
      if (p < nP) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = 16 * rb + 4 * g + r;
            if (h < a.H) dcs[static_cast<size_t>(p) * a.H + h] = dCa[rb][cb][r];
          }
      }
    }
  }

  // ---- per-sample tails: carry -> halo / du tail; d theta -> slab ----
  for (int bl = 0; bl < nb; ++bl) {
    const int b = b_lo + bl;
    for (int q = lane; q < a.k; q += 64) {
      const float v = mycarry[bl * KP + q];
      if (chn == a.n_chunks - 1) du[static_cast<size_t>(b) * a.L + a.Lout + q] = v;
      else halo[(static_cast<size_t>(b) * a.n_chunks + chn) * a.k + q] = v;
    }
    if (lane < a.H) dth_slab[(static_cast<size_t>(chn) * a.B + b) * a.H + lane] = dthl[w][bl][lane];
  }

  // ---- weight-gradient partials of this work item (layout of flow4's n_wgrad) ----
  const int H = a.H;
  const int nW = a.k * H + NH * H * H + 3 * NH * H + 2 * H + 2;
  float* ws = dW_slab + static_cast<size_t>(item) * nW;
#pragma unroll
  for (int jb = 0; jb < JB; ++jb)
#pragma unroll
    for (int hb = 0; hb < 4; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * jb + 4 * g + r, h = 16 * hb + c;
        if (j < a.k && h < H) ws[j * H + h] = dWe[jb][hb][r];
      }
  const int off_w = a.k * H, off_b = off_w + NH * H * H;
#pragma unroll
  for (int ib = 0; ib < 4; ++ib)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hi = 16 * ib + 4 * g + r, ho = 16 * ob + c;
        if (ho < H) {
          if (hi < H) ws[off_w + hi * H + ho] = dW[ib][ob][r];
          else if (hi == 63) ws[off_b + ho] = dW[ib][ob][r];  // the ones row: bias gradient
        }
      }
  // bn gamma / beta partials: zero (no BN on this path)
  for (int i = lane; i < 2 * NH * H; i += 64) ws[off_b + NH * H + i] = 0.f;
  const int off_h = off_b + 3 * NH * H;
  if (c < 2) {
#pragma unroll
    for (int hb = 0; hb < 4; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * hb + 4 * g + r;
        if (h < H) ws[off_h + h * 2 + c] = dWh[hb][r];
        else if (h == 63) ws[off_h + 2 * H + c] = dWh[hb][r];  // ones row: head bias gradient
      }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct Geom {
  int s, Lout, Lh, S, n_groups, n_tiles, CH, n_chunks, n_items;
};

static Geom geom(const VissmFlowDesc* d, bool backward) {
  Geom g;
  g.s = d->stride2 ? 2 : 1;
  g.Lout = d->L - d->k;
  g.Lh = g.Lout / g.s;
  g.S = (backward && d->n_win > 1) ? 1 : S;
  g.n_groups = (d->B + g.S - 1) / g.S;
  g.n_tiles = (g.Lh + P - 1) / P;
  int ch_min_tiles = ((d->k + g.s - 1) / g.s + P - 1) / P;
  if (ch_min_tiles < 1) ch_min_tiles = 1;
  const int target_items = 8192;
  int want = (target_items + g.n_groups - 1) / g.n_groups;
  int max_chunks = g.n_tiles / ch_min_tiles;
  if (max_chunks < 1) max_chunks = 1;
  int nc = want < max_chunks ? want : max_chunks;
  if (nc < 1) nc = 1;
  int tiles_per_chunk = (g.n_tiles + nc - 1) / nc;
  if (tiles_per_chunk < ch_min_tiles) tiles_per_chunk = ch_min_tiles;
  g.CH = tiles_per_chunk * P;
  g.n_chunks = (g.Lh + g.CH - 1) / g.CH;
  g.n_items = g.n_groups * g.n_chunks;
  return g;
}

static int n_wgrad(const VissmFlowDesc* d) {
  const int H = d->H, k = d->k, nh = d->n_hidden;
  return k * H + nh * H * H + 3 * nh * H + 2 * H + 2;
}

static int jb_of(int k) { return (k + 15) / 16; }
static int np_of(const VissmFlowDesc* d) { return d->precision == VISSM_PREC_BF16X3 ? 3 : 1; }

struct Ws {
  bf8* img;
  float* cst;
  float* ls_slab;                                        // fwd
  float *dC_slab, *dth_slab, *dW_slab, *halo, *wred;     // bwd
};

static size_t ws_layout(const VissmFlowDesc* d, const Geom& g, bool backward, char* base, Ws* w) {
  size_t off = 0;
  auto take = [&](size_t nbytes) { char* p = base ? base + off : nullptr; off += align_up(nbytes); return p; };
  Ws t{};
  const int JB = jb_of(d->k), KB = (JB + 1) / 2;
  const int NPL = np_of(d) == 3 ? 2 : 1;
  t.img = reinterpret_cast<bf8*>(take(static_cast<size_t>(n_frags(d->n_hidden, KB, JB)) * NPL * 64 * sizeof(bf8)));
  t.cst = reinterpret_cast<float*>(take(((d->n_hidden + 2) * HP + 4) * sizeof(float)));
  if (!backward) {
    t.ls_slab = reinterpret_cast<float*>(take(static_cast<size_t>(g.n_chunks) * d->B * 4));
  } else {
    t.dC_slab = reinterpret_cast<float*>(take(static_cast<size_t>(g.n_groups) * g.Lh * d->H * 4));
    t.dth_slab = reinterpret_cast<float*>(take(static_cast<size_t>(g.n_chunks) * d->B * d->H * 4));
    t.dW_slab = reinterpret_cast<float*>(take(static_cast<size_t>(g.n_items) * n_wgrad(d) * 4));
    t.halo = reinterpret_cast<float*>(take(static_cast<size_t>(d->B) * g.n_chunks * d->k * 4));
    t.wred = reinterpret_cast<float*>(take(static_cast<size_t>(n_wgrad(d)) * 4));
  }
  if (w) *w = t;
  return off;
}

static KArgs make_args(const VissmFlowDesc* d, const Geom& g) {
  KArgs a;
  a.B = d->B; a.L = d->L; a.k = d->k; a.H = d->H; a.s = g.s; a.swap_out = d->swap_out;
  a.n_logsig = d->n_logsig; a.Lout = g.Lout; a.Lh = g.Lh; a.CH = g.CH; a.n_chunks = g.n_chunks; a.S = g.S;
  a.n_groups = g.n_groups; a.n_items = g.n_items;
  return a;
}

// from flow_v4.hip (shared epilogue kernels)
__global__ void halo_fixup_kernel(float* __restrict__ du, const float* __restrict__ halo, int B, int L, int k,
                                  int n_chunks, int s, int CH) {
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < (n_chunks - 1) * k; i += blockDim.x) {
    const int c = i / k, q = i % k;
    const int pos = s * (c + 1) * CH + q;
    if (pos < L) du[static_cast<size_t>(b) * L + pos] += halo[(static_cast<size_t>(b) * n_chunks + c) * k + q];
  }
}

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

__global__ void scatter_wgrad_kernel(const float* __restrict__ red, VissmFlowGrads g, int k, int H, int nh) {
  const int nW = k * H + nh * H * H + 3 * nh * H + 2 * H + 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nW; i += gridDim.x * blockDim.x) {
    const float v = red[i];
    int off = 0;
    if (i < (off += k * H)) { g.w_eps[i] = v; continue; }
    if (i < off + nh * H * H) { g.w_hid[i - off] = v; continue; }
    off += nh * H * H;
    if (i < off + nh * H) { g.b_hid[i - off] = v; continue; }
    off += nh * H;
    if (i < off + nh * H) continue;  // bn gamma (no BN on this path)
    off += nh * H;
    if (i < off + nh * H) continue;  // bn beta
    off += nh * H;
    if (i < off + 2 * H) { g.w_head[i - off] = v; continue; }
    off += 2 * H;
    g.b_head[i - off] = v;
  }
}

}  // namespace flow5

using namespace flow5;

bool flow5_supports(const VissmFlowDesc* d) {
  // bf16x3 keeps hi and lo images in LDS: k <= 32 there (k <= 64 for bf16)
  return (d->precision == VISSM_PREC_BF16 || (d->precision == VISSM_PREC_BF16X3 && d->k <= 32)) &&
         d->n_hidden == 1 && !d->bn && d->H <= 63 && d->k <= 64;
}

size_t flow5_workspace_size(const VissmFlowDesc* d, int backward) {
  Geom g = geom(d, backward != 0);
  return ws_layout(d, g, backward != 0, nullptr, nullptr);
}

#define FLOW5_DISPATCH(KERNEL, JB, NP, ...)                                                        \
  do {                                                                                             \
    if (NP == 3) {                                                                                 \
      switch (JB) {                                                                                \
        case 1: hipLaunchKernelGGL((KERNEL<1, 1, 1, 3>), __VA_ARGS__); break;                       \
        default: hipLaunchKernelGGL((KERNEL<1, 1, 2, 3>), __VA_ARGS__); break;                      \
      }                                                                                            \
    } else {                                                                                       \
      switch (JB) {                                                                                \
        case 1: hipLaunchKernelGGL((KERNEL<1, 1, 1, 1>), __VA_ARGS__); break;                       \
        case 2: hipLaunchKernelGGL((KERNEL<1, 1, 2, 1>), __VA_ARGS__); break;                       \
        case 3: hipLaunchKernelGGL((KERNEL<1, 2, 3, 1>), __VA_ARGS__); break;                       \
        default: hipLaunchKernelGGL((KERNEL<1, 2, 4, 1>), __VA_ARGS__); break;                      \
      }                                                                                            \
    }                                                                                              \
  } while (0)

static void launch_prep(const VissmFlowDesc* d, const VissmFlowParams* w, const Ws& ws, hipStream_t st) {
  const int JB = jb_of(d->k), KB = (JB + 1) / 2;
  hipLaunchKernelGGL(prep_kernel, dim3(n_frags(d->n_hidden, KB, JB)), dim3(64), 0, st, *w, d->H, d->k, d->n_hidden,
                     np_of(d), KB, JB, ws.img, ws.cst);
}

int flow5_fwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
              const float* theta_term, float* u_next, float* logsig, void* workspace, size_t ws_bytes,
              hipStream_t st) {
  Geom g = geom(d, false);
  VISSM_CHECK_ARG(workspace && ws_bytes >= ws_layout(d, g, false, nullptr, nullptr), "flow_fwd: workspace too small");
  Ws ws;
  ws_layout(d, g, false, reinterpret_cast<char*>(workspace), &ws);
  launch_prep(d, w, ws, st);
  VISSM_CHECK_LAUNCH("flow5_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid((g.n_items + NW - 1) / NW);
  prof_begin(VISSM_PROF_FLOW_FWD, st);
  FLOW5_DISPATCH(fwd_kernel, jb_of(d->k), np_of(d), grid, dim3(NT), 0, st, a, u, C, wn, theta_term, ws.img, ws.cst,
                 u_next, ws.ls_slab);
  VISSM_CHECK_LAUNCH("flow5_fwd");
  prof_end(VISSM_PROF_FLOW_FWD, st);
  return launch_reduce_rows(ws.ls_slab, logsig, g.n_chunks, d->B, st);
}

int flow5_bwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
              const float* theta_term, const float* du_next, const float* dlogsig, float* du, float* dC,
              float* dtheta_term, const VissmFlowGrads* gr, void* workspace, size_t ws_bytes, hipStream_t st) {
  Geom g = geom(d, true);
  VISSM_CHECK_ARG(workspace && ws_bytes >= ws_layout(d, g, true, nullptr, nullptr), "flow_bwd: workspace too small");
  Ws ws;
  ws_layout(d, g, true, reinterpret_cast<char*>(workspace), &ws);
  launch_prep(d, w, ws, st);
  VISSM_CHECK_LAUNCH("flow5_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid((g.n_items + NW - 1) / NW);
  prof_begin(VISSM_PROF_FLOW_BWD, st);
  FLOW5_DISPATCH(bwd_kernel, jb_of(d->k), np_of(d), grid, dim3(NT), 0, st, a, u, C, wn, theta_term, du_next, dlogsig,
                 ws.img, ws.cst, du, ws.dC_slab, ws.dth_slab, ws.dW_slab, ws.halo);
  VISSM_CHECK_LAUNCH("flow5_bwd");
  prof_end(VISSM_PROF_FLOW_BWD, st);
  if (g.n_chunks > 1) {
    hipLaunchKernelGGL(flow5::halo_fixup_kernel, dim3(d->B), dim3(256), 0, st, du, ws.halo, d->B, d->L, d->k,
                       g.n_chunks, g.s, g.CH);
    VISSM_CHECK_LAUNCH("flow5_halo");
  }
  const int64_t nC = static_cast<int64_t>(g.Lh) * d->H;
  int rc;
  if (d->n_win == 1) {
    rc = launch_reduce_rows(ws.dC_slab, dC, g.n_groups, nC, st);
    if (rc) return rc;
  } else {
    dim3 rg(static_cast<unsigned>((nC + 255) / 256), d->n_win);
    hipLaunchKernelGGL(flow5::reduce_by_window_kernel, rg, dim3(256), 0, st, ws.dC_slab, win, dC, d->B,
                       static_cast<int>(nC));
    VISSM_CHECK_LAUNCH("flow5_reduce_window");
  }
  rc = launch_reduce_rows(ws.dth_slab, dtheta_term, g.n_chunks, static_cast<int64_t>(d->B) * d->H, st);
  if (rc) return rc;
  const int nW = n_wgrad(d);
  rc = launch_reduce_rows(ws.dW_slab, ws.wred, g.n_items, nW, st);
  if (rc) return rc;
  hipLaunchKernelGGL(flow5::scatter_wgrad_kernel, dim3((nW + 255) / 256), dim3(256), 0, st, ws.wred, *gr, d->k,
                     d->H, d->n_hidden);
  VISSM_CHECK_LAUNCH("flow5_scatter");
  return VISSM_OK;
}

}  // namespace vissm
