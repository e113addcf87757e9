// IAF flow of the neural-MA sampler on the bf16 matrix cores (fp32 accumulation):
// forward and backward.
//
// Precision: VISSM_PREC_BF16 (bf16 operands, one product per MFMA),
// VISSM_PREC_BF16X3 (split operands a = a_hi + a_lo, products a_hi b_hi + a_hi b_lo
// + a_lo b_hi: ~2^-16 relative per product, fp32-class results), or VISSM_PREC_BF16X2 (forward
// kernel only: split weights, bf16 activations, products w_hi x + w_lo x -- the weights' rounding
// is the same at every position and adds up coherently over a path; the activations' is not).
//
// Reference: IAF._create_flow / IAF.slp (AR.py:50-89), stride-2 head
// (lotka_volterra_partial.py:97-104), Permute fused into the store (swap_out).
//
// Design (wave-centric: no block barriers on the step path):
//   * a work unit = one (sample, tile of P = 16 head positions) is processed by ONE
//     wave; a block's 4 waves run independent work items and share only the weight
//     fragments staged in LDS once per block;
//   * activations are MFMA accumulators X[rb] (lane (g, c) holds rows
//     h = 16 rb + 4 g + r, position p = c).  Products that contract over h (hidden
//     layer, head, dX = W dZ, dcon = w_eps dA0, the dC identity-selection) take the
//     accumulators directly as the B operand of v_mfma_f32_16x16x32_bf16: k-step ks
//     packs rows 32 ks + 16 (j >> 2) + 4 g + (j & 3) of the lane's own registers and
//     the weight fragments are pre-permuted to that k order (hperm) -- no LDS round
//     trip, no lane movement;
//   * products that contract over positions (dW = X dZ^T, dW_eps = U dA0^T,
//     d theta = dA0 1, dW_head = X1 G^T) use v_mfma_f32_16x16x16_bf16 on fragments
//     read from a wave-private swizzled [p][h] LDS image with ds_read_b64_tr_b16
//     (one read per fragment);
//   * bias gradients come free from a row of ones in the padded activations (row 63:
//     W is zero there, so the forward is unchanged and dW[63][:] = sum_p dZ);
//   * grid decomposition, carries, halo and fixed-order partial slabs follow
//     flow_v4.hip (sample groups x t-chunks; the backward walks tiles outer / samples
//     inner so the window-shared dC tile is summed over the group in accumulators).
// Supported (flow5_supports): H <= 50, k <= 64; bf16 with one hidden layer (AR) or three hidden layers with
// the BN affine folded into the weights (LV / SV / FHN heads: bwd_kernel<3, ...>, one wave per SIMD -- its
// three dW accumulator sets take 192 of the 512 registers), bf16x3 / bf16x2 with one hidden layer and k <= 32.
// The AR configurations' backward (bf16, one hidden layer, k <= 8, stride 1, one window) runs bwd2_kernel and the
// three-hidden-layer one-window shapes (LV / FHN / SV) bwd2n_kernel: two samples per unit, see below.  The forward of
// every one-window shape with k <= 64 (one hidden layer at bf16 / bf16x2 with k <= 32, three hidden layers at bf16)
// runs fwd2_kernel.  The AR kernels take the theta term folded into their layer-0 product when the caller passes the
// theta branch's factors (VissmFlowParams.theta_rank); the fused last AR flow also runs at bf16x2 (split-weight
// recompute).  Everything else runs on flow_v4 / flow_v2 (exact fp32).
#include "common.hpp"

// flow_v5n.hip compiles this file a second time, without the SLP vectorizer, under its own namespace and entry
// point names: the three-hidden-layer shapes (LV / SV / FHN) dispatch there (flow_api.hip)
#ifndef VISSM_FLOW5_NS
#define VISSM_FLOW5_NS flow5
#define VISSM_FLOW5_API(name) name
#endif

#include <cstdlib>
// VISSM_ABL_STORES (diagnostic builds only, results wrong): bit 0 drops the fused variant's x stores, bit 1 the du
// stores, bit 2 the dC slab stores -- per-buffer attribution of the backward's PMC WRITE_SIZE
#ifndef VISSM_ABL_STORES
#define VISSM_ABL_STORES 0
#endif

namespace vissm {
namespace VISSM_FLOW5_NS {

constexpr int P = 16;
constexpr int HP = 64;
constexpr int S = 16;
constexpr int NW = 4;
constexpr int NT = 64 * NW;
constexpr int UW = 128;
constexpr int DTH = 56;  // d theta rows kept per sample (H <= DTH): keeps the backward block <= 80 KB of LDS  // u window staged per unit: s * P + k <= 96

typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf4 lds_bf4;

// fragments: hi (and lo for NP == 3; NP == 2: lo of the weight operand only)
template <int NP>
struct Fr8 {
  bf8 h, l;
};
template <int NP>
struct Fr4 {
  bf4 h, l;
};

__device__ __forceinline__ f4 mfma32(bf8 a, bf8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 mfma16(bf4 a, bf4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s4, a), __builtin_bit_cast(s4, b), c, 0, 0, 0);
}

// the three-layer backward's accumulators in AGPRs (below): on in flow_v5n.hip, the translation unit built with the
// VGPR-form MFMAs that runs those kernels
#ifndef VISSM_BWD2N_AACC
#define VISSM_BWD2N_AACC 0
#endif
// accumulator-file MFMAs (inline asm): C / D pinned to AGPRs ("+a"), A / B in VGPRs.  For item-lifetime weight-gradient
// accumulators that only MFMAs touch, beside a chain that needs the 256 VGPRs (bwd2n_kernel).  hipcc pads no hazard
// inside the string: the opening s_nop 1 covers a VALU / v_accvgpr_write producer of an operand; accumulating into the
// previous MFMA's D needs none; readers of D after the loop wait through agpr_drain4().
__device__ __forceinline__ void mfma32_a(bf8 a, bf8 b, f4& c) {
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma32_a4(bf8 a, const bf8 (&b)[4], f4& c0, f4& c1, f4& c2, f4& c3) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %4, %5, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %4, %6, %1\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %4, %7, %2\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %4, %8, %3"
      : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3)
      : "v"(a), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]));
}
// the same with a shared B operand: c_x = A_x B
__device__ __forceinline__ void mfma32_a4b(const bf8 (&a)[4], bf8 b, f4& c0, f4& c1, f4& c2, f4& c3) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %4, %8, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %5, %8, %1\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %6, %8, %2\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %7, %8, %3"
      : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(b));
}
// 12 wait states (an 8-pass MFMA's D before any non-MFMA reader), tied to the accumulators so that no read of them can
// be scheduled above it
__device__ __forceinline__ void agpr_drain4(f4& c0, f4& c1, f4& c2, f4& c3) {
  asm volatile("s_nop 7\n\ts_nop 3" : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3));
}

template <int NP>
__device__ __forceinline__ f4 mm(const Fr8<NP>& a, const Fr8<NP>& b, f4 c) {
  if constexpr (NP >= 2) c = mfma32(a.l, b.h, c);  // a: the weight operand
  if constexpr (NP == 3) c = mfma32(a.h, b.l, c);
  return mfma32(a.h, b.h, c);
}
template <int NP>
__device__ __forceinline__ f4 mm(const Fr4<NP>& a, const Fr4<NP>& b, f4 c) {
  if constexpr (NP == 3) {
    c = mfma16(a.l, b.h, c);
    c = mfma16(a.h, b.l, c);
  }
  return mfma16(a.h, b.h, c);
}
// K = 16 product with the WEIGHT as the A operand: NP = 2 (split weights, bf16 activations) adds a_lo b_hi
template <int NP>
__device__ __forceinline__ f4 mm_w4(const Fr4<NP>& a, const Fr4<NP>& b, f4 c) {
  if constexpr (NP >= 2) c = mfma16(a.l, b.h, c);
  if constexpr (NP == 3) c = mfma16(a.h, b.l, c);
  return mfma16(a.h, b.h, c);
}
// one operand exact in bf16 (ones / selections)
template <int NP>
__device__ __forceinline__ f4 mm_ax(bf8 a, const Fr8<NP>& b, f4 c) {
  if constexpr (NP == 3) c = mfma32(a, b.l, c);
  return mfma32(a, b.h, c);
}
template <int NP>
__device__ __forceinline__ f4 mm_bx(const Fr4<NP>& a, bf4 b, f4 c) {
  if constexpr (NP == 3) c = mfma16(a.l, b, c);
  return mfma16(a.h, b, c);
}

__device__ __forceinline__ unsigned cvt2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f2){a, b}, bf2));
}
__device__ __forceinline__ float lo_of(float x, unsigned packed, int half) {
  // x - float(bf16 half of packed)
  const unsigned bits = half ? (packed & 0xffff0000u) : (packed << 16);
  return x - __builtin_bit_cast(float, bits);
}

template <int NP>
__device__ __forceinline__ Fr8<NP> split8(const f4& x0, const f4& x1) {
  Fr8<NP> f;
  const u4 h = {cvt2(x0[0], x0[1]), cvt2(x0[2], x0[3]), cvt2(x1[0], x1[1]), cvt2(x1[2], x1[3])};
  f.h = __builtin_bit_cast(bf8, h);
  if constexpr (NP == 3) {
    const u4 l = {cvt2(lo_of(x0[0], h[0], 0), lo_of(x0[1], h[0], 1)), cvt2(lo_of(x0[2], h[1], 0), lo_of(x0[3], h[1], 1)),
                  cvt2(lo_of(x1[0], h[2], 0), lo_of(x1[1], h[2], 1)), cvt2(lo_of(x1[2], h[3], 0), lo_of(x1[3], h[3], 1))};
    f.l = __builtin_bit_cast(bf8, l);
  }
  return f;
}
template <int NP>
__device__ __forceinline__ Fr4<NP> split4(const f4& x) {
  Fr4<NP> f;
  const u2 h = {cvt2(x[0], x[1]), cvt2(x[2], x[3])};
  f.h = __builtin_bit_cast(bf4, h);
  if constexpr (NP == 3) {
    const u2 l = {cvt2(lo_of(x[0], h[0], 0), lo_of(x[1], h[0], 1)), cvt2(lo_of(x[2], h[1], 0), lo_of(x[3], h[1], 1))};
    f.l = __builtin_bit_cast(bf4, l);
  }
  return f;
}

// chain B fragment of activations X (one column block): k-step ks = rows 32ks .. 32ks + 31
template <int NP>
__device__ __forceinline__ Fr8<NP> chain_frag(const f4 (&X)[4], int ks) {
  return split8<NP>(X[2 * ks], X[2 * ks + 1]);
}

// hidden row of element j of k-step ks in lane group g (the chain k order)
// Hidden unit h <-> padded row: swap the two 2-bit fields, h = 16a + 4b + c <-> row 16a + 4c + b
// (an involution; 63 -> 63).  Row 16 rb + 4 g + r sits in register (rb, r) of lane group g, so
// units fill whole registers: for H <= 50 registers (3, 1..3) hold only padding and the ones row
// and skip the elementwise work (NR below).
__host__ __device__ constexpr int swz(int i) { return (i & ~15) | ((i & 3) << 2) | ((i >> 2) & 3); }
constexpr int kMaxH = 50;  // units fit rows 0..47 and 48, 52 (dthl keeps DTH = 56 rows)
constexpr int NR = 13;     // registers (rb, r) with 4 rb + r < NR carry units

__host__ __device__ __forceinline__ int hperm(int ks, int g, int j) {
  return 32 * ks + 16 * (j >> 2) + 4 * g + (j & 3);
}

// Hidden activations live in log2-scaled units: the kernels carry x' = log2(e) x and
// y' = log2(e) ELU(x) (the scale folds into C, theta, w_eps, the biases and the head), so
// ELU is one v_exp_f32 and one FMA: y' = x' > 0 ? x' : log2(e) (2^x' - 1), and
// dy'/dx' = 2^x' = y' ln 2 + 1 below zero.
constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
// MED3: the select as med3(x', y'_neg, 0) (log2(e)(2^t - 1) >= t on both sides of zero), one
// instruction shorter; measured faster in the forward kernel, slower in the backward's recompute
template <bool MED3>
__device__ __forceinline__ float elu_fast(float x) {
  const float en = __builtin_fmaf(kLog2e, __builtin_amdgcn_exp2f(x), -kLog2e);
  if constexpr (MED3) return __builtin_amdgcn_fmed3f(x, en, 0.f);
  return x > 0.f ? x : en;
}
// (min(y', 0) as a median: fminf would add a NaN-canonicalising v_max per element)
__device__ __forceinline__ float elu_d(float y) {
  return __builtin_fmaf(__builtin_amdgcn_fmed3f(y, -3.0e38f, 0.f), kLn2, 1.f);
}
// The two-sample backward kernels take elu' from the recompute itself: the exponential clamped to [0, 1] (the clamp
// folds into v_exp_f32) IS the derivative, min(2^x', 1), and with it the ELU is max(x', log2(e)(d - 1)) -- the same
// three instructions as elu_fast<true>, bitwise the same value.  d is kept as f16 pairs (v_cvt_pk_f16_f32: 2^-11
// relative, below the bf16 rounding the products apply next) and applied by v_fma_mix_f32 (fp32 x f16 half, one
// instruction per element) instead of re-deriving elu' from the activation (unpack, med3, fma, mul: four).
// Levels: 0 off, 1 elu'(A0) only (in the registers of the bf16 A0 pairs it replaces), 2 every level (AR; LV / FHN at
// k <= 32 in the first flow's variant without du).  The pair unit issues 7 % (AR) / 15 % (LV) fewer instructions, but
// the kernels are latency-bound, so the time moves little: first measured slower (AR-cfg middle-flow backward 20.4 ->
// 23.2 ms) because the scheduler sank the packing to the pairs' use and spilled an accumulator in the loop
// (profiles/r06/ab_r06e.log); with the pairs pinned where they are computed (pin_pair) and flow_v5 / flow_v5f built
// without the SLP vectorizer (which otherwise unpacks the halves for v_pk_fma_f32 instead of v_fma_mix_f32): AR-cfg
// step 79.6 -> 79.3 ms (first flow 18.3 -> 17.9, middle 20.65 -> 20.47, fused unchanged), LV no-du backward 12.8 ->
// 12.2 ms but the du variant 15.8 -> 16.6 (off there), FHN alike (profiles/r06/ab_r06g.log).
#ifndef VISSM_DERIV16
#define VISSM_DERIV16 2
#endif
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float elu_dv(float x, float& d) {
  d = __builtin_amdgcn_fmed3f(__builtin_amdgcn_exp2f(x), 0.f, 1.f);
  return __builtin_amdgcn_fmed3f(x, __builtin_fmaf(kLog2e, d, -kLog2e), 3.0e38f);
}
__device__ __forceinline__ unsigned pk_f16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f2){a, b}, h2v));
}
// materialise a pair where it is computed (left alone, the scheduler sinks the packing to the pair's use and keeps the
// fp32 derivatives live across the recompute's MFMA chains instead: a spilled accumulator in the loop)
__device__ __forceinline__ void pin_pair(u2& v) { asm volatile("" : "+v"(v[0]), "+v"(v[1])); }
// x * (f16 half `half` of pk) as v_fma_mix_f32 (a plain product would unpack first)
__device__ __forceinline__ float mul_h(float x, unsigned pk, int half) {
  return __builtin_fmaf(x, static_cast<float>(__builtin_bit_cast(h2v, pk)[half]), 0.f);
}
// (the forward kernels take log sigma on v_log_f32: sigma >= 1e-10 is a normal float; AR-cfg fwd 7.56 -> 7.34 ms)
// softplus on v_exp_f32 / v_log_f32 directly (__logf adds a denormal-scaling and refinement sequence; 1 + e^-|x|
// lies in [1, 2]) and max(x, 0) as a median
__device__ __forceinline__ float softplus_fast(float x) {
  return __builtin_amdgcn_fmed3f(x, 0.f, 3.0e38f) +
         __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(-kLog2e * fabsf(x))) * kLn2;
}
// v_rcp_f32 (1 ulp) instead of the correctly rounded division sequence of __frcp_rn (-1.1 ms per AR-cfg step)
__device__ __forceinline__ float rcp_f(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float sigmoid_fast(float x) { return rcp_f(1.f + __expf(-x)); }

// ---------------------------------------------------------------------------
// weight fragments (8 bf16 per lane): [frag][plane (hi, lo)][lane]
//   WF(l, ob, ks)  l*8 + ob*2 + ks          forward hidden l   A[h_out][h_in perm]
//   WB(l, ib, ks)  8NH + l*8 + ib*2 + ks    dI = W dZ          A[h_in][h_out perm]
//   WE(kb, ob)     16NH + kb*4 + ob         layer 0            A[h][j]
//   WC(jb, ks)     16NH + 4KB + jb*2 + ks   dcon               A[j][h perm]
//   WH(ks)         16NH + 4KB + 2JB + ks    head               A[o][h perm]
// With batch_normalization(training=False) after each hidden ELU (LV / SV / FHN), the BN affine
// x = gamma' e + beta is folded into the layer that consumes it: W~ = diag(gamma') W and
// b~ = b + W^T beta (head likewise), so the kernels only see ELU outputs E; the BN and
// unfolded weight gradients are recovered from the reduced sums in scatter_wgrad_kernel.
// ---------------------------------------------------------------------------
// (head fragments replicate the two output rows into every lane group)
__host__ __device__ constexpr int n_frags(int NH, int KB, int JB) { return 16 * NH + 4 * KB + 2 * JB + 2; }

struct KArgs {
  int B, L, k, H, s, swap_out, n_logsig, Lout, Lh, CH, n_chunks, S, n_groups, n_items;
  int pL, pLo;  // row strides of u / du and u_next / du_next (VissmFlowDesc.u_pitch / out_pitch)
  int dc16;  // backward, bf16 products, one window: the dC slab holds bf16 partials (half the reduce's reads)
  int ncu;  // compute units of the device (the backward's wave priority pattern)
};

// The last flow of the AR(1) stack fused with its ELBO terms (vissm_flow_ar_elbo_fused): the backward
// kernel recomputes the flow's output x = u_next itself, so it evaluates the gradient of the AR(1)
// transition and observation terms on the fly instead of reading an upstream gradient; the flow's
// forward launch is not needed.  Loss part: -scale sum_b (sde_b + obs_b + logsig_b) (AR.py:168-185).
// A tile computes 16 columns but produces the gradients of 15 positions: column 15 is the next
// position's x (the head of the transition out of position 14); x at the previous tile's last position
// rides in a per-sample carry, and a chunk other than the first starts one tile early (outputs
// discarded) to obtain it.  The kernel writes x (for the per-sample sde / obs / d theta sums, which a
// streaming kernel takes afterwards) and per-column log sigma partial sums (fixed order: tiles, then
// the 16 columns at the item's end) to a [n_chunks][B] slab.
struct FzArgs {
  const float* theta;  // [B][3] AR(1) theta per sample
  const float* obs;    // [n_win][M] observations y_t (pairs with x_{t+1})
  const float* bin;    // [n_win][M] observation mask
  float* x;            // [B][M + 1] the flow's output (the latent path)
  float* lsl;          // [n_chunks][B] log sigma partial sums
  float scale;         // T / M
  float iosd;          // 1 / obs_std
  int M;               // transitions (x has M + 1 entries = the flow's Lout)
};
// x of the neighbouring column within a 16-lane row (DPP row shifts: no LDS)
__device__ __forceinline__ float row_prev(float v) {  // lane c <- lane c - 1 (c = 0 keeps v)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                                               0x111, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_next(float v) {  // lane c <- lane c + 1 (c = 15 keeps v)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                                               0x101, 0xf, 0xf, false));
}

// bf16 dC slab partials at bf16 products, one window (read by launch_reduce_rows_bf16).  (Summing the dC tiles over
// a block's groups through LDS before the slab -- slab 4.1 -> 1.0 GB and its reduce 0.74 -> 0.19 ms per AR-cfg
// launch -- cost the kernel 0.8 ms in tile-barrier wave skew: 126.9 vs 125.8 ms per step, round 1; removed.)

// folded hidden weight W~_l[hin][hout] and head weight W~_h[h][o]
__device__ __forceinline__ float wt_hid(const VissmFlowParams& w, int H, int bn, int l, int hin, int hout) {
  const float x = w.w_hid[(static_cast<size_t>(l) * H + hin) * H + hout];
  return (bn && l > 0) ? x * w.bn_g[(l - 1) * H + hin] * kBnScale : x;
}
__device__ __forceinline__ float wt_head(const VissmFlowParams& w, int H, int bn, int nh, int h, int o) {
  const float x = w.w_head[h * 2 + o];
  return (bn && nh > 0) ? x * w.bn_g[(nh - 1) * H + h] * kBnScale : x;
}

// folded hidden bias b~_l[hout] = b_l + W_l^T beta_{l-1} and head bias (BN after the previous layer)
__device__ __forceinline__ float bias_hid(const VissmFlowParams& w, int H, int bn, int l, int hout) {
  float bb = w.b_hid[l * H + hout];
  if (bn && l > 0)
    for (int hi = 0; hi < H; ++hi) bb += w.w_hid[(static_cast<size_t>(l) * H + hi) * H + hout] * w.bn_b[(l - 1) * H + hi];
  return bb;
}
__device__ __forceinline__ float bias_head(const VissmFlowParams& w, int H, int bn, int nh, int o) {
  float bb = w.b_head[o];
  if (bn && nh > 0)
    for (int h = 0; h < H; ++h) bb += w.w_head[h * 2 + o] * w.bn_b[(nh - 1) * H + h];
  return bb;
}

// theta fold (VissmFlowParams.theta_rank = R > 0, k <= 16): K rows 16 + kk of the layer-0 product carry the theta
// term, theta_term[h] = sum_i w_theta[i][h] theta[i], as w_hi theta_hi + w_hi theta_lo + w_lo theta_hi:
// kk < R: (w_hi[kk], theta_hi[kk]); R <= kk < 2R: (w_hi[kk - R], theta_lo[kk - R]); 2R <= kk < 3R: (w_lo, theta_hi)
constexpr int kFoldRow = 16;
__host__ __device__ __forceinline__ int fold_index(int kk, int R, int* which) {
  if (kk < R) { *which = 0; return kk; }
  if (kk < 2 * R) { *which = 1; return kk - R; }
  if (kk < 3 * R) { *which = 2; return kk - 2 * R; }
  *which = -1;
  return -1;
}
__device__ __forceinline__ float bf16_hi(float x) { return static_cast<float>(static_cast<__bf16>(x)); }

// the split-weight forward's 8-wave blocks keep the hidden layer's hi planes in registers (122 VGPRs, still four waves per
// SIMD): 8.46 -> 8.39 ms per AR-cfg launch, profiles/r06/ab_r06j.log
#ifndef VISSM_X2_HIDREG
#define VISSM_X2_HIDREG 1
#endif
#ifndef VISSM_NO_LOFOLD
#define VISSM_NO_LOFOLD 0  // (A/B switch: 1 keeps the separate lo MFMAs)
#endif
constexpr bool kLoFoldOff = VISSM_NO_LOFOLD;
// lofold (the two-sample kernels' split-weight products, k <= 8): the lo planes of the layer-0 and head weights ride in
// the hi plane's otherwise zero rows -- layer-0 K rows 8..15 (lane group 1, whose B operand then repeats the taps
// 0..7) and head output rows 4q + 2, 4q + 3 (lo of mu, r: the kernel adds d[2], d[3] to d[0], d[1]) -- so those
// products need no second MFMA (kLoFold below)
__global__ void prep_kernel(VissmFlowParams w, int H, int k, int nh, int bn, int NP, int KB, int JB,
                            bf8* __restrict__ img, float* __restrict__ cst, int fold, int lofold) {
  const int f = blockIdx.x, lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const int NPL = NP >= 2 ? 2 : 1;
  float v[8];
  for (int j = 0; j < 8; ++j) {
    float x = 0.f;
    int r = f;
    if (r < 8 * nh) {  // WF (row 63 of the input carries ones: the folded bias rides in the MFMA)
      const int l = r >> 3, ob = (r >> 1) & 3, ks = r & 1;
      const int hin = swz(hperm(ks, g, j)), hout = swz(16 * ob + c);
      if (hin < H && hout < H) x = wt_hid(w, H, bn, l, hin, hout);
      else if (hin == HP - 1 && hout < H) x = bias_hid(w, H, bn, l, hout) * kLog2e;
    } else if ((r -= 8 * nh) < 8 * nh) {  // WB
      const int l = r >> 3, ib = (r >> 1) & 3, ks = r & 1;
      const int hin = swz(16 * ib + c), hout = swz(hperm(ks, g, j));
      if (hin < H && hout < H) x = wt_hid(w, H, bn, l, hin, hout);
    } else if ((r -= 8 * nh) < 4 * KB) {  // WE
      const int kb = r >> 2, ob = r & 3;
      const int jt = 32 * kb + 8 * g + j, h = swz(16 * ob + c);
      if (jt < k && h < H) x = w.w_eps[jt * H + h] * kLog2e;
      else if (lofold && kb == 0 && jt >= 8 && jt < 16 && jt - 8 < k && h < H) {  // lo of the taps 0..7
        const float wv = w.w_eps[(jt - 8) * H + h] * kLog2e;
        x = wv - bf16_hi(wv);
      } else if (fold && kb == 0 && jt >= kFoldRow && h < H) {  // the theta term's rows (theta fold)
        int which;
        const int i = fold_index(jt - kFoldRow, w.theta_rank, &which);
        if (i >= 0) {
          const float wv = w.w_theta[i * H + h] * kLog2e, hi = bf16_hi(wv);
          x = which == 2 ? bf16_hi(wv - hi) : hi;
        }
      }
    } else if ((r -= 4 * KB) < 2 * JB) {  // WC
      const int jb = r >> 1, ks = r & 1;
      const int jt = 16 * jb + c, h = swz(hperm(ks, g, j));
      if (jt < k && h < H) x = w.w_eps[jt * H + h] * kLog2e;
    } else {  // WH
      r -= 2 * JB;
      const int h = swz(hperm(r, g, j));
      // output rows o' = 4 q + o (o = 0: mu, 1: sigma) for every q: each lane group receives (mu, r) of its
      // column in registers 0, 1 of the head MFMA (no shuffle)
      const int o = c & 3;
      if (o < 2 && h < H) x = wt_head(w, H, bn, nh, h, o) * kLn2;
      else if (o < 2 && h == HP - 1) x = bias_head(w, H, bn, nh, o);
      else if (lofold && h < H) x = wt_head(w, H, bn, nh, h, o - 2) * kLn2 - bf16_hi(wt_head(w, H, bn, nh, h, o - 2) * kLn2);
      else if (lofold && h == HP - 1) x = bias_head(w, H, bn, nh, o - 2) - bf16_hi(bias_head(w, H, bn, nh, o - 2));
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
    // constants: folded biases [nh][64], folded head weights [2][64], folded head bias [2]
    const int hu = swz(lane);  // cst rows are padded rows
    for (int l = 0; l < nh; ++l) cst[l * HP + lane] = hu < H ? bias_hid(w, H, bn, l, hu) * kLog2e : 0.f;
    // folded head weights as bf16 pairs (mu, r) per row h: hi plane, then lo plane (the A
    // fragment of the head backward)
    {
      const float wm = hu < H ? wt_head(w, H, bn, nh, hu, 0) * kLn2 : 0.f;
      const float wr = hu < H ? wt_head(w, H, bn, nh, hu, 1) * kLn2 : 0.f;
      const __bf16 hm = (__bf16)wm, hr = (__bf16)wr;
      const __bf16 lm = (__bf16)(wm - (float)hm), lr = (__bf16)(wr - (float)hr);
      const bf2 ph = {hm, hr}, pl = {lm, lr};
      cst[nh * HP + lane] = __builtin_bit_cast(float, ph);
      cst[(nh + 1) * HP + lane] = __builtin_bit_cast(float, pl);
    }
    if (lane < 2) cst[(nh + 2) * HP + lane] = bias_head(w, H, bn, nh, lane);
  }
}

// zero-padded 64-wide copies of C [n_win][Lh][H] (+ the theta fold's bias) and of the theta term [B][H],
// log2(e)-scaled
__global__ void pad_kernel(const float* __restrict__ src, float* __restrict__ dst, int64_t rows, int H,
                           const float* __restrict__ bias) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= rows * HP) return;
  const int64_t r = i / HP;
  const int h = swz(static_cast<int>(i % HP));
  dst[i] = h < H ? (bias ? src[r * H + h] + bias[h] : src[r * H + h]) * kLog2e : 0.f;
}

// theta fold: per sample the B-operand rows 16..31 of the layer-0 product (lane groups 2, 3), as bf16:
// tf[b][gg] = 8 values, kk = 8 gg + j (fold_index order)
__global__ void theta_frag_kernel(const float* __restrict__ theta, int B, int R, u4* __restrict__ tf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * B) return;
  const int b = i >> 1, gg = i & 1;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int which;
    const int t = fold_index(8 * gg + j, R, &which);
    float x = 0.f;
    if (t >= 0) {
      const float th = theta[static_cast<size_t>(b) * R + t], hi = bf16_hi(th);
      x = which == 1 ? bf16_hi(th - hi) : hi;
    }
    v[j] = x;
  }
  tf[i] = u4{cvt2(v[0], v[1]), cvt2(v[2], v[3]), cvt2(v[4], v[5]), cvt2(v[6], v[7])};
}

template <int NH, int KB, int JB, int NP>
struct Shared {
  static constexpr int NFR = n_frags(NH, KB, JB);
  static constexpr int NPL = NP >= 2 ? 2 : 1;
  static constexpr int NCST = (NH + 2) * HP + 4;
  bf8 img[NFR][NPL][64];
  float cst[NCST];
};

// Compiler-only fence: keeps the (loop-invariant) LDS weight-fragment loads next to their
// use instead of hoisted out of the unit loop with ~100-200 VGPRs live.
__device__ __forceinline__ void fence() { asm volatile("" ::: "memory"); }
// Forward kernel: the 8 NH + 4 KB + 2 weight fragments it uses live in registers for the whole item (its
// footprint allows it) and it has no fences; measured 11.8 -> 10.4 ms per AR-cfg launch.  The bf16x2 forward
// (split weights) keeps the hi planes in registers and reads the lo planes from LDS per use (both planes in
// registers 12.5, both from LDS 12.9 ms against 11.6).  The backward keeps its fences between phases: at ~250
// VGPRs nothing may be hoisted.
//
// Backward design decisions (A/B measurements, docs/DESIGN_HISTORY.md §4 / §8): one hidden layer -- the head gradient rides in
// the dZ image (no G fragment via LDS), elu'(I_0) from the bf16 pairs the recompute keeps in registers, the dX and
// dcon weight fragments, dW's I_0 and dW_eps's u fragments all read before the head-backward VALU block; the dW /
// dW_head MFMAs (off the unit's critical path) issued after the du section's dcon stores (105.6 -> 104.3 ms per
// step; after the dA0 image store 105.1, after the dW_eps / d theta products 105.5, profiles/r02/dw_late_ab.log);
// the fused AR(1) variant reads the previous tile's last x (LDS carry) with the unit's inputs (104.6 -> 104.2);
// the per-sample d theta read-modify-writes branch-free with their reads issued together (no-return LDS adds: no
// change); k = 8: a straight-line transposed-conv sum, reads first, then a pairwise tree; per-sample window index /
// d log q read once per item into lane b, then v_readlane per unit; the four head-backward A fragments read
// unconditionally up front (a masked read per MFMA serialised four LDS round trips).  Rejected: the ELU select as
// v_med3 in the one-sample recompute (30.4 vs 29.7 ms), per-position LDS writes by every lane instead of a branch.
// value of lane `bl` of v (bl wave-uniform)
__device__ __forceinline__ int lane_i(int v, int bl) { return __builtin_amdgcn_readlane(v, bl); }
__device__ __forceinline__ float lane_f(float v, int bl) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), bl));
}
// unit_forward's fences: in the backward's recompute only
template <bool BWD>
__device__ __forceinline__ void fence_uf() {
  if constexpr (BWD) fence();
}

template <int NH, int KB, int JB, int NP>
__device__ __forceinline__ Fr8<NP> wfrag(const Shared<NH, KB, JB, NP>& sh, int f, int lane) {
  Fr8<NP> r;
  r.h = sh.img[f][0][lane];
  if constexpr (NP >= 2) r.l = sh.img[f][1][lane];
  return r;
}

template <int NH, int KB, int JB, int NP, int NTHR = NT>
__device__ __forceinline__ void load_shared(Shared<NH, KB, JB, NP>& sh, const bf8* __restrict__ img,
                                            const float* __restrict__ cst) {
  using SH = Shared<NH, KB, JB, NP>;
  constexpr int N = SH::NFR * SH::NPL * 64;
  for (int i = threadIdx.x; i < N; i += NTHR) (&sh.img[0][0][0])[i] = img[i];
  for (int i = threadIdx.x; i < SH::NCST; i += NTHR) sh.cst[i] = cst[i];
}

// transposed image: [p = 16 rows][64 h] bf16, 16 chunks of 4 per 128-byte row; chunk ch of row p
// sits at slot ch ^ p ^ ((p & 2) << 2).  Conflict-free for all three accesses (bank rules of
// MI355X_MICROARCH.md §LDS): the image store (ds_write_b64, 16-lane groups of one g: the XOR is a
// bijection of p), the own-entry read (ds_read_b64, 32-lane halves: the two g of a half differ in
// slot bit 0 and so in row parity, i.e. in the 128-B half of the bank row), and the transposed read
// (ds_read_b64_tr_b16, 32-lane halves = rows 8h .. 8h + 7 x chunks 4hb .. 4hb + 3: the four rows of
// one parity take four different 4-slot blocks through slot bits 2-3 = (p2, p3 ^ p1)).  The plain
// `ch ^ p` layout gave the transposed reads 2-way conflicts (rows p and p ^ 2 shared slot blocks):
// SQ_LDS_BANK_CONFLICT per bf16 backward launch 2.16e8 -> 4.1e7 cycles, step 118.5 -> 117.5 ms (A/B,
// profiles/r02/lds_swizzle_ab.log).  A full bit permutation of p that is equally conflict-free cost 26 more
// instructions and a spill: 121.6 ms.
__host__ __device__ constexpr int timg_perm(int p) { return p ^ ((p & 2) << 2); }
__device__ __forceinline__ int timg_off(int p, int ch) { return p * HP + 4 * (ch ^ timg_perm(p)); }

template <int NP>
__device__ __forceinline__ void put_image(__bf16* hi, __bf16* lo, const f4 (&X)[4], int g, int c) {
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const u2 h = {cvt2(X[rb][0], X[rb][1]), cvt2(X[rb][2], X[rb][3])};
    const int off = timg_off(c, 4 * rb + g);
    *reinterpret_cast<u2*>(hi + off) = h;
    if constexpr (NP == 3) {
      const u2 l = {cvt2(lo_of(X[rb][0], h[0], 0), lo_of(X[rb][1], h[0], 1)),
                    cvt2(lo_of(X[rb][2], h[1], 0), lo_of(X[rb][3], h[1], 1))};
      *reinterpret_cast<u2*>(lo + off) = l;
    }
  }
}

// a lane's own entries of an image it wrote, as fp32 (hi + lo)
template <int NP>
__device__ __forceinline__ f4 get_own(const __bf16* hi, const __bf16* lo, int rb, int g, int c) {
  const int off = timg_off(c, 4 * rb + g);
  const u2 h = *reinterpret_cast<const u2*>(hi + off);
  f4 r = {__builtin_bit_cast(float, h[0] << 16), __builtin_bit_cast(float, h[0] & 0xffff0000u),
          __builtin_bit_cast(float, h[1] << 16), __builtin_bit_cast(float, h[1] & 0xffff0000u)};
  if constexpr (NP == 3) {
    const u2 l = *reinterpret_cast<const u2*>(lo + off);
    r += f4{__builtin_bit_cast(float, l[0] << 16), __builtin_bit_cast(float, l[0] & 0xffff0000u),
            __builtin_bit_cast(float, l[1] << 16), __builtin_bit_cast(float, l[1] & 0xffff0000u)};
  }
  return r;
}

// K = 16 fragment over positions: lane (g, c) receives X[h = 16 hb + c][p = 4 g + jj], jj = 0..3
__device__ __forceinline__ bf4 tr_read(const __bf16* img, int hb, int g, int c) {
  const int row = 4 * g + (c >> 2), ch = 4 * hb + (c & 3);
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf4*)(img + timg_off(row, ch)));
}
template <int NP>
__device__ __forceinline__ Fr4<NP> tr_frag(const __bf16* hi, const __bf16* lo, int hb, int g, int c) {
  Fr4<NP> f;
  f.h = tr_read(hi, hb, g, c);
  if constexpr (NP == 3) f.l = tr_read(lo, hb, g, c);
  return f;
}

__device__ __forceinline__ int clampi(int i, int n) { return i < n ? i : n - 1; }

// Per-unit inputs, loaded branch-free: the u window [t0, t0 + 64 WU) and (backward) the
// upstream-gradient window [t0, t0 + 64), staged in the wave's LDS; C + theta term for the
// lane's 16 (h, p = c) entries from the zero-padded 64-wide copies (pad_kernel).
// (positions p >= nP read the last valid row: finite, their outputs are dropped and their
//  upstream gradient is zero.)  WU = 1 suffices for k <= 32: every read stays below s * 15 + 32.
template <int WU>
struct Win {
  float u[WU];
  float gv;
};

template <int WU>
__device__ __forceinline__ void fetch_win(const KArgs& a, const float* __restrict__ ub, const float* __restrict__ gb,
                                          int t0, Win<WU>& wn) {
  const int lane = threadIdx.x & 63;
  // only the entries a unit reads are fetched (u: s P + k, upstream gradient: s P); the rest of the
  // window is zero (it meets zero weights or discarded rows).  Fetching the whole 64-entry windows
  // re-read each row ~2.5x from beyond L2 in the backward, whose tiles-outer order revisits a
  // sample's row 16 units later.
  const int nu = a.s * P + a.k;
#pragma unroll
  for (int i = 0; i < WU; ++i) wn.u[i] = 64 * i + lane < nu ? ub[clampi(t0 + 64 * i + lane, a.L)] : 0.f;
  wn.gv = 0.f;
  if (gb && lane < a.s * P) {
    const int o = t0 + lane;
    wn.gv = gb[clampi(a.swap_out ? (o ^ 1) : o, a.Lout)];
  }
}

template <int WU>
__device__ __forceinline__ void stage_win(const Win<WU>& wn, float* uw, float* gw) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < WU; ++i) uw[64 * i + lane] = wn.u[i];
  if (gw) gw[lane] = wn.gv;
}

__device__ __forceinline__ void load_ct(const float* __restrict__ Cw, const float* __restrict__ thb, int m0, int nP,
                                        f4 (&cin)[4]) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const f4* crow = reinterpret_cast<const f4*>(Cw + static_cast<size_t>(m0 + clampi(c, nP)) * HP) + g;
  const f4* trow = reinterpret_cast<const f4*>(thb) + g;
  f4 cr[4], tr[4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    cr[rb] = crow[4 * rb];
    tr[rb] = trow[4 * rb];
  }
  // all eight loads in flight before the first use (left alone, the scheduler may pair them with
  // a full vmcnt(0) drain each to save registers)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) cin[rb] = cr[rb] + tr[rb];
}

// layer-0 B fragment: U[j = 32 kb + 8 g + jj][p = c] = u[t0 + s c + j] (weights are zero for j >= k)
template <int NP>
__device__ __forceinline__ Fr8<NP> u_frag(const float* uw, int s, int kb, int g, int c) {
  const float* q = uw + s * c + 32 * kb + 8 * g;
  return split8<NP>(f4{q[0], q[1], q[2], q[3]}, f4{q[4], q[5], q[6], q[7]});
}

// dW_eps A fragment (K = 16 positions): U[j = 16 jb + c][p = 4 g + jj] = u[t0 + s p + j]
// (rows j >= k are discarded; positions p >= nP meet dA0 = 0)
template <int NP>
__device__ __forceinline__ Fr4<NP> ua_frag(const float* uw, int s, int jb, int g, int c) {
  const float* q = uw + s * 4 * g + 16 * jb + c;
  return split4<NP>(f4{q[0], q[s], q[2 * s], q[3 * s]});
}

// forward of one unit from its staged inputs: X holds C + theta on entry and the last layer's
// ELU output I_NH (its row 63 set to one) on return; mu / rr are the head outputs at p = c.  The
// inputs of every product carry ones in row 63, where the fragments hold the (folded, scaled)
// biases.  With IMG, the hidden layers' inputs I_0 .. I_{NH-1} are written to images[0 .. NH-1].
// the forward's weight fragments held in registers (forward kernel: WF, WE, WH in that order)
template <int NH, int KB, int NP>
struct FwdRegs {
  static constexpr int N = 8 * NH + 4 * KB + 2;
  Fr8<NP> f[N];
};

template <int NH, int KB, int JB, int NP, bool IMG, bool REGW = false>
__device__ __forceinline__ void unit_forward(const KArgs& a, const Shared<NH, KB, JB, NP>& sh, const float* uw,
                                             f4 (&X)[4], float& mu, float& rr, __bf16* const* ih,
                                             __bf16* const* il, const FwdRegs<NH, KB, NP>* wr = nullptr,
                                             u2* i0p = nullptr) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  // fragment f of the shared image, or its register copy (index i in FwdRegs order)
  auto W = [&](int f, int i) -> Fr8<NP> {
    if constexpr (REGW && NP == 2) {  // hi planes from registers, lo planes from LDS
      Fr8<NP> r;
      r.h = wr->f[i].h;
      r.l = sh.img[f][1][lane];
      return r;
    } else if constexpr (REGW) {
      return wr->f[i];
    } else {
      return wfrag(sh, f, lane);
    }
  };
  // layer 0: the MFMA accumulates onto C + theta (its C operand), so no separate add
  f4 acc[4];
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) acc[ob] = X[ob];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const Fr8<NP> uf = u_frag<NP>(uw, a.s, kb, g, c);
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) acc[ob] = mm<NP>(W(16 * NH + kb * 4 + ob, 8 * NH + kb * 4 + ob), uf, acc[ob]);
  }
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      X[rb][r] = 4 * rb + r < NR ? elu_fast<!IMG>(acc[rb][r]) : 0.f;
#pragma unroll
  for (int l = 0; l < NH; ++l) {
    fence_uf<IMG>();
    if (g == 3) X[3][3] = 1.f;  // the ones row: bias of layer l (and its gradient)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) acc[ob] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const Fr8<NP> xf = chain_frag<NP>(X, ks);
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) acc[ob] = mm<NP>(W(l * 8 + ob * 2 + ks, l * 8 + ob * 2 + ks), xf, acc[ob]);
    }
    if constexpr (IMG) put_image<NP>(ih[l], il[l], X, g, c);  // I_l with its ones row -> image l
    if (IMG && l == 0 && i0p) {  // the bf16 pairs of I_0 kept in registers as well (hi plane)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) i0p[rb] = u2{cvt2(X[rb][0], X[rb][1]), cvt2(X[rb][2], X[rb][3])};
    }
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) X[rb][r] = 4 * rb + r < NR ? elu_fast<!IMG>(acc[rb][r]) : 0.f;
  }
  // head (16 output rows, o = 0: mu, o = 1: sigma pre-softplus; bias on the ones row)
  fence_uf<IMG>();
  if (g == 3) X[3][3] = 1.f;
  const int fh = 16 * NH + 4 * KB + 2 * JB;
  f4 d = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) d = mm<NP>(W(fh + ks, 8 * NH + 4 * KB + ks), chain_frag<NP>(X, ks), d);
  mu = d[0];
  rr = d[1];
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
  __shared__ float uwin[NW][UW];
  load_shared(sh, img, cst);
  // static wave priority = dispatch round mod 4 (four blocks per CU; see bwd_kernel): 9.45 -> 9.15 ms per launch
  {
    const int r = __builtin_amdgcn_readfirstlane(blockIdx.x / a.ncu) & 3;
    if (r == 1) __builtin_amdgcn_s_setprio(1);
    else if (r == 2) __builtin_amdgcn_s_setprio(2);
    else if (r == 3) __builtin_amdgcn_s_setprio(3);
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * NW + w);  // wave-uniform: scalar loads of per-sample data
  if (item >= a.n_items) return;
  const int grp = item / a.n_chunks, ch = item % a.n_chunks;
  const int m_lo = ch * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int b_lo = grp * a.S, nb = min(a.S, a.B - b_lo);
  float* uw = uwin[w];
  FwdRegs<NH, KB, NP> wr;
#pragma unroll
  for (int i = 0; i < 8 * NH; ++i) wr.f[i] = wfrag(sh, i, lane);
#pragma unroll
  for (int i = 0; i < 4 * KB; ++i) wr.f[8 * NH + i] = wfrag(sh, 16 * NH + i, lane);
#pragma unroll
  for (int i = 0; i < 2; ++i) wr.f[8 * NH + 4 * KB + i] = wfrag(sh, 16 * NH + 4 * KB + 2 * JB + i, lane);
  const int lwi = (win && lane < nb) ? win[b_lo + lane] : 0;
  for (int bl = 0; bl < nb; ++bl) {
    const int b = b_lo + bl;
    const float* ub = u + static_cast<size_t>(b) * a.pL;
    float* ob = u_next + static_cast<size_t>(b) * a.pLo;
    const int wi = lane_i(lwi, bl);
    const float* Cw = C + static_cast<size_t>(wi) * a.Lh * HP;
    float ls = 0.f;
    for (int m0 = m_lo; m0 < m_hi; m0 += P) {
      const int nP = min(P, m_hi - m0), t0 = a.s * m0;
      f4 X[4];
      float mu, rr;
      {
        Win<KB> wn;
        fetch_win<KB>(a, ub, nullptr, t0, wn);
        load_ct(Cw, tht + static_cast<size_t>(b) * HP, m0, nP, X);
        stage_win<KB>(wn, uw, nullptr);
      }
      unit_forward<NH, KB, JB, NP, false, true>(a, sh, uw, X, mu, rr, nullptr, nullptr, &wr);
      if (g == 0 && c < nP) {
        const float sg = softplus_fast(rr) + 1e-10f;
        const int oq = a.s * c + (a.s - 1);
        const int o = t0 + oq;
        ob[a.swap_out ? (o ^ 1) : o] = uw[oq + a.k] * sg + mu;
        if (a.s == 2) {
          const int oe = t0 + 2 * c;
          ob[a.swap_out ? (oe ^ 1) : oe] = uw[2 * c + a.k];
        }
        if (o >= a.Lout - a.n_logsig) ls += __builtin_amdgcn_logf(sg) * kLn2;
      }
    }
    const float v = wave_sum(ls);
    if (lane == 0) ls_slab[static_cast<size_t>(ch) * a.B + b] = v;
  }
}

// ---------------------------------------------------------------------------
// backward kernel: one work item per wave; tiles outer, samples inner
// ---------------------------------------------------------------------------
template <int NH, int KB, int JB, int NP, bool FZ = false, bool DU = true>
__global__ __launch_bounds__(NT, 2) void bwd_kernel(KArgs a, const float* __restrict__ u, const float* __restrict__ C,
                                                    const int32_t* __restrict__ win, const float* __restrict__ tht,
                                                    const float* __restrict__ gout, const float* __restrict__ dls,
                                                    const bf8* __restrict__ img, const float* __restrict__ cst,
                                                    float* __restrict__ du, float* __restrict__ dC_slab,
                                                    float* __restrict__ dth_slab, float* __restrict__ dW_slab,
                                                    float* __restrict__ halo, FzArgs fz = FzArgs{}) {
  static_assert(!FZ || NH == 1, "the fused AR(1) ELBO variant has one hidden layer");
  // !DU (du == NULL): the gradient w.r.t. u is not wanted (the first flow's input is the base noise):
  // the transposed convolution, its carries and the du stores are compiled out (a runtime branch
  // around them measured 5 % slower for the launches that do need du)
  constexpr int wdu = DU ? 1 : 0;
  constexpr int PO = FZ ? P - 1 : P;  // output positions per tile (FZ: column 15 is look-ahead only)
  constexpr int NPL = NP == 3 ? 2 : 1;
  constexpr int KP = 16 * JB;  // carry slots (k <= KP)
  constexpr int NS = NH + 1;   // images: I_0 .. I_NH (reused for dZ_l and dA0)
  constexpr bool GI = NH == 1;              // the head gradient rides in the dZ image
  constexpr bool I0R = NH == 1 && NP == 1;  // elu'(I_0) from the recompute's bf16 pairs in registers
  __shared__ Shared<NH, KB, JB, NP> sh;
  __shared__ __bf16 timg[NW][NS][NPL][P * HP];  // [wave][slot][plane][p][h]
  __shared__ float dthl[NW][S][DTH];
  __shared__ __attribute__((aligned(16))) float dths[NW][4];  // sink for the d theta rows beyond DTH
  __shared__ float carry[NW][S][KP];
  __shared__ float gsc[NW][3][P];              // sigma, d r, go even (stride 2)
  __shared__ float uwin[NW][UW];
  __shared__ float gwin[NW][64];
  // dcon[j][p] stored at its output position q = s p + j of row j (other columns stay zero),
  // so du[q] = sum_{j<k} row_j[q] needs no masks
  // (k > 32: the [j][p] layout, row stride P + 1, summed along the diagonal q = s p + j -- at most P terms per q
  // -- keeps the block's LDS in bounds)
  constexpr bool PADDED = JB <= 2;
  constexpr int QW = PADDED ? 2 * P + KP : P + 1;
  __shared__ float dscr[NW][KP][QW];
  __shared__ float zls[FZ ? NW : 1][FZ ? S : 1][P];  // FZ: per-sample, per-column log sigma sums over the tiles
  __shared__ float zcar[FZ ? NW : 1][FZ ? S : 1];     // FZ: x at the previous tile's last position
  load_shared(sh, img, cst);
  // Static wave priority.  Each CU holds two blocks, so each SIMD one wave of each; blocks are dispatched
  // in rounds of (CU count) blocks and finish roughly in dispatch order, so a block of round r shares its
  // CU with one of round r - 1 or r + 1.  VALU issue between the two waves goes by priority, then age
  // (MI355X_MICROARCH.md, two waves per SIMD): the younger wave of a pair loses every tie and stalls.
  // Priority = dispatch round mod 4 makes the younger wave of a pair the prioritized one (except across
  // the wrap): 29.6 -> 28.8 ms per launch for the two-level (round & 1) form, 28.9 -> 28.8 more for mod 4;
  // by blockIdx parity (pairs of equal priority) no change; capped at 3 (ties from round 3 on) 29.5 ms;
  // by the wave's slot on its SIMD (hwreg HW_ID) 30.0 ms.
  {
    const int r = __builtin_amdgcn_readfirstlane(blockIdx.x / a.ncu) & 3;
    if (r == 1) __builtin_amdgcn_s_setprio(1);
    else if (r == 2) __builtin_amdgcn_s_setprio(2);
    else if (r == 3) __builtin_amdgcn_s_setprio(3);
  }
  if constexpr (FZ) {
    for (int i = threadIdx.x; i < NW * S * P; i += NT) (&zls[0][0][0])[i] = 0.f;
    for (int i = threadIdx.x; i < NW * S; i += NT) (&zcar[0][0])[i] = 0.f;
  }
  for (int i = threadIdx.x; i < NW * S * DTH; i += NT) (&dthl[0][0][0])[i] = 0.f;
  for (int i = threadIdx.x; i < NW * S * KP; i += NT) (&carry[0][0][0])[i] = 0.f;
  if constexpr (PADDED)
    for (int i = threadIdx.x; i < NW * KP * QW; i += NT) (&dscr[0][0][0])[i] = 0.f;
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  // Work items (sample group x t-chunk), one per wave; a block's waves are independent (no block-level
  // synchronisation follows)
  const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * NW + w);  // wave-uniform: scalar loads of per-sample data
  const int grp = item / a.n_chunks, chn = item % a.n_chunks;
  if (grp >= a.n_groups) return;
  const int m_lo = chn * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int b_lo = grp * a.S, nb = min(a.S, a.B - b_lo);
  __bf16* ih[NS];
  __bf16* il[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    ih[i] = timg[w][i][0];
    il[i] = timg[w][i][NPL - 1];
  }
  float* dsc = &dscr[w][0][0];
  float* mycarry = &carry[w][0][0];
  float* uw = uwin[w];
  float* gw = gwin[w];
  const unsigned* whp = reinterpret_cast<const unsigned*>(&sh.cst[NH * HP]);  // (mu, r) bf16 pairs

  f4 dW[NH][4][4], dWe[JB][4], dWh[4];
#pragma unroll
  for (int l = 0; l < NH; ++l)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int o = 0; o < 4; ++o) dW[l][i][o] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < JB; ++i)
#pragma unroll
    for (int o = 0; o < 4; ++o) dWe[i][o] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) dWh[i] = f4{0.f, 0.f, 0.f, 0.f};
  const bf4 ones4 = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};
  const int fwc = 16 * NH + 4 * KB;

  const int lwi = (win && lane < nb) ? win[b_lo + lane] : 0;
  const float ldl = (!FZ && lane < nb) ? dls[b_lo + lane] : 0.f;
  float lt0 = 0.f, lt1 = 0.f, lis = 0.f;  // FZ: theta_0, theta_1, e^{-theta_2} of sample b_lo + lane
  if constexpr (FZ) {
    if (lane < nb) {
      const float* tp = fz.theta + static_cast<size_t>(b_lo + lane) * 3;
      lt0 = tp[0];
      lt1 = tp[1];
      lis = __expf(-tp[2]);
    }
  }
  // FZ: a chunk after the first starts one tile early; that tile only provides x at position m_lo - 1
  const int m_start = (FZ && chn > 0) ? m_lo - PO : m_lo;
  for (int m0 = m_start; m0 < m_hi; m0 += PO) {
    const bool discard = FZ && m0 < m_lo;  // wave-uniform
    const int nP = discard ? 0 : min(PO, m_hi - m0), t0 = a.s * m0, fin = a.s * nP;
    const int nZ = FZ ? min(P, a.Lh - m0) : nP;  // columns with real inputs
    f4 dCa[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) dCa[rb] = f4{0.f, 0.f, 0.f, 0.f};
    for (int bl = 0; bl < nb; ++bl) {
      fence();
      const int b = b_lo + bl;
      const int wi = lane_i(lwi, bl);
      const float* Cw = C + static_cast<size_t>(wi) * a.Lh * HP;
      const float dl = FZ ? -fz.scale : lane_f(ldl, bl);
      f4 XN[4];
      float mu, rr;
      float fz_yp = 0.f, fz_bp = 0.f;  // FZ: the observation of x_t (row t - 1), loaded with the unit's inputs
      {
        if constexpr (FZ) {
          const size_t wo = static_cast<size_t>(wi) * fz.M + min(max(m0 + c - 1, 0), fz.M - 1);
          fz_yp = fz.obs[wo];
          fz_bp = fz.bin[wo];
        }
        Win<KB> wn;
        fetch_win<KB>(a, u + static_cast<size_t>(b) * a.pL, FZ ? nullptr : gout + static_cast<size_t>(b) * a.pLo, t0, wn);
        load_ct(Cw, tht + static_cast<size_t>(b) * HP, m0, nZ, XN);
        stage_win<KB>(wn, uw, gw);
      }
      // FZ: the previous tile's last x read with the unit's inputs, not after the recompute
      const float fz_zc = FZ ? zcar[w][bl] : 0.f;
      u2 i0p[4];
      unit_forward<NH, KB, JB, NP, true>(a, sh, uw, XN, mu, rr, ih, il, nullptr, I0R ? i0p : nullptr);
      // I_NH (the head input) with its ones row -> image NH, for dW_head
      put_image<NP>(ih[NH], il[NH], XN, g, c);

      // ---- head backward (per position p = c, redundant over g) ----
      const int oq = a.s * c + (a.s - 1);
      const bool pv = c < nP;
      const float sig = softplus_fast(rr) + 1e-10f;
      float gmu;
      if constexpr (FZ) {
        // x at t = m0 + c (column c < nZ), its neighbours from the adjacent columns / the carry
        const float x = uw[c + a.k] * sig + mu;
        float xp = row_prev(x);
        const float xn = row_next(x);
        if (c == 0) xp = fz_zc;
        if (discard) {
          if (lane == PO - 1) zcar[w][bl] = x;
          continue;
        }
        const float th0 = lane_f(lt0, bl), th1 = lane_f(lt1, bl), is = lane_f(lis, bl);
        const int t = m0 + c;
        // branch-free: every lane loads (clamped indices) and masks with 0 / 1 factors
        const float fh = (pv && t < fz.M) ? 1.f : 0.f;  // transition t: x_t -> x_{t+1}
        const float ft = (pv && t >= 1) ? 1.f : 0.f;    // transition t - 1 and its observation of x_t
        const float yp = fz_yp, bp = fz_bp * ft;
        const float zt = fh * (xn - th1 * x - th0) * is;
        const float zp = ft * (x - th1 * xp - th0) * is;
        // d(sde + obs)/dx_t
        const float de = th1 * zt * is - zp * is - bp * (x - yp) * (fz.iosd * fz.iosd);
        gmu = -fz.scale * de;  // 0 for columns without an output
        const float lsg = (t0 + oq >= a.Lout - a.n_logsig) ? __logf(sig) : 0.f;
        if (g == 0) {
          gw[c] = gmu;  // the upstream-gradient window the rest of the unit reads
          if (pv) {
            fz.x[static_cast<size_t>(b) * (fz.M + 1) + t] = x;
            zls[w][bl][c] += lsg;
          }
        }
        if (lane == PO - 1 && nP == PO) zcar[w][bl] = x;
      } else {
        gmu = pv ? gw[oq] : 0.f;
      }
      float dsig = gmu * uw[oq + a.k];
      if (pv && t0 + oq >= a.Lout - a.n_logsig) dsig += dl * rcp_f(sig);
      const float gr = dsig * sigmoid_fast(rr);
      if (g == 0) {
        gsc[w][0][c] = sig;
        if constexpr (!GI) gsc[w][1][c] = gr;
        if (a.s == 2) gsc[w][2][c] = pv ? gw[2 * c] : 0.f;
      }
      fence();
      // GI: the head gradient G rides in two padding rows of the dZ image (below); the I_NH
      // fragments of dW_head are read now, before that image overwrites I_NH's slot
      Fr4<NP> i1f[4];
      if constexpr (GI) {
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) i1f[hb] = tr_frag<NP>(ih[NH], il[NH], hb, g, c);
      } else {
        // dW_head[h][o] += sum_p I_NH[h][p] G[o][p]: B fragment G[p = 4 g + jj][o = c]
        f4 gv4;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int p = 4 * g + jj;
          const float g0 = p < nP ? gw[a.s * p + (a.s - 1)] : 0.f;
          const float g1 = gsc[w][1][p];
          gv4[jj] = c == 0 ? g0 : (c == 1 ? g1 : 0.f);
        }
        const Fr4<NP> gf = split4<NP>(gv4);
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) dWh[hb] = mm<NP>(tr_frag<NP>(ih[NH], il[NH], hb, g, c), gf, dWh[hb]);
      }
      // dZ_{NH-1} = (w~_mu gmu + w~_r gr) * elu'(I_NH) -> image NH: the rank-2 outer product is
      // one K = 16 MFMA per row block, A[h][o] = W~h[16 rb + h][o], B[o][p] = (gmu, gr)[o] at p = c
      // (only k-group g = 0 carries the two nonzero k rows)
      // (one hidden layer: the dX weight fragments, dW's I_0 fragments and dW_eps's u fragments read before the
      // head-backward VALU)
      Fr8<NP> wb[8];
      Fr4<NP> xa0[4];
      Fr4<NP> uaf[JB];
      if constexpr (NH == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) wb[i] = wfrag(sh, 8 * NH + i, lane);
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) xa0[ib] = tr_frag<NP>(ih[0], il[0], ib, g, c);
#pragma unroll
        for (int jb = 0; jb < JB; ++jb) uaf[jb] = ua_frag<NP>(uw, a.s, jb, g, c);
        __builtin_amdgcn_sched_barrier(0);
      }
      f4 D[4];
      {
        const bool g0 = g == 0;
        const Fr4<NP> gf2 = split4<NP>(f4{g0 ? gmu : 0.f, g0 ? gr : 0.f, 0.f, 0.f});
        unsigned wvh[4], wvl[4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          wvh[rb] = whp[16 * rb + c];
          if constexpr (NP >= 2) wvl[rb] = whp[HP + 16 * rb + c];
        }
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          Fr4<NP> wa;
          wa.h = __builtin_bit_cast(bf4, u2{g0 ? wvh[rb] : 0u, 0u});
          if constexpr (NP >= 2) wa.l = __builtin_bit_cast(bf4, u2{g0 ? wvl[rb] : 0u, 0u});
          D[rb] = mm_w4<NP>(wa, gf2, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int r = 0; r < 4; ++r) D[rb][r] = 4 * rb + r < NR ? D[rb][r] * elu_d(XN[rb][r]) : 0.f;
        }
        if constexpr (GI) {
          // padding rows 53, 54 (register (3, 1), (3, 2) of lane group 1): (g_mu, g_r) at p = c.
          // The dX weights are zero there and dW ignores those rows.
          D[3][1] = g == 1 ? gmu : 0.f;
          D[3][2] = g == 1 ? gr : 0.f;
        }
      }
      put_image<NP>(ih[NH], il[NH], D, g, c);
      Fr8<NP> wcp[2 * JB];  // (one hidden layer: the dcon fragments, read before elu'(I_0))
      // (DWL, one hidden layer: the dW / dW_head MFMAs deferred past the du section's dcon stores, from the dZ
      //  image's four fragments read at their usual place; block 3 is also dW_head's B operand)
      constexpr bool DWL = NH == 1;
      Fr4<NP> dzf[4];
      auto dw_late = [&]() {
#pragma unroll
        for (int ib = 0; ib < 4; ++ib)
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) dW[0][ib][ob] = mm<NP>(xa0[ib], dzf[ob], dW[0][ib][ob]);
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) dWh[hb] = mm<NP>(i1f[hb], dzf[3], dWh[hb]);
      };
      // hidden layers, top down: dI_l = W~_l dZ_l (chain); dW_l += I_l dZ_l^T; dZ_{l-1} = dI_l elu'(I_l)
#pragma unroll
      for (int l = NH - 1; l >= 0; --l) {
        fence();
        f4 dX[4];
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) dX[ib] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const Fr8<NP> df = chain_frag<NP>(D, ks);
#pragma unroll
          for (int ib = 0; ib < 4; ++ib)
            dX[ib] = mm<NP>(NH == 1 ? wb[ib * 2 + ks] : wfrag(sh, 8 * NH + l * 8 + ib * 2 + ks, lane), df, dX[ib]);
        }
        fence();
        if constexpr (DWL) {
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) dzf[ob] = tr_frag<NP>(ih[1], il[1], ob, g, c);
        }
#pragma unroll
        for (int ib = 0; ib < 4 * !DWL; ++ib) {
          const Fr4<NP> xa = tr_frag<NP>(ih[l], il[l], ib, g, c);
#pragma unroll
          for (int ob = 0; ob < 4; ++ob)
            dW[l][ib][ob] = mm<NP>(xa, tr_frag<NP>(ih[l + 1], il[l + 1], ob, g, c), dW[l][ib][ob]);
        }
        if constexpr (GI && !DWL) {
          // dW_head[h][o] += sum_p I_1[h][p] G[o][p]: B = rows 48..63 of the dZ image, columns
          // c = 5, 6 of the product hold o = 0, 1 (padding rows 53, 54)
          const Fr4<NP> gb = tr_frag<NP>(ih[NH], il[NH], 3, g, c);
#pragma unroll
          for (int hb = 0; hb < 4; ++hb) dWh[hb] = mm<NP>(i1f[hb], gb, dWh[hb]);
        }
        if constexpr (NH == 1) {
#pragma unroll
          for (int i = 0; i < 2 * JB; ++i) wcp[i] = wfrag(sh, fwc + i, lane);
          __builtin_amdgcn_sched_barrier(0);
        }
        // D <- dZ_{l-1} (or dA0 for l = 0) from I_l (read back from its image; row 63 held 1
        // where dI is 0)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          f4 x;
          if constexpr (I0R) {  // I_0 from the registers the forward left (same bf16 values as the image)
            x = f4{__builtin_bit_cast(float, i0p[rb][0] << 16), __builtin_bit_cast(float, i0p[rb][0] & 0xffff0000u),
                   __builtin_bit_cast(float, i0p[rb][1] << 16), __builtin_bit_cast(float, i0p[rb][1] & 0xffff0000u)};
          } else {
            x = get_own<NP>(ih[l], il[l], rb, g, c);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) D[rb][r] = 4 * rb + r < NR ? dX[rb][r] * elu_d(x[r]) : 0.f;
        }
        if (l > 0) put_image<NP>(ih[l], il[l], D, g, c);
      }
      // dcon[j][p] = sum_h w_eps[j][h] dA0[h][p]; dC tile += dA0
      fence();
      f4 dcn[JB];
#pragma unroll
      for (int jb = 0; jb < JB; ++jb) dcn[jb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2 * wdu; ++ks) {
        const Fr8<NP> df = chain_frag<NP>(D, ks);
#pragma unroll
        for (int jb = 0; jb < JB; ++jb)
          dcn[jb] = mm<NP>(NH == 1 ? wcp[jb * 2 + ks] : wfrag(sh, fwc + jb * 2 + ks, lane), df, dcn[jb]);
      }
      // dC tile += dA0 (same lane layout): fp32 adds on the unit-carrying registers (an identity-selection MFMA
      // measured slower in this kernel)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * rb + r < NR) dCa[rb][r] += D[rb][r];
      // dA0 -> image 1; dW_eps and d theta from its position-contracted fragments
      put_image<NP>(ih[1], il[1], D, g, c);
      fence();
      f4 dth4[4] = {};
#pragma unroll
      for (int hb = 0; hb < 4; ++hb) {
        const Fr4<NP> ta = tr_frag<NP>(ih[1], il[1], hb, g, c);
        dth4[hb] = mm_bx<NP>(ta, ones4, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int jb = 0; jb < JB; ++jb)
          dWe[jb][hb] = mm<NP>(NH == 1 ? uaf[jb] : ua_frag<NP>(uw, a.s, jb, g, c), ta, dWe[jb][hb]);
      }
      // the four read-modify-writes with their reads issued together: rows 16 hb + 4 g beyond DTH (hb = 3, g >= 2:
      // padding and the ones row) go to a per-wave scratch slot instead of a branch around them (every column of
      // dth4 holds the same sums)
      if (c == 0) {
        float* base = &dthl[w][bl][4 * g];
        f4* dp[4];
#pragma unroll
        for (int hb = 0; hb < 4; ++hb)
          dp[hb] = reinterpret_cast<f4*>(16 * hb + 4 * g < DTH ? base + 16 * hb : &dths[w][0]);
        f4 o[4];
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) o[hb] = *dp[hb];
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) *dp[hb] = o[hb] + dth4[hb];
      }
      if constexpr (DU) {
#pragma unroll
      for (int jb = 0; jb < JB; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 16 * jb + 4 * g + r;
          dsc[j * QW + (PADDED ? a.s * c + j : c)] = dcn[jb][r];
        }
      }
      if constexpr (DWL) dw_late();
      // du over local positions q in [0, fin + k): transposed conv + pass-through + carry
      if constexpr (DU) {
        float* db = du + static_cast<size_t>(b) * a.pL;
        // fin + k <= 64 when PADDED (k <= 32), <= 96 otherwise
        constexpr int NBASE = PADDED ? 1 : 2;
        const int lim = fin + a.k;
#pragma unroll
        for (int it = 0; it < NBASE; ++it) {
          const int base = 64 * it;
          if (base >= lim) break;
          const int q = base + lane;
          float v = 0.f;
          if constexpr (PADDED) {
            const int qc = q < QW ? q : QW - 1;
            if (a.k == 8) {
              // k = 8 (the AR configurations): all reads issued before the first add, then a pairwise sum (a chain of
              // serial adds had the compiler wait on each read in turn)
              constexpr int KF = 8;
              float t[KF];
#pragma unroll
              for (int j = 0; j < KF; ++j) t[j] = dsc[j * QW + qc];
#pragma unroll
              for (int w2 = 1; w2 < KF; w2 *= 2)
#pragma unroll
                for (int j = 0; j + w2 < KF; j += 2 * w2) t[j] += t[j + w2];
              v = t[0];
            } else {
#pragma unroll 4
              for (int j = 0; j < a.k; ++j) v += dsc[j * QW + qc];
            }
          } else {
            // the diagonal q = s p + j over the tile's P positions (columns p >= nP hold zeros: their gradients
            // are zero); row stride P + 1 puts the 64 lanes' reads of one p in 64 distinct banks.  (Round 2 summed
            // all k rows with a mask per term: SV's k = 50 made the du section 46 % of the launch.)
#pragma unroll
            for (int p = 0; p < P; ++p) {
              const int j = q - a.s * p;
              const bool ok = static_cast<unsigned>(j) < static_cast<unsigned>(a.k);
              const float x = dsc[(ok ? j : 0) * QW + p];
              v += ok ? x : 0.f;
            }
          }
          const int oq2 = q - a.k;
          if (oq2 >= 0 && oq2 < fin) {
            if (a.s == 1) v += gw[oq2] * gsc[w][0][oq2];
            else v += (oq2 & 1) ? gw[oq2] * gsc[w][0][oq2 >> 1] : gsc[w][2][oq2 >> 1];
          }
          const float cin = mycarry[bl * KP + (q < a.k ? q : 0)];
          if (q < a.k) v += cin;
          if (q < fin) db[t0 + q] = v;
          else if (q < fin + a.k) mycarry[bl * KP + q - fin] = v;
        }
      }
    }
    // tile done: its dC over the group
    if (c < nP) {
      const size_t row = (static_cast<size_t>(grp) * a.Lh + m0 + c) * a.H;
      if (a.dc16) {  // (bf16 partials: each rounding is independent, the reduce sums 4096 of them in fp32)
        __bf16* dcs = reinterpret_cast<__bf16*>(dC_slab) + row;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = swz(16 * rb + 4 * g + r);
            if (h < a.H) dcs[h] = static_cast<__bf16>(dCa[rb][r] * kLog2e);
          }
      } else {
        float* dcs = dC_slab + row;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = swz(16 * rb + 4 * g + r);
            if (h < a.H) dcs[h] = dCa[rb][r] * kLog2e;
          }
      }
    }
  }

  if constexpr (FZ) {
    if (lane < nb) {  // lane bl: its sample's columns in order
      float v = 0.f;
#pragma unroll
      for (int cc = 0; cc < P; ++cc) v += zls[w][lane][cc];
      fz.lsl[static_cast<size_t>(chn) * a.B + b_lo + lane] = v;
    }
  }
  // ---- per-sample tails: carry -> halo / du tail; d theta -> slab ----
  for (int bl = 0; bl < nb; ++bl) {
    const int b = b_lo + bl;
    for (int q = lane; q < a.k * wdu; q += 64) {
      const float v = mycarry[bl * KP + q];
      if (chn == a.n_chunks - 1) du[static_cast<size_t>(b) * a.pL + a.Lout + q] = v;
      else halo[(static_cast<size_t>(b) * a.n_chunks + chn) * a.k + q] = v;
    }
    if (lane < a.H) dth_slab[(static_cast<size_t>(chn) * a.B + b) * a.H + lane] = dthl[w][bl][swz(lane)] * kLog2e;
  }

  // ---- weight-gradient partials of this work item (layout of flow4's n_wgrad; folded-BN form:
  //      scatter_wgrad_kernel recovers the BN and unfolded weight gradients) ----
  const int H = a.H;
  const int nW = a.k * H + NH * H * H + 3 * NH * H + 2 * H + 2;
  float* ws = dW_slab + static_cast<size_t>(item) * nW;
#pragma unroll
  for (int jb = 0; jb < JB; ++jb)
#pragma unroll
    for (int hb = 0; hb < 4; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * jb + 4 * g + r, h = swz(16 * hb + c);
        if (j < a.k && h < H) ws[j * H + h] = dWe[jb][hb][r] * kLog2e;
      }
  const int off_w = a.k * H, off_b = off_w + NH * H * H;
#pragma unroll
  for (int l = 0; l < NH; ++l)
#pragma unroll
    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
      for (int ob = 0; ob < 4; ++ob)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int hi = swz(16 * ib + 4 * g + r), ho = swz(16 * ob + c);
          if (ho < H) {
            if (hi < H) ws[off_w + (l * H + hi) * H + ho] = dW[l][ib][ob][r];
            else if (hi == 63) ws[off_b + l * H + ho] = dW[l][ib][ob][r] * kLog2e;  // ones row: bias
          }
        }
  for (int i = lane; i < 2 * NH * H; i += 64) ws[off_b + NH * H + i] = 0.f;  // bn: recovered at scatter
  const int off_h = off_b + 3 * NH * H;
  const int oh = GI ? c - 5 : c;  // output column of dW_head's product -> head output o
  if (oh == 0 || oh == 1) {
#pragma unroll
    for (int hb = 0; hb < 4; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = swz(16 * hb + 4 * g + r);
        if (h < H) ws[off_h + h * 2 + oh] = dWh[hb][r] * kLn2;
        else if (h == 63) ws[off_h + 2 * H + oh] = dWh[hb][r];  // ones row: head bias gradient
      }
  }
}

// ---------------------------------------------------------------------------
// backward kernel, two samples per unit ("bwd2"): the AR configurations' flow shape (one hidden layer,
// bf16 products, k <= KP2, stride 1, one window)
//
// A unit is (two samples of the group) x (tile of 16 head positions).  The two samples' dependency chains
// (recompute -> head backward -> dX -> dA0 -> dcon -> transposed conv) run interleaved in one wave, so each
// covers the other's MFMA and LDS latencies; the weight fragments, the C rows and the dC tile accumulator
// are shared by the pair; and every product that contracts over positions (dW, dW_head, dW_eps, d theta)
// contracts over the pair's 32 columns with one v_mfma_f32_16x16x32_bf16 (K = 32: k = 8g + jj is sample
// jj >> 2, position 4g + (jj & 3), i.e. the two samples' ds_read_b64_tr_b16 fragments side by side), half
// the 16x16x16 instructions of the one-sample kernel at the same matrix-pipe cycles each.  d theta is per
// sample: one MFMA against a ones operand split by sample (columns 0-7 sample A, 8-15 sample B).
// Blocks of 8 waves (one block per CU, two waves per SIMD) stage the weight images once.
// A group with an odd sample count pairs its last sample with a ghost (sample A again, upstream gradient
// zero: every contribution of the ghost is exactly zero and its stores are skipped).
// ---------------------------------------------------------------------------
constexpr int NW2 = 8;
constexpr int NT2 = 64 * NW2;
// lanes 32..63 of v into lanes 0..31 (v_permlane32_swap); lanes 32..63 of the result keep v's
__device__ __forceinline__ float swap_hi_lo(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                  false, false);
  return __builtin_bit_cast(float, static_cast<unsigned>(r[1]));
}
constexpr int KP2 = 8;  // carry slots / dcon rows (k <= 8)
// Design decisions (A/B, AR-cfg launches; docs/DESIGN_HISTORY.md §4 / §8):
//  * compiler fences between the unit's phases in the fused (FZ) variant (without them: middle flows 23.3 ->
//    22.4 ms, the fused one 26.8 -> 28.2, the first flow unchanged) and, since round 5, in the first flow's variant
//    without du (18.31 -> 18.07 ms; the middle flows with them 20.57 -> 20.88: profiles/r05/ab_sched_strategies.log);
//  * the recompute's ELU select as v_med3 (one instruction fewer per element): 93.3 -> 91.4 ms per AR-cfg step;
//  * a t-chunk's look-back tile (fused variant) runs the whole unit with every gradient zero (nP = 0 masks them): a
//    branch out after the recompute split the unit into basic blocks the scheduler cannot interleave across;
//  * the dC tile summed by a K = 32 MFMA over the pair's dA0 image fragments against a position-selection B operand
//    instead of fp32 VALU adds of the dA0 accumulators (-0.4 ms per step);
//  * dW_eps accumulated transposed ([h][tap]) by one K = 32 MFMA per row block whose B operand's columns 8..15 carry
//    one-hot sample columns: the same product sums d theta for 8 samples, flushed to the LDS rows every fourth pair
//    (4 MFMAs and 3 of 4 read-modify-writes fewer per pair; -1.7 ms per step);
//  * fused variant: the tile's observations (per position) loaded once per tile; log sigma on v_log_f32 (sigma >=
//    1e-10 is a normal float); per-sample log sigma column sums in LDS at bf16 (through two padding rows of the dA0
//    image into the merged dW_eps / d theta product in the split-weight recompute variant, whose lo weight planes
//    take that LDS; no change at bf16).
// Rejected: elu'(I_1) = min(2^x', 1) from the recompute's exp kept to the head backward (+1 ms per step: registers);
// per-sample d theta for the whole item in a [h][16 samples] MFMA accumulator (16 more registers: 60 spilled);
// s_setprio 1 for the second wave on each SIMD (-0.2 ms, noise).
#ifndef VISSM_NODU_FENCES
#define VISSM_NODU_FENCES 1   // (A/B switch: 0 leaves the first flow's variant without phase fences)
#endif
template <bool FZ>
__device__ __forceinline__ void fence2() {
  if constexpr (FZ) fence();
}

// the K = 32 fragment of a position contraction: sample A's transposed fragment then sample B's
__device__ __forceinline__ bf8 cat8(bf4 a, bf4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf8 tr_frag2(const __bf16* img, int hb, int g, int c) {
  return cat8(tr_read(img, hb, g, c), tr_read(img + P * HP, hb, g, c));
}

// NPR = 2: the forward recompute -- the values that reach the ELBO through x and log sigma, and every activation
// the backward differentiates at -- on split weights (w_hi u + w_lo u, the bf16x2 forward's products; lo planes of
// the recompute's fragments in LDS).  SB (split backward, needs NPR = 2; VISSM_PREC_BF16X2): the backward chain's
// weight products too -- the head backward W~h (g_mu, g_r), dX = W~ dZ, dcon = w_eps dA0 -- as w_hi x + w_lo x; the
// position contractions (dW, dW_eps, dW_head, d theta, dC: activation x gradient operands) stay single bf16
// products, whose independent per-position roundings average out.  CPU emulation at the AR-cfg length
// (scripts/bf16_grad_emul.py): gradient 2.5e-3 (bf16) / 2.2e-3 (bf16x2f: split forward only) -> 7e-5 with SB.
// NPR = 2 without SB: the bf16x2f host mode's fused last flow (VISSM_PREC_BF16X2_BF16: backward products bf16).
template <bool FZ, bool DU, bool TF, int NPR = 1, bool SB = false>
__global__ __launch_bounds__(NT2, 2) void bwd2_kernel(KArgs a, const float* __restrict__ u, const float* __restrict__ C,
                                                      const float* __restrict__ tht, const float* __restrict__ gout,
                                                      const float* __restrict__ dls, const bf8* __restrict__ img,
                                                      const float* __restrict__ cst, float* __restrict__ du,
                                                      float* __restrict__ dC_slab, float* __restrict__ dth_slab,
                                                      float* __restrict__ dW_slab, float* __restrict__ halo,
                                                      const u4* __restrict__ thf, FzArgs fz = FzArgs{}) {
  static_assert(!SB || NPR == 2, "the split backward chain goes with the split recompute");
  constexpr int NH = 1, KB = 1, JB = 1, NP = 1;
  constexpr bool LOF = NPR == 2 && !kLoFoldOff;  // the recompute's layer-0 / head lo products in spare rows (k <= 8)
  constexpr int PO = FZ ? P - 1 : P;
  constexpr int QW2 = P + KP2;  // dcon[j][p] stored at column p + j: du[q] = sum_j row_j[q], no masks
  // u window entries: the layer-0 fragment reads up to c + 8 g + 7 <= 46 (48 in the split-weight variants, whose
  // lo planes need the LDS; 64 otherwise: an unmasked store, the measured bf16 code)
  constexpr int UWN = NPR == 2 ? 48 : 64;
  __shared__ Shared<NH, KB, JB, NP> sh;
  __shared__ __bf16 timg[NW2][2][2 * P * HP];  // [wave][slot][row 16 cb + position][64 h]
  __shared__ float dthl[NW2][S][DTH];
  __shared__ __attribute__((aligned(16))) float dths[NW2][4];
  __shared__ float carry[NW2][S][KP2];
  __shared__ float uwin[NW2][2][UWN];
  // the upstream gradient g_mu at p (read by the head backward); NPR = 2 (LDS for the lo planes): then overwritten
  // with g_mu sigma, the du pass-through term, instead of keeping sigma in gsc
  __shared__ float gwin[NW2][2][P];
  __shared__ float gsc[NPR == 2 ? 1 : NW2][2][P];
  __shared__ float dscr[NW2][2][KP2][QW2];
  constexpr bool ZLS = FZ && NPR == 1;  // per-column log sigma sums in LDS
  __shared__ float zls[ZLS ? NW2 : 1][ZLS ? S : 1][P];
  // lo planes: NPR = 2 the recompute's WF 0..7 and WH 0..1 (slo[0..9]); SB the backward chain's WB 0..7 and WC 0..1
  // (slo[RO..RO + 9]); the layer-0 WE 0..3 lo planes are nonzero in lane group 0 only (rows j < k <= 8; the theta
  // fold's rows are exact bf16 splits): swe[ob][c]
  constexpr int RO = NPR == 2 ? 10 : 0, NLO = RO + (SB ? 10 : 0);
  __shared__ bf8 slo[NLO > 0 ? NLO : 1][64];
  __shared__ bf8 swe[NPR == 2 ? 4 : 1][16];
  __shared__ float zcar[FZ ? NW2 : 1][FZ ? S : 1];
  if constexpr (NPR == 2) {  // the image holds [frag][hi, lo][lane]: hi planes to sh, the lo planes to slo / swe
    constexpr int NFR = Shared<NH, KB, JB, NP>::NFR;
    for (int i = threadIdx.x; i < NFR * 64; i += NT2) sh.img[i >> 6][0][i & 63] = img[((i >> 6) * 2) * 64 + (i & 63)];
    for (int i = threadIdx.x; i < NLO * 64; i += NT2) {
      const int j = i >> 6;
      const int f = j < 8 ? j                                            // WF
                  : j < 10 ? 16 * NH + 4 * KB + 2 * JB + (j - 8)         // WH
                  : j < 18 ? 8 * NH + (j - 10)                           // WB
                           : 16 * NH + 4 * KB + (j - 18);                // WC
      slo[j][i & 63] = img[(f * 2 + 1) * 64 + (i & 63)];
    }
    for (int i = threadIdx.x; i < 4 * 16; i += NT2) swe[i >> 4][i & 15] = img[((16 * NH + (i >> 4)) * 2 + 1) * 64 + (i & 15)];
    for (int i = threadIdx.x; i < Shared<NH, KB, JB, NP>::NCST; i += NT2) sh.cst[i] = cst[i];
  } else {
    load_shared<NH, KB, JB, NP, NT2>(sh, img, cst);
  }
  if constexpr (FZ) {
    if constexpr (ZLS)
      for (int i = threadIdx.x; i < NW2 * S * P; i += NT2) (&zls[0][0][0])[i] = 0.f;
    for (int i = threadIdx.x; i < NW2 * S; i += NT2) (&zcar[0][0])[i] = 0.f;
  }
  for (int i = threadIdx.x; i < NW2 * S * DTH; i += NT2) (&dthl[0][0][0])[i] = 0.f;
  for (int i = threadIdx.x; i < NW2 * S * KP2; i += NT2) (&carry[0][0][0])[i] = 0.f;
  for (int i = threadIdx.x; i < NW2 * 2 * KP2 * QW2; i += NT2) (&dscr[0][0][0][0])[i] = 0.f;
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * NW2 + w);
  const int grp = __builtin_amdgcn_readfirstlane(item / a.n_chunks);
  const int chn = __builtin_amdgcn_readfirstlane(item % a.n_chunks);
  if (grp >= a.n_groups) return;
  const int m_lo = chn * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int b_lo = grp * a.S, nb = min(a.S, a.B - b_lo);
  __bf16* const im0 = timg[w][0];  // I_0
  __bf16* const im1 = timg[w][1];  // I_1, then dZ, then dA0
  const unsigned* whp = reinterpret_cast<const unsigned*>(&sh.cst[NH * HP]);  // (mu, r) bf16 pairs

  f4 dW[4][4], dWe[4], dWh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int o = 0; o < 4; ++o) dW[i][o] = f4{0.f, 0.f, 0.f, 0.f};
    dWe[i] = f4{0.f, 0.f, 0.f, 0.f};
    dWh[i] = f4{0.f, 0.f, 0.f, 0.f};
  }
  const int fwc = 16 * NH + 4 * KB;
  // the dC selection operand: B[k = 8g + jj][n = c] = 1 if k's position 4g + (jj & 3) is column n (either sample)
  bf8 sel_p;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) sel_p[jj] = (__bf16)((4 * g + (jj & 3) == c) ? 1.f : 0.f);

  const float ldl = (!FZ && lane < nb) ? dls[b_lo + lane] : 0.f;
  float lt0 = 0.f, lt1 = 0.f, lis = 0.f;
  if constexpr (FZ) {
    if (lane < nb) {
      const float* tp = fz.theta + static_cast<size_t>(b_lo + lane) * 3;
      lt0 = tp[0];
      lt1 = tp[1];
      lis = __expf(-tp[2]);
    }
  }
  const int m_start = (FZ && chn > 0) ? m_lo - PO : m_lo;
  const int nu = a.k + P;  // u entries a unit reads (stride 1)
  for (int m0 = m_start; m0 < m_hi; m0 += PO) {
    const bool discard = FZ && m0 < m_lo;
    const int nP = discard ? 0 : min(PO, m_hi - m0), t0 = m0;
    const int nZ = FZ ? min(P, a.Lh - m0) : nP;
    f4 dCa[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) dCa[rb] = f4{0.f, 0.f, 0.f, 0.f};
    float fz_yt = 0.f, fz_bt = 0.f;  // FZ: the observation of x_t (row t - 1) at p = c, once per tile
    if constexpr (FZ) {
      const int wo = min(max(m0 + c - 1, 0), fz.M - 1);
      fz_yt = fz.obs[wo];
      fz_bt = fz.bin[wo];
    }
    for (int bl = 0; bl < nb; bl += 2) {
      fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
      const bool two = bl + 1 < nb;  // wave-uniform; else the second slot is a ghost
      const int blv[2] = {bl, two ? bl + 1 : bl};
      const int bv[2] = {b_lo + blv[0], b_lo + blv[1]};
      // ---- inputs: the two u windows (and upstream-gradient windows), the shared C rows + each theta row
      f4 X[2][4];
      bf8 tfr[2];
      float fz_yp = fz_yt, fz_bp = fz_bt, fz_zc[2] = {0.f, 0.f};
      {
        float uv[2], gv[2] = {0.f, 0.f};
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const float* ub = u + static_cast<size_t>(bv[cb]) * a.pL;
          uv[cb] = lane < nu ? ub[clampi(t0 + lane, a.L)] : 0.f;
          if constexpr (!FZ) {
            if (lane < P) gv[cb] = gout[static_cast<size_t>(bv[cb]) * a.pLo + clampi(t0 + lane, a.Lout)];
          }
        }
        if (!two) gv[1] = 0.f;
        const f4* crow = reinterpret_cast<const f4*>(C + static_cast<size_t>(m0 + clampi(c, nZ)) * HP) + g;
        f4 cr[4], tr[2][4];
        if constexpr (TF) {  // the theta fold: the pair's theta rows of the layer-0 B operand (lane groups 2, 3)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) tfr[cb] = __builtin_bit_cast(bf8, thf[2 * static_cast<size_t>(bv[cb]) + (g & 1)]);
        }
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          cr[rb] = crow[4 * rb];
          if constexpr (!TF) {
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
              tr[cb][rb] = (reinterpret_cast<const f4*>(tht + static_cast<size_t>(bv[cb]) * HP) + g)[4 * rb];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          if (UWN == 64 || lane < UWN) uwin[w][cb][lane] = uv[cb];
          if (lane < P) gwin[w][cb][lane] = gv[cb];
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) X[cb][rb] = TF ? cr[rb] : cr[rb] + tr[cb][rb];
        }
        if constexpr (FZ) {
          fz_zc[0] = zcar[w][blv[0]];
          fz_zc[1] = zcar[w][blv[1]];
        }
      }
      // ---- forward recompute of both samples (shared weight fragments)
      u2 i0p[2][4];
      u2 d0p[2][4], d1p[2][4];  // VISSM_DERIV16: elu'(A0), elu'(A1) as f16 pairs
      float mu[2], rr[2];
      {
        f4 acc[2][4];
        fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
        const int gu = (LOF && g == 1) ? 0 : g;  // LOF: lane group 1's K rows repeat the taps 0..7 (lo weights)
        Fr8<NP> uf[2] = {u_frag<NP>(uwin[w][0], 1, 0, gu, c), u_frag<NP>(uwin[w][1], 1, 0, gu, c)};
        if constexpr (TF) {
          if (g >= 2) {
            uf[0].h = tfr[0];
            uf[1].h = tfr[1];
          }
        }
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) {
          const Fr8<NP> wf = wfrag(sh, 16 * NH + ob, lane);
          bf8 wel = {};
          if constexpr (NPR == 2 && !LOF) {
            const bf8 v = swe[ob][c];
            if (g == 0) wel = v;
          }
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            acc[cb][ob] = X[cb][ob];
            if constexpr (NPR == 2 && !LOF) acc[cb][ob] = mfma32(wel, uf[cb].h, acc[cb][ob]);
            acc[cb][ob] = mm<NP>(wf, uf[cb], acc[cb][ob]);
          }
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            float e[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (VISSM_DERIV16 >= 1) X[cb][rb][r] = 4 * rb + r < NR ? elu_dv(acc[cb][rb][r], e[r]) : 0.f;
              else X[cb][rb][r] = 4 * rb + r < NR ? elu_fast<true>(acc[cb][rb][r]) : 0.f;
            }
            if (VISSM_DERIV16 >= 1) {
              d0p[cb][rb] = u2{pk_f16(e[0], e[1]), 4 * rb + 2 < NR ? pk_f16(e[2], e[3]) : 0u};
              pin_pair(d0p[cb][rb]);
            }
          }
        fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          if (g == 3) X[cb][3][3] = 1.f;  // the ones row: bias of the hidden layer
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) acc[cb][ob] = f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          Fr8<NP> xf[2] = {chain_frag<NP>(X[0], ks), chain_frag<NP>(X[1], ks)};
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) {
            const Fr8<NP> wf = wfrag(sh, ob * 2 + ks, lane);
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
              if constexpr (NPR == 2) acc[cb][ob] = mfma32(slo[ob * 2 + ks][lane], xf[cb].h, acc[cb][ob]);
              acc[cb][ob] = mm<NP>(wf, xf[cb], acc[cb][ob]);
            }
          }
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          put_image<NP>(im0 + cb * P * HP, nullptr, X[cb], g, c);  // I_0 with its ones row
          if (VISSM_DERIV16 == 0) {
#pragma unroll
            for (int rb = 0; rb < 4; ++rb) i0p[cb][rb] = u2{cvt2(X[cb][rb][0], X[cb][rb][1]), cvt2(X[cb][rb][2], X[cb][rb][3])};
          }
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            float e[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (VISSM_DERIV16 >= 2) X[cb][rb][r] = 4 * rb + r < NR ? elu_dv(acc[cb][rb][r], e[r]) : 0.f;
              else X[cb][rb][r] = 4 * rb + r < NR ? elu_fast<true>(acc[cb][rb][r]) : 0.f;
            }
            if (VISSM_DERIV16 >= 2) {
              d1p[cb][rb] = u2{pk_f16(e[0], e[1]), 4 * rb + 2 < NR ? pk_f16(e[2], e[3]) : 0u};
              pin_pair(d1p[cb][rb]);
            }
          }
        fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
        const int fh = 16 * NH + 4 * KB + 2 * JB;
        f4 d[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          if (g == 3) X[cb][3][3] = 1.f;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const Fr8<NP> wf = wfrag(sh, fh + ks, lane);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            const Fr8<NP> xk = chain_frag<NP>(X[cb], ks);
            if constexpr (NPR == 2 && !LOF) d[cb] = mfma32(slo[8 + ks][lane], xk.h, d[cb]);
            d[cb] = mm<NP>(wf, xk, d[cb]);
          }
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          mu[cb] = LOF ? d[cb][0] + d[cb][2] : d[cb][0];
          rr[cb] = LOF ? d[cb][1] + d[cb][3] : d[cb][1];
          put_image<NP>(im1 + cb * P * HP, nullptr, X[cb], g, c);  // I_1 (head input) with its ones row
        }
      }
      // ---- head backward
      const bool pv = c < nP;
      float gmu[2], gr[2];
      float lsv[2] = {0.f, 0.f};  // fused variant without the LDS column sums: the output columns' log sigma
      if constexpr (FZ) {
        // Fused last flow: both samples' head backward in one pass: lane groups 0, 1 evaluate sample A's columns and
        // 2, 3 sample B's (the head MFMA left every column's (mu, r) in all four groups), so the softplus / sigmoid /
        // AR(1) transition and observation gradient work runs once per pair instead of once per sample;
        // v_permlane32_swap then brings B's (g_mu, g_r) from groups 2, 3 to 0, 1, where the dZ product's B operand
        // (group 0) and the I_1 image rows (group 1) take them.  Fused flow 23.8 -> 23.4 ms per AR-cfg launch; the
        // unfused variants' lighter head gains nothing from it (first flow +0.3 ms, middle +0.0,
        // profiles/r05/ab_step.log), so they keep the per-sample form below.
        const int hs = g >> 1;                      // the sample of this lane's head work
        const bool hv = hs == 0 || two;             // not the ghost
        const float mu_h = hs ? mu[1] : mu[0], rr_h = hs ? rr[1] : rr[0];
        const float sig_h = softplus_fast(rr_h) + 1e-10f;
        const float uk = uwin[w][hs][c + a.k];
        const float x = uk * sig_h + mu_h;
        float xp = row_prev(x);
        const float xn = row_next(x);
        if (c == 0) xp = hs ? fz_zc[1] : fz_zc[0];
        const int bl2 = hs ? blv[1] : blv[0];
        const float th0 = hs ? lane_f(lt0, blv[1]) : lane_f(lt0, blv[0]);
        const float th1 = hs ? lane_f(lt1, blv[1]) : lane_f(lt1, blv[0]);
        const float is = hs ? lane_f(lis, blv[1]) : lane_f(lis, blv[0]);
        const int t = m0 + c;
        const float fh = (pv && t < fz.M) ? 1.f : 0.f;
        const float ft = (pv && t >= 1) ? 1.f : 0.f;
        const float bp = fz_bp * ft;
        const float zt = fh * (xn - th1 * x - th0) * is;
        const float zp = ft * (x - th1 * xp - th0) * is;
        const float de = th1 * zt * is - zp * is - bp * (x - fz_yp) * (fz.iosd * fz.iosd);
        const float gmu_h = hv ? -fz.scale * de : 0.f;
        const float lsg = (t0 + c >= a.Lout - a.n_logsig) ? __builtin_amdgcn_logf(sig_h) * kLn2 : 0.f;
        if ((g & 1) == 0) {  // lane groups 0 (A) and 2 (B)
          if constexpr (NPR == 1) gwin[w][hs][c] = gmu_h;  // the upstream-gradient window the du section reads
          if (pv && hv) {
            if constexpr (!(VISSM_ABL_STORES & 1)) fz.x[static_cast<size_t>(b_lo + bl2) * (fz.M + 1) + t] = x;
            if constexpr (ZLS) zls[w][bl2][c] += lsg;
          }
        }
        if ((lane & 31) == PO - 1 && (nP == PO || discard) && hv) zcar[w][bl2] = x;
        float dsig = gmu_h * uk;
        if (pv && hv && t0 + c >= a.Lout - a.n_logsig) dsig += -fz.scale * rcp_f(sig_h);
        const float gr_h = dsig * sigmoid_fast(rr_h);
        if ((g & 1) == 0) {
          if constexpr (NPR == 2) {
            if constexpr (DU) gwin[w][hs][c] = gmu_h * sig_h;  // (after the reads of g_mu above: LDS order)
          } else {
            gsc[w][hs][c] = sig_h;
          }
        }
        gmu[0] = gmu_h;
        gr[0] = gr_h;
        gmu[1] = swap_hi_lo(gmu_h);
        gr[1] = swap_hi_lo(gr_h);
        if constexpr (!ZLS) {
          const float lsv_h = (pv && hv) ? lsg : 0.f;
          lsv[0] = lsv_h;
          lsv[1] = swap_hi_lo(lsv_h);
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          if (g == 1) {  // G = (g_mu, g_r) into the I_1 image's padding rows 53, 54 (as below)
            const int off = timg_off(c, 4 * 3 + 1);
            *reinterpret_cast<u2*>(im1 + cb * P * HP + off) = u2{cvt2(X[cb][3][0], gmu[cb]), cvt2(gr[cb], X[cb][3][3])};
          }
        }
      } else {
        float sig[2];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          sig[cb] = softplus_fast(rr[cb]) + 1e-10f;
          gmu[cb] = pv ? gwin[w][cb][c] : 0.f;
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const float dl = lane_f(ldl, blv[cb]);
          float dsig = gmu[cb] * uwin[w][cb][c + a.k];
          if (pv && (cb == 0 || two) && t0 + c >= a.Lout - a.n_logsig) dsig += dl * rcp_f(sig[cb]);
          gr[cb] = dsig * sigmoid_fast(rr[cb]);
          if (g == 0) {
            if constexpr (NPR == 2) {
              if constexpr (DU) gwin[w][cb][c] = gmu[cb] * sig[cb];  // (after the reads of g_mu above: LDS order)
            } else {
              gsc[w][cb][c] = sig[cb];
            }
          }
          // the head gradient G = (g_mu, g_r) at p = c into the I_1 image's padding rows 53, 54 (register (3, 1),
          // (3, 2) of lane group 1; unit 49 in row 52 rewritten unchanged): dW_head = I_1 G^T then takes both
          // operands from this one image, before the dZ image overwrites its slot
          if (g == 1) {
            const int off = timg_off(c, 4 * 3 + 1);
            *reinterpret_cast<u2*>(im1 + cb * P * HP + off) = u2{cvt2(X[cb][3][0], gmu[cb]), cvt2(gr[cb], X[cb][3][3])};
          }
        }
      }
      fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
      // dW_head[h][o] += sum over both samples' positions of I_1[h][p] G[o][p] (K = 32): block 3 of the same
      // fragments is the B operand (its columns 5, 6 are the G rows)
      {
        bf8 i1f[4];
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) i1f[hb] = tr_frag2(im1, hb, g, c);
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) dWh[hb] = mfma32(i1f[hb], i1f[3], dWh[hb]);
      }
      // dZ = (w~_mu g_mu + w~_r g_r) * elu'(I_1): one K = 16 MFMA per row block per sample
      f4 D[2][4];
      {
        unsigned wvh[4], wvl[4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          wvh[rb] = whp[16 * rb + c];
          if constexpr (SB) wvl[rb] = whp[HP + 16 * rb + c];  // the lo plane of the (mu, r) pairs
        }
        const bool g0 = g == 0;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const bf4 gf2 = __builtin_bit_cast(bf4, u2{cvt2(g0 ? gmu[cb] : 0.f, g0 ? gr[cb] : 0.f), 0u});
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            const bf4 wa = __builtin_bit_cast(bf4, u2{g0 ? wvh[rb] : 0u, 0u});
            f4 d0 = f4{0.f, 0.f, 0.f, 0.f};
            if constexpr (SB) d0 = mfma16(__builtin_bit_cast(bf4, u2{g0 ? wvl[rb] : 0u, 0u}), gf2, d0);
            D[cb][rb] = mfma16(wa, gf2, d0);
          }
        }
        fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
          for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (VISSM_DERIV16 >= 2) D[cb][rb][r] = 4 * rb + r < NR ? mul_h(D[cb][rb][r], d1p[cb][rb][r >> 1], r & 1) : 0.f;
              else D[cb][rb][r] = 4 * rb + r < NR ? D[cb][rb][r] * elu_d(X[cb][rb][r]) : 0.f;
            }
          put_image<NP>(im1 + cb * P * HP, nullptr, D[cb], g, c);
        }
      }
      fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
      // dX = W~ dZ (chain), both samples
      f4 dX[2][4];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) dX[cb][ib] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        Fr8<NP> df[2] = {chain_frag<NP>(D[0], ks), chain_frag<NP>(D[1], ks)};
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) {
          const Fr8<NP> wb = wfrag(sh, 8 * NH + ib * 2 + ks, lane);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            if constexpr (SB) dX[cb][ib] = mfma32(slo[RO + ib * 2 + ks][lane], df[cb].h, dX[cb][ib]);
            dX[cb][ib] = mm<NP>(wb, df[cb], dX[cb][ib]);
          }
        }
      }
      fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
      // dW += I_0 dZ^T over both samples' positions (K = 32), from the two images
      {
        bf8 dzf[4];
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) dzf[ob] = tr_frag2(im1, ob, g, c);
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) {
          const bf8 xa = tr_frag2(im0, ib, g, c);
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) dW[ib][ob] = mfma32(xa, dzf[ob], dW[ib][ob]);
        }
      }
      // dA0 = dX * elu'(I_0) (I_0 from the registers the forward left: the image's bf16 values)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          if (VISSM_DERIV16 >= 1) {
#pragma unroll
            for (int r = 0; r < 4; ++r) D[cb][rb][r] = 4 * rb + r < NR ? mul_h(dX[cb][rb][r], d0p[cb][rb][r >> 1], r & 1) : 0.f;
          } else {
            const f4 x = {__builtin_bit_cast(float, i0p[cb][rb][0] << 16), __builtin_bit_cast(float, i0p[cb][rb][0] & 0xffff0000u),
                          __builtin_bit_cast(float, i0p[cb][rb][1] << 16), __builtin_bit_cast(float, i0p[cb][rb][1] & 0xffff0000u)};
#pragma unroll
            for (int r = 0; r < 4; ++r) D[cb][rb][r] = 4 * rb + r < NR ? dX[cb][rb][r] * elu_d(x[r]) : 0.f;
          }
        }
      // dcon[j][p] = sum_h w_eps[j][h] dA0[h][p] per sample; the dC tile += dA0 of both
      f4 dcn[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
      if constexpr (DU) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const Fr8<NP> wc = wfrag(sh, fwc + ks, lane);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            const Fr8<NP> dk = chain_frag<NP>(D[cb], ks);
            if constexpr (SB) dcn[cb] = mfma32(slo[RO + 8 + ks][lane], dk.h, dcn[cb]);
            dcn[cb] = mm<NP>(wc, dk, dcn[cb]);
          }
        }
      }
      if constexpr (FZ && !ZLS) {
        // the log sigma of the pair's output columns rides in two padding rows of the dA0 image (register (3, 1):
        // row 49 = unit 52 <- hi, row 53 = unit 53 <- lo of a split-bf16 pair), so the merged dW_eps / d theta
        // product sums it per sample with d theta (its other outputs there are discarded padding units)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const float hi = bf16_hi(lsv[cb]);
          D[cb][3][1] = g == 0 ? hi : (g == 1 ? lsv[cb] - hi : 0.f);
        }
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) put_image<NP>(im1 + cb * P * HP, nullptr, D[cb], g, c);  // dA0 -> slot 1
      if constexpr (DU) {
        // dcon stores (rows j < KP2: lane groups 0, 1)
        if (g < KP2 / 4) {
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r) dscr[w][cb][4 * g + r][c + 4 * g + r] = dcn[cb][r];
        }
      }
      fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
      // dW_eps and d theta from dA0's position-contracted fragments (K = 32)
      {
        const unsigned one2 = 0x3F803F80u;
        bf8 uaf;
        {
          const Fr4<NP> ua = ua_frag<NP>(uwin[w][0], 1, 0, g, c), ub = ua_frag<NP>(uwin[w][1], 1, 0, g, c);
          uaf = cat8(ua.h, ub.h);
        }
        // one B operand for dW_eps^T (columns j < 8: the u windows) and the d theta of the pair's two samples
        // (columns 8 + slot: one-hot by sample, slot = sample mod 8)
        bf8 bcomb = uaf;
        {
          const unsigned ta_ = c - 8 == (blv[0] & 7) ? one2 : 0u, tb_ = (two && c - 8 == (blv[1] & 7)) ? one2 : 0u;
          if (c >= 8) bcomb = __builtin_bit_cast(bf8, u4{ta_, ta_, tb_, tb_});
        }
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) {
          const bf8 ta = tr_frag2(im1, hb, g, c);
          dWe[hb] = mfma32(ta, bcomb, dWe[hb]);
          dCa[hb] = mfma32(ta, sel_p, dCa[hb]);
        }
      }
      // the eight sample columns flushed into the per-sample d theta rows after every fourth pair and after the
      // tile's last, then cleared
      {
        if ((bl & 7) == 6 || bl + 2 >= nb) {
          const int smp = (bl & ~7) + c - 8;
          if (c >= 8 && smp < nb) {
            float* base = &dthl[w][smp][4 * g];
            f4* dp[4];
#pragma unroll
            for (int hb = 0; hb < 4; ++hb)
              dp[hb] = reinterpret_cast<f4*>(16 * hb + 4 * g < DTH ? base + 16 * hb : &dths[w][0]);
            f4 o[4];
#pragma unroll
            for (int hb = 0; hb < 4; ++hb) o[hb] = *dp[hb];
#pragma unroll
            for (int hb = 0; hb < 4; ++hb) *dp[hb] = o[hb] + dWe[hb];
          }
#pragma unroll
          for (int hb = 0; hb < 4; ++hb)
            if (c >= 8) dWe[hb] = f4{0.f, 0.f, 0.f, 0.f};
        }
      }
      // du over local positions q in [0, nP + k) for both samples at once: lane = 32 cb + q
      if constexpr (DU) {
        fence2<FZ || (!DU && VISSM_NODU_FENCES)>();
        const int cbq = lane >> 5, q = lane & 31;
        const int lim = nP + a.k;
        const bool act = q < lim && (cbq == 0 || two);
        const int blq = cbq ? blv[1] : blv[0];
        float v = 0.f;
        if (act) {
          const int qc = q < QW2 ? q : QW2 - 1;
          float t[KP2];
#pragma unroll
          for (int j = 0; j < KP2; ++j) t[j] = dscr[w][cbq][j][qc];
#pragma unroll
          for (int w2 = 1; w2 < KP2; w2 *= 2)
#pragma unroll
            for (int j = 0; j + w2 < KP2; j += 2 * w2) t[j] += t[j + w2];
          v = t[0];
          const int oq2 = q - a.k;
          if (oq2 >= 0 && oq2 < nP) v += NPR == 2 ? gwin[w][cbq][oq2] : gwin[w][cbq][oq2] * gsc[w][cbq][oq2];
          if (q < a.k) v += carry[w][blq][q];
        }
        // (16-byte du stores of full aligned tiles -- four lanes' values gathered by DPP row shifts -- measured 0.2 ms
        // slower per middle-flow launch and no fewer PMC write bytes (4.05 vs 4.07 GB), profiles/r05/ab_step.log)
        if (act) {
          float* const dur = du + static_cast<size_t>(b_lo + blq) * a.pL + t0;
          if (q < nP) {
            if constexpr (!(VISSM_ABL_STORES & 2)) dur[q] = v;
          } else {
            carry[w][blq][q - nP] = v;
          }
        }
      }
    }
    // tile done: its dC over the group (both samples of every pair)
    if (c < nP && !(VISSM_ABL_STORES & 4)) {
      const size_t row = (static_cast<size_t>(grp) * a.Lh + m0 + c) * a.H;
      if (a.dc16) {
        __bf16* dcs = reinterpret_cast<__bf16*>(dC_slab) + row;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = swz(16 * rb + 4 * g + r);
            if (h < a.H) dcs[h] = static_cast<__bf16>(dCa[rb][r] * kLog2e);
          }
      } else {
        float* dcs = dC_slab + row;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = swz(16 * rb + 4 * g + r);
            if (h < a.H) dcs[h] = dCa[rb][r] * kLog2e;
          }
      }
    }
  }

  if constexpr (FZ) {
    if (lane < nb) {
      float v = 0.f;
      if constexpr (!ZLS) {
        v = dthl[w][lane][49] + dthl[w][lane][53];
      } else {
#pragma unroll
        for (int cc = 0; cc < P; ++cc) v += zls[w][lane][cc];
      }
      fz.lsl[static_cast<size_t>(chn) * a.B + b_lo + lane] = v;
    }
  }
  for (int bl = 0; bl < nb; ++bl) {
    const int b = b_lo + bl;
    if constexpr (DU) {
      if (lane < a.k) {
        const float v = carry[w][bl][lane];
        if (chn == a.n_chunks - 1) du[static_cast<size_t>(b) * a.pL + a.Lout + lane] = v;
        else halo[(static_cast<size_t>(b) * a.n_chunks + chn) * a.k + lane] = v;
      }
    }
    if (lane < a.H) dth_slab[(static_cast<size_t>(chn) * a.B + b) * a.H + lane] = dthl[w][bl][swz(lane)] * kLog2e;
  }

  // weight-gradient partials of this work item (the layout of bwd_kernel's)
  const int H = a.H;
  const int nW = a.k * H + NH * H * H + 3 * NH * H + 2 * H + 2;
  float* ws = dW_slab + static_cast<size_t>(item) * nW;
#pragma unroll
  for (int hb = 0; hb < 4; ++hb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // dWe^T: lane column c = tap, rows h
      const int ht = swz(16 * hb + 4 * g + r);
      if (c < a.k && ht < H) ws[c * H + ht] = dWe[hb][r] * kLog2e;
    }
  const int off_w = a.k * H, off_b = off_w + NH * H * H;
#pragma unroll
  for (int ib = 0; ib < 4; ++ib)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hi = swz(16 * ib + 4 * g + r), ho = swz(16 * ob + c);
        if (ho < H) {
          if (hi < H) ws[off_w + hi * H + ho] = dW[ib][ob][r];
          else if (hi == 63) ws[off_b + ho] = dW[ib][ob][r] * kLog2e;
        }
      }
  for (int i = lane; i < 2 * NH * H; i += 64) ws[off_b + NH * H + i] = 0.f;
  const int off_h = off_b + 3 * NH * H;
  const int oh = c - 5;
  if (oh == 0 || oh == 1) {
#pragma unroll
    for (int hb = 0; hb < 4; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = swz(16 * hb + 4 * g + r);
        if (h < H) ws[off_h + h * 2 + oh] = dWh[hb][r] * kLn2;
        else if (h == 63) ws[off_h + 2 * H + oh] = dWh[hb][r];
      }
  }
}

// ---------------------------------------------------------------------------
// forward kernel, two samples per unit ("fwd2"): the AR configurations' shape (one hidden layer, bf16, k <= 16,
// stride 1, one window).  Pairs of samples outer, tiles inner: the pair's two chains run interleaved in one
// wave and share the tile's C rows and every weight fragment (register-resident).  It also runs the three-hidden-
// layer forward (LV / FHN heads, k <= 32; SV's 32 < k <= 64 at stride 1 with two layer-0 K blocks and a 128-entry u
// window) and the bf16x2 forward of the parity-precision modes.
// ---------------------------------------------------------------------------
// TF: the theta fold (VissmFlowParams.theta_rank): the theta term rides in the layer-0 product's K rows 16..31
// (lane groups 2, 3 of the B operand: the sample's fragment thf[b][g - 2], loaded once per pair) instead of a
// [64] theta_term row per sample and tile added to the C rows
// NP = 2: the bf16x2 forward (split weights w_hi x + w_lo x, bf16 activations; the parity-precision modes'
// forward): hi planes register-resident, lo planes read from LDS per use
// NH / JB: one hidden layer (AR) or three with the BN affine folded (LV / SV / FHN heads: stride-2 head with the
// pass-through of the even outputs and the fused pair swap), k <= 32 (one layer-0 K block)
// LOF (NP = 2, k <= 8: prep_kernel's lofold): the layer-0 and head lo products ride in the hi fragments' spare rows
template <bool TF, int NP, int NH, int JB, int NWF = NW, bool LOF = false>
__global__ __launch_bounds__(64 * NWF, 2) void fwd2_kernel(KArgs a, const float* __restrict__ u,
                                                                  const float* __restrict__ C,
                                                                  const float* __restrict__ tht,
                                                                  const bf8* __restrict__ img,
                                                                  const float* __restrict__ cst,
                                                                  float* __restrict__ u_next,
                                                                  float* __restrict__ ls_slab,
                                                                  const u4* __restrict__ thf) {
  constexpr int KB = (JB + 1) / 2;  // layer-0 K blocks (k > 32: two, a 128-entry u window)
  __shared__ Shared<NH, KB, JB, NP> sh;
  __shared__ float uwin[NWF][2][64 * KB];
  load_shared<NH, KB, JB, NP, 64 * NWF>(sh, img, cst);
  {  // static wave priority = dispatch round mod 4 (as fwd_kernel)
    const int r = __builtin_amdgcn_readfirstlane(blockIdx.x / a.ncu) & 3;
    if (r == 1) __builtin_amdgcn_s_setprio(1);
    else if (r == 2) __builtin_amdgcn_s_setprio(2);
    else if (r == 3) __builtin_amdgcn_s_setprio(3);
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * NWF + w);
  if (item >= a.n_items) return;
  const int grp = item / a.n_chunks, ch = item % a.n_chunks;
  const int m_lo = ch * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int b_lo = grp * a.S, nb = min(a.S, a.B - b_lo);
  // weight hi planes register-resident in 4-wave blocks; 8-wave blocks read every plane from LDS (fewer registers, and
  // the block's LDS image serves twice the waves)
  constexpr bool HIREG = NWF == NW;
  constexpr int NWR = HIREG ? 8 * NH + 4 * KB + 2 : 1;
  bf8 wr[NWR];
  // (VISSM_X2_HIDREG, 8-wave split-weight blocks with lofold: the hidden layer's hi planes register-resident)
  constexpr bool HIDREG = !HIREG && LOF && VISSM_X2_HIDREG;
  bf8 wrh[HIDREG ? 8 * NH : 1];
  if constexpr (HIDREG) {
#pragma unroll
    for (int i = 0; i < 8 * NH; ++i) wrh[i] = sh.img[i][0][lane];
  }
  if constexpr (HIREG) {
#pragma unroll
    for (int i = 0; i < 8 * NH; ++i) wr[i] = sh.img[i][0][lane];
#pragma unroll
    for (int i = 0; i < 4 * KB; ++i) wr[8 * NH + i] = sh.img[16 * NH + i][0][lane];
#pragma unroll
    for (int i = 0; i < 2; ++i) wr[8 * NH + 4 * KB + i] = sh.img[16 * NH + 4 * KB + 2 * JB + i][0][lane];
  }
  // fragment f: its hi plane's register copy (index i); NP = 2: with its lo plane from LDS
  auto W = [&](int f, int i) -> Fr8<NP> {
    Fr8<NP> r;
    if constexpr (HIREG) r.h = wr[i];
    else if (HIDREG && f < 8 * NH) r.h = wrh[HIDREG ? f : 0];
    else r.h = sh.img[f][0][lane];
    if constexpr (NP == 2) r.l = sh.img[f][1][lane];
    return r;
  };
  // weight (A) x activation (B, bf16) product at the kernel's precision
  auto mmw = [](const Fr8<NP>& a, const bf8& b, f4 cc) -> f4 {
    if constexpr (NP == 2) cc = mfma32(a.l, b, cc);
    return mfma32(a.h, b, cc);
  };
  // one hidden layer: the AR shape (stride 1, no swap: fwd2_ok) as compile-time constants
  const int ss = NH == 1 ? 1 : a.s;
  const bool swp = NH == 1 ? false : a.swap_out != 0;
  const int nu = ss * P + a.k;  // u entries a unit reads (<= 64 KB)
  for (int bl = 0; bl < nb; bl += 2) {
    const bool two = bl + 1 < nb;
    const int bv[2] = {b_lo + bl, b_lo + (two ? bl + 1 : bl)};
    float ls[2] = {0.f, 0.f};
    bf8 tfr[2];  // TF: the pair's theta rows of the B operand (lane groups 2, 3)
    if constexpr (TF) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) tfr[cb] = __builtin_bit_cast(bf8, thf[2 * static_cast<size_t>(bv[cb]) + (g & 1)]);
    }
    for (int m0 = m_lo; m0 < m_hi; m0 += P) {
      const int nP = min(P, m_hi - m0), t0 = ss * m0;
      f4 X[2][4];
      {
        float uv[2][KB];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int i = 0; i < KB; ++i)
            uv[cb][i] = 64 * i + lane < nu ? u[static_cast<size_t>(bv[cb]) * a.pL + clampi(t0 + 64 * i + lane, a.L)] : 0.f;
        const f4* crow = reinterpret_cast<const f4*>(C + static_cast<size_t>(m0 + clampi(c, nP)) * HP) + g;
        f4 cr[4], tr[2][4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          cr[rb] = crow[4 * rb];
          if constexpr (!TF) {
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
              tr[cb][rb] = (reinterpret_cast<const f4*>(tht + static_cast<size_t>(bv[cb]) * HP) + g)[4 * rb];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
          for (int i = 0; i < KB; ++i) uwin[w][cb][64 * i + lane] = uv[cb][i];
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) X[cb][rb] = TF ? cr[rb] : cr[rb] + tr[cb][rb];
        }
      }
      f4 acc[2][4];
      {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          const int gu = (LOF && g == 1) ? 0 : g;  // LOF: lane group 1's K rows repeat the taps 0..7 (lo weights)
          bf8 uf[2] = {u_frag<1>(uwin[w][0], ss, kb, gu, c).h, u_frag<1>(uwin[w][1], ss, kb, gu, c).h};
          if constexpr (TF) {
            if (g >= 2) {
              uf[0] = tfr[0];
              uf[1] = tfr[1];
            }
          }
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) {
            if constexpr (LOF) {
              const bf8 wh = HIREG ? wr[8 * NH + 4 * kb + ob] : sh.img[16 * NH + 4 * kb + ob][0][lane];
#pragma unroll
              for (int cb = 0; cb < 2; ++cb) acc[cb][ob] = mfma32(wh, uf[cb], kb == 0 ? X[cb][ob] : acc[cb][ob]);
            } else {
              const Fr8<NP> wf = W(16 * NH + 4 * kb + ob, 8 * NH + 4 * kb + ob);
#pragma unroll
              for (int cb = 0; cb < 2; ++cb) acc[cb][ob] = mmw(wf, uf[cb], kb == 0 ? X[cb][ob] : acc[cb][ob]);
            }
          }
        }
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) X[cb][rb][r] = 4 * rb + r < NR ? elu_fast<true>(acc[cb][rb][r]) : 0.f;
#pragma unroll
      for (int l = 0; l < NH; ++l) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          if (g == 3) X[cb][3][3] = 1.f;  // the ones row: bias of layer l
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) acc[cb][ob] = f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf8 xf[2] = {chain_frag<1>(X[0], ks).h, chain_frag<1>(X[1], ks).h};
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) {
            const Fr8<NP> wf = W(l * 8 + ob * 2 + ks, l * 8 + ob * 2 + ks);
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) acc[cb][ob] = mmw(wf, xf[cb], acc[cb][ob]);
          }
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) X[cb][rb][r] = 4 * rb + r < NR ? elu_fast<true>(acc[cb][rb][r]) : 0.f;
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
        if (g == 3) X[cb][3][3] = 1.f;
      const int fh = 16 * NH + 4 * KB + 2 * JB;
      f4 d[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (LOF) {
          const bf8 wh = HIREG ? wr[8 * NH + 4 * KB + ks] : sh.img[fh + ks][0][lane];
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) d[cb] = mfma32(wh, chain_frag<1>(X[cb], ks).h, d[cb]);
        } else {
          const Fr8<NP> wf = W(fh + ks, 8 * NH + 4 * KB + ks);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) d[cb] = mmw(wf, chain_frag<1>(X[cb], ks).h, d[cb]);
        }
      }
      if constexpr (LOF) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          d[cb][0] += d[cb][2];
          d[cb][1] += d[cb][3];
        }
      }
      if (g == 0 && c < nP) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          if (cb == 1 && !two) break;
          const float sg = softplus_fast(d[cb][1]) + 1e-10f;
          const int oq = ss * c + (ss - 1), o = t0 + oq;
          float* ob = u_next + static_cast<size_t>(bv[cb]) * a.pLo;
          ob[swp ? (o ^ 1) : o] = uwin[w][cb][oq + a.k] * sg + d[cb][0];
          if (ss == 2) {  // the even outputs pass through (lotka_volterra_partial.py:97-104)
            const int oe = t0 + 2 * c;
            ob[swp ? (oe ^ 1) : oe] = uwin[w][cb][2 * c + a.k];
          }
          if (o >= a.Lout - a.n_logsig) ls[cb] += __builtin_amdgcn_logf(sg) * kLn2;
        }
      }
    }
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const float v = wave_sum(ls[cb]);
      if (lane == 0 && (cb == 0 || two)) ls_slab[static_cast<size_t>(ch) * a.B + bv[cb]] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// backward kernel for three hidden layers (LV / SV / FHN heads, BN affine folded), two samples per unit
// ("bwd2n").  The one-sample kernel above holds dW for three layers (192 registers) and runs one wave per
// SIMD with nothing to cover its latencies (round-3 counters: half of a wave's cycles parked at s_waitcnt,
// profiles/r03/bwd_nh3_counters_lv_B4096.txt).  Here the wave interleaves two samples' chains as bwd2_kernel
// does, with the position contractions at K = 32 over the pair; the hidden activations I_0 .. I_3 stay in
// registers as bf16 pairs (what the one-sample kernel read back from its images) and each is written into the
// wave's image slot 0 only when its weight gradient is formed, next to D_l in slot 1, so two 32-row image
// slots per wave suffice (the one-sample kernel kept four 16-row slots).  k <= 24 (any stride) or 32 < k <= 64
// (stride 1: SV), one window.
// ---------------------------------------------------------------------------
constexpr int NW3 = 4;
constexpr int NT3 = 64 * NW3;

__device__ __forceinline__ void put_pairs(__bf16* img, const u2 (&v)[4], int g, int c) {
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) *reinterpret_cast<u2*>(img + timg_off(c, 4 * rb + g)) = v[rb];
}
__device__ __forceinline__ f4 unpack_pair(u2 v) {
  return f4{__builtin_bit_cast(float, v[0] << 16), __builtin_bit_cast(float, v[0] & 0xffff0000u),
            __builtin_bit_cast(float, v[1] << 16), __builtin_bit_cast(float, v[1] & 0xffff0000u)};
}

template <int JB, bool S2, bool DU>
__global__ __launch_bounds__(NT3, 1) void bwd2n_kernel(KArgs a, const float* __restrict__ u, const float* __restrict__ C,
                                                       const float* __restrict__ tht, const float* __restrict__ gout,
                                                       const float* __restrict__ dls, const bf8* __restrict__ img,
                                                       const float* __restrict__ cst, float* __restrict__ du,
                                                       float* __restrict__ dC_slab, float* __restrict__ dth_slab,
                                                       float* __restrict__ dW_slab, float* __restrict__ halo) {
  constexpr int NH = 3, KB = (JB + 1) / 2, NP = 1;
  static_assert(JB <= 2 || !S2, "k > 32: stride 1 only");
  constexpr int s = S2 ? 2 : 1;
  constexpr int KP = 16 * JB;
  // dcon rows: k <= 24 (JB <= 2) at column s p + j of row j (padded: du[q] = sum_j row_j[q], no masks); k > 32 in
  // [j][p] rows of stride P + 1 (no room for padded rows), summed along the diagonal q = p + j (at most P terms)
  constexpr bool DIAG = JB > 2;
  // dW / dW_eps / dW_head accumulate in AGPRs through inline asm (mfma32_a*) at k <= 32; at k > 32 (SV) the compiler
  // copies those operands between register files around the statements (scripts/check_agpr_asm.py finds the copies
  // within an MFMA's wait states), so the builtin form stays there
  constexpr bool AACC = VISSM_BWD2N_AACC && JB <= 2;
  // elu' as f16 pairs (VISSM_DERIV16) at k <= 32 in the variant without du (with du: LV 15.8 -> 16.6 ms per launch);
  // SV's k > 32 build has no registers to spare for them
  constexpr bool DV = VISSM_DERIV16 >= 2 && JB <= 2 && !DU;
  constexpr int KR = JB == 1 ? 16 : JB == 2 ? 24 : KP;
  constexpr int QWR = DIAG ? P + 1 : s * P + KR;
  constexpr int UWN = KB == 1 ? 64 : 128;    // u entries staged per sample (s P + k of them read)
  __shared__ Shared<NH, KB, JB, NP> sh;
  __shared__ __bf16 timg[NW3][2][2 * P * HP];  // slot 0: I_l, slot 1: D_l, then dA0
  __shared__ float dthl[NW3][S][DTH];
  __shared__ __attribute__((aligned(16))) float dths[NW3][4];
  __shared__ float carry[NW3][S][KP];
  __shared__ float gsc[NW3][2][2][P];  // per sample: sigma, the even outputs' pass-through gradient (stride 2)
  __shared__ float uwin[NW3][2][UWN];
  __shared__ float gwin[NW3][2][s * P];
  __shared__ float dscr[NW3][KR][QWR];  // one sample at a time
  load_shared<NH, KB, JB, NP, NT3>(sh, img, cst);
  for (int i = threadIdx.x; i < NW3 * S * DTH; i += NT3) (&dthl[0][0][0])[i] = 0.f;
  for (int i = threadIdx.x; i < NW3 * S * KP; i += NT3) (&carry[0][0][0])[i] = 0.f;
  for (int i = threadIdx.x; i < NW3 * KR * QWR; i += NT3) (&dscr[0][0][0])[i] = 0.f;
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * NW3 + w);
  const int grp = __builtin_amdgcn_readfirstlane(item / a.n_chunks);
  const int chn = __builtin_amdgcn_readfirstlane(item % a.n_chunks);
  if (grp >= a.n_groups) return;
  const int m_lo = chn * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int b_lo = grp * a.S, nb = min(a.S, a.B - b_lo);
  __bf16* const im0 = timg[w][0];
  __bf16* const im1 = timg[w][1];
  const unsigned* whp = reinterpret_cast<const unsigned*>(&sh.cst[NH * HP]);

  f4 dW[NH][4][4], dWe[JB][4], dWh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int l = 0; l < NH; ++l)
#pragma unroll
      for (int o = 0; o < 4; ++o) dW[l][i][o] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jb = 0; jb < JB; ++jb) dWe[jb][i] = f4{0.f, 0.f, 0.f, 0.f};
    dWh[i] = f4{0.f, 0.f, 0.f, 0.f};
  }
  const int fwc = 16 * NH + 4 * KB, fh = 16 * NH + 4 * KB + 2 * JB;
  bf8 ones_ab;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) ones_ab[jj] = (__bf16)(((jj < 4) == (c < 8)) ? 1.f : 0.f);
  const float ldl = lane < nb ? dls[b_lo + lane] : 0.f;
  const int nu = s * P + a.k;
  for (int m0 = m_lo; m0 < m_hi; m0 += P) {
    const int nP = min(P, m_hi - m0), t0 = s * m0, fin = s * nP;
    f4 dCa[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) dCa[rb] = f4{0.f, 0.f, 0.f, 0.f};
    for (int bl = 0; bl < nb; bl += 2) {
      fence();
      const bool two = bl + 1 < nb;
      const int blv[2] = {bl, two ? bl + 1 : bl};
      const int bv[2] = {b_lo + blv[0], b_lo + blv[1]};
      f4 X[2][4];
      {
        float uv[2][UWN / 64], gv[2] = {0.f, 0.f};
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
          for (int i = 0; i < UWN / 64; ++i)
            uv[cb][i] = lane + 64 * i < nu ? u[static_cast<size_t>(bv[cb]) * a.pL + clampi(t0 + lane + 64 * i, a.L)] : 0.f;
          if (lane < s * P) {
            const int o = t0 + lane;
            gv[cb] = gout[static_cast<size_t>(bv[cb]) * a.pLo + clampi(a.swap_out ? (o ^ 1) : o, a.Lout)];
          }
        }
        if (!two) gv[1] = 0.f;
        const f4* crow = reinterpret_cast<const f4*>(C + static_cast<size_t>(m0 + clampi(c, nP)) * HP) + g;
        f4 cr[4], tr[2][4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          cr[rb] = crow[4 * rb];
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
            tr[cb][rb] = (reinterpret_cast<const f4*>(tht + static_cast<size_t>(bv[cb]) * HP) + g)[4 * rb];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
          for (int i = 0; i < UWN / 64; ++i) uwin[w][cb][lane + 64 * i] = uv[cb][i];
          if (lane < s * P) gwin[w][cb][lane] = gv[cb];
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) X[cb][rb] = cr[rb] + tr[cb][rb];
        }
      }
      // ---- forward recompute of both samples; I_0 .. I_NH kept as bf16 pairs (with the ones row)
      u2 ip[NH + 1][2][4];
      u2 dp[DV ? NH + 1 : 1][2][4];  // DV: elu'(I_0 .. I_NH) as f16 pairs (VISSM_DERIV16)
      // the ELU of both samples' accumulators, with (DV) its derivative pairs
      auto elu_pairs = [&](const f4 (&ac)[2][4], f4 (&Y)[2][4], u2 (&dd)[2][4]) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            float e[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if constexpr (DV) Y[cb][rb][r] = 4 * rb + r < NR ? elu_dv(ac[cb][rb][r], e[r]) : 0.f;
              else Y[cb][rb][r] = 4 * rb + r < NR ? elu_fast<true>(ac[cb][rb][r]) : 0.f;
            }
            if constexpr (DV) {
              dd[cb][rb] = u2{pk_f16(e[0], e[1]), 4 * rb + 2 < NR ? pk_f16(e[2], e[3]) : 0u};
              pin_pair(dd[cb][rb]);
            }
          }
      };
      float mu[2], rr[2];
      {
        f4 acc[2][4];
        fence();
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          const Fr8<NP> uf[2] = {u_frag<NP>(uwin[w][0], s, kb, g, c), u_frag<NP>(uwin[w][1], s, kb, g, c)};
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) {
            const Fr8<NP> wf = wfrag(sh, 16 * NH + kb * 4 + ob, lane);
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) acc[cb][ob] = mm<NP>(wf, uf[cb], kb == 0 ? X[cb][ob] : acc[cb][ob]);
          }
        }
        elu_pairs(acc, X, dp[0]);
#pragma unroll
        for (int l = 0; l < NH; ++l) {
          fence();
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            if (g == 3) X[cb][3][3] = 1.f;
#pragma unroll
            for (int rb = 0; rb < 4; ++rb) {
              ip[l][cb][rb] = u2{cvt2(X[cb][rb][0], X[cb][rb][1]), cvt2(X[cb][rb][2], X[cb][rb][3])};
              acc[cb][rb] = f4{0.f, 0.f, 0.f, 0.f};
            }
          }
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const Fr8<NP> xf[2] = {chain_frag<NP>(X[0], ks), chain_frag<NP>(X[1], ks)};
#pragma unroll
            for (int ob = 0; ob < 4; ++ob) {
              const Fr8<NP> wf = wfrag(sh, l * 8 + ob * 2 + ks, lane);
#pragma unroll
              for (int cb = 0; cb < 2; ++cb) acc[cb][ob] = mm<NP>(wf, xf[cb], acc[cb][ob]);
            }
          }
          elu_pairs(acc, X, dp[l + 1]);
        }
        fence();
        f4 d[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          if (g == 3) X[cb][3][3] = 1.f;
#pragma unroll
          for (int rb = 0; rb < 4; ++rb)
            ip[NH][cb][rb] = u2{cvt2(X[cb][rb][0], X[cb][rb][1]), cvt2(X[cb][rb][2], X[cb][rb][3])};
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const Fr8<NP> wf = wfrag(sh, fh + ks, lane);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) d[cb] = mm<NP>(wf, chain_frag<NP>(X[cb], ks), d[cb]);
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          mu[cb] = d[cb][0];
          rr[cb] = d[cb][1];
        }
      }
      // ---- head backward per sample; G rides in the I_NH image's padding rows 53, 54
      const bool pv = c < nP;
      const int oq = s * c + (s - 1);
      float gmu[2], gr[2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const float sig = softplus_fast(rr[cb]) + 1e-10f;
        gmu[cb] = pv ? gwin[w][cb][oq] : 0.f;
        float dsig = gmu[cb] * uwin[w][cb][oq + a.k];
        if (pv && (cb == 0 || two) && t0 + oq >= a.Lout - a.n_logsig) dsig += lane_f(ldl, blv[cb]) * rcp_f(sig);
        gr[cb] = dsig * sigmoid_fast(rr[cb]);
        if (g == 0) {
          gsc[w][cb][0][c] = sig;
          if constexpr (S2) gsc[w][cb][1][c] = pv ? gwin[w][cb][2 * c] : 0.f;
        }
        u2 v3[4] = {ip[NH][cb][0], ip[NH][cb][1], ip[NH][cb][2], ip[NH][cb][3]};
        if (g == 1) v3[3] = u2{cvt2(X[cb][3][0], gmu[cb]), cvt2(gr[cb], X[cb][3][3])};
        put_pairs(im0 + cb * P * HP, v3, g, c);
      }
      fence();
      {
        bf8 i1f[4];
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) i1f[hb] = tr_frag2(im0, hb, g, c);
        if constexpr (AACC) {
          mfma32_a4b(i1f, i1f[3], dWh[0], dWh[1], dWh[2], dWh[3]);
        } else {
#pragma unroll
          for (int hb = 0; hb < 4; ++hb) dWh[hb] = mfma32(i1f[hb], i1f[3], dWh[hb]);
        }
      }
      f4 D[2][4];
      {
        unsigned wvh[4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) wvh[rb] = whp[16 * rb + c];
        const bool g0 = g == 0;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const bf4 gf2 = __builtin_bit_cast(bf4, u2{cvt2(g0 ? gmu[cb] : 0.f, g0 ? gr[cb] : 0.f), 0u});
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            const bf4 wa = __builtin_bit_cast(bf4, u2{g0 ? wvh[rb] : 0u, 0u});
            D[cb][rb] = mfma16(wa, gf2, f4{0.f, 0.f, 0.f, 0.f});
          }
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if constexpr (DV) D[cb][rb][r] = 4 * rb + r < NR ? mul_h(D[cb][rb][r], dp[NH][cb][rb][r >> 1], r & 1) : 0.f;
              else D[cb][rb][r] = 4 * rb + r < NR ? D[cb][rb][r] * elu_d(X[cb][rb][r]) : 0.f;
            }
      }
      // ---- hidden layers, top down: D = dZ_l; dW_l += I_l D^T; D <- (W_l D) * elu'(I_l)
#pragma unroll
      for (int l = NH - 1; l >= 0; --l) {
        fence();
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          put_image<NP>(im1 + cb * P * HP, nullptr, D[cb], g, c);
          put_pairs(im0 + cb * P * HP, ip[l][cb], g, c);
        }
        f4 dX[2][4];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int ib = 0; ib < 4; ++ib) dX[cb][ib] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const Fr8<NP> df[2] = {chain_frag<NP>(D[0], ks), chain_frag<NP>(D[1], ks)};
#pragma unroll
          for (int ib = 0; ib < 4; ++ib) {
            const Fr8<NP> wb = wfrag(sh, 8 * NH + l * 8 + ib * 2 + ks, lane);
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) dX[cb][ib] = mm<NP>(wb, df[cb], dX[cb][ib]);
          }
        }
        fence();
        {
          bf8 dzf[4];
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) dzf[ob] = tr_frag2(im1, ob, g, c);
#pragma unroll
          for (int ib = 0; ib < 4; ++ib) {
            const bf8 xa = tr_frag2(im0, ib, g, c);
            if constexpr (AACC) {
              mfma32_a4(xa, dzf, dW[l][ib][0], dW[l][ib][1], dW[l][ib][2], dW[l][ib][3]);
            } else {
#pragma unroll
              for (int ob = 0; ob < 4; ++ob) dW[l][ib][ob] = mfma32(xa, dzf[ob], dW[l][ib][ob]);
            }
          }
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            if constexpr (DV) {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                D[cb][rb][r] = 4 * rb + r < NR ? mul_h(dX[cb][rb][r], dp[l][cb][rb][r >> 1], r & 1) : 0.f;
            } else {
              const f4 x = unpack_pair(ip[l][cb][rb]);
#pragma unroll
              for (int r = 0; r < 4; ++r) D[cb][rb][r] = 4 * rb + r < NR ? dX[cb][rb][r] * elu_d(x[r]) : 0.f;
            }
          }
      }
      // ---- D = dA0: dC tile, dcon, dW_eps, d theta
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * rb + r < NR) dCa[rb][r] += D[0][rb][r] + D[1][rb][r];
      fence();
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) put_image<NP>(im1 + cb * P * HP, nullptr, D[cb], g, c);
      f4 dcn_keep[2][JB];
      if constexpr (DU) {
        f4 dcn[2][JB];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int jb = 0; jb < JB; ++jb) dcn[cb][jb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const Fr8<NP> df[2] = {chain_frag<NP>(D[0], ks), chain_frag<NP>(D[1], ks)};
#pragma unroll
          for (int jb = 0; jb < JB; ++jb) {
            const Fr8<NP> wc = wfrag(sh, fwc + jb * 2 + ks, lane);
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) dcn[cb][jb] = mm<NP>(wc, df[cb], dcn[cb][jb]);
          }
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int jb = 0; jb < JB; ++jb) dcn_keep[cb][jb] = dcn[cb][jb];
      }
      // dW_eps and d theta from dA0's position-contracted fragments (K = 32 over the pair)
      auto dth_block = [&]() {
      fence();
      f4 dth4[4];
      {
        bf8 uaf[JB];
#pragma unroll
        for (int jb = 0; jb < JB; ++jb)
          uaf[jb] = cat8(ua_frag<NP>(uwin[w][0], s, jb, g, c).h, ua_frag<NP>(uwin[w][1], s, jb, g, c).h);
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) {
          const bf8 ta = tr_frag2(im1, hb, g, c);
          dth4[hb] = mfma32(ta, ones_ab, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int jb = 0; jb < JB; ++jb) {
            if constexpr (AACC) mfma32_a(uaf[jb], ta, dWe[jb][hb]);
            else dWe[jb][hb] = mfma32(uaf[jb], ta, dWe[jb][hb]);
          }
        }
      }
      if (c == 0 || (c == 8 && two)) {
        float* base = &dthl[w][c == 0 ? blv[0] : blv[1]][4 * g];
        f4* dp[4];
#pragma unroll
        for (int hb = 0; hb < 4; ++hb)
          dp[hb] = reinterpret_cast<f4*>(16 * hb + 4 * g < DTH ? base + 16 * hb : &dths[w][0]);
        f4 o[4];
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) o[hb] = *dp[hb];
#pragma unroll
        for (int hb = 0; hb < 4; ++hb) *dp[hb] = o[hb] + dth4[hb];
      }
      };
      auto du_block = [&]() {
      // ---- du over local positions q in [0, fin + k) of each sample in turn: its dcon into the padded rows,
      //      then one lane per position sums the rows (reads first, then a pairwise sum)
      if constexpr (DU) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          if (cb == 1 && !two) break;
          fence();
#pragma unroll
          for (int jb = 0; jb < JB; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int j = 16 * jb + 4 * g + r;
              if (DIAG) dscr[w][j][c] = dcn_keep[cb][jb][r];
              else if (j < KR && j < a.k) dscr[w][j][s * c + j] = dcn_keep[cb][jb][r];
            }
#pragma unroll
          for (int base = 0; base < (DIAG ? 128 : 64); base += 64) {
          const int q = base + lane;
          if (q < fin + a.k) {
            float v;
            if constexpr (DIAG) {
              v = 0.f;
#pragma unroll
              for (int p = 0; p < P; ++p) {
                const int j = q - p;
                const bool ok = static_cast<unsigned>(j) < static_cast<unsigned>(a.k);
                const float x = dscr[w][ok ? j : 0][p];
                v += ok ? x : 0.f;
              }
            } else {
              const int qc = q < QWR ? q : QWR - 1;
              float t[KR];
#pragma unroll
              for (int j = 0; j < KR; ++j) t[j] = dscr[w][j][qc];
#pragma unroll
              for (int w2 = 1; w2 < KR; w2 *= 2)
#pragma unroll
                for (int j = 0; j + w2 < KR; j += 2 * w2) t[j] += t[j + w2];
              v = t[0];
            }
            const int oq2 = q - a.k;
            if (oq2 >= 0 && oq2 < fin) {
              if constexpr (S2) v += (oq2 & 1) ? gwin[w][cb][oq2] * gsc[w][cb][0][oq2 >> 1] : gsc[w][cb][1][oq2 >> 1];
              else v += gwin[w][cb][oq2] * gsc[w][cb][0][oq2];
            }
            const int blq = blv[cb];
            if (q < a.k) v += carry[w][blq][q];
            if (q < fin) du[static_cast<size_t>(bv[cb]) * a.pL + t0 + q] = v;
            else carry[w][blq][q - fin] = v;
          }
          }
        }
      }
      };
      // k > 32: the du section first, so the pair's dcon tiles are not live across the dW_eps / d theta products
      if constexpr (DIAG) {
        du_block();
        dth_block();
      } else {
        dth_block();
        du_block();
      }
    }
    if (c < nP) {
      const size_t row = (static_cast<size_t>(grp) * a.Lh + m0 + c) * a.H;
      float* dcs = dC_slab + row;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = swz(16 * rb + 4 * g + r);
          if (h < a.H) {
            if (a.dc16) reinterpret_cast<__bf16*>(dC_slab)[row + h] = static_cast<__bf16>(dCa[rb][r] * kLog2e);
            else dcs[h] = dCa[rb][r] * kLog2e;
          }
        }
    }
  }
  for (int bl = 0; bl < nb; ++bl) {
    const int b = b_lo + bl;
    if constexpr (DU) {
      for (int q = lane; q < a.k; q += 64) {
        const float v = carry[w][bl][q];
        if (chn == a.n_chunks - 1) du[static_cast<size_t>(b) * a.pL + a.Lout + q] = v;
        else halo[(static_cast<size_t>(b) * a.n_chunks + chn) * a.k + q] = v;
      }
    }
    if (lane < a.H) dth_slab[(static_cast<size_t>(chn) * a.B + b) * a.H + lane] = dthl[w][bl][swz(lane)] * kLog2e;
  }
  if constexpr (AACC) {
    // the accumulators leave the AGPRs only through these statements: their wait states precede every read
#pragma unroll
    for (int l = 0; l < NH; ++l)
#pragma unroll
      for (int ib = 0; ib < 4; ++ib) agpr_drain4(dW[l][ib][0], dW[l][ib][1], dW[l][ib][2], dW[l][ib][3]);
#pragma unroll
    for (int jb = 0; jb < JB; ++jb) agpr_drain4(dWe[jb][0], dWe[jb][1], dWe[jb][2], dWe[jb][3]);
    agpr_drain4(dWh[0], dWh[1], dWh[2], dWh[3]);
  }
  const int H = a.H;
  const int nW = a.k * H + NH * H * H + 3 * NH * H + 2 * H + 2;
  float* ws = dW_slab + static_cast<size_t>(item) * nW;
#pragma unroll
  for (int jb = 0; jb < JB; ++jb)
#pragma unroll
    for (int hb = 0; hb < 4; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * jb + 4 * g + r, h = swz(16 * hb + c);
        if (j < a.k && h < H) ws[j * H + h] = dWe[jb][hb][r] * kLog2e;
      }
  const int off_w = a.k * H, off_b = off_w + NH * H * H;
#pragma unroll
  for (int l = 0; l < NH; ++l)
#pragma unroll
    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
      for (int ob = 0; ob < 4; ++ob)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int hi = swz(16 * ib + 4 * g + r), ho = swz(16 * ob + c);
          if (ho < H) {
            if (hi < H) ws[off_w + (l * H + hi) * H + ho] = dW[l][ib][ob][r];
            else if (hi == 63) ws[off_b + l * H + ho] = dW[l][ib][ob][r] * kLog2e;
          }
        }
  for (int i = lane; i < 2 * NH * H; i += 64) ws[off_b + NH * H + i] = 0.f;
  const int off_h = off_b + 3 * NH * H;
  const int oh = c - 5;
  if (oh == 0 || oh == 1) {
#pragma unroll
    for (int hb = 0; hb < 4; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = swz(16 * hb + 4 * g + r);
        if (h < H) ws[off_h + h * 2 + oh] = dWh[hb][r] * kLn2;
        else if (h == 63) ws[off_h + 2 * H + oh] = dWh[hb][r];
      }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct Geom {
  int s, Lout, Lh, S, n_groups, n_tiles, CH, n_chunks, n_items;
  int blocks;  // grid size of the 4-wave kernels
};

// work items (sample group x t-chunk) a launch aims for (4096 / 12288 / 16384: within +-0.3 ms at the AR-cfg shape)
constexpr int kTargetItems = 8192;
static Geom geom(const VissmFlowDesc* d, bool backward, int po = P) {
  Geom g;
  g.s = d->stride2 ? 2 : 1;
  g.Lout = d->L - d->k;
  g.Lh = g.Lout / g.s;
  g.S = (backward && d->n_win > 1) ? 1 : S;
  g.n_groups = (d->B + g.S - 1) / g.S;
  g.n_tiles = (g.Lh + po - 1) / po;
  int ch_min_tiles = ((d->k + g.s - 1) / g.s + po - 1) / po;
  if (ch_min_tiles < 1) ch_min_tiles = 1;
  int want = (kTargetItems + g.n_groups - 1) / g.n_groups;
  int max_chunks = g.n_tiles / ch_min_tiles;
  if (max_chunks < 1) max_chunks = 1;
  int nc = want < max_chunks ? want : max_chunks;
  if (nc < 1) nc = 1;
  int tiles_per_chunk = (g.n_tiles + nc - 1) / nc;
  if (d->chunk_tiles > 0) tiles_per_chunk = d->chunk_tiles;  // caller-forced chunk geometry (tests)
  if (tiles_per_chunk < ch_min_tiles) tiles_per_chunk = ch_min_tiles;
  g.CH = tiles_per_chunk * po;
  g.n_chunks = (g.Lh + g.CH - 1) / g.CH;
  g.n_items = g.n_groups * g.n_chunks;
  g.blocks = (g.n_items + NW - 1) / NW;
  return g;
}

static int n_wgrad(const VissmFlowDesc* d) {
  const int H = d->H, k = d->k, nh = d->n_hidden;
  return k * H + nh * H * H + 3 * nh * H + 2 * H + 2;
}

static int jb_of(int k) { return (k + 15) / 16; }
static int np_of(const VissmFlowDesc* d) {
  return d->precision == VISSM_PREC_BF16X3 ? 3
       : (d->precision == VISSM_PREC_BF16X2 || d->precision == VISSM_PREC_BF16X2_BF16) ? 2 : 1;
}

struct Ws {
  bf8* img;
  float* cst;
  float *Cp, *thp;
  u4* thf;                                               // theta fold: [B][2] B-operand rows
  float* ls_slab;                                        // fwd
  float *dC_slab, *dth_slab, *dW_slab, *halo, *wred;     // bwd
  float* zsl;                                            // fused AR(1) ELBO: per-chunk per-sample sums
};

static size_t ws_layout(const VissmFlowDesc* d, const Geom& g, bool backward, char* base, Ws* w, bool fused = false) {
  size_t off = 0;
  auto take = [&](size_t nbytes) { char* p = base ? base + off : nullptr; off += align_up(nbytes); return p; };
  Ws t{};
  const int JB = jb_of(d->k), KB = (JB + 1) / 2;
  const int NPL = np_of(d) >= 2 ? 2 : 1;
  t.img = reinterpret_cast<bf8*>(take(static_cast<size_t>(n_frags(d->n_hidden, KB, JB)) * NPL * 64 * sizeof(bf8)));
  t.cst = reinterpret_cast<float*>(take(((d->n_hidden + 2) * HP + 4) * sizeof(float)));
  t.Cp = reinterpret_cast<float*>(take(static_cast<size_t>(d->n_win) * g.Lh * HP * 4));
  t.thp = reinterpret_cast<float*>(take(static_cast<size_t>(d->B) * HP * 4));
  t.thf = reinterpret_cast<u4*>(take(static_cast<size_t>(d->B) * 2 * sizeof(u4)));
  if (!backward) {
    t.ls_slab = reinterpret_cast<float*>(take(static_cast<size_t>(g.n_chunks) * d->B * 4));
  } else {
    t.dC_slab = reinterpret_cast<float*>(take(static_cast<size_t>(g.n_groups) * g.Lh * d->H * 4));
    t.dth_slab = reinterpret_cast<float*>(take(static_cast<size_t>(g.n_chunks) * d->B * d->H * 4));
    t.dW_slab = reinterpret_cast<float*>(take(static_cast<size_t>(g.n_items) * n_wgrad(d) * 4));
    t.halo = reinterpret_cast<float*>(take(static_cast<size_t>(d->B) * g.n_chunks * d->k * 4));
    t.wred = reinterpret_cast<float*>(take(static_cast<size_t>(n_wgrad(d)) * 4));
    if (fused) t.zsl = reinterpret_cast<float*>(take(static_cast<size_t>(g.n_chunks) * d->B * 4));
  }
  if (w) *w = t;
  return off;
}

// compute units of the current device (cached per device)
static int device_cus() {
  static int cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
  if (dev < 16 && cache[dev]) return cache[dev];
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  if (dev < 16) cache[dev] = n;
  return n;
}

static KArgs make_args(const VissmFlowDesc* d, const Geom& g) {
  KArgs a;
  a.B = d->B; a.L = d->L; a.k = d->k; a.H = d->H; a.s = g.s; a.swap_out = d->swap_out;
  a.pL = d->u_pitch ? d->u_pitch : d->L; a.pLo = d->out_pitch ? d->out_pitch : g.Lout;
  a.n_logsig = d->n_logsig; a.Lout = g.Lout; a.Lh = g.Lh; a.CH = g.CH; a.n_chunks = g.n_chunks; a.S = g.S;
  a.n_groups = g.n_groups; a.n_items = g.n_items;
  a.dc16 = (d->n_win == 1 && d->precision != VISSM_PREC_FP32 && d->precision != VISSM_PREC_BF16X3) ? 1 : 0;
  a.ncu = device_cus();
  return a;
}

// Scatter the reduced partials into the caller's gradient buffers, undoing the BN folding:
// for a layer fed by BN (gamma', beta) the kernel accumulated dWE = sum_p E dZ^T and
// db = sum_p dZ, so  dW = diag(gamma') dWE + beta db^T,  d gamma' = rowsum(W o dWE),
// d beta = W db  (and d gamma = kBnScale d gamma').  Without BN the partials are the gradients.
__global__ void scatter_wgrad_kernel(const float* __restrict__ red, VissmFlowParams p, VissmFlowGrads g, int k, int H,
                                     int nh, int bn) {
  const int off_w = k * H, off_b = off_w + nh * H * H, off_h = off_b + 3 * nh * H;
  const int nW = off_h + 2 * H + 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nW; i += gridDim.x * blockDim.x) {
    const float v = red[i];
    if (i < off_w) {
      g.w_eps[i] = v;
    } else if (i < off_b) {
      const int r = i - off_w, l = r / (H * H), hi = (r / H) % H, ho = r % H;
      float x = v;
      if (bn && l > 0)
        x = p.bn_g[(l - 1) * H + hi] * kBnScale * v + p.bn_b[(l - 1) * H + hi] * red[off_b + l * H + ho];
      g.w_hid[r] = x;
    } else if (i < off_b + nh * H) {
      g.b_hid[i - off_b] = v;
    } else if (i < off_h) {
      // bn gamma (first nh*H) / beta (next nh*H) of layer l: BN_l feeds layer l + 1 or the head
      const int r = i - off_b - nh * H, which = r / (nh * H), l = (r / H) % nh, h = r % H;
      if (!bn) continue;
      float s = 0.f;
      if (l + 1 < nh) {
        const float* W = p.w_hid + static_cast<size_t>(l + 1) * H * H;
        const float* dWE = red + off_w + static_cast<size_t>(l + 1) * H * H;
        const float* db = red + off_b + (l + 1) * H;
        for (int o = 0; o < H; ++o) s += W[h * H + o] * (which == 0 ? dWE[h * H + o] : db[o]);
      } else {
        for (int o = 0; o < 2; ++o)
          s += p.w_head[h * 2 + o] * (which == 0 ? red[off_h + h * 2 + o] : red[off_h + 2 * H + o]);
      }
      if (which == 0) g.bn_g[l * H + h] = s * kBnScale;
      else g.bn_b[l * H + h] = s;
    } else if (i < off_h + 2 * H) {
      const int r = i - off_h, h = r / 2, o = r % 2;
      float x = v;
      if (bn && nh > 0)
        x = p.bn_g[(nh - 1) * H + h] * kBnScale * v + p.bn_b[(nh - 1) * H + h] * red[off_h + 2 * H + o];
      g.w_head[r] = x;
    } else {
      g.b_head[i - off_h - 2 * H] = v;
    }
  }
}

// the two-sample backward covers the AR configurations' flow shape, at bf16 and bf16x2 (split weights: SB)
static bool bwd2_ok(const VissmFlowDesc* d, const Geom& g) {
  return (d->precision == VISSM_PREC_BF16 || d->precision == VISSM_PREC_BF16X2) && d->n_hidden == 1 && !d->bn && !d->stride2 && !d->swap_out &&
         d->k <= KP2 && d->H <= kMaxH && d->n_win == 1 && g.S == S;
}

// the three-hidden-layer two-sample backward: LV / FHN heads (k <= 24: padded dcon rows), SV (32 < k <= 64, stride 1:
// the diagonal du sum), one window
static bool bwd2n_ok(const VissmFlowDesc* d, const Geom& g) {
  return d->precision == VISSM_PREC_BF16 && d->n_hidden == 3 &&
         (d->k <= 24 || (d->k > 32 && d->k <= 64 && !d->stride2)) && d->H <= kMaxH && d->n_win == 1 && g.S == S;
}

// the two-sample forward covers the AR configurations' flow shape
static bool fwd2_ok(const VissmFlowDesc* d, const Geom& g) {
  if (d->H > kMaxH || d->n_win != 1 || g.S != S || d->k > 64) return false;
  if (d->k > 32 && (d->n_hidden != 3 || d->stride2)) return false;  // two K blocks: SV's shape
  if (d->n_hidden == 1)
    return !d->bn && !d->stride2 && !d->swap_out &&
           (d->precision == VISSM_PREC_BF16 || d->precision == VISSM_PREC_BF16X2);
  return d->n_hidden == 3 && d->precision == VISSM_PREC_BF16;
}

}  // namespace VISSM_FLOW5_NS

using namespace VISSM_FLOW5_NS;

bool VISSM_FLOW5_API(flow5_supports)(const VissmFlowDesc* d) {
  // one hidden layer (AR): bf16 and bf16x3 (k <= 32: hi + lo images in LDS); three hidden layers
  // with or without BN (LV / SV / FHN heads): bf16
  if (d->H > kMaxH || d->k > 64) return false;
  if (d->precision == VISSM_PREC_BF16) return d->n_hidden == 1 || d->n_hidden == 3;
  if (d->precision == VISSM_PREC_BF16X3) return d->n_hidden == 1 && d->k <= 32;
  if (d->precision == VISSM_PREC_BF16X2) return d->n_hidden == 1 && d->k <= 32;
  return false;
}

size_t VISSM_FLOW5_API(flow5_workspace_size)(const VissmFlowDesc* d, int backward) {
  Geom g = geom(d, backward != 0);
  return ws_layout(d, g, backward != 0, nullptr, nullptr);
}

// which: 0 forward, 1 backward, 2 the fused last AR flow (15 outputs per 16-column tile)
void VISSM_FLOW5_API(flow5_geometry)(const VissmFlowDesc* d, int which, int32_t* out) {
  const int po = which == 2 ? P - 1 : P;
  Geom g = geom(d, which != 0, po);
  out[0] = po; out[1] = g.CH / po; out[2] = g.n_chunks; out[3] = g.n_groups;
}

#define FLOW5_DISPATCH(KERNEL, NHd, JB, NP, ...)                                                  \
  do {                                                                                             \
    if (NP == 3) {                                                                                 \
      if (JB == 1) hipLaunchKernelGGL((KERNEL<1, 1, 1, 3>), __VA_ARGS__);                           \
      else hipLaunchKernelGGL((KERNEL<1, 1, 2, 3>), __VA_ARGS__);                                   \
    } else if (NP == 2) {                                                                          \
      if (JB == 1) hipLaunchKernelGGL((KERNEL<1, 1, 1, 2>), __VA_ARGS__);                           \
      else hipLaunchKernelGGL((KERNEL<1, 1, 2, 2>), __VA_ARGS__);                                   \
    } else if (NHd == 1) {                                                                         \
      switch (JB) {                                                                                \
        case 1: hipLaunchKernelGGL((KERNEL<1, 1, 1, 1>), __VA_ARGS__); break;                       \
        case 2: hipLaunchKernelGGL((KERNEL<1, 1, 2, 1>), __VA_ARGS__); break;                       \
        case 3: hipLaunchKernelGGL((KERNEL<1, 2, 3, 1>), __VA_ARGS__); break;                       \
        default: hipLaunchKernelGGL((KERNEL<1, 2, 4, 1>), __VA_ARGS__); break;                      \
      }                                                                                            \
    } else {                                                                                       \
      switch (JB) {                                                                                \
        case 1: hipLaunchKernelGGL((KERNEL<3, 1, 1, 1>), __VA_ARGS__); break;                       \
        case 2: hipLaunchKernelGGL((KERNEL<3, 1, 2, 1>), __VA_ARGS__); break;                       \
        case 3: hipLaunchKernelGGL((KERNEL<3, 2, 3, 1>), __VA_ARGS__); break;                       \
        default: hipLaunchKernelGGL((KERNEL<3, 2, 4, 1>), __VA_ARGS__); break;                      \
      }                                                                                            \
    }                                                                                              \
  } while (0)

#define COMMA ,
// as FLOW5_DISPATCH with trailing template arguments TAIL (write their commas as COMMA)
#define FLOW5_DISPATCH_T(KERNEL, TAIL, NHd, JB, NP, ...)                                                  \
  do {                                                                                             \
    if (NP == 3) {                                                                                 \
      if (JB == 1) hipLaunchKernelGGL((KERNEL<1, 1, 1, 3, TAIL>), __VA_ARGS__);                           \
      else hipLaunchKernelGGL((KERNEL<1, 1, 2, 3, TAIL>), __VA_ARGS__);                                   \
    } else if (NP == 2) {                                                                          \
      if (JB == 1) hipLaunchKernelGGL((KERNEL<1, 1, 1, 2, TAIL>), __VA_ARGS__);                           \
      else hipLaunchKernelGGL((KERNEL<1, 1, 2, 2, TAIL>), __VA_ARGS__);                                   \
    } else if (NHd == 1) {                                                                         \
      switch (JB) {                                                                                \
        case 1: hipLaunchKernelGGL((KERNEL<1, 1, 1, 1, TAIL>), __VA_ARGS__); break;                       \
        case 2: hipLaunchKernelGGL((KERNEL<1, 1, 2, 1, TAIL>), __VA_ARGS__); break;                       \
        case 3: hipLaunchKernelGGL((KERNEL<1, 2, 3, 1, TAIL>), __VA_ARGS__); break;                       \
        default: hipLaunchKernelGGL((KERNEL<1, 2, 4, 1, TAIL>), __VA_ARGS__); break;                      \
      }                                                                                            \
    } else {                                                                                       \
      switch (JB) {                                                                                \
        case 1: hipLaunchKernelGGL((KERNEL<3, 1, 1, 1, TAIL>), __VA_ARGS__); break;                       \
        case 2: hipLaunchKernelGGL((KERNEL<3, 1, 2, 1, TAIL>), __VA_ARGS__); break;                       \
        case 3: hipLaunchKernelGGL((KERNEL<3, 2, 3, 1, TAIL>), __VA_ARGS__); break;                       \
        default: hipLaunchKernelGGL((KERNEL<3, 2, 4, 1, TAIL>), __VA_ARGS__); break;                      \
      }                                                                                            \
    }                                                                                              \
  } while (0)

// the caller supplied the theta branch's factors (VissmFlowParams.theta_rank) and the shape leaves K rows 16..31 of
// the layer-0 product free
static bool fold_ok(const VissmFlowDesc* d, const VissmFlowParams* w) {
  return w->theta_rank >= 1 && w->theta_rank <= 5 && w->theta_x && w->w_theta && w->b_theta &&
         d->k <= kFoldRow && d->n_hidden == 1;
}

// the split-weight (bf16x2) two-sample kernels' layer-0 / head lo products in the hi fragments' spare rows (prep_kernel)
static bool lofold_ok(const VissmFlowDesc* d) {
  return np_of(d) == 2 && d->k <= 8 && d->n_hidden == 1 && !kLoFoldOff;
}

// padded C (+ b_theta when folding) and either the padded theta term or the theta fold's B-operand rows
static void launch_pad(const VissmFlowDesc* d, const VissmFlowParams* w, const Geom& g, const float* C,
                       const float* tht, const Ws& ws, bool fold, hipStream_t st) {
  const int64_t nC = static_cast<int64_t>(d->n_win) * g.Lh, nT = d->B;
  hipLaunchKernelGGL(pad_kernel, dim3(static_cast<unsigned>((nC * HP + 255) / 256)), dim3(256), 0, st, C, ws.Cp, nC,
                     d->H, fold ? w->b_theta : static_cast<const float*>(nullptr));
  if (fold)
    hipLaunchKernelGGL(theta_frag_kernel, dim3(static_cast<unsigned>((2 * nT + 255) / 256)), dim3(256), 0, st,
                       w->theta_x, d->B, w->theta_rank, ws.thf);
  else
    hipLaunchKernelGGL(pad_kernel, dim3(static_cast<unsigned>((nT * HP + 255) / 256)), dim3(256), 0, st, tht, ws.thp,
                       nT, d->H, static_cast<const float*>(nullptr));
}

static void launch_prep(const VissmFlowDesc* d, const VissmFlowParams* w, const Ws& ws, bool fold, hipStream_t st,
                        bool lofold = false) {
  const int JB = jb_of(d->k), KB = (JB + 1) / 2;
  hipLaunchKernelGGL(prep_kernel, dim3(n_frags(d->n_hidden, KB, JB)), dim3(64), 0, st, *w, d->H, d->k, d->n_hidden,
                     d->bn, np_of(d), KB, JB, ws.img, ws.cst, fold ? 1 : 0, lofold ? 1 : 0);
}

int VISSM_FLOW5_API(flow5_fwd)(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
              const float* theta_term, float* u_next, float* logsig, void* workspace, size_t ws_bytes,
              hipStream_t st) {
  Geom g = geom(d, false);
  VISSM_CHECK_ARG(workspace && ws_bytes >= ws_layout(d, g, false, nullptr, nullptr), "flow_fwd: workspace too small");
  Ws ws;
  ws_layout(d, g, false, reinterpret_cast<char*>(workspace), &ws);
  const bool f2 = fwd2_ok(d, g), fold = f2 && fold_ok(d, w);
  const bool lof = f2 && lofold_ok(d);
  launch_prep(d, w, ws, fold, st, lof);
  launch_pad(d, w, g, C, theta_term, ws, fold, st);
  VISSM_CHECK_LAUNCH("flow5_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid((g.n_items + NW - 1) / NW);
  prof_begin(VISSM_PROF_FLOW_FWD, st);
  if (f2) {
// 8-wave blocks with every weight plane read from LDS for the split-weight forward (155 -> 93 VGPRs: bf16x2 forward
// 9.81 -> 9.19 ms per AR-cfg launch) and three hidden layers (225 -> 126: LV 3.68 -> 3.51 ms, FHN 0.77 -> 0.69 ms): the
// block's weight image then serves twice the waves and the LDS no longer caps them at 2-3 per SIMD; the bf16 AR forward
// keeps 4-wave blocks with register-resident hi planes (8-wave blocks: 6.90 -> 7.16 ms, still four waves per SIMD at
// 103 VGPRs), profiles/r04/ab_fwd_blocks_steps.log
#ifndef VISSM_X2_NWF
#define VISSM_X2_NWF 8  // split-weight forward with lofold: 8-wave blocks reading every plane from LDS (4-wave blocks with
                        // the hi planes register-resident, 155 VGPRs: 8.47 -> 9.06 ms per AR-cfg launch,
                        // profiles/r06/ab_r06i.log)
#endif
#define FWD2_LAUNCH(TF_, NP_, NH_, JB_, LOF_)                                                                      \
  do {                                                                                                           \
    constexpr int nwf = (NP_ == 2 && LOF_) ? VISSM_X2_NWF : (NP_ == 2 || NH_ == 3) ? 8 : NW;                      \
    hipLaunchKernelGGL((fwd2_kernel<TF_, NP_, NH_, JB_, nwf, LOF_>), dim3((g.n_items + nwf - 1) / nwf),            \
                       dim3(64 * nwf), 0, st, a, u, ws.Cp, ws.thp, ws.img, ws.cst, u_next, ws.ls_slab, ws.thf);   \
  } while (0)
    const int jb = jb_of(d->k);
    if (d->n_hidden == 3) {
      if (jb == 1) FWD2_LAUNCH(false, 1, 3, 1, false);
      else if (jb == 2) FWD2_LAUNCH(false, 1, 3, 2, false);
      else if (jb == 3) FWD2_LAUNCH(false, 1, 3, 3, false);
      else FWD2_LAUNCH(false, 1, 3, 4, false);
    }
    else if (jb == 2) { if (np_of(d) == 2) FWD2_LAUNCH(false, 2, 1, 2, false); else FWD2_LAUNCH(false, 1, 1, 2, false); }
    else if (np_of(d) == 2 && lof) { if (fold) FWD2_LAUNCH(true, 2, 1, 1, true); else FWD2_LAUNCH(false, 2, 1, 1, true); }
    else if (np_of(d) == 2) { if (fold) FWD2_LAUNCH(true, 2, 1, 1, false); else FWD2_LAUNCH(false, 2, 1, 1, false); }
    else { if (fold) FWD2_LAUNCH(true, 1, 1, 1, false); else FWD2_LAUNCH(false, 1, 1, 1, false); }
#undef FWD2_LAUNCH
  } else if (np_of(d) == 2) {
    if (jb_of(d->k) == 1)
      hipLaunchKernelGGL((fwd_kernel<1, 1, 1, 2>), grid, dim3(NT), 0, st, a, u, ws.Cp, wn, ws.thp, ws.img, ws.cst, u_next,
                         ws.ls_slab);
    else
      hipLaunchKernelGGL((fwd_kernel<1, 1, 2, 2>), grid, dim3(NT), 0, st, a, u, ws.Cp, wn, ws.thp, ws.img, ws.cst, u_next,
                         ws.ls_slab);
  } else {
    FLOW5_DISPATCH(fwd_kernel, d->n_hidden, jb_of(d->k), np_of(d), grid, dim3(NT), 0, st, a, u, ws.Cp, wn, ws.thp, ws.img,
                   ws.cst, u_next, ws.ls_slab);
  }
  VISSM_CHECK_LAUNCH("flow5_fwd");
  prof_end(VISSM_PROF_FLOW_FWD, st);
  return launch_reduce_rows(ws.ls_slab, logsig, g.n_chunks, d->B, st);
}

int VISSM_FLOW5_API(flow5_bwd)(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
              const float* theta_term, const float* du_next, const float* dlogsig, float* du, float* dC,
              float* dtheta_term, const VissmFlowGrads* gr, void* workspace, size_t ws_bytes, hipStream_t st) {
  Geom g = geom(d, true);
  VISSM_CHECK_ARG(workspace && ws_bytes >= ws_layout(d, g, true, nullptr, nullptr), "flow_bwd: workspace too small");
  Ws ws;
  ws_layout(d, g, true, reinterpret_cast<char*>(workspace), &ws);
  const bool b2 = !bwd2n_ok(d, g) && bwd2_ok(d, g), fold = b2 && fold_ok(d, w);
  launch_prep(d, w, ws, fold, st, b2 && lofold_ok(d));
  launch_pad(d, w, g, C, theta_term, ws, fold, st);
  VISSM_CHECK_LAUNCH("flow5_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid(g.blocks);
  const int pvar = du ? VISSM_PROF_FLOW_BWD_DU : VISSM_PROF_FLOW_BWD_NODU;
  prof_begin(VISSM_PROF_FLOW_BWD, st);
  prof_begin(pvar, st);
  if (bwd2n_ok(d, g)) {
    const dim3 grid3((g.n_items + NW3 - 1) / NW3);
#define BWD2N_LAUNCH(JB_, S2_, DU_)                                                                              \
  hipLaunchKernelGGL((bwd2n_kernel<JB_, S2_, DU_>), grid3, dim3(NT3), 0, st, a, u, ws.Cp, ws.thp, du_next, dlogsig, \
                     ws.img, ws.cst, du, ws.dC_slab, ws.dth_slab, ws.dW_slab, ws.halo)
    const int jb = jb_of(d->k);
    if (d->stride2) {
      if (jb == 1) { if (du) BWD2N_LAUNCH(1, true, true); else BWD2N_LAUNCH(1, true, false); }
      else { if (du) BWD2N_LAUNCH(2, true, true); else BWD2N_LAUNCH(2, true, false); }
    } else {
      if (jb == 1) { if (du) BWD2N_LAUNCH(1, false, true); else BWD2N_LAUNCH(1, false, false); }
      else if (jb == 2) { if (du) BWD2N_LAUNCH(2, false, true); else BWD2N_LAUNCH(2, false, false); }
      else if (jb == 3) { if (du) BWD2N_LAUNCH(3, false, true); else BWD2N_LAUNCH(3, false, false); }
      else { if (du) BWD2N_LAUNCH(4, false, true); else BWD2N_LAUNCH(4, false, false); }
    }
#undef BWD2N_LAUNCH
  } else if (b2) {
    const dim3 grid2((g.n_items + NW2 - 1) / NW2);
#define BWD2_LAUNCH(DU_, TF_, NPR_, SB_)                                                                          \
  hipLaunchKernelGGL((bwd2_kernel<false, DU_, TF_, NPR_, SB_>), grid2, dim3(NT2), 0, st, a, u, ws.Cp, ws.thp, du_next, \
                     dlogsig, ws.img, ws.cst, du, ws.dC_slab, ws.dth_slab, ws.dW_slab, ws.halo, ws.thf, FzArgs{})
    if (np_of(d) == 2) {  // bf16x2: split-weight recompute and backward chain
      if (du) { if (fold) BWD2_LAUNCH(true, true, 2, true); else BWD2_LAUNCH(true, false, 2, true); }
      else { if (fold) BWD2_LAUNCH(false, true, 2, true); else BWD2_LAUNCH(false, false, 2, true); }
    } else {
      if (du) { if (fold) BWD2_LAUNCH(true, true, 1, false); else BWD2_LAUNCH(true, false, 1, false); }
      else { if (fold) BWD2_LAUNCH(false, true, 1, false); else BWD2_LAUNCH(false, false, 1, false); }
    }
#undef BWD2_LAUNCH
  } else if (du)
    FLOW5_DISPATCH_T(bwd_kernel, false COMMA true, d->n_hidden, jb_of(d->k), np_of(d), grid, dim3(NT), 0, st, a, u,
                     ws.Cp, wn, ws.thp, du_next, dlogsig, ws.img, ws.cst, du, ws.dC_slab, ws.dth_slab, ws.dW_slab,
                     ws.halo, FzArgs{});
  else
    FLOW5_DISPATCH_T(bwd_kernel, false COMMA false, d->n_hidden, jb_of(d->k), np_of(d), grid, dim3(NT), 0, st, a, u,
                     ws.Cp, wn, ws.thp, du_next, dlogsig, ws.img, ws.cst, du, ws.dC_slab, ws.dth_slab, ws.dW_slab,
                     ws.halo, FzArgs{});
  VISSM_CHECK_LAUNCH("flow5_bwd");
  prof_end(pvar, st);
  prof_end(VISSM_PROF_FLOW_BWD, st);
  int rc = du ? launch_halo_fixup(du, ws.halo, d->B, d->L, a.pL, d->k, g.n_chunks, g.s, g.CH, st) : VISSM_OK;
  if (rc) return rc;
  const int64_t nC = static_cast<int64_t>(g.Lh) * d->H;
  if (d->n_win == 1) {
    rc = a.dc16 ? launch_reduce_rows_bf16(ws.dC_slab, dC, g.n_groups, nC, st)
                : launch_reduce_rows_inplace(ws.dC_slab, dC, g.n_groups, nC, st);
    if (rc) return rc;
  } else {
    rc = launch_reduce_by_window(ws.dC_slab, win, dC, d->B, d->n_win, nC, st);
    if (rc) return rc;
  }
  rc = launch_reduce_rows(ws.dth_slab, dtheta_term, g.n_chunks, static_cast<int64_t>(d->B) * d->H, st);
  if (rc) return rc;
  const int nW = n_wgrad(d);
  rc = launch_reduce_rows_inplace(ws.dW_slab, ws.wred, g.n_items, nW, st);
  if (rc) return rc;
  hipLaunchKernelGGL(VISSM_FLOW5_NS::scatter_wgrad_kernel, dim3((nW + 255) / 256), dim3(256), 0, st, ws.wred, *w, *gr, d->k,
                     d->H, d->n_hidden, d->bn);
  VISSM_CHECK_LAUNCH("flow5_scatter");
  return VISSM_OK;
}


// ---- the last AR(1) flow fused with its ELBO terms (vissm_flow_ar_elbo_fused) ----
bool VISSM_FLOW5_API(flow5_ar_fused_supports)(const VissmFlowDesc* d) {
  const bool shape = d->n_hidden == 1 && !d->bn && !d->stride2 && !d->swap_out && d->k <= 32 && d->H <= kMaxH &&
                     d->n_win >= 1;
  if (d->precision == VISSM_PREC_BF16X2 || d->precision == VISSM_PREC_BF16X2_BF16)  // the two-sample kernel's shape only
    return shape && d->k <= KP2 && d->n_win == 1;
  return (d->precision == VISSM_PREC_BF16 || d->precision == VISSM_PREC_BF16X3) && shape;
}

size_t VISSM_FLOW5_API(flow5_ar_fused_workspace_size)(const VissmFlowDesc* d) {
  Geom g = geom(d, true, P - 1);
  return ws_layout(d, g, true, nullptr, nullptr, true);
}

#define FLOW5_FZ_DISPATCH(JB, NP, ...)                                                     \
  do {                                                                                     \
    if (NP == 3) {                                                                         \
      if (JB == 1) hipLaunchKernelGGL((bwd_kernel<1, 1, 1, 3, true>), __VA_ARGS__);        \
      else hipLaunchKernelGGL((bwd_kernel<1, 1, 2, 3, true>), __VA_ARGS__);                \
    } else {                                                                               \
      if (JB == 1) hipLaunchKernelGGL((bwd_kernel<1, 1, 1, 1, true>), __VA_ARGS__);        \
      else hipLaunchKernelGGL((bwd_kernel<1, 1, 2, 1, true>), __VA_ARGS__);                \
    }                                                                                      \
  } while (0)

int VISSM_FLOW5_API(flow5_ar_fused)(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
                   const float* theta_term, const float* theta, const float* obs, const float* obs_bin, float obs_std,
                   float scale, float* x, float* logsig, float* du, float* dC, float* dtheta_term,
                   const VissmFlowGrads* gr, void* workspace, size_t ws_bytes, hipStream_t st) {
  Geom g = geom(d, true, P - 1);
  VISSM_CHECK_ARG(workspace && ws_bytes >= ws_layout(d, g, true, nullptr, nullptr, true),
                  "flow_ar_elbo_fused: workspace too small");
  Ws ws;
  ws_layout(d, g, true, reinterpret_cast<char*>(workspace), &ws, true);
  // bf16x2: split-weight recompute and backward chain; bf16x2_bf16: split-weight recompute, bf16 backward products
  const bool x2 = d->precision == VISSM_PREC_BF16X2 || d->precision == VISSM_PREC_BF16X2_BF16;
  const bool sb = d->precision == VISSM_PREC_BF16X2;
  // bf16x2 has only the two-sample kernel: it must meet that kernel's geometry (bwd2_ok minus the precision test)
  VISSM_CHECK_ARG(!x2 || (g.S == S && d->n_win == 1 && d->k <= KP2),
                  "flow_ar_elbo_fused: bf16x2 needs the two-sample kernel's geometry (one window, k <= %d)", KP2);
  const bool b2 = x2 || bwd2_ok(d, g), fold = b2 && fold_ok(d, w);
  launch_prep(d, w, ws, fold, st, x2 && lofold_ok(d));
  launch_pad(d, w, g, C, theta_term, ws, fold, st);
  VISSM_CHECK_LAUNCH("flow5_fused_prep");
  KArgs a = make_args(d, g);
  FzArgs fz;
  fz.theta = theta;
  fz.obs = obs;
  fz.bin = obs_bin;
  fz.x = x;
  fz.lsl = ws.zsl;
  fz.scale = scale;
  fz.iosd = 1.f / obs_std;
  fz.M = d->L - d->k - 1;
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  prof_begin(VISSM_PROF_FLOW_BWD, st);
  prof_begin(VISSM_PROF_FLOW_FUSED, st);
  if (b2) {
#define BWD2F_LAUNCH(TF_, NPR_, SB_)                                                                                 \
  hipLaunchKernelGGL((bwd2_kernel<true, true, TF_, NPR_, SB_>), dim3((g.n_items + NW2 - 1) / NW2), dim3(NT2), 0, st, a, u, \
                     ws.Cp, ws.thp, static_cast<const float*>(nullptr), static_cast<const float*>(nullptr), ws.img,     \
                     ws.cst, du, ws.dC_slab, ws.dth_slab, ws.dW_slab, ws.halo, ws.thf, fz)
    if (sb) { if (fold) BWD2F_LAUNCH(true, 2, true); else BWD2F_LAUNCH(false, 2, true); }
    else if (x2) { if (fold) BWD2F_LAUNCH(true, 2, false); else BWD2F_LAUNCH(false, 2, false); }
    else { if (fold) BWD2F_LAUNCH(true, 1, false); else BWD2F_LAUNCH(false, 1, false); }
#undef BWD2F_LAUNCH
  } else
    FLOW5_FZ_DISPATCH(jb_of(d->k), np_of(d), dim3(g.blocks), dim3(NT), 0, st, a, u, ws.Cp, wn, ws.thp,
                      static_cast<const float*>(nullptr), static_cast<const float*>(nullptr), ws.img, ws.cst, du,
                      ws.dC_slab, ws.dth_slab, ws.dW_slab, ws.halo, fz);
  VISSM_CHECK_LAUNCH("flow5_fused");
  prof_end(VISSM_PROF_FLOW_FUSED, st);
  prof_end(VISSM_PROF_FLOW_BWD, st);
  int rc = launch_halo_fixup(du, ws.halo, d->B, d->L, a.pL, d->k, g.n_chunks, g.s, g.CH, st);
  if (rc) return rc;
  const int64_t nC = static_cast<int64_t>(g.Lh) * d->H;
  if (d->n_win == 1) {
    rc = a.dc16 ? launch_reduce_rows_bf16(ws.dC_slab, dC, g.n_groups, nC, st)
                : launch_reduce_rows_inplace(ws.dC_slab, dC, g.n_groups, nC, st);
  } else {
    rc = launch_reduce_by_window(ws.dC_slab, win, dC, d->B, d->n_win, nC, st);
  }
  if (rc) return rc;
  rc = launch_reduce_rows(ws.dth_slab, dtheta_term, g.n_chunks, static_cast<int64_t>(d->B) * d->H, st);
  if (rc) return rc;
  rc = launch_reduce_rows(ws.zsl, logsig, g.n_chunks, d->B, st);
  if (rc) return rc;
  const int nW = n_wgrad(d);
  rc = launch_reduce_rows_inplace(ws.dW_slab, ws.wred, g.n_items, nW, st);
  if (rc) return rc;
  hipLaunchKernelGGL(VISSM_FLOW5_NS::scatter_wgrad_kernel, dim3((nW + 255) / 256), dim3(256), 0, st, ws.wred, *w, *gr, d->k,
                     d->H, d->n_hidden, d->bn);
  VISSM_CHECK_LAUNCH("flow5_fused_scatter");
  return VISSM_OK;
}

}  // namespace vissm
