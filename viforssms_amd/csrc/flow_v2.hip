// IAF flow of the neural-MA sampler on the matrix cores (exact fp32:
// v_mfma_f32_16x16x4_f32), forward and backward.
//
// Reference: IAF._create_flow / IAF.slp (AR.py:50-89); stride-2 head with
// (0,1) interleave and BN affine (lotka_volterra_partial.py:93-104,
// fitz_nag_NVP.py:90-105); Permute fused into the store (swap_out).
//
// Work unit: one (sample, tile of P = 32 head positions), processed by a whole
// 256-thread block (4 waves).  Activations live in LDS as [h][p] tiles (h =
// hidden unit, padded to 64; p = position).  Wave w owns hidden rows
// 16w .. 16w+15 of every [64 x 32] activation tile, i.e. two 16x16 MFMA
// output blocks, so
//   * forward products  Z[h_out][p] = sum_h_in W[h_in][h_out] X[h_in][p]
//   * backward products dX[h_in][p] = sum_h_out W[h_in][h_out] dZ[h_out][p]
// are computed without cross-wave sums (K = 4 hidden units per MFMA), while
//   * weight gradients  dW[h_in][h_out] = sum_p X[h_in][p] dZ[h_out][p]
// contract over positions (K = 4 positions per MFMA) by reading the same LDS
// tiles along the other axis; wave w accumulates rows h_in = 16w .. 16w+15 of
// every layer's dW in registers for the block's whole lifetime.
//
// Grid decomposition, carries, halo and partial slabs are those of flow_v1.hip
// (sample groups x t-chunks; backward walks tiles outer / samples inner so the
// window-shared dC tile is summed over the group in registers).
#include "common.hpp"

namespace vissm {
namespace flow2 {

constexpr int P = 32;    // head positions per tile (MFMA columns: 2 blocks of 16)
constexpr int S = 16;    // samples per group
constexpr int HP = 64;   // padded hidden width
constexpr int PS = 33;   // LDS row stride of [h][p] tiles
constexpr int NT = 256;
constexpr int US = 2 * P + 64 + 8;  // u window staging

using f4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f4 mma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct Geom {
  int s, Lout, Lh, S, n_groups, n_tiles, CH, n_chunks;
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
  const int target_blocks = 2048;
  int want = (target_blocks + g.n_groups - 1) / g.n_groups;
  int max_chunks = g.n_tiles / ch_min_tiles;
  if (max_chunks < 1) max_chunks = 1;
  int nc = want < max_chunks ? want : max_chunks;
  if (nc < 1) nc = 1;
  int tiles_per_chunk = (g.n_tiles + nc - 1) / nc;
  if (d->chunk_tiles > 0) tiles_per_chunk = d->chunk_tiles;  // caller-forced chunk geometry (tests)
  if (tiles_per_chunk < ch_min_tiles) tiles_per_chunk = ch_min_tiles;
  g.CH = tiles_per_chunk * P;
  g.n_chunks = (g.Lh + g.CH - 1) / g.CH;
  return g;
}

static int n_wgrad(const VissmFlowDesc* d) {
  const int H = d->H, k = d->k, nh = d->n_hidden;
  return k * H + nh * H * H + 3 * nh * H + 2 * H + 2;
}

// padded weight images in the workspace (all [64][64] fp32, zero padded)
struct WImg {
  float* wp;     // [nh][h_in][h_out]
  float* wtp;    // [nh][h_out][h_in]
  float* weps;   // [j][h]
  float* wepsT;  // [h][j]
  float* bh;     // [nh][64]
  float* bng;    // [nh][64] (gamma * bn scale)
  float* bnb;    // [nh][64]
  float* whead;  // [2][64] + [2]
};

struct WsF {
  WImg w;
  float* ls_slab;
};
struct WsB {
  WImg w;
  float *dC_slab, *dth_slab, *dW_slab, *halo, *wred;
};

template <class F>
static size_t take_wimg(const VissmFlowDesc* d, F take, WImg* w) {
  const int nh = d->n_hidden > 0 ? d->n_hidden : 1;
  w->wp = take(static_cast<size_t>(nh) * HP * HP);
  w->wtp = take(static_cast<size_t>(nh) * HP * HP);
  w->weps = take(HP * HP);
  w->wepsT = take(HP * HP);
  w->bh = take(nh * HP);
  w->bng = take(nh * HP);
  w->bnb = take(nh * HP);
  w->whead = take(2 * HP + 2);
  return 0;
}

static size_t fwd_ws_layout(const VissmFlowDesc* d, const Geom& g, char* base, WsF* w) {
  size_t off = 0;
  auto take = [&](size_t nfl) { float* p = base ? reinterpret_cast<float*>(base + off) : nullptr; off += align_up(nfl * 4); return p; };
  WsF t;
  take_wimg(d, take, &t.w);
  t.ls_slab = take(static_cast<size_t>(g.n_chunks) * d->B);
  if (w) *w = t;
  return off;
}

static size_t bwd_ws_layout(const VissmFlowDesc* d, const Geom& g, char* base, WsB* w) {
  size_t off = 0;
  auto take = [&](size_t nfl) { float* p = base ? reinterpret_cast<float*>(base + off) : nullptr; off += align_up(nfl * 4); return p; };
  WsB t;
  take_wimg(d, take, &t.w);
  t.dC_slab = take(static_cast<size_t>(g.n_groups) * g.Lh * d->H);
  t.dth_slab = take(static_cast<size_t>(g.n_chunks) * d->B * d->H);
  t.dW_slab = take(static_cast<size_t>(g.n_groups) * g.n_chunks * n_wgrad(d));
  t.halo = take(static_cast<size_t>(d->B) * g.n_chunks * d->k);
  t.wred = take(n_wgrad(d));
  if (w) *w = t;
  return off;
}

__global__ void prep_kernel(VissmFlowParams w, int H, int k, int nh, int bn, WImg img) {
  const int i = threadIdx.x & 63, j = threadIdx.x >> 6;  // 64 x 4 threads
  for (int r = j; r < HP; r += 4) {
    for (int l = 0; l < nh; ++l) {
      const float v = (r < H && i < H) ? w.w_hid[(static_cast<size_t>(l) * H + r) * H + i] : 0.f;
      img.wp[(l * HP + r) * HP + i] = v;   // [h_in = r][h_out = i]
      img.wtp[(l * HP + i) * HP + r] = v;  // [h_out = i][h_in = r]
    }
    const float e = (r < k && i < H) ? w.w_eps[r * H + i] : 0.f;
    img.weps[r * HP + i] = e;   // [j = r][h = i]
    img.wepsT[i * HP + r] = e;  // [h = i][j = r]
  }
  if (j == 0) {
    for (int l = 0; l < nh; ++l) {
      img.bh[l * HP + i] = i < H ? w.b_hid[l * H + i] : 0.f;
      img.bng[l * HP + i] = (bn && i < H) ? w.bn_g[l * H + i] * kBnScale : 1.f;
      img.bnb[l * HP + i] = (bn && i < H) ? w.bn_b[l * H + i] : 0.f;
    }
    img.whead[i] = i < H ? w.w_head[i * 2 + 0] : 0.f;
    img.whead[HP + i] = i < H ? w.w_head[i * 2 + 1] : 0.f;
    if (i < 2) img.whead[2 * HP + i] = w.b_head[i];
  }
}

struct KArgs {
  int B, L, k, H, bn, s, swap_out, n_logsig, n_win, Lout, Lh, CH, n_chunks, S;
  int pL, pLo;  // row strides of u / du and u_next / du_next (VissmFlowDesc.u_pitch / out_pitch)
  int KS;  // k-steps of the sample-channel conv: ceil(k/4)
  int HK;  // k-steps over hidden units: ceil(H/4)
};

// shared-memory image of one work unit
template <int NH>
struct Smem {
  float act[NH + 1][HP][PS];  // post-ELU activations E_l [h][p]
  float dz[HP][PS];           // gradient scratch [h][p]
  float us[US];               // u window
  float go[2 * P];            // upstream gradient of the tile's outputs
  float red[4][2][P];         // head partial sums per wave
  float mu[P], rr[P], sig[P], gmu[P], gr[P];
  float ths[HP];              // theta term of the sample
  float bng[NH > 0 ? NH : 1][HP], bnb[NH > 0 ? NH : 1][HP];
};

// ---------------------------------------------------------------------------
// forward of one work unit.  On return: act[] filled, xh[cb][r] (the head's
// input for this lane's rows/cols) in registers, mu/rr/sig in LDS.
// ---------------------------------------------------------------------------
template <int NH, int HK, int KS>
__device__ __forceinline__ void unit_forward(const KArgs& a, Smem<NH>& sm, const WImg& W, const f4 (&cinit)[2],
                                             f4 (&xh)[2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  // ---- layer 0: A0^T = W_eps^T U + C^T + theta ----
  f4 acc[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    acc[cb] = cinit[cb];
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[cb][r] += sm.ths[16 * w + 4 * lk + r];
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int j = 4 * s + lk;
    const float wa = W.weps[j * HP + 16 * w + li];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) acc[cb] = mma(wa, sm.us[a.s * (16 * cb + li) + j], acc[cb]);
  }
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 16 * w + 4 * lk + r;
      const float e = h < a.H ? elu_f(acc[cb][r]) : 0.f;
      acc[cb][r] = e;
      sm.act[0][h][16 * cb + li] = e;
    }
  // ---- hidden layers ----
#pragma unroll
  for (int l = 0; l < NH; ++l) {
    __syncthreads();
    f4 z[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) z[cb][r] = W.bh[l * HP + 16 * w + 4 * lk + r];
    const float* wl = W.wp + l * HP * HP;
#pragma unroll 4
    for (int s = 0; s < HK; ++s) {
      const int hin = 4 * s + lk;
      const float wa = wl[hin * HP + 16 * w + li];
      float g = 1.f, be = 0.f;
      if (l > 0) {
        g = sm.bng[l - 1][hin];
        be = sm.bnb[l - 1][hin];
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) z[cb] = mma(wa, fmaf(g, sm.act[l][hin][16 * cb + li], be), z[cb]);
    }
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * w + 4 * lk + r;
        const float e = h < a.H ? elu_f(z[cb][r]) : 0.f;
        sm.act[l + 1][h][16 * cb + li] = e;
        acc[cb][r] = a.bn ? fmaf(sm.bng[l][h], e, sm.bnb[l][h]) : e;
      }
  }
  // ---- head: mu, r = X_nh . w_head + b ----
  {
    float pm[2], pr[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      float m = 0.f, q = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * w + 4 * lk + r;
        m = fmaf(acc[cb][r], W.whead[h], m);
        q = fmaf(acc[cb][r], W.whead[HP + h], q);
      }
      m += __shfl_xor(m, 16, 64);
      m += __shfl_xor(m, 32, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      pm[cb] = m;
      pr[cb] = q;
      xh[cb] = acc[cb];
    }
    if (lk == 0) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        sm.red[w][0][16 * cb + li] = pm[cb];
        sm.red[w][1][16 * cb + li] = pr[cb];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < P) {
    const int p = threadIdx.x;
    const float m = sm.red[0][0][p] + sm.red[1][0][p] + sm.red[2][0][p] + sm.red[3][0][p] + W.whead[2 * HP];
    const float q = sm.red[0][1][p] + sm.red[1][1][p] + sm.red[2][1][p] + sm.red[3][1][p] + W.whead[2 * HP + 1];
    sm.mu[p] = m;
    sm.rr[p] = q;
    sm.sig[p] = softplus_f(q) + 1e-10f;
  }
  __syncthreads();
}

// initial accumulator = C^T tile for the lane's rows / columns
__device__ __forceinline__ void load_cinit(const KArgs& a, const float* __restrict__ C, int win, int m0, int nP,
                                           f4 (&ci)[2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int p = 16 * cb + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 16 * w + 4 * lk + r;
      ci[cb][r] = (p < nP && h < a.H) ? C[(static_cast<size_t>(win) * a.Lh + m0 + p) * a.H + h] : 0.f;
    }
  }
}

template <int NH>
__device__ __forceinline__ void load_unit_inputs(const KArgs& a, Smem<NH>& sm, const float* __restrict__ ub,
                                                 const float* __restrict__ thb, int t0) {
  const int tid = threadIdx.x;
  const int span = a.s * P + a.k + 2;
  for (int q = tid; q < US; q += NT) sm.us[q] = (q < span && t0 + q < a.L) ? ub[t0 + q] : 0.f;
  if (tid < HP) sm.ths[tid] = tid < a.H ? thb[tid] : 0.f;
}

template <int NH>
__device__ __forceinline__ void load_bn(const KArgs& a, Smem<NH>& sm, const WImg& W) {
  const int tid = threadIdx.x;
  for (int i = tid; i < (NH > 0 ? NH : 1) * HP; i += NT) {
    (&sm.bng[0][0])[i] = NH > 0 ? W.bng[i] : 1.f;
    (&sm.bnb[0][0])[i] = NH > 0 ? W.bnb[i] : 0.f;
  }
}

// ---------------------------------------------------------------------------
// forward kernel: samples outer, tiles inner
// ---------------------------------------------------------------------------
template <int NH, int HK, int KS>
__global__ __launch_bounds__(NT, 2) void fwd_kernel(KArgs a, const float* __restrict__ u, const float* __restrict__ C,
                                                    const int32_t* __restrict__ win, const float* __restrict__ tht,
                                                    WImg W, float* __restrict__ u_next,
                                                    float* __restrict__ ls_slab) {
  __shared__ Smem<NH> sm;
  const int tid = threadIdx.x;
  const int g = blockIdx.x, c = blockIdx.y;
  const int m_lo = c * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  load_bn<NH>(a, sm, W);
  for (int bl = 0; bl < a.S; ++bl) {
    const int b = g * a.S + bl;
    if (b >= a.B) break;
    const int wi = win ? win[b] : 0;
    const float* ub = u + static_cast<size_t>(b) * a.pL;
    float* ob = u_next + static_cast<size_t>(b) * a.pLo;
    float ls_acc = 0.f;
    for (int m0 = m_lo; m0 < m_hi; m0 += P) {
      const int nP = min(P, m_hi - m0);
      const int t0 = a.s * m0;
      __syncthreads();
      load_unit_inputs<NH>(a, sm, ub, tht + static_cast<size_t>(b) * a.H, t0);
      f4 ci[2], xh[2];
      load_cinit(a, C, wi, m0, nP, ci);
      __syncthreads();
      unit_forward<NH, HK, KS>(a, sm, W, ci, xh);
      if (tid < nP) {
        const int p = tid;
        const float sg = sm.sig[p];
        const int o = t0 + a.s * p + (a.s - 1);
        ob[a.swap_out ? (o ^ 1) : o] = sm.us[a.s * p + (a.s - 1) + a.k] * sg + sm.mu[p];
        if (a.s == 2) {
          const int oe = t0 + 2 * p;
          ob[a.swap_out ? (oe ^ 1) : oe] = sm.us[2 * p + a.k];
        }
        if (o >= a.Lout - a.n_logsig) ls_acc += logf(sg);
      }
    }
    const float v = wave_sum(tid < 64 ? ls_acc : 0.f);
    if (tid == 0) ls_slab[static_cast<size_t>(c) * a.B + b] = v;
  }
}

// sum over the 16 lanes that share lk (xor over li)
__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

// ---------------------------------------------------------------------------
// backward kernel: tiles outer, samples inner
// ---------------------------------------------------------------------------
template <int NH, int HK, int KS>
__global__ __launch_bounds__(NT, 2) void bwd_kernel(KArgs a, const float* __restrict__ u, const float* __restrict__ C,
                                                    const int32_t* __restrict__ win, const float* __restrict__ tht,
                                                    const float* __restrict__ gout, const float* __restrict__ dls,
                                                    WImg W, float* __restrict__ du, float* __restrict__ dC_slab,
                                                    float* __restrict__ dth_slab, float* __restrict__ dW_slab,
                                                    float* __restrict__ halo) {
  __shared__ Smem<NH> sm;
  __shared__ float carry[S][64];
  __shared__ float dth[S][HP];
  __shared__ float dul[US];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int g = blockIdx.x, c = blockIdx.y;
  const int m_lo = c * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int b_lo = g * a.S, nb = min(a.S, a.B - b_lo);
  constexpr int NHA = NH > 0 ? NH : 1;
  constexpr int njb = (4 * KS + 15) >> 4;  // row blocks of dW_eps / dcon (j)

  // weight-gradient accumulators (wave w: rows 16w..16w+15 of dW_l; column block w of dW_eps)
  f4 dWl[NHA][4];
  f4 dWe[njb];
  float dbl[NHA][4], dgl[NHA][4], dbe[NHA][4];
  float dwh0[4], dwh1[4];
  float dbh0 = 0.f, dbh1 = 0.f;
#pragma unroll
  for (int l = 0; l < NHA; ++l)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dWl[l][r] = f4{0.f, 0.f, 0.f, 0.f};
      dbl[l][r] = dgl[l][r] = dbe[l][r] = 0.f;
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) dwh0[r] = dwh1[r] = 0.f;
#pragma unroll
  for (int r = 0; r < njb; ++r) dWe[r] = f4{0.f, 0.f, 0.f, 0.f};
  load_bn<NH>(a, sm, W);
  for (int i = tid; i < S * 64; i += NT) {
    (&carry[0][0])[i] = 0.f;
    (&dth[0][0])[i] = 0.f;
  }

  for (int m0 = m_lo; m0 < m_hi; m0 += P) {
    const int nP = min(P, m_hi - m0);
    const int t0 = a.s * m0;
    f4 dCa[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
    f4 ci[2];
    int cached = -1;

    for (int bl = 0; bl < nb; ++bl) {
      const int b = b_lo + bl;
      const int wi = win ? win[b] : 0;
      const float* ub = u + static_cast<size_t>(b) * a.pL;
      const float* gb = gout + static_cast<size_t>(b) * a.pLo;
      __syncthreads();
      load_unit_inputs<NH>(a, sm, ub, tht + static_cast<size_t>(b) * a.H, t0);
      for (int q = tid; q < 2 * P; q += NT) {
        const int o = t0 + q;
        sm.go[q] = (q < a.s * nP) ? gb[a.swap_out ? (o ^ 1) : o] : 0.f;
      }
      for (int q = tid; q < US; q += NT) dul[q] = 0.f;
      if (wi != cached) {
        load_cinit(a, C, wi, m0, nP, ci);
        cached = wi;
      }
      __syncthreads();
      f4 xh[2];
      unit_forward<NH, HK, KS>(a, sm, W, ci, xh);

      // ---- head backward (per position) ----
      if (tid < P) {
        const int p = tid;
        const float r = sm.rr[p], sg = sm.sig[p];
        const int oq = a.s * p + (a.s - 1);
        const float gv = p < nP ? sm.go[oq] : 0.f;
        float dsig = gv * sm.us[oq + a.k];
        if (p < nP && t0 + oq >= a.Lout - a.n_logsig) dsig += dls[b] / sg;
        const float dr = dsig * sigmoid_f(r);
        sm.gmu[p] = gv;
        sm.gr[p] = dr;
        dbh0 += gv;
        dbh1 += dr;
      }
      __syncthreads();
      f4 dx[2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const float gm = sm.gmu[16 * cb + li], gq = sm.gr[16 * cb + li];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = 16 * w + 4 * lk + r;
          dx[cb][r] = W.whead[h] * gm + W.whead[HP + h] * gq;
          dwh0[r] = fmaf(xh[cb][r], gm, dwh0[r]);
          dwh1[r] = fmaf(xh[cb][r], gq, dwh1[r]);
        }
      }

      // ---- hidden layers backward ----
#pragma unroll
      for (int l = NH - 1; l >= 0; --l) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = 16 * w + 4 * lk + r;
            const float e = sm.act[l + 1][h][16 * cb + li];
            float de = dx[cb][r];
            if (a.bn) {
              dgl[l][r] = fmaf(de, e, dgl[l][r]);
              dbe[l][r] += de;
              de *= sm.bng[l][h];
            }
            const float dzv = de * elu_grad_from_out(e);
            dbl[l][r] += dzv;
            sm.dz[h][16 * cb + li] = dzv;
          }
        __syncthreads();
        // dX_l[h_in][p] = sum_h_out W[h_in][h_out] dz[h_out][p]   (rows h_in of this wave)
        f4 nx[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
        const float* wt = W.wtp + l * HP * HP;
#pragma unroll 4
        for (int s = 0; s < HK; ++s) {
          const int ho = 4 * s + lk;
          const float wa = wt[ho * HP + 16 * w + li];
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) nx[cb] = mma(wa, sm.dz[ho][16 * cb + li], nx[cb]);
        }
        // dW_l[h_in][h_out] += sum_p X_l[h_in][p] dz[h_out][p]   (h_in rows 16w.., all h_out blocks)
        {
          const int hin = 16 * w + li;
          float gi = 1.f, bi = 0.f;
          if (l > 0) {
            gi = sm.bng[l - 1][hin];
            bi = sm.bnb[l - 1][hin];
          }
#pragma unroll
          for (int s = 0; s < P / 4; ++s) {
            const int p = 4 * s + lk;
            const float xa = fmaf(gi, sm.act[l][hin][p], bi);
#pragma unroll
            for (int ob = 0; ob < 4; ++ob) dWl[l][ob] = mma(xa, sm.dz[16 * ob + li][p], dWl[l][ob]);
          }
        }
        __syncthreads();
        dx[0] = nx[0];
        dx[1] = nx[1];
      }

      // ---- first layer ----
      {
        float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = 16 * w + 4 * lk + r;
            const int p = 16 * cb + li;
            const float da = (p < nP) ? dx[cb][r] * elu_grad_from_out(sm.act[0][h][p]) : 0.f;
            dCa[cb][r] += da;
            rs[r] += da;
            sm.dz[h][p] = da;
          }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = sum16(rs[r]);
          if (li == 0) dth[bl][16 * w + 4 * lk + r] += v;
        }
      }
      __syncthreads();
      // dW_eps[j][h] += sum_p U[j][p] dA0[h][p]   (wave w: h block w, all j blocks)
#pragma unroll
      for (int s = 0; s < P / 4; ++s) {
        const int p = 4 * s + lk;
        const float bz = sm.dz[16 * w + li][p];
#pragma unroll
        for (int jb = 0; jb < njb; ++jb) dWe[jb] = mma(sm.us[a.s * p + 16 * jb + li], bz, dWe[jb]);
      }
      // dcon[j][p] = sum_h w_eps[j][h] dA0[h][p]  (block pairs (jb, cb) spread over waves)
      f4 dcn[2];
      int npair = 0;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int pair = w + 4 * q;
        dcn[q] = f4{0.f, 0.f, 0.f, 0.f};
        if (pair < 2 * njb) {
          const int jb = pair >> 1, cb = pair & 1;
#pragma unroll 4
          for (int s = 0; s < HK; ++s) {
            const int hh = 4 * s + lk;
            dcn[q] = mma(W.wepsT[hh * HP + 16 * jb + li], sm.dz[hh][16 * cb + li], dcn[q]);
          }
          npair = q + 1;
        }
      }
      __syncthreads();
      // park dcon in act[0] (free now): [j][p]
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (q < npair) {
          const int pair = w + 4 * q;
          const int jb = pair >> 1, cb = pair & 1;
#pragma unroll
          for (int r = 0; r < 4; ++r) sm.act[0][16 * jb + 4 * lk + r][16 * cb + li] = dcn[q][r];
        }
      }
      __syncthreads();
      // du over local positions q in [0, s*nP + k)
      const int fin = a.s * nP;
      float* db = du + static_cast<size_t>(b) * a.pL;
      for (int q = tid; q < fin + a.k; q += NT) {
        float v = 0.f;
        for (int j = 0; j < a.k; ++j) {
          const int t = q - j;
          if (t >= 0) {
            if (a.s == 1) {
              if (t < nP) v += sm.act[0][j][t];
            } else if (!(t & 1) && (t >> 1) < nP) {
              v += sm.act[0][j][t >> 1];
            }
          }
        }
        const int oq = q - a.k;
        if (oq >= 0 && oq < fin) {
          if (a.s == 1) v += sm.go[oq] * sm.sig[oq];
          else v += (oq & 1) ? sm.go[oq] * sm.sig[oq >> 1] : sm.go[oq];
        }
        if (q < a.k) v += carry[bl][q];
        if (q < fin) db[t0 + q] = v;
        else dul[q - fin] = v;
      }
      __syncthreads();
      for (int q = tid; q < a.k; q += NT) carry[bl][q] = dul[q];
    }  // samples

    // dC tile of this group
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * w + 4 * lk + r, p = 16 * cb + li;
        if (p < nP && h < a.H) dC_slab[(static_cast<size_t>(g) * a.Lh + m0 + p) * a.H + h] = dCa[cb][r];
      }
  }  // tiles

  __syncthreads();
  for (int bl = 0; bl < nb; ++bl) {
    const int b = b_lo + bl;
    for (int q = tid; q < a.k; q += NT) {
      if (c == a.n_chunks - 1) du[static_cast<size_t>(b) * a.pL + a.Lout + q] = carry[bl][q];
      else halo[(static_cast<size_t>(b) * a.n_chunks + c) * a.k + q] = carry[bl][q];
    }
    if (tid < a.H) dth_slab[(static_cast<size_t>(c) * a.B + b) * a.H + tid] = dth[bl][tid];
  }

  // ---- weight-gradient partials of this block ----
  const int H = a.H;
  const int nW = a.k * H + NH * H * H + 3 * NH * H + 2 * H + 2;
  float* ws = dW_slab + (static_cast<size_t>(g) * a.n_chunks + c) * nW;
  // w_eps [k][H]: dWe[jb][r] = dW_eps[j = 16 jb + 4 lk + r][h = 16 w + li]
#pragma unroll
  for (int jb = 0; jb < njb; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jb + 4 * lk + r, h = 16 * w + li;
      if (j < a.k && h < H) ws[j * H + h] = dWe[jb][r];
    }
  int off = a.k * H;
  // w_hid [l][h_in][h_out]: dWl[l][ob][r] = dW[h_in = 16 w + 4 lk + r][h_out = 16 ob + li]
#pragma unroll
  for (int l = 0; l < NH; ++l)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hi = 16 * w + 4 * lk + r, ho = 16 * ob + li;
        if (hi < H && ho < H) ws[off + (l * H + hi) * H + ho] = dWl[l][ob][r];
      }
  off += NH * H * H;
  // per-row sums over the lane's columns: reduce over li, lane li == 0 writes
  auto put_rows = [&](const float (&v)[4], int dst, int stride) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = sum16(v[r]);
      const int h = 16 * w + 4 * lk + r;
      if (li == 0 && h < H) ws[dst + h * stride] = s;
    }
  };
#pragma unroll
  for (int l = 0; l < NH; ++l) put_rows(dbl[l], off + l * H, 1);
  off += NH * H;
#pragma unroll
  for (int l = 0; l < NH; ++l) put_rows(dgl[l], off + l * H, 1);  // d gamma (x bn scale applied below)
  off += NH * H;
#pragma unroll
  for (int l = 0; l < NH; ++l) put_rows(dbe[l], off + l * H, 1);
  off += NH * H;
  put_rows(dwh0, off + 0, 2);
  put_rows(dwh1, off + 1, 2);
  off += 2 * H;
  // b_head: threads 0..31 of wave 0 hold per-position partials
  float s0 = (tid < P) ? dbh0 : 0.f, s1 = (tid < P) ? dbh1 : 0.f;
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  if (tid == 0) {
    ws[off + 0] = s0;
    ws[off + 1] = s1;
  }
}

static KArgs make_args(const VissmFlowDesc* d, const Geom& g) {
  KArgs a;
  a.B = d->B; a.L = d->L; a.k = d->k; a.H = d->H; a.bn = d->bn; a.s = g.s; a.swap_out = d->swap_out;
  a.pL = d->u_pitch ? d->u_pitch : d->L; a.pLo = d->out_pitch ? d->out_pitch : g.Lout;
  a.n_logsig = d->n_logsig; a.n_win = d->n_win; a.Lout = g.Lout; a.Lh = g.Lh; a.CH = g.CH; a.n_chunks = g.n_chunks;
  a.S = g.S;
  a.KS = (d->k + 3) / 4;
  a.HK = (d->H + 3) / 4;
  return a;
}

}  // namespace flow2

// ---------------------------------------------------------------------------
// entry points used by flow_api.cpp
// ---------------------------------------------------------------------------
// (HK, KS) buckets: hidden k-steps ceil(H/4) and sample-channel k-steps ceil(k/4), rounded up to
// the shapes of the reference configs; the generic <NH, 16, 16> covers any H <= 64, k <= 64 (the
// padded weight images are zero beyond H and k, so extra k-steps add zeros).
#define FLOW2_CASES(KERNEL, nh, hk, ks, ...)                                                      \
  do {                                                                                            \
    if (hk == 13 && ks == 2 && nh == 1) hipLaunchKernelGGL((KERNEL<1, 13, 2>), __VA_ARGS__);      \
    else if (hk == 13 && ks == 13 && nh == 1) hipLaunchKernelGGL((KERNEL<1, 13, 13>), __VA_ARGS__); \
    else if (hk == 13 && ks == 5 && nh == 3) hipLaunchKernelGGL((KERNEL<3, 13, 5>), __VA_ARGS__);  \
    else if (hk == 13 && ks == 13 && nh == 3) hipLaunchKernelGGL((KERNEL<3, 13, 13>), __VA_ARGS__); \
    else switch (nh) {                                                                            \
        case 0: hipLaunchKernelGGL((KERNEL<0, 16, 16>), __VA_ARGS__); break;                      \
        case 1: hipLaunchKernelGGL((KERNEL<1, 16, 16>), __VA_ARGS__); break;                      \
        case 2: hipLaunchKernelGGL((KERNEL<2, 16, 16>), __VA_ARGS__); break;                      \
        case 3: hipLaunchKernelGGL((KERNEL<3, 16, 16>), __VA_ARGS__); break;                      \
        default: hipLaunchKernelGGL((KERNEL<4, 16, 16>), __VA_ARGS__); break;                     \
      }                                                                                           \
  } while (0)

static void buckets(const VissmFlowDesc* d, int* hk, int* ks) {
  *hk = d->H <= 52 ? 13 : 16;
  const int kk = (d->k + 3) / 4;
  *ks = kk <= 2 ? 2 : kk <= 5 ? 5 : kk <= 13 ? 13 : 16;
  if (*hk == 16) *ks = 16;
}

size_t flow2_workspace_size(const VissmFlowDesc* d, int backward) {
  using namespace flow2;
  Geom g = geom(d, backward != 0);
  return backward ? bwd_ws_layout(d, g, nullptr, nullptr) : fwd_ws_layout(d, g, nullptr, nullptr);
}

void flow2_geometry(const VissmFlowDesc* d, int backward, int32_t* out) {
  using namespace flow2;
  Geom g = geom(d, backward != 0);
  out[0] = P; out[1] = g.CH / P; out[2] = g.n_chunks; out[3] = g.n_groups;
}

int flow2_fwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
              const float* theta_term, float* u_next, float* logsig, void* workspace, size_t ws_bytes,
              hipStream_t st) {
  using namespace flow2;
  Geom g = geom(d, false);
  VISSM_CHECK_ARG(workspace && ws_bytes >= fwd_ws_layout(d, g, nullptr, nullptr), "flow_fwd: workspace too small");
  WsF ws;
  fwd_ws_layout(d, g, reinterpret_cast<char*>(workspace), &ws);
  hipLaunchKernelGGL(prep_kernel, dim3(1), dim3(256), 0, st, *w, d->H, d->k, d->n_hidden, d->bn, ws.w);
  VISSM_CHECK_LAUNCH("flow2_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid(g.n_groups, g.n_chunks);
  int hk, ks;
  buckets(d, &hk, &ks);
  prof_begin(VISSM_PROF_FLOW_FWD, st);
  FLOW2_CASES(fwd_kernel, d->n_hidden, hk, ks, grid, dim3(NT), 0, st, a, u, C, wn, theta_term, ws.w, u_next,
              ws.ls_slab);
  VISSM_CHECK_LAUNCH("flow2_fwd");
  prof_end(VISSM_PROF_FLOW_FWD, st);
  return launch_reduce_rows(ws.ls_slab, logsig, g.n_chunks, d->B, st);
}

int flow2_bwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
              const float* theta_term, const float* du_next, const float* dlogsig, float* du, float* dC,
              float* dtheta_term, const VissmFlowGrads* gr, void* workspace, size_t ws_bytes, hipStream_t st) {
  using namespace flow2;
  Geom g = geom(d, true);
  VISSM_CHECK_ARG(workspace && ws_bytes >= bwd_ws_layout(d, g, nullptr, nullptr), "flow_bwd: workspace too small");
  WsB ws;
  bwd_ws_layout(d, g, reinterpret_cast<char*>(workspace), &ws);
  hipLaunchKernelGGL(prep_kernel, dim3(1), dim3(256), 0, st, *w, d->H, d->k, d->n_hidden, d->bn, ws.w);
  VISSM_CHECK_LAUNCH("flow2_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid(g.n_groups, g.n_chunks);
  int hk, ks;
  buckets(d, &hk, &ks);
  prof_begin(VISSM_PROF_FLOW_BWD, st);
  prof_begin(VISSM_PROF_FLOW_BWD_DU, st);
  FLOW2_CASES(bwd_kernel, d->n_hidden, hk, ks, grid, dim3(NT), 0, st, a, u, C, wn, theta_term, du_next, dlogsig, ws.w,
              du, ws.dC_slab, ws.dth_slab, ws.dW_slab, ws.halo);
  VISSM_CHECK_LAUNCH("flow2_bwd");
  prof_end(VISSM_PROF_FLOW_BWD_DU, st);
  prof_end(VISSM_PROF_FLOW_BWD, st);
  int rc = launch_halo_fixup(du, ws.halo, d->B, d->L, a.pL, d->k, g.n_chunks, g.s, g.CH, st);
  if (rc) return rc;
  const int64_t nC = static_cast<int64_t>(g.Lh) * d->H;
  if (d->n_win == 1) {
    rc = launch_reduce_rows(ws.dC_slab, dC, g.n_groups, nC, st);
    if (rc) return rc;
  } else {
    rc = launch_reduce_by_window(ws.dC_slab, win, dC, d->B, d->n_win, nC, st);
    if (rc) return rc;
  }
  rc = launch_reduce_rows(ws.dth_slab, dtheta_term, g.n_chunks, static_cast<int64_t>(d->B) * d->H, st);
  if (rc) return rc;
  const int nW = n_wgrad(d);
  rc = launch_reduce_rows(ws.dW_slab, ws.wred, static_cast<int64_t>(g.n_groups) * g.n_chunks, nW, st);
  if (rc) return rc;
  return launch_scatter_wgrad(ws.wred, gr, d->k, d->H, d->n_hidden, d->bn, st);
}

}  // namespace vissm
