// IAF flow of the neural-MA sampler on the matrix cores (exact fp32:
// v_mfma_f32_16x16x4_f32), forward and backward -- latency-hiding version.
//
// Changes over flow_v2.hip (same algorithm, same decomposition), all aimed at
// the 74 % of wave cycles that v2/v3 spent waiting (rocprofv3 SQ_WAIT_ANY):
//   * [h][p] LDS tiles are 32-float rows with an XOR swizzle that makes both the
//     row reads (forward / dX products) and the column reads (dW products)
//     bank-conflict free (v2: SQ_LDS_BANK_CONFLICT > LDS instruction cycles);
//   * the next work unit's inputs (u window, upstream gradient, theta term,
//     window index, d logsig) are prefetched into registers while the current
//     unit computes; vmcnt retires loads in issue order, so the compute phase
//     issues no other global loads: biases / head / BN vectors live in LDS and,
//     for one hidden layer (the AR configs), each wave keeps its MFMA A-operand
//     weight slices in VGPRs for the block's lifetime;
//   * fewer block barriers per unit (head finalised redundantly per lane, dcon
//     parked without an extra barrier, carry ping-pong buffer).
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
namespace flow4 {

constexpr int P = 32;    // head positions per tile (MFMA columns: 2 blocks of 16)
constexpr int S = 16;    // samples per group
constexpr int HP = 64;   // padded hidden width
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

// XOR-swizzled [h][32] tile index: rows h and h+1 use opposite bank halves
// (row reads of 16 columns x 2 rows), and 16 consecutive rows map to 16 distinct
// bank pairs (column reads of 16 rows x 2 adjacent columns).
__device__ __forceinline__ int sw(int h, int p) {
  return (h << 5) | (p ^ (((h & 1) << 4) | (((h >> 1) & 7) << 1)));
}

template <int NH>
struct Smem {
  float act[NH + 1][HP * P];  // post-ELU activations E_l, swizzled [h][p]
  float dz[HP * P];           // gradient scratch, swizzled [h][p]
  float us[US];               // u window
  float go[2 * P];            // upstream gradient of the tile's outputs
  float red[4][2][P];         // head partial sums per wave
  float ths[HP];              // theta term of the sample
  float bh[NH > 0 ? NH : 1][HP];
  float bng[NH > 0 ? NH : 1][HP], bnb[NH > 0 ? NH : 1][HP];
  float whead[2 * HP + 2];
  float sig[P];               // sigma per head position (for the pass-through gradient)
  float dls;                  // d loss / d logsig of the sample
};

// for s in [0, N): fully unrolled when the body indexes VGPR-resident arrays
// (a runtime index would send them to scratch), unrolled by 4 otherwise.
template <bool FULL, int N, class F>
__device__ __forceinline__ void kloop(F&& f) {
  if constexpr (FULL) {
#pragma unroll
    for (int s = 0; s < N; ++s) f(s);
  } else {
#pragma unroll 4
    for (int s = 0; s < N; ++s) f(s);
  }
}

// per-wave MFMA A-operand weight slices (VGPR-resident when WREG)
// dcon block pairs (jb, column block): 2 * ceil(4 KS / 16), spread as w, w + 4
template <int KS>
struct Pairs {
  static constexpr int njb = (4 * KS + 15) >> 4;
  static constexpr int per_wave = (2 * njb + 3) / 4;
};

template <int HK, int KS, bool WREG>
struct WRegs {
  float wf[WREG ? HK : 1], wb[WREG ? HK : 1], we[WREG ? KS : 1];
  float wc[WREG ? Pairs<KS>::per_wave : 1][WREG ? HK : 1];
};

struct Lane {
  int lane, w, li, lk;
  __device__ Lane() : lane(threadIdx.x & 63), w(threadIdx.x >> 6), li((threadIdx.x & 63) & 15),
                      lk((threadIdx.x & 63) >> 4) {}
  __device__ int row(int r) const { return 16 * w + 4 * lk + r; }
};

template <int NH>
__device__ __forceinline__ void load_block_consts(Smem<NH>& sm, const WImg& W) {
  constexpr int NHA = NH > 0 ? NH : 1;
  for (int i = threadIdx.x; i < NHA * HP; i += NT) {
    (&sm.bh[0][0])[i] = NH > 0 ? W.bh[i] : 0.f;
    (&sm.bng[0][0])[i] = NH > 0 ? W.bng[i] : 1.f;
    (&sm.bnb[0][0])[i] = NH > 0 ? W.bnb[i] : 0.f;
  }
  for (int i = threadIdx.x; i < 2 * HP + 2; i += NT) sm.whead[i] = W.whead[i];
}

template <int HK, int KS, bool WREG>
__device__ __forceinline__ void load_wregs(const WImg& W, WRegs<HK, KS, WREG>& R, int njb) {
  if constexpr (WREG) {
    const Lane L;
#pragma unroll
    for (int s = 0; s < HK; ++s) {
      R.wf[s] = W.wp[(4 * s + L.lk) * HP + 16 * L.w + L.li];
      R.wb[s] = W.wtp[(4 * s + L.lk) * HP + 16 * L.w + L.li];
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) R.we[s] = W.weps[(4 * s + L.lk) * HP + 16 * L.w + L.li];
#pragma unroll
    for (int q = 0; q < Pairs<KS>::per_wave; ++q) {
      const int pair = L.w + 4 * q;
      const int pjb = pair >> 1;
      if (pair < 2 * njb) {
#pragma unroll
        for (int s = 0; s < HK; ++s) R.wc[q][s] = W.wepsT[(4 * s + L.lk) * HP + 16 * pjb + L.li];
      }
    }
  }
}

// prefetched inputs of one work unit (registers of the thread that stores them)
struct Pre {
  float u, go, th, dls;
  int win;
};

__device__ __forceinline__ void prefetch(const KArgs& a, const float* __restrict__ u, const float* __restrict__ gout,
                                         const float* __restrict__ tht, const float* __restrict__ dls,
                                         const int32_t* __restrict__ win, int b, int t0, int nP, Pre& pf) {
  const int tid = threadIdx.x;
  const int span = a.s * P + a.k + 2;
  pf.u = (tid < span && t0 + tid < a.L) ? u[static_cast<size_t>(b) * a.pL + t0 + tid] : 0.f;
  pf.go = 0.f;
  if (gout && tid < a.s * nP) {
    const int o = t0 + tid;
    pf.go = gout[static_cast<size_t>(b) * a.pLo + (a.swap_out ? (o ^ 1) : o)];
  }
  pf.th = tid < a.H ? tht[static_cast<size_t>(b) * a.H + tid] : 0.f;
  pf.dls = (dls && tid == 0) ? dls[b] : 0.f;
  pf.win = (win && (tid & 63) == 0) ? win[b] : 0;  // lane 0 of every wave (broadcast by __shfl)
}

template <int NH>
__device__ __forceinline__ void stage(Smem<NH>& sm, const Pre& pf) {
  const int tid = threadIdx.x;
  if (tid < US) sm.us[tid] = pf.u;
  if (tid < 2 * P) sm.go[tid] = pf.go;
  if (tid < HP) sm.ths[tid] = pf.th;
  if (tid == 0) sm.dls = pf.dls;
}

// initial accumulator = C^T tile at the lane's rows / columns
__device__ __forceinline__ void load_cinit(const KArgs& a, const float* __restrict__ C, int win, int m0, int nP,
                                           f4 (&ci)[2]) {
  const Lane L;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int p = 16 * cb + L.li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = L.row(r);
      ci[cb][r] = (p < nP && h < a.H) ? C[(static_cast<size_t>(win) * a.Lh + m0 + p) * a.H + h] : 0.f;
    }
  }
}

// ---------------------------------------------------------------------------
// forward of one work unit.  On return: act[] filled, xh[cb] (the head input at
// this lane's rows / columns) in registers, and per lane the head outputs of its
// two columns: mu[cb], rr[cb] (pre-softplus) -- finalised redundantly per lane.
// ---------------------------------------------------------------------------
template <int NH, int HK, int KS, bool WREG>
__device__ __forceinline__ void unit_forward(const KArgs& a, Smem<NH>& sm, const WImg& W,
                                             const WRegs<HK, KS, WREG>& R, const f4 (&cinit)[2], f4 (&xh)[2],
                                             float (&mu)[2], float (&rr)[2]) {
  const Lane L;
  const int w = L.w, li = L.li, lk = L.lk;
  // ---- layer 0: A0^T = W_eps^T U + C^T + theta ----
  f4 acc[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    acc[cb] = cinit[cb];
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[cb][r] += sm.ths[L.row(r)];
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int j = 4 * s + lk;
    const float wa = WREG ? R.we[WREG ? s : 0] : W.weps[j * HP + 16 * w + li];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) acc[cb] = mma(wa, sm.us[a.s * (16 * cb + li) + j], acc[cb]);
  }
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = L.row(r);
      const float e = h < a.H ? elu_f(acc[cb][r]) : 0.f;
      acc[cb][r] = e;
      sm.act[0][sw(h, 16 * cb + li)] = e;
    }
  // ---- hidden layers ----
#pragma unroll
  for (int l = 0; l < NH; ++l) {
    __syncthreads();
    f4 z[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) z[cb][r] = sm.bh[l][L.row(r)];
    const float* wl = W.wp + l * HP * HP;
    kloop<WREG, HK>([&](int s) {
      const int hin = 4 * s + lk;
      const float wa = WREG ? R.wf[WREG ? s : 0] : wl[hin * HP + 16 * w + li];
      float g = 1.f, be = 0.f;
      if (l > 0) {
        g = sm.bng[l - 1][hin];
        be = sm.bnb[l - 1][hin];
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) z[cb] = mma(wa, fmaf(g, sm.act[l][sw(hin, 16 * cb + li)], be), z[cb]);
    });
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = L.row(r);
        const float e = h < a.H ? elu_f(z[cb][r]) : 0.f;
        sm.act[l + 1][sw(h, 16 * cb + li)] = e;
        acc[cb][r] = a.bn ? fmaf(sm.bng[l][h], e, sm.bnb[l][h]) : e;
      }
  }
  // ---- head partial sums: mu, r = X_nh . w_head ----
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    float m = 0.f, q = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = L.row(r);
      m = fmaf(acc[cb][r], sm.whead[h], m);
      q = fmaf(acc[cb][r], sm.whead[HP + h], q);
    }
    m += __shfl_xor(m, 16, 64);
    m += __shfl_xor(m, 32, 64);
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    xh[cb] = acc[cb];
    if (lk == 0) {
      sm.red[w][0][16 * cb + li] = m;
      sm.red[w][1][16 * cb + li] = q;
    }
  }
  __syncthreads();
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int p = 16 * cb + li;
    mu[cb] = sm.red[0][0][p] + sm.red[1][0][p] + sm.red[2][0][p] + sm.red[3][0][p] + sm.whead[2 * HP];
    rr[cb] = sm.red[0][1][p] + sm.red[1][1][p] + sm.red[2][1][p] + sm.red[3][1][p] + sm.whead[2 * HP + 1];
  }
}

// unit sequence helpers
struct UnitPos {
  int bl, m0;
};

// ---------------------------------------------------------------------------
// forward kernel: samples outer, tiles inner
// ---------------------------------------------------------------------------
template <int NH, int HK, int KS>
__global__ __launch_bounds__(NT, 2) void fwd_kernel(KArgs a, const float* __restrict__ u, const float* __restrict__ C,
                                                    const int32_t* __restrict__ win, const float* __restrict__ tht,
                                                    WImg W, float* __restrict__ u_next,
                                                    float* __restrict__ ls_slab) {
  constexpr bool WREG = NH <= 1;
  __shared__ Smem<NH> sm;
  const Lane L;
  const int tid = threadIdx.x;
  const int g = blockIdx.x, c = blockIdx.y;
  const int m_lo = c * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int nb = min(a.S, a.B - g * a.S);
  WRegs<HK, KS, WREG> R;
  load_wregs<HK, KS, WREG>(W, R, 0);
  load_block_consts<NH>(sm, W);
  Pre pf;
  UnitPos cur{0, m_lo};
  prefetch(a, u, nullptr, tht, nullptr, win, g * a.S, a.s * m_lo, min(P, m_hi - m_lo), pf);
  float ls_acc = 0.f;
  while (cur.bl < nb) {
    const int b = g * a.S + cur.bl;
    const int m0 = cur.m0;
    const int nP = min(P, m_hi - m0);
    const int t0 = a.s * m0;
    __syncthreads();
    stage<NH>(sm, pf);
    int wi = pf.win;
    wi = __shfl(wi, 0, 64);
    if (win == nullptr) wi = 0;
    f4 ci[2];
    load_cinit(a, C, wi, m0, nP, ci);  // issued before the prefetch: waiting on it never waits on the prefetch
    UnitPos nxt = cur;
    nxt.m0 += P;
    if (nxt.m0 >= m_hi) {
      nxt.m0 = m_lo;
      ++nxt.bl;
    }
    if (nxt.bl < nb)
      prefetch(a, u, nullptr, tht, nullptr, win, g * a.S + nxt.bl, a.s * nxt.m0, min(P, m_hi - nxt.m0), pf);
    __syncthreads();
    f4 xh[2];
    float mu[2], rr[2];
    unit_forward<NH, HK, KS, WREG>(a, sm, W, R, ci, xh, mu, rr);
    // lanes of wave 0 with lk == 0 own the 32 columns: outputs and log sigma
    if (L.w == 0 && L.lk == 0) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int p = 16 * cb + L.li;
        if (p < nP) {
          const float sg = softplus_f(rr[cb]) + 1e-10f;
          float* ob = u_next + static_cast<size_t>(b) * a.pLo;
          const int o = t0 + a.s * p + (a.s - 1);
          ob[a.swap_out ? (o ^ 1) : o] = sm.us[a.s * p + (a.s - 1) + a.k] * sg + mu[cb];
          if (a.s == 2) {
            const int oe = t0 + 2 * p;
            ob[a.swap_out ? (oe ^ 1) : oe] = sm.us[2 * p + a.k];
          }
          if (o >= a.Lout - a.n_logsig) ls_acc += logf(sg);
        }
      }
    }
    if (nxt.bl != cur.bl) {  // sample finished: its log-sigma partial for this chunk
      const float v = wave_sum(tid < 64 ? ls_acc : 0.f);
      if (tid == 0) ls_slab[static_cast<size_t>(c) * a.B + b] = v;
      ls_acc = 0.f;
    }
    cur = nxt;
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
  constexpr bool WREG = NH <= 1;
  constexpr int NHA = NH > 0 ? NH : 1;
  constexpr int njb = (4 * KS + 15) >> 4;  // row blocks (j) of dW_eps / dcon
  __shared__ Smem<NH> sm;
  __shared__ float carry[2][S][64];        // ping-pong by tile parity
  __shared__ float dth[S][HP];
  const Lane L;
  const int tid = threadIdx.x, w = L.w, li = L.li, lk = L.lk;
  const int g = blockIdx.x, c = blockIdx.y;
  const int m_lo = c * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int b_lo = g * a.S, nb = min(a.S, a.B - b_lo);

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
  WRegs<HK, KS, WREG> R;
  load_wregs<HK, KS, WREG>(W, R, njb);
  load_block_consts<NH>(sm, W);
  for (int i = tid; i < 2 * S * 64; i += NT) (&carry[0][0][0])[i] = 0.f;
  for (int i = tid; i < S * HP; i += NT) (&dth[0][0])[i] = 0.f;

  Pre pf;
  prefetch(a, u, gout, tht, dls, win, b_lo, a.s * m_lo, min(P, m_hi - m_lo), pf);
  f4 dCa[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  f4 ci[2];
  int cached = -1;
  int tile = 0;
  UnitPos cur{0, m_lo};
  while (cur.m0 < m_hi) {
    const int bl = cur.bl, m0 = cur.m0;
    const int b = b_lo + bl;
    const int nP = min(P, m_hi - m0);
    const int t0 = a.s * m0;
    const int par = tile & 1;
    __syncthreads();
    stage<NH>(sm, pf);
    int wi = __shfl(pf.win, 0, 64);
    if (win == nullptr) wi = 0;
    if (bl == 0) cached = -1;
    if (wi != cached) {
      load_cinit(a, C, wi, m0, nP, ci);
      cached = wi;
    }
    UnitPos nxt = cur;
    if (++nxt.bl >= nb) {
      nxt.bl = 0;
      nxt.m0 += P;
    }
    if (nxt.m0 < m_hi)
      prefetch(a, u, gout, tht, dls, win, b_lo + nxt.bl, a.s * nxt.m0, min(P, m_hi - nxt.m0), pf);
    __syncthreads();
    f4 xh[2];
    float mu[2], rr[2];
    unit_forward<NH, HK, KS, WREG>(a, sm, W, R, ci, xh, mu, rr);

    // ---- head backward (redundant per lane for its two columns) ----
    float gmu[2], gr[2], sig[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int p = 16 * cb + li;
      const int oq = a.s * p + (a.s - 1);
      sig[cb] = softplus_f(rr[cb]) + 1e-10f;
      const float gv = p < nP ? sm.go[oq] : 0.f;
      float dsig = gv * sm.us[oq + a.k];
      if (p < nP && t0 + oq >= a.Lout - a.n_logsig) dsig += sm.dls / sig[cb];
      gmu[cb] = gv;
      gr[cb] = dsig * sigmoid_f(rr[cb]);
    }
    if (w == 0 && lk == 0) {
      dbh0 += gmu[0] + gmu[1];
      dbh1 += gr[0] + gr[1];
      sm.sig[li] = sig[0];
      sm.sig[16 + li] = sig[1];
    }
    f4 dx[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = L.row(r);
        dx[cb][r] = sm.whead[h] * gmu[cb] + sm.whead[HP + h] * gr[cb];
        dwh0[r] = fmaf(xh[cb][r], gmu[cb], dwh0[r]);
        dwh1[r] = fmaf(xh[cb][r], gr[cb], dwh1[r]);
      }

    // ---- hidden layers backward ----
#pragma unroll
    for (int l = NH - 1; l >= 0; --l) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = L.row(r);
          const int idx = sw(h, 16 * cb + li);
          const float e = sm.act[l + 1][idx];
          float de = dx[cb][r];
          if (a.bn) {
            dgl[l][r] = fmaf(de, e, dgl[l][r]);
            dbe[l][r] += de;
            de *= sm.bng[l][h];
          }
          const float dzv = de * elu_grad_from_out(e);
          dbl[l][r] += dzv;
          sm.dz[idx] = dzv;
        }
      __syncthreads();
      // dX_l[h_in][p] = sum_h_out W[h_in][h_out] dz[h_out][p]
      f4 nx[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
      const float* wt = W.wtp + l * HP * HP;
      kloop<WREG, HK>([&](int s) {
        const int ho = 4 * s + lk;
        const float wa = WREG ? R.wb[WREG ? s : 0] : wt[ho * HP + 16 * w + li];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) nx[cb] = mma(wa, sm.dz[sw(ho, 16 * cb + li)], nx[cb]);
      });
      // dW_l[h_in][h_out] += sum_p X_l[h_in][p] dz[h_out][p]
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
          const float xa = fmaf(gi, sm.act[l][sw(hin, p)], bi);
#pragma unroll
          for (int ob = 0; ob < 4; ++ob) dWl[l][ob] = mma(xa, sm.dz[sw(16 * ob + li, p)], dWl[l][ob]);
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
          const int h = L.row(r);
          const int p = 16 * cb + li;
          const int idx = sw(h, p);
          const float da = (p < nP) ? dx[cb][r] * elu_grad_from_out(sm.act[0][idx]) : 0.f;
          dCa[cb][r] += da;
          rs[r] += da;
          sm.dz[idx] = da;
        }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sum16(rs[r]);
        if (li == 0) dth[bl][L.row(r)] += v;
      }
    }
    __syncthreads();
    // dW_eps[j][h] += sum_p U[j][p] dA0[h][p]   (wave w: h block w, all j blocks)
#pragma unroll
    for (int s = 0; s < P / 4; ++s) {
      const int p = 4 * s + lk;
      const float bz = sm.dz[sw(16 * w + li, p)];
#pragma unroll
      for (int jb = 0; jb < njb; ++jb) dWe[jb] = mma(sm.us[a.s * p + 16 * jb + li], bz, dWe[jb]);
    }
    // dcon[j][p] = sum_h w_eps[j][h] dA0[h][p]   (block pairs (jb, cb) = (pair >> 1, pair & 1), pair = w + 4 q)
#pragma unroll
    for (int q = 0; q < Pairs<KS>::per_wave; ++q) {
      const int pair = w + 4 * q;
      const int pjb = pair >> 1, pcb = pair & 1;
      if (pair < 2 * njb) {
        f4 dcn = f4{0.f, 0.f, 0.f, 0.f};
        kloop<WREG, HK>([&](int s) {
          const int hh = 4 * s + lk;
          const float wa = WREG ? R.wc[WREG ? q : 0][WREG ? s : 0] : W.wepsT[hh * HP + 16 * pjb + li];
          dcn = mma(wa, sm.dz[sw(hh, 16 * pcb + li)], dcn);
        });
        // park dcon [j][p] in act[0]: no wave reads act[0] after the first-layer barrier above
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.act[0][sw(16 * pjb + 4 * lk + r, 16 * pcb + li)] = dcn[r];
      }
    }
    __syncthreads();
    // du over local positions q in [0, s*nP + k); the overhang beyond the tile becomes the new carry
    {
      const int fin = a.s * nP;
      float* db = du + static_cast<size_t>(b) * a.pL;
      for (int q = tid; q < fin + a.k; q += NT) {
        float v = 0.f;
        for (int j = 0; j < a.k; ++j) {
          const int t = q - j;
          if (t >= 0) {
            if (a.s == 1) {
              if (t < nP) v += sm.act[0][sw(j, t)];
            } else if (!(t & 1) && (t >> 1) < nP) {
              v += sm.act[0][sw(j, t >> 1)];
            }
          }
        }
        const int oq = q - a.k;
        if (oq >= 0 && oq < fin) {
          if (a.s == 1) {
            v += sm.go[oq] * sm.sig[oq];
          } else {
            v += (oq & 1) ? sm.go[oq] * sm.sig[oq >> 1] : sm.go[oq];
          }
        }
        if (q < a.k) v += carry[par][bl][q];
        if (q < fin) db[t0 + q] = v;
        else carry[par ^ 1][bl][q - fin] = v;
      }
    }
    if (nxt.bl == 0 || nxt.m0 >= m_hi) {
      // tile finished: its dC over the group
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = L.row(r), p = 16 * cb + li;
          if (p < nP && h < a.H) dC_slab[(static_cast<size_t>(g) * a.Lh + m0 + p) * a.H + h] = dCa[cb][r];
          dCa[cb][r] = 0.f;
        }
      ++tile;
    }
    cur = nxt;
  }

  __syncthreads();
  const int par = tile & 1;
  for (int bl = 0; bl < nb; ++bl) {
    const int b = b_lo + bl;
    for (int q = tid; q < a.k; q += NT) {
      if (c == a.n_chunks - 1) du[static_cast<size_t>(b) * a.pL + a.Lout + q] = carry[par][bl][q];
      else halo[(static_cast<size_t>(b) * a.n_chunks + c) * a.k + q] = carry[par][bl][q];
    }
    if (tid < a.H) dth_slab[(static_cast<size_t>(c) * a.B + b) * a.H + tid] = dth[bl][tid];
  }

  // ---- weight-gradient partials of this block ----
  const int H = a.H;
  const int nW = a.k * H + NH * H * H + 3 * NH * H + 2 * H + 2;
  float* ws = dW_slab + (static_cast<size_t>(g) * a.n_chunks + c) * nW;
#pragma unroll
  for (int jb = 0; jb < njb; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jb + 4 * lk + r, h = 16 * w + li;
      if (j < a.k && h < H) ws[j * H + h] = dWe[jb][r];
    }
  int off = a.k * H;
#pragma unroll
  for (int l = 0; l < NH; ++l)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hi = L.row(r), ho = 16 * ob + li;
        if (hi < H && ho < H) ws[off + (l * H + hi) * H + ho] = dWl[l][ob][r];
      }
  off += NH * H * H;
  auto put_rows = [&](const float (&v)[4], int dst, int stride) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = sum16(v[r]);
      const int h = L.row(r);
      if (li == 0 && h < H) ws[dst + h * stride] = s;
    }
  };
#pragma unroll
  for (int l = 0; l < NH; ++l) put_rows(dbl[l], off + l * H, 1);
  off += NH * H;
#pragma unroll
  for (int l = 0; l < NH; ++l) put_rows(dgl[l], off + l * H, 1);  // d gamma (bn scale applied at scatter)
  off += NH * H;
#pragma unroll
  for (int l = 0; l < NH; ++l) put_rows(dbe[l], off + l * H, 1);
  off += NH * H;
  put_rows(dwh0, off + 0, 2);
  put_rows(dwh1, off + 1, 2);
  off += 2 * H;
  const float s0 = wave_sum(w == 0 ? dbh0 : 0.f), s1 = wave_sum(w == 0 ? dbh1 : 0.f);
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

}  // namespace flow4

// ---------------------------------------------------------------------------
// entry points used by flow_api.cpp
// ---------------------------------------------------------------------------
// (HK, KS) buckets: hidden k-steps ceil(H/4) and sample-channel k-steps ceil(k/4), rounded up to
// the shapes of the reference configs; the generic <NH, 16, 16> covers any H <= 64, k <= 64 (the
// padded weight images are zero beyond H and k, so extra k-steps add zeros).
#define FLOW4_CASES(KERNEL, nh, hk, ks, ...)                                                      \
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

size_t flow4_workspace_size(const VissmFlowDesc* d, int backward) {
  using namespace flow4;
  Geom g = geom(d, backward != 0);
  return backward ? bwd_ws_layout(d, g, nullptr, nullptr) : fwd_ws_layout(d, g, nullptr, nullptr);
}

void flow4_geometry(const VissmFlowDesc* d, int backward, int32_t* out) {
  using namespace flow4;
  Geom g = geom(d, backward != 0);
  out[0] = P; out[1] = g.CH / P; out[2] = g.n_chunks; out[3] = g.n_groups;
}

int flow4_fwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
              const float* theta_term, float* u_next, float* logsig, void* workspace, size_t ws_bytes,
              hipStream_t st) {
  using namespace flow4;
  Geom g = geom(d, false);
  VISSM_CHECK_ARG(workspace && ws_bytes >= fwd_ws_layout(d, g, nullptr, nullptr), "flow_fwd: workspace too small");
  WsF ws;
  fwd_ws_layout(d, g, reinterpret_cast<char*>(workspace), &ws);
  hipLaunchKernelGGL(prep_kernel, dim3(1), dim3(256), 0, st, *w, d->H, d->k, d->n_hidden, d->bn, ws.w);
  VISSM_CHECK_LAUNCH("flow4_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid(g.n_groups, g.n_chunks);
  int hk, ks;
  buckets(d, &hk, &ks);
  prof_begin(VISSM_PROF_FLOW_FWD, st);
  FLOW4_CASES(fwd_kernel, d->n_hidden, hk, ks, grid, dim3(NT), 0, st, a, u, C, wn, theta_term, ws.w, u_next,
              ws.ls_slab);
  VISSM_CHECK_LAUNCH("flow4_fwd");
  prof_end(VISSM_PROF_FLOW_FWD, st);
  return launch_reduce_rows(ws.ls_slab, logsig, g.n_chunks, d->B, st);
}

int flow4_bwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
              const float* theta_term, const float* du_next, const float* dlogsig, float* du, float* dC,
              float* dtheta_term, const VissmFlowGrads* gr, void* workspace, size_t ws_bytes, hipStream_t st) {
  using namespace flow4;
  Geom g = geom(d, true);
  VISSM_CHECK_ARG(workspace && ws_bytes >= bwd_ws_layout(d, g, nullptr, nullptr), "flow_bwd: workspace too small");
  WsB ws;
  bwd_ws_layout(d, g, reinterpret_cast<char*>(workspace), &ws);
  hipLaunchKernelGGL(prep_kernel, dim3(1), dim3(256), 0, st, *w, d->H, d->k, d->n_hidden, d->bn, ws.w);
  VISSM_CHECK_LAUNCH("flow4_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid(g.n_groups, g.n_chunks);
  int hk, ks;
  buckets(d, &hk, &ks);
  prof_begin(VISSM_PROF_FLOW_BWD, st);
  prof_begin(VISSM_PROF_FLOW_BWD_DU, st);
  FLOW4_CASES(bwd_kernel, d->n_hidden, hk, ks, grid, dim3(NT), 0, st, a, u, C, wn, theta_term, du_next, dlogsig, ws.w,
              du, ws.dC_slab, ws.dth_slab, ws.dW_slab, ws.halo);
  VISSM_CHECK_LAUNCH("flow4_bwd");
  prof_end(VISSM_PROF_FLOW_BWD_DU, st);
  prof_end(VISSM_PROF_FLOW_BWD, st);
  int rc = launch_halo_fixup(du, ws.halo, d->B, d->L, a.pL, d->k, g.n_chunks, g.s, g.CH, st);
  if (rc) return rc;
  const int64_t nC = static_cast<int64_t>(g.Lh) * d->H;
  if (d->n_win == 1) {
    rc = launch_reduce_rows_inplace(ws.dC_slab, dC, g.n_groups, nC, st);
    if (rc) return rc;
  } else {
    rc = launch_reduce_by_window(ws.dC_slab, win, dC, d->B, d->n_win, nC, st);
    if (rc) return rc;
  }
  rc = launch_reduce_rows(ws.dth_slab, dtheta_term, g.n_chunks, static_cast<int64_t>(d->B) * d->H, st);
  if (rc) return rc;
  const int nW = n_wgrad(d);
  rc = launch_reduce_rows_inplace(ws.dW_slab, ws.wred, static_cast<int64_t>(g.n_groups) * g.n_chunks, nW, st);
  if (rc) return rc;
  return launch_scatter_wgrad(ws.wred, gr, d->k, d->H, d->n_hidden, d->bn, st);
}

}  // namespace vissm
