// IAF flow of the neural-MA sampler, forward and backward (fp32, LDS-tiled).
//
// Reference: IAF._create_flow / IAF.slp (AR.py:50-89); stride-2 head with
// (0,1) interleave and BN affine (lotka_volterra_partial.py:93-104,
// fitz_nag_NVP.py:90-105); Permute flow (lotka_volterra_partial.py:137-159)
// fused into the output store (swap_out).
//
// Decomposition (both passes): grid = (sample groups of S) x (t-chunks of
// head positions).  A block walks its chunk in tiles of P head positions.
//   forward : samples outer, tiles inner; log-sigma partials per (chunk, sample).
//   backward: tiles outer, samples inner, so that the window-shared gradient
//             dC of a tile is summed over the group's samples in registers and
//             written once per (group, tile); the transposed conv's overhang
//             into the next tile is carried per sample in LDS; the carry out of
//             a chunk goes to a halo slab added by a fix-up kernel.
// All cross-block sums go through partial slabs reduced in fixed order.
#include "common.hpp"

namespace vissm {
namespace flow1 {

constexpr int P = 16;      // head positions per tile
constexpr int S = 32;      // samples per group
constexpr int HP = 64;     // padded hidden width
constexpr int HS = 65;     // LDS row stride (bank padding)
constexpr int NT = 256;    // threads per block
constexpr int PPT = P / 4; // positions per thread (4 position groups)

struct Geom {
  int s, Lout, Lh, S, n_groups, n_tiles, CH, n_chunks;
};

// backward with several windows runs one sample per group so that the dC rows
// are per sample (reduced by window afterwards); everything else uses groups of S.
static Geom geom(const VissmFlowDesc* d, bool backward) {
  Geom g;
  g.s = d->stride2 ? 2 : 1;
  g.Lout = d->L - d->k;
  g.Lh = g.Lout / g.s;
  g.S = (backward && d->n_win > 1) ? 1 : S;
  g.n_groups = (d->B + g.S - 1) / g.S;
  g.n_tiles = (g.Lh + P - 1) / P;
  int ch_min_tiles = ((d->k + g.s - 1) / g.s + P - 1) / P;  // chunk must span >= k positions
  if (ch_min_tiles < 1) ch_min_tiles = 1;
  int want = (1024 + g.n_groups - 1) / g.n_groups;
  int max_chunks = g.n_tiles / ch_min_tiles;
  if (max_chunks < 1) max_chunks = 1;
  int nc = want < max_chunks ? want : max_chunks;
  if (nc < 1) nc = 1;
  int tiles_per_chunk = (g.n_tiles + nc - 1) / nc;
  if (tiles_per_chunk < ch_min_tiles) tiles_per_chunk = ch_min_tiles;
  g.CH = tiles_per_chunk * P;
  g.n_chunks = (g.Lh + g.CH - 1) / g.CH;
  return g;
}

// number of floats of the per-block dW partial
static int n_wgrad(const VissmFlowDesc* d) {
  const int H = d->H, k = d->k, nh = d->n_hidden;
  return k * H + nh * H * H + nh * H + 2 * nh * H + 2 * H + 2;
}

struct WsF {  // forward workspace
  float *wp, *bh, *bng, *bnb, *weps, *whead, *ls_slab;
};
struct WsB {  // backward workspace
  float *wp, *wTp, *bh, *bng, *bnb, *weps, *wepsT, *whead;
  float *dC_slab, *dth_slab, *dW_slab, *halo, *wred;
};

static size_t fwd_ws_layout(const VissmFlowDesc* d, const Geom& g, char* base, WsF* w) {
  size_t off = 0;
  auto take = [&](size_t nfl) { float* p = base ? reinterpret_cast<float*>(base + off) : nullptr; off += align_up(nfl * 4); return p; };
  const int nh = d->n_hidden > 0 ? d->n_hidden : 1;
  WsF t;
  t.wp = take(static_cast<size_t>(nh) * HP * HP);
  t.bh = take(nh * HP);
  t.bng = take(nh * HP);
  t.bnb = take(nh * HP);
  t.weps = take(HP * HP);
  t.whead = take(2 * HP + 2);
  t.ls_slab = take(static_cast<size_t>(g.n_chunks) * d->B);
  if (w) *w = t;
  return off;
}

static size_t bwd_ws_layout(const VissmFlowDesc* d, const Geom& g, char* base, WsB* w) {
  size_t off = 0;
  auto take = [&](size_t nfl) { float* p = base ? reinterpret_cast<float*>(base + off) : nullptr; off += align_up(nfl * 4); return p; };
  const int nh = d->n_hidden > 0 ? d->n_hidden : 1;
  WsB t;
  t.wp = take(static_cast<size_t>(nh) * HP * HP);
  t.wTp = take(static_cast<size_t>(nh) * HP * HP);
  t.bh = take(nh * HP);
  t.bng = take(nh * HP);
  t.bnb = take(nh * HP);
  t.weps = take(HP * HP);
  t.wepsT = take(HP * HP);
  t.whead = take(2 * HP + 2);
  t.dC_slab = take(static_cast<size_t>(g.n_groups) * g.Lh * d->H);
  t.dth_slab = take(static_cast<size_t>(g.n_chunks) * d->B * d->H);
  t.dW_slab = take(static_cast<size_t>(g.n_groups) * g.n_chunks * n_wgrad(d));
  t.halo = take(static_cast<size_t>(d->B) * g.n_chunks * d->k);
  t.wred = take(n_wgrad(d));
  if (w) *w = t;
  return off;
}

// ---------------------------------------------------------------------------
// weight prep: zero-padded [64][64] copies (and transposes) in the workspace
// ---------------------------------------------------------------------------
__global__ void prep_weights_kernel(VissmFlowParams w, int H, int k, int nh, int bn, float* wp, float* wTp,
                                    float* bh, float* bng, float* bnb, float* weps, float* wepsT, float* whead) {
  const int i = threadIdx.x & 63, j = threadIdx.x >> 6;  // 64 x 4
  for (int r = j; r < HP; r += 4) {
    for (int l = 0; l < nh; ++l) {
      float v = (r < H && i < H) ? w.w_hid[(static_cast<size_t>(l) * H + r) * H + i] : 0.f;
      wp[(l * HP + r) * HP + i] = v;  // [l][h_in=r][h_out=i]
      if (wTp) wTp[(l * HP + i) * HP + r] = v;  // [l][h_out=i][h_in=r]
    }
    float e = (r < k && i < H) ? w.w_eps[r * H + i] : 0.f;
    weps[r * HP + i] = e;           // [j=r][h=i]
    if (wepsT) wepsT[i * HP + r] = e;  // [h=i][j=r]
  }
  if (j == 0) {
    for (int l = 0; l < nh; ++l) {
      bh[l * HP + i] = i < H ? w.b_hid[l * H + i] : 0.f;
      bng[l * HP + i] = (bn && i < H) ? w.bn_g[l * H + i] : 1.f;
      bnb[l * HP + i] = (bn && i < H) ? w.bn_b[l * H + i] : 0.f;
    }
    whead[i] = i < H ? w.w_head[i * 2 + 0] : 0.f;
    whead[HP + i] = i < H ? w.w_head[i * 2 + 1] : 0.f;
    if (i < 2) whead[2 * HP + i] = w.b_head[i];
  }
}

struct KArgs {
  int B, L, k, H, bn, s, swap_out, n_logsig, n_win, Lout, Lh, CH, n_chunks, S;
};

// forward recompute of one (tile, sample) into LDS.
//   us  : u[b][t0 + q], q < s*P + k + 2 (zero beyond L)
//   Cs  : C tile [P][HS] (zero for invalid rows / h >= H)
//   ths : theta_term[b] padded [HP]
// produces E[l][p][h] (post-ELU), X[l][p][h] (layer inputs, post-BN) for l = 0..NH,
// and mu_s[p], r_s[p] (head outputs, pre-softplus r).
template <int NH>
__device__ __forceinline__ void tile_forward(const KArgs& a, const float* __restrict__ us, const float (*Cs)[HS],
                                             const float* __restrict__ ths, const float* __restrict__ weps,
                                             const float* __restrict__ wp, const float* __restrict__ bh,
                                             const float* __restrict__ bng, const float* __restrict__ bnb,
                                             const float* __restrict__ whead, float (*E)[P][HS], float (*X)[P][HS],
                                             float* mu_s, float* r_s) {
  const int h = threadIdx.x & 63, pg = threadIdx.x >> 6;
  // first layer: conv over the sample channel + C + theta term
  {
    float acc[PPT];
#pragma unroll
    for (int i = 0; i < PPT; ++i) acc[i] = Cs[pg * PPT + i][h] + ths[h];
    for (int j = 0; j < a.k; ++j) {
      const float w = weps[j * HP + h];
#pragma unroll
      for (int i = 0; i < PPT; ++i) acc[i] = fmaf(us[a.s * (pg * PPT + i) + j], w, acc[i]);
    }
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      float e = h < a.H ? elu_f(acc[i]) : 0.f;
      E[0][pg * PPT + i][h] = e;
    }
  }
  __syncthreads();
#pragma unroll
  for (int l = 0; l < NH; ++l) {
    const float(*xin)[HS] = (a.bn && l > 0) ? X[l] : E[l];
    float acc[PPT];
    const float bias = bh[l * HP + h];
#pragma unroll
    for (int i = 0; i < PPT; ++i) acc[i] = bias;
    const float* wl = wp + l * HP * HP;
    for (int hi = 0; hi < a.H; ++hi) {
      const float w = wl[hi * HP + h];
#pragma unroll
      for (int i = 0; i < PPT; ++i) acc[i] = fmaf(xin[pg * PPT + i][hi], w, acc[i]);
    }
    const float g = bng[l * HP + h] * kBnScale, be = bnb[l * HP + h];
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      float e = h < a.H ? elu_f(acc[i]) : 0.f;
      E[l + 1][pg * PPT + i][h] = e;
      if (a.bn) X[l + 1][pg * PPT + i][h] = h < a.H ? fmaf(g, e, be) : 0.f;
    }
    __syncthreads();
  }
  // head (wave pg owns positions pg*PPT .. +PPT-1)
  {
    const float(*xl)[HS] = (a.bn && NH > 0) ? X[NH] : E[NH];
    const float w0 = whead[h], w1 = whead[HP + h];
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const float xv = xl[pg * PPT + i][h];
      float m = wave_sum(xv * w0), r = wave_sum(xv * w1);
      if (h == 0) {
        mu_s[pg * PPT + i] = m + whead[2 * HP + 0];
        r_s[pg * PPT + i] = r + whead[2 * HP + 1];
      }
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// forward kernel
// ---------------------------------------------------------------------------
template <int NH>
__global__ __launch_bounds__(NT) void flow_fwd_kernel(KArgs a, const float* __restrict__ u,
                                                      const float* __restrict__ C, const int32_t* __restrict__ win,
                                                      const float* __restrict__ tht, const float* __restrict__ wp,
                                                      const float* __restrict__ bh, const float* __restrict__ bng,
                                                      const float* __restrict__ bnb, const float* __restrict__ weps,
                                                      const float* __restrict__ whead, float* __restrict__ u_next,
                                                      float* __restrict__ ls_slab) {
  __shared__ float E[NH + 1][P][HS];
  __shared__ float X[NH + 1][P][HS];
  __shared__ float Cs[P][HS];
  __shared__ float us[2 * P + 64 + 4];
  __shared__ float ths[HP];
  __shared__ float mu_s[P], r_s[P];

  const int tid = threadIdx.x, h = tid & 63, pg = tid >> 6;
  const int g = blockIdx.x, c = blockIdx.y;
  const int m_lo = c * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int span = a.s * P + a.k + 2;

  for (int bl = 0; bl < a.S; ++bl) {
    const int b = g * a.S + bl;
    if (b >= a.B) break;
    const int w = win ? win[b] : 0;
    const float* ub = u + static_cast<size_t>(b) * a.L;
    float* ob = u_next + static_cast<size_t>(b) * a.Lout;
    if (tid < HP) ths[tid] = tid < a.H ? tht[static_cast<size_t>(b) * a.H + tid] : 0.f;
    float ls_acc = 0.f;
    for (int m0 = m_lo; m0 < m_hi; m0 += P) {
      const int nP = min(P, m_hi - m0);
      const int t0 = a.s * m0;
      __syncthreads();
      for (int q = tid; q < span; q += NT) us[q] = (t0 + q < a.L) ? ub[t0 + q] : 0.f;
      for (int i = 0; i < PPT; ++i) {
        const int p = pg * PPT + i;
        Cs[p][h] = (p < nP && h < a.H) ? C[(static_cast<size_t>(w) * a.Lh + m0 + p) * a.H + h] : 0.f;
      }
      __syncthreads();
      tile_forward<NH>(a, us, Cs, ths, weps, wp, bh, bng, bnb, whead, E, X, mu_s, r_s);
      if (tid < nP) {
        const int p = tid;
        const float sig = softplus_f(r_s[p]) + 1e-10f;
        const int o = t0 + a.s * p + (a.s - 1);  // transformed output position
        const float y = us[a.s * p + (a.s - 1) + a.k] * sig + mu_s[p];
        ob[a.swap_out ? (o ^ 1) : o] = y;
        if (a.s == 2) {
          const int oe = t0 + 2 * p;  // pass-through (sigma = 1, mu = 0)
          ob[a.swap_out ? (oe ^ 1) : oe] = us[2 * p + a.k];
        }
        if (o >= a.Lout - a.n_logsig) ls_acc += logf(sig);
      }
    }
    // sum the per-thread log-sigma partials (threads 0..P-1) in fixed order
    float v = wave_sum(tid < 64 ? ls_acc : 0.f);
    if (tid == 0) ls_slab[static_cast<size_t>(c) * a.B + b] = v;
  }
}

// ---------------------------------------------------------------------------
// backward kernel
// ---------------------------------------------------------------------------
template <int NH>
__global__ __launch_bounds__(NT) void flow_bwd_kernel(KArgs a, const float* __restrict__ u,
                                                      const float* __restrict__ C, const int32_t* __restrict__ win,
                                                      const float* __restrict__ tht, const float* __restrict__ gout,
                                                      const float* __restrict__ dls, const float* __restrict__ wp,
                                                      const float* __restrict__ wTp, const float* __restrict__ bh,
                                                      const float* __restrict__ bng, const float* __restrict__ bnb,
                                                      const float* __restrict__ weps, const float* __restrict__ wepsT,
                                                      const float* __restrict__ whead, float* __restrict__ du,
                                                      float* __restrict__ dC_slab, float* __restrict__ dth_slab,
                                                      float* __restrict__ dW_slab, float* __restrict__ halo) {
  __shared__ float E[NH + 1][P][HS];
  __shared__ float X[NH + 1][P][HS];
  __shared__ float Cs[P][HS];
  __shared__ float G[P][HS];
  __shared__ float DZ[P][HS];
  __shared__ float us[2 * P + 64 + 4];
  __shared__ float go[2 * P];
  __shared__ float ths[HP];
  __shared__ float mu_s[P], r_s[P], sig_s[P];
  __shared__ float carry[S][64];
  __shared__ float dth[S][HP];
  __shared__ float red4[4][HP];
  __shared__ float dul[2 * P + 64 + 4];

  const int tid = threadIdx.x, h = tid & 63, pg = tid >> 6;
  const int g = blockIdx.x, c = blockIdx.y;
  const int m_lo = c * a.CH, m_hi = min(a.Lh, m_lo + a.CH);
  const int span = a.s * P + a.k + 2;
  const int b_lo = g * a.S, nb = min(a.S, a.B - b_lo);
  const float cb = kBnScale;

  // per-thread weight-gradient accumulators
  float dWl[NH > 0 ? NH : 1][16];
  float dbl[NH > 0 ? NH : 1], dgl[NH > 0 ? NH : 1], dbe[NH > 0 ? NH : 1];
  float dwe[16];
  float dwh0 = 0.f, dwh1 = 0.f, dbh0 = 0.f, dbh1 = 0.f;
#pragma unroll
  for (int l = 0; l < (NH > 0 ? NH : 1); ++l) {
    dbl[l] = dgl[l] = dbe[l] = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) dWl[l][r] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) dwe[r] = 0.f;

  for (int i = tid; i < S * 64; i += NT) {
    (&carry[0][0])[i] = 0.f;
    (&dth[0][0])[i] = 0.f;
  }
  int cached_w = -1;

  for (int m0 = m_lo; m0 < m_hi; m0 += P) {
    const int nP = min(P, m_hi - m0);
    const int t0 = a.s * m0;
    float dCacc[PPT];
#pragma unroll
    for (int i = 0; i < PPT; ++i) dCacc[i] = 0.f;
    cached_w = -1;

    for (int bl = 0; bl < nb; ++bl) {
      const int b = b_lo + bl;
      const int w = win ? win[b] : 0;
      const float* ub = u + static_cast<size_t>(b) * a.L;
      const float* gb = gout + static_cast<size_t>(b) * a.Lout;
      const float gls = dls[b];
      __syncthreads();
      for (int q = tid; q < span; q += NT) {
        us[q] = (t0 + q < a.L) ? ub[t0 + q] : 0.f;
        dul[q] = 0.f;
      }
      for (int q = tid; q < a.s * P; q += NT) {
        const int o = t0 + q;
        go[q] = (q < a.s * nP) ? gb[a.swap_out ? (o ^ 1) : o] : 0.f;
      }
      if (tid < HP) ths[tid] = tid < a.H ? tht[static_cast<size_t>(b) * a.H + tid] : 0.f;
      if (w != cached_w) {
        for (int i = 0; i < PPT; ++i) {
          const int p = pg * PPT + i;
          Cs[p][h] = (p < nP && h < a.H) ? C[(static_cast<size_t>(w) * a.Lh + m0 + p) * a.H + h] : 0.f;
        }
        cached_w = w;
      }
      __syncthreads();
      tile_forward<NH>(a, us, Cs, ths, weps, wp, bh, bng, bnb, whead, E, X, mu_s, r_s);

      // ---- head backward ----
      const float(*xl)[HS] = (a.bn && NH > 0) ? X[NH] : E[NH];
      {
        const float w0 = whead[h], w1 = whead[HP + h];
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
          const int p = pg * PPT + i;
          const float r = r_s[p];
          const float sig = softplus_f(r) + 1e-10f;
          const int oq = a.s * p + (a.s - 1);
          const float gv = (p < nP) ? go[oq] : 0.f;
          const int o = t0 + oq;
          float dsig = gv * us[oq + a.k];
          if (p < nP && o >= a.Lout - a.n_logsig) dsig += gls / sig;
          const float dmu = gv;
          const float dr = dsig * sigmoid_f(r);
          const float xv = xl[p][h];
          dwh0 = fmaf(xv, dmu, dwh0);
          dwh1 = fmaf(xv, dr, dwh1);
          if (h == 0) {
            dbh0 += dmu;
            dbh1 += dr;
            sig_s[p] = sig;
          }
          G[p][h] = h < a.H ? dmu * w0 + dr * w1 : 0.f;
        }
      }
      __syncthreads();

      // ---- hidden layers backward ----
#pragma unroll
      for (int l = NH - 1; l >= 0; --l) {
        const float gm = bng[l * HP + h] * cb;
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
          const int p = pg * PPT + i;
          const float dx = G[p][h];
          const float e = E[l + 1][p][h];
          float de = dx;
          if (a.bn) {
            dgl[l] = fmaf(dx, e * cb, dgl[l]);
            dbe[l] += dx;
            de = dx * gm;
          }
          const float dz = de * elu_grad_from_out(e);
          DZ[p][h] = dz;
          dbl[l] += dz;
        }
        __syncthreads();
        // dX[l] = dz W_l^T
        {
          float acc[PPT];
#pragma unroll
          for (int i = 0; i < PPT; ++i) acc[i] = 0.f;
          const float* wt = wTp + l * HP * HP;
          for (int ho = 0; ho < a.H; ++ho) {
            const float wv = wt[ho * HP + h];
#pragma unroll
            for (int i = 0; i < PPT; ++i) acc[i] = fmaf(DZ[pg * PPT + i][ho], wv, acc[i]);
          }
          // dW_l[hin][h] += sum_p xin[p][hin] dz[p][h], hin = pg + 4r
          const float(*xin)[HS] = (a.bn && l > 0) ? X[l] : E[l];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int hin = pg + 4 * r;
            float s = 0.f;
#pragma unroll
            for (int p = 0; p < P; ++p) s = fmaf(xin[p][hin], DZ[p][h], s);
            dWl[l][r] += s;
          }
          __syncthreads();
#pragma unroll
          for (int i = 0; i < PPT; ++i) G[pg * PPT + i][h] = acc[i];
        }
        __syncthreads();
      }

      // ---- first layer: da0 ----
      {
        float tsum = 0.f;
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
          const int p = pg * PPT + i;
          const float da = (p < nP) ? G[p][h] * elu_grad_from_out(E[0][p][h]) : 0.f;
          DZ[p][h] = da;
          dCacc[i] += da;
          tsum += da;
        }
        red4[pg][h] = tsum;
      }
      __syncthreads();
      if (pg == 0) dth[bl][h] += red4[0][h] + red4[1][h] + red4[2][h] + red4[3][h];
      // dW_eps[j][h] += sum_p u[s p + j] da0[p][h], j = pg + 4r
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = pg + 4 * r;
        if (j < a.k) {
          float s = 0.f;
#pragma unroll
          for (int p = 0; p < P; ++p) s = fmaf(us[a.s * p + j], DZ[p][h], s);
          dwe[r] += s;
        }
      }
      // dcon[p][j] = sum_h da0[p][h] w_eps[j][h]  (thread: j = tid&63, positions of pg) -> G
      {
        const int j = h;
        float acc[PPT];
#pragma unroll
        for (int i = 0; i < PPT; ++i) acc[i] = 0.f;
        for (int hh = 0; hh < a.H; ++hh) {
          const float wv = wepsT[hh * HP + j];
#pragma unroll
          for (int i = 0; i < PPT; ++i) acc[i] = fmaf(DZ[pg * PPT + i][hh], wv, acc[i]);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PPT; ++i) G[pg * PPT + i][j] = acc[i];
      }
      __syncthreads();
      // assemble du over local positions q in [0, s*nP + k)
      const int fin = a.s * nP;
      for (int q = tid; q < fin + a.k; q += NT) {
        float v = 0.f;
        for (int j = 0; j < a.k; ++j) {
          const int t = q - j;
          if (t >= 0 && (t % a.s) == 0 && t / a.s < nP) v += G[t / a.s][j];
        }
        const int oq = q - a.k;  // output index whose pass-through lands here
        if (oq >= 0 && oq < fin) {
          if (a.s == 1) v += go[oq] * sig_s[oq];
          else v += (oq & 1) ? go[oq] * sig_s[oq >> 1] : go[oq];
        }
        if (q < a.k) v += carry[bl][q];
        dul[q] = v;
      }
      __syncthreads();
      float* db = du + static_cast<size_t>(b) * a.L;
      for (int q = tid; q < fin + a.k; q += NT) {
        if (q < fin) db[t0 + q] = dul[q];
        else carry[bl][q - fin] = dul[q];
      }
    }  // samples

    // dC tile of this group: one row per group (= per sample in multi-window mode)
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int p = pg * PPT + i;
      if (p < nP && h < a.H) dC_slab[(static_cast<size_t>(g) * a.Lh + m0 + p) * a.H + h] = dCacc[i];
    }
  }  // tiles

  __syncthreads();
  // chunk end: carries -> halo (or the last k entries of du), dtheta partial
  for (int bl = 0; bl < nb; ++bl) {
    const int b = b_lo + bl;
    for (int q = tid; q < a.k; q += NT) {
      if (c == a.n_chunks - 1) {
        du[static_cast<size_t>(b) * a.L + a.Lout + q] = carry[bl][q];
      } else {
        halo[(static_cast<size_t>(b) * a.n_chunks + c) * a.k + q] = carry[bl][q];
      }
    }
    if (tid < a.H) dth_slab[(static_cast<size_t>(c) * a.B + b) * a.H + tid] = dth[bl][tid];
  }

  // weight-gradient partials of this block
  const int nW = a.k * a.H + NH * a.H * a.H + 3 * NH * a.H + 2 * a.H + 2;
  float* ws = dW_slab + (static_cast<size_t>(g) * a.n_chunks + c) * nW;
  // w_eps [k][H]
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = pg + 4 * r;
    if (j < a.k && h < a.H) ws[j * a.H + h] = dwe[r];
  }
  int off = a.k * a.H;
#pragma unroll
  for (int l = 0; l < NH; ++l) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int hin = pg + 4 * r;
      if (hin < a.H && h < a.H) ws[off + (l * a.H + hin) * a.H + h] = dWl[l][r];
    }
  }
  off += NH * a.H * a.H;
  // per-(h) sums over the 4 position groups: b_hid, bn_g, bn_b, w_head cols
  auto combine = [&](float v, int dst) {
    __syncthreads();
    red4[pg][h] = v;
    __syncthreads();
    if (pg == 0 && h < a.H) ws[dst + h] = red4[0][h] + red4[1][h] + red4[2][h] + red4[3][h];
  };
#pragma unroll
  for (int l = 0; l < NH; ++l) combine(dbl[l], off + l * a.H);
  off += NH * a.H;
#pragma unroll
  for (int l = 0; l < NH; ++l) combine(dgl[l], off + l * a.H);
  off += NH * a.H;
#pragma unroll
  for (int l = 0; l < NH; ++l) combine(dbe[l], off + l * a.H);
  off += NH * a.H;
  // w_head [H][2] interleaved: write col 0 and col 1 via two combines into scratch then interleave
  __syncthreads();
  red4[pg][h] = dwh0;
  __syncthreads();
  if (pg == 0 && h < a.H) ws[off + h * 2 + 0] = red4[0][h] + red4[1][h] + red4[2][h] + red4[3][h];
  __syncthreads();
  red4[pg][h] = dwh1;
  __syncthreads();
  if (pg == 0 && h < a.H) ws[off + h * 2 + 1] = red4[0][h] + red4[1][h] + red4[2][h] + red4[3][h];
  off += 2 * a.H;
  __syncthreads();
  red4[pg][h] = (h == 0) ? dbh0 : 0.f;
  __syncthreads();
  if (tid == 0) {
    ws[off + 0] = red4[0][0] + red4[1][0] + red4[2][0] + red4[3][0];
  }
  __syncthreads();
  red4[pg][h] = (h == 0) ? dbh1 : 0.f;
  __syncthreads();
  if (tid == 0) ws[off + 1] = red4[0][0] + red4[1][0] + red4[2][0] + red4[3][0];
}

__global__ void halo_fixup_kernel(float* __restrict__ du, const float* __restrict__ halo, int B, int L, int k,
                                  int n_chunks, int s, int CH) {
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < (n_chunks - 1) * k; i += blockDim.x) {
    const int c = i / k, q = i % k;
    const int pos = s * (c + 1) * CH + q;
    if (pos < L) du[static_cast<size_t>(b) * L + pos] += halo[(static_cast<size_t>(b) * n_chunks + c) * k + q];
  }
}

// dC[w] = sum over rows r with win_of_row(r) == w  (n_win > 1: rows are samples)
__global__ void reduce_by_window_kernel(const float* __restrict__ slab, const int32_t* __restrict__ win,
                                        float* __restrict__ out, int B, int N) {
  const int w = blockIdx.y;
  const int cidx = blockIdx.x * blockDim.x + threadIdx.x;
  if (cidx >= N) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b)
    if (win[b] == w) s += slab[static_cast<size_t>(b) * N + cidx];
  out[static_cast<size_t>(w) * N + cidx] = s;
}

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
    if (i < off + nh * H) { if (bn && g.bn_g) g.bn_g[i - off] = v; continue; }
    off += nh * H;
    if (i < off + nh * H) { if (bn && g.bn_b) g.bn_b[i - off] = v; continue; }
    off += nh * H;
    if (i < off + 2 * H) { g.w_head[i - off] = v; continue; }
    off += 2 * H;
    g.b_head[i - off] = v;
  }
}

static KArgs make_args(const VissmFlowDesc* d, const Geom& g) {
  KArgs a;
  a.B = d->B; a.L = d->L; a.k = d->k; a.H = d->H; a.bn = d->bn; a.s = g.s; a.swap_out = d->swap_out;
  a.n_logsig = d->n_logsig; a.n_win = d->n_win; a.Lout = g.Lout; a.Lh = g.Lh; a.CH = g.CH; a.n_chunks = g.n_chunks;
  a.S = g.S;
  return a;
}

}  // namespace flow1

using namespace flow1;

#define FLOW_DISPATCH(NHV, KERNEL, ...)                                                 \
  switch (NHV) {                                                                        \
    case 0: hipLaunchKernelGGL(KERNEL<0>, __VA_ARGS__); break;                          \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                          \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                          \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                          \
    default: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                         \
  }


size_t flow1_workspace_size(const VissmFlowDesc* d, int backward) {
  Geom g = geom(d, backward != 0);
  return backward ? bwd_ws_layout(d, g, nullptr, nullptr) : fwd_ws_layout(d, g, nullptr, nullptr);
}

int flow1_fwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C,
              const int32_t* win, const float* theta_term, float* u_next, float* logsig, void* workspace,
              size_t ws_bytes, hipStream_t st) {
  Geom g = geom(d, false);
  VISSM_CHECK_ARG(workspace && ws_bytes >= fwd_ws_layout(d, g, nullptr, nullptr), "flow_fwd: workspace too small");
  WsF ws;
  fwd_ws_layout(d, g, reinterpret_cast<char*>(workspace), &ws);
  hipLaunchKernelGGL(prep_weights_kernel, dim3(1), dim3(256), 0, st, *w, d->H, d->k, d->n_hidden, d->bn, ws.wp,
                     nullptr, ws.bh, ws.bng, ws.bnb, ws.weps, nullptr, ws.whead);
  VISSM_CHECK_LAUNCH("flow_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid(g.n_groups, g.n_chunks);
  prof_begin(VISSM_PROF_FLOW_FWD, st);
  FLOW_DISPATCH(d->n_hidden, flow_fwd_kernel, grid, dim3(NT), 0, st, a, u, C, wn, theta_term, ws.wp, ws.bh, ws.bng,
                ws.bnb, ws.weps, ws.whead, u_next, ws.ls_slab);
  VISSM_CHECK_LAUNCH("flow_fwd");
  prof_end(VISSM_PROF_FLOW_FWD, st);
  return launch_reduce_rows(ws.ls_slab, logsig, g.n_chunks, d->B, st);
}

int flow1_bwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C,
              const int32_t* win, const float* theta_term, const float* du_next, const float* dlogsig,
              float* du, float* dC, float* dtheta_term, const VissmFlowGrads* gr, void* workspace,
              size_t ws_bytes, hipStream_t st) {
  int rc;
  Geom g = geom(d, true);
  VISSM_CHECK_ARG(workspace && ws_bytes >= bwd_ws_layout(d, g, nullptr, nullptr), "flow_bwd: workspace too small");
  WsB ws;
  bwd_ws_layout(d, g, reinterpret_cast<char*>(workspace), &ws);
  hipLaunchKernelGGL(prep_weights_kernel, dim3(1), dim3(256), 0, st, *w, d->H, d->k, d->n_hidden, d->bn, ws.wp,
                     ws.wTp, ws.bh, ws.bng, ws.bnb, ws.weps, ws.wepsT, ws.whead);
  VISSM_CHECK_LAUNCH("flow_prep");
  KArgs a = make_args(d, g);
  const int32_t* wn = d->n_win > 1 ? win : nullptr;
  dim3 grid(g.n_groups, g.n_chunks);
  prof_begin(VISSM_PROF_FLOW_BWD, st);
  FLOW_DISPATCH(d->n_hidden, flow_bwd_kernel, grid, dim3(NT), 0, st, a, u, C, wn, theta_term, du_next, dlogsig,
                ws.wp, ws.wTp, ws.bh, ws.bng, ws.bnb, ws.weps, ws.wepsT, ws.whead, du, ws.dC_slab, ws.dth_slab,
                ws.dW_slab, ws.halo);
  VISSM_CHECK_LAUNCH("flow_bwd");
  prof_end(VISSM_PROF_FLOW_BWD, st);
  if (g.n_chunks > 1) {
    hipLaunchKernelGGL(halo_fixup_kernel, dim3(d->B), dim3(256), 0, st, du, ws.halo, d->B, d->L, d->k, g.n_chunks,
                       g.s, g.CH);
    VISSM_CHECK_LAUNCH("flow_halo");
  }
  const int64_t nC = static_cast<int64_t>(g.Lh) * d->H;
  if (d->n_win == 1) {
    rc = launch_reduce_rows(ws.dC_slab, dC, g.n_groups, nC, st);
    if (rc) return rc;
  } else {
    dim3 rg(static_cast<unsigned>((nC + 255) / 256), d->n_win);
    hipLaunchKernelGGL(reduce_by_window_kernel, rg, dim3(256), 0, st, ws.dC_slab, win, dC, d->B,
                       static_cast<int>(nC));
    VISSM_CHECK_LAUNCH("flow_reduce_window");
  }
  rc = launch_reduce_rows(ws.dth_slab, dtheta_term, g.n_chunks, static_cast<int64_t>(d->B) * d->H, st);
  if (rc) return rc;
  const int nW = n_wgrad(d);
  rc = launch_reduce_rows(ws.dW_slab, ws.wred, static_cast<int64_t>(g.n_groups) * g.n_chunks, nW, st);
  if (rc) return rc;
  hipLaunchKernelGGL(scatter_wgrad_kernel, dim3((nW + 255) / 256), dim3(256), 0, st, ws.wred, *gr, d->k, d->H,
                     d->n_hidden, d->bn);
  VISSM_CHECK_LAUNCH("flow_scatter");
  return VISSM_OK;
}


}  // namespace vissm
