// The window-shared feature branch of a flow and the first conv's feature channels, fused
// (vissm_feat_fwd / vissm_feat_bwd).
//
// Reference: AR.py:53-62 (SV_dense.py:53-62, fitz_nag_NVP.py:71-79) -- four tf.layers.dense with ELU over the
// window's time features, then the conv1d over [eps, features] (kernel [k][1 + H][H], bias, stride 1 or 2);
// this computes the feature channels' part of that conv,
//   C[w][m][o] = conv_b[o] + sum_{j < k} sum_{i < H} F[w][s m + j][i] conv_w[j][1 + i][o],
//   F = elu(elu(elu(elu(h0 W0 + b0) W1 + b1) W2 + b2) W3 + b3),
// which every sample of a window shares (the sample channel, conv_w[j][0][o] eps, is the flow kernel's).
// These products are tiny ([~5000 x 50] x [50 x 50] per layer) and run as ~40 library / elementwise launches per
// flow in torch; here one block computes a tile of kT output positions from its rows of F (recomputing the k - s
// halo rows its neighbour also computes) with the weights staged in LDS, fp32 FMAs throughout.  The backward
// partitions F's rows the same way: the transposed conv (dF), the conv's weight gradient over the tile's
// positions, the MLP backward; per-block weight-gradient partials go to a slab summed in a fixed order
// (deterministic; no atomics).
#include "common.hpp"

#include <cstdlib>
#include <type_traits>

namespace vissm {
namespace feat {

// output positions per block (forward) / per m-range of a block (backward): KT = 32, 16 or 8, fewer where the
// 32-position grid would leave most CUs idle (AR-cfg: one window of 5017 positions is 157 blocks for 256 CUs; pick_kt)
constexpr int kNT = 256;   // 4 waves: lane = output unit, wave = row group
constexpr int kMaxH = 64, kMaxCin = 63, kMaxK = 64;

struct Args {
  int n_win, Lf, Cin, H, k, s, Lh, Lu;   // Lu = s (Lh - 1) + k: the rows of F any output reads
  int64_t in_ws;                         // floats between windows of h0 (rows of Cin floats)
};

struct Params {
  const float* w[4];
  const float* b[4];
  const float* cw;   // conv kernel [k][1 + H][H]
  const float* cb;
};

__device__ __forceinline__ float elu(float x) { return x > 0.f ? x : expm1f(x); }
__device__ __forceinline__ float elu_d_out(float y) { return y > 0.f ? 1.f : y + 1.f; }  // from the output

// weights [nin][H] (row pitch H in global) into LDS with row pitch wp
__device__ __forceinline__ void stage_w(float* Ws, int wp, const float* g, int nin, int H) {
  for (int idx = threadIdx.x; idx < nin * H; idx += kNT) Ws[(idx / H) * wp + idx % H] = g[idx];
}
// the feature channels of conv tap j, [H in][H out], with row pitch wp
__device__ __forceinline__ void stage_tap(float* Ws, int wp, const float* cw, int j, int H) {
  const float* g = cw + static_cast<size_t>(j) * (1 + H) * H + H;
  for (int idx = threadIdx.x; idx < H * H; idx += kNT) Ws[(idx / H) * wp + idx % H] = g[idx];
}

// out[r][o] = elu(b[o] + sum_i in[r][i] W[i][o]) for r < R (rows in eight-row groups: rows up to the next
// multiple of 32 are read, the buffers hold them); rows r < n_store also go to gout (row pitch H)
__device__ void dense_elu(const float* in, int ip, int nin, const float* Ws, int wp, const float* bg, float* out,
                          int op, int R, int H, float* gout, int n_store) {
  const int o = threadIdx.x & 63, rg = threadIdx.x >> 6;
  if (o >= H) return;
  const float bo = bg[o];
  for (int r0 = rg * 8; r0 < R; r0 += 32) {
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = bo;
    for (int i = 0; i < nin; ++i) {
      const float wv = Ws[i * wp + o];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = fmaf(in[(r0 + q) * ip + i], wv, acc[q]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = r0 + q;
      if (r < R) {
        const float y = elu(acc[q]);
        out[r * op + o] = y;
        if (r < n_store) gout[static_cast<size_t>(r) * H + o] = y;
      }
    }
  }
}

// LDS layout (floats) shared by both kernels: rows padded to the next multiple of 32
__host__ __device__ inline int rows_pad(int r) { return (r + 31) / 32 * 32; }

// forward: grid (ceil(Lh / KT), n_win)
template <int KT>
__global__ __launch_bounds__(kNT) void feat_fwd_kernel(Args a, Params p, const float* __restrict__ h0,
                                                       float* __restrict__ C, float* __restrict__ act) {
  constexpr int kT = KT, RQ = KT / 4;   // output rows per wave in the conv
  extern __shared__ float sm[];
  const int H = a.H, hp = H + 1, ip = a.Cin + 1;
  const int w = blockIdx.y, m0 = blockIdx.x * kT;
  const int nm = min(kT, a.Lh - m0);
  const int r0 = a.s * m0;                                   // first row of F this block computes
  const int R = min(a.s * (kT - 1) + a.k, a.Lu - r0);        // rows it computes
  const bool last = m0 + kT >= a.Lh;
  const int n_own = last ? R : min(a.s * kT, R);              // rows it stores (the next block recomputes the rest)
  const int RP = rows_pad(a.s * (kT - 1) + a.k);
  float* hA = sm;                                // [RP][max(Cin, H) + 1]
  float* hB = hA + RP * max(ip, hp);             // [RP][H + 1]
  float* Ws = hB + RP * hp;                      // [max(Cin, H)][H + 1]
  const float* src = h0 + static_cast<int64_t>(w) * a.in_ws + static_cast<int64_t>(r0) * a.Cin;
  for (int idx = threadIdx.x; idx < RP * a.Cin; idx += kNT) {
    const int r = idx / a.Cin, c = idx % a.Cin;
    hA[r * ip + c] = r < R ? src[idx] : 0.f;
  }
  for (int idx = threadIdx.x; idx < RP * hp; idx += kNT) hB[idx] = 0.f;
  stage_w(Ws, hp, p.w[0], a.Cin, H);
  __syncthreads();
  const size_t plane = static_cast<size_t>(a.n_win) * a.Lf * H;
  float* ab = act + (static_cast<size_t>(w) * a.Lf + r0) * H;
  dense_elu(hA, ip, a.Cin, Ws, hp, p.b[0], hB, hp, R, H, ab, n_own);
  __syncthreads();
  stage_w(Ws, hp, p.w[1], H, H);
  __syncthreads();
  dense_elu(hB, hp, H, Ws, hp, p.b[1], hA, hp, R, H, ab + plane, n_own);
  __syncthreads();
  stage_w(Ws, hp, p.w[2], H, H);
  __syncthreads();
  dense_elu(hA, hp, H, Ws, hp, p.b[2], hB, hp, R, H, ab + 2 * plane, n_own);
  __syncthreads();
  stage_w(Ws, hp, p.w[3], H, H);
  __syncthreads();
  dense_elu(hB, hp, H, Ws, hp, p.b[3], hA, hp, R, H, ab + 3 * plane, n_own);   // F in hA (pitch hp)
  // rows of hA at and past R hold the previous layer's values: zero them (the conv reads up to RP rows)
  for (int idx = threadIdx.x; idx < (RP - R) * hp; idx += kNT) hA[R * hp + idx] = 0.f;
  // the conv over the feature channels: thread (o, rg) owns output rows rg*RQ .. rg*RQ + RQ - 1
  const int o = threadIdx.x & 63, rg = threadIdx.x >> 6;
  float acc[RQ];
#pragma unroll
  for (int q = 0; q < RQ; ++q) acc[q] = 0.f;
  for (int j = 0; j < a.k; ++j) {
    __syncthreads();
    stage_tap(Ws, hp, p.cw, j, H);
    __syncthreads();
    if (o < H) {
      const float* Fr = hA + (a.s * rg * RQ + j) * hp;
      for (int i = 0; i < H; ++i) {
        const float wv = Ws[i * hp + o];
#pragma unroll
        for (int q = 0; q < RQ; ++q) acc[q] = fmaf(Fr[a.s * q * hp + i], wv, acc[q]);
      }
    }
  }
  if (o < H) {
    const float bo = p.cb[o];
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int m = rg * RQ + q;
      if (m < nm) C[(static_cast<size_t>(w) * a.Lh + m0 + m) * H + o] = acc[q] + bo;
    }
  }
}

// gradient slab row layout: W0 [Cin][H], b0, W1, b1, W2, b2, W3, b3 ([H][H], [H]), conv taps [k][H][H], conv b [H]
struct Off {
  int w[4], b[4], cw, cb, n;
};
__host__ __device__ inline Off offsets(int Cin, int H, int k) {
  Off f;
  int o = 0;
  for (int l = 0; l < 4; ++l) {
    f.w[l] = o;
    o += (l == 0 ? Cin : H) * H;
    f.b[l] = o;
    o += H;
  }
  f.cw = o;
  o += k * H * H;
  f.cb = o;
  o += H;
  f.n = o;
  return f;
}

// part[i][o] = sum_{r < nr} X[r][i] G[r][o] for i < nin (thread (o, ig): i = ig, ig + 4, ...); written to slab
__device__ void wgrad(const float* X, int xp, int nin, const float* G, int gp, int nr, int H, float* out) {
  const int o = threadIdx.x & 63, ig = threadIdx.x >> 6;
  if (o >= H) return;
  for (int i0 = ig; i0 < nin; i0 += 64) {   // 16 inputs per pass: i0 + 4 t
    float acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = 0.f;
    for (int r = 0; r < nr; ++r) {
      const float g = G[r * gp + o];
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[t] = fmaf(X[r * xp + min(i0 + 4 * t, nin - 1)], g, acc[t]);
    }
#pragma unroll
    for (int t = 0; t < 16; ++t)
      if (i0 + 4 * t < nin) out[(i0 + 4 * t) * H + o] = acc[t];
  }
}

// backward: grid (ceil(Lu / (s KT)), n_win); block b owns F rows [b s KT, (b + 1) s KT) and positions
// m in [b KT, (b + 1) KT)
template <int KT>
__global__ __launch_bounds__(kNT) void feat_bwd_kernel(Args a, Params p, const float* __restrict__ h0,
                                                       const float* __restrict__ act, const float* __restrict__ dC,
                                                       float* __restrict__ slab) {
  constexpr int kT = KT;
  extern __shared__ float sm[];
  const int H = a.H, hp = H + 1, ip = a.Cin + 1, k = a.k, s = a.s;
  const int w = blockIdx.y, b = blockIdx.x;
  const int TR = s * kT;
  const int r0 = b * TR, nr = min(TR, a.Lu - r0);            // own rows of F
  const int m0 = b * kT, nm = max(0, min(kT, a.Lh - m0));    // own positions
  const int m_lo = r0 - (k - 1) >= 0 ? (r0 - (k - 1)) / s : -((k - 1 - r0 + s - 1) / s);  // floor((r0-k+1)/s)
  const int nd = m0 + kT - m_lo;                              // staged dC rows [m_lo, m0 + kT)
  const int RF = s * (kT - 1) + k;                            // staged F rows [r0, r0 + RF) for the conv gradient
  const int DP = rows_pad(nd), FP = rows_pad(RF), GP = rows_pad(TR);
  float* dCs = sm;                      // [DP][hp]
  float* Fs = dCs + DP * hp;            // [FP][hp]
  float* G0 = Fs + FP * hp;             // [GP][hp]  gradient rows (ping)
  float* G1 = G0 + GP * hp;             // [GP][hp]  (pong)
  float* Xs = G1 + GP * hp;             // [GP][max(ip, hp)]  a layer's input rows
  float* Ws = Xs + GP * max(ip, hp);    // [max(Cin, H)][hp]
  const size_t plane = static_cast<size_t>(a.n_win) * a.Lf * H;
  const float* dCw = dC + static_cast<size_t>(w) * a.Lh * H;
  for (int idx = threadIdx.x; idx < DP * hp; idx += kNT) {
    const int r = idx / hp, c = idx % hp, m = m_lo + r;
    dCs[idx] = (c < H && r < nd && m >= 0 && m < a.Lh) ? dCw[static_cast<size_t>(m) * H + c] : 0.f;
  }
  const float* F = act + 3 * plane + static_cast<size_t>(w) * a.Lf * H;
  for (int idx = threadIdx.x; idx < FP * hp; idx += kNT) {
    const int r = idx / hp, c = idx % hp, rr = r0 + r;
    Fs[idx] = (c < H && r < RF && rr < a.Lu) ? F[static_cast<size_t>(rr) * H + c] : 0.f;
  }
  __syncthreads();
  const Off of = offsets(a.Cin, H, k);
  float* out = slab + (static_cast<size_t>(w) * gridDim.x + b) * of.n;
  const int o = threadIdx.x & 63, rg = threadIdx.x >> 6;
  // conv bias: sum of the own positions' dC
  if (rg == 0 && o < H) {
    float sb = 0.f;
    for (int m = 0; m < nm; ++m) sb += dCs[(m0 + m - m_lo) * hp + o];
    out[of.cb + o] = sb;
  }
  // conv taps: dW_j[i][o] = sum_{own m} F[s m + j][i] dC[m][o] (F row s m + j - r0 = s (m - m0) + j)
  if (o < H) {
    for (int j = 0; j < k; ++j)
      for (int i0 = rg; i0 < H; i0 += 64) {
        float acc[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) acc[t] = 0.f;
        for (int m = 0; m < nm; ++m) {
          const float g = dCs[(m0 + m - m_lo) * hp + o];
          const float* Fr = Fs + (s * m + j) * hp;
#pragma unroll
          for (int t = 0; t < 16; ++t) acc[t] = fmaf(Fr[min(i0 + 4 * t, H - 1)], g, acc[t]);
        }
#pragma unroll
        for (int t = 0; t < 16; ++t)
          if (i0 + 4 * t < H) out[of.cw + (j * H + i0 + 4 * t) * H + o] = acc[t];
      }
  }
  // dF[r][i] = sum_j sum_o dC[(r - j) / s][o] W_j[i][o] over (r - j) divisible by s: thread (i, rg) rows
  // rg*Q .. rg*Q + Q - 1 of each 4Q-row group (Q = 8, or 4 when the block owns 16 rows)
  auto dF_pass = [&](auto qtag) {
    constexpr int Q = decltype(qtag)::value;
    const int i = o;
    for (int rb = 0; rb < TR; rb += 4 * Q) {
      float acc[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) acc[q] = 0.f;
      for (int j = 0; j < k; ++j) {
        __syncthreads();
        stage_tap(Ws, hp, p.cw, j, H);
        __syncthreads();
        if (i < H) {
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            const int r = r0 + rb + rg * Q + q - j;    // s m for the tap's position m
            if (r % s != 0) continue;                    // wave-uniform (one row per wave and q)
            const int mi = (r >= 0 ? r / s : -((-r + s - 1) / s)) - m_lo;
            if (mi < 0 || mi >= nd) continue;
            const float* dr = dCs + mi * hp;
            float v = 0.f;
            for (int oo = 0; oo < H; ++oo) v = fmaf(dr[oo], Ws[i * hp + oo], v);
            acc[q] += v;
          }
        }
      }
      // dz4 = dF * elu'(F) (F from the staged rows: row r - r0 of Fs)
      if (i < H) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int rl = rb + rg * Q + q;
          if (rl < GP) G0[rl * hp + i] = rl < nr ? acc[q] * elu_d_out(Fs[rl * hp + i]) : 0.f;
        }
      }
    }
    // rows [4Q ceil(TR / 4Q), GP) stay for the MLP backward below to read as zeros
    for (int rl = (TR + 4 * Q - 1) / (4 * Q) * (4 * Q) + threadIdx.x / 64; rl < GP; rl += 4)
      if (i < H) G0[rl * hp + i] = 0.f;
  };
  if (TR >= 32) dF_pass(std::integral_constant<int, 8>{});
  else if (TR >= 16) dF_pass(std::integral_constant<int, 4>{});
  else dF_pass(std::integral_constant<int, 2>{});
  // the MLP backward, layer 3 down to 0: dW_l = X_l^T dz, db_l = sum dz, dz_prev = (dz W_l^T) * elu'(X_l)
  float* Gc = G0;
  float* Gn = G1;
  for (int l = 3; l >= 0; --l) {
    const int nin = l == 0 ? a.Cin : H, xp = l == 0 ? ip : hp;
    __syncthreads();
    if (l == 0) {
      const float* src = h0 + static_cast<int64_t>(w) * a.in_ws + static_cast<int64_t>(r0) * a.Cin;
      for (int idx = threadIdx.x; idx < GP * a.Cin; idx += kNT) {
        const int r = idx / a.Cin, c = idx % a.Cin;
        Xs[r * ip + c] = r < nr ? src[idx] : 0.f;
      }
    } else {
      const float* X = act + (l - 1) * plane + (static_cast<size_t>(w) * a.Lf + r0) * H;
      for (int idx = threadIdx.x; idx < GP * hp; idx += kNT) {
        const int r = idx / hp, c = idx % hp;
        Xs[idx] = (r < nr && c < H) ? X[static_cast<size_t>(r) * H + c] : 0.f;
      }
    }
    if (l > 0) stage_w(Ws, hp, p.w[l], H, H);
    __syncthreads();
    wgrad(Xs, xp, nin, Gc, hp, nr, H, out + of.w[l]);
    if (rg == 0 && o < H) {
      float sb = 0.f;
      for (int r = 0; r < nr; ++r) sb += Gc[r * hp + o];
      out[of.b[l] + o] = sb;
    }
    if (l > 0) {
      const int i = o;
      if (i < H) {
        for (int r0b = rg * 8; r0b < GP; r0b += 32) {
          float acc[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] = 0.f;
          for (int oo = 0; oo < H; ++oo) {
            const float wv = Ws[i * hp + oo];
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[q] = fmaf(Gc[(r0b + q) * hp + oo], wv, acc[q]);
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int r = r0b + q;
            Gn[r * hp + i] = r < nr ? acc[q] * elu_d_out(Xs[r * hp + i]) : 0.f;
          }
        }
      }
      float* t = Gc;
      Gc = Gn;
      Gn = t;
    }
  }
}

// red [n] (the reduced slab row) -> the caller's gradient tensors; the conv kernel's sample channel gets 0
__global__ void feat_scatter_kernel(const float* __restrict__ red, int Cin, int H, int k, float* gw0, float* gb0,
                                    float* gw1, float* gb1, float* gw2, float* gb2, float* gw3, float* gb3,
                                    float* gcw, float* gcb) {
  const Off of = offsets(Cin, H, k);
  float* gw[4] = {gw0, gw1, gw2, gw3};
  float* gb[4] = {gb0, gb1, gb2, gb3};
  const int n_cw = k * (1 + H) * H;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < of.n - k * H * H + n_cw; i += gridDim.x * blockDim.x) {
    if (i < of.cw) {
      int l = 3;
      while (l > 0 && i < of.w[l]) --l;
      if (i < of.b[l]) gw[l][i - of.w[l]] = red[i];
      else gb[l][i - of.b[l]] = red[i];
    } else if (i < of.cw + n_cw) {
      const int e = i - of.cw, j = e / ((1 + H) * H), c = (e / H) % (1 + H), oo = e % H;
      gcw[e] = c == 0 ? 0.f : red[of.cw + (j * H + c - 1) * H + oo];
    } else {
      gcb[i - of.cw - n_cw] = red[of.cb + i - of.cw - n_cw];
    }
  }
}

// output positions per block: the largest of 32 / 16 / 8 that still gives two blocks per CU, else 8 (forward: fewer
// positions per block recompute more halo rows, k - s per block).  Same-box A/B (profiles/r06/ab_r06b.log,
// ab_r06d.log): FHN-cfg step 14.08 (torch form) -> 14.20 (16) -> 13.88 ms (8); AR-cfg 79.11 (16) / 78.82 (32) /
// 78.61 ms (8), within noise.  VISSM_FEAT_KT / VISSM_FEAT_KT_BWD = 8 | 16 | 32 override (A/B timing; the backward's
// choice also sizes its workspace: set it before vissm_feat_workspace_size)
static int env_kt(const char* name) {
  const char* e = std::getenv(name);
  const int v = e ? std::atoi(e) : 0;
  return (v == 8 || v == 16 || v == 32) ? v : 0;
}
static int pick_kt(const Args& a, bool bwd) {
  const int forced = env_kt(bwd ? "VISSM_FEAT_KT_BWD" : "VISSM_FEAT_KT");
  if (forced) return forced;
  for (int kt = 32; kt > 8; kt /= 2)
    if (static_cast<int64_t>((a.Lh + kt - 1) / kt) * a.n_win >= 512) return kt;
  return 8;
}
static int bwd_blocks(const Args& a, int kT) { return (a.Lu + a.s * kT - 1) / (a.s * kT); }

static size_t fwd_smem(const Args& a, int kT) {
  const int RP = rows_pad(a.s * (kT - 1) + a.k), hp = a.H + 1, wp = std::max(a.Cin, a.H) + 1;
  return static_cast<size_t>(RP * wp + RP * hp + wp * hp) * sizeof(float);
}
static size_t bwd_smem(const Args& a, int kT) {
  const int hp = a.H + 1, ip = a.Cin + 1;
  const int nd = kT + (a.k - 1 + a.s - 1) / a.s + 1;   // upper bound of the staged dC rows
  const int DP = rows_pad(nd), FP = rows_pad(a.s * (kT - 1) + a.k), GP = rows_pad(a.s * kT);
  return static_cast<size_t>(DP * hp + FP * hp + 2 * GP * hp + GP * std::max(ip, hp) + std::max(a.Cin, a.H) * hp) *
         sizeof(float);
}

// dynamic LDS above the default 64 KB (the backward at k = 20 / 50 takes 70-85 KB): raise the kernels' limit once
static int allow_lds() {
  static int rc = [] {
    const void* fs[6] = {reinterpret_cast<const void*>(feat_fwd_kernel<8>),
                         reinterpret_cast<const void*>(feat_fwd_kernel<16>),
                         reinterpret_cast<const void*>(feat_fwd_kernel<32>),
                         reinterpret_cast<const void*>(feat_bwd_kernel<8>),
                         reinterpret_cast<const void*>(feat_bwd_kernel<16>),
                         reinterpret_cast<const void*>(feat_bwd_kernel<32>)};
    for (const void* f : fs)
      if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) return 1;
    return 0;
  }();
  return rc;
}

static int make(const VissmFeatDesc* d, Args* a) {
  VISSM_CHECK_ARG(d && d->n_win >= 1 && d->Lf >= 1 && d->Cin >= 1 && d->Cin <= kMaxCin && d->H >= 1 &&
                      d->H <= kMaxH && d->k >= 1 && d->k <= kMaxK && (d->stride == 1 || d->stride == 2),
                  "feat: bad shape (n_win >= 1, Cin <= %d, H <= %d, k <= %d, stride 1 | 2)", kMaxCin, kMaxH, kMaxK);
  a->n_win = d->n_win;
  a->Lf = d->Lf;
  a->Cin = d->Cin;
  a->H = d->H;
  a->k = d->k;
  a->s = d->stride;
  a->Lh = d->Lh;
  VISSM_CHECK_ARG(d->Lh >= 1 && d->stride * (d->Lh - 1) + d->k <= d->Lf, "feat: Lh = %d needs s (Lh - 1) + k <= Lf = %d",
                  d->Lh, d->Lf);
  // a forward block computes s (kT - 1) + k rows and the backward reads its s kT own rows: k >= s keeps every row the
  // backward reads written by some forward block (k < s would leave row s kT - 1 of each block unwritten)
  VISSM_CHECK_ARG(d->k >= d->stride, "feat: kernel_len %d < stride %d", d->k, d->stride);
  a->Lu = d->stride * (d->Lh - 1) + d->k;
  a->in_ws = d->in_win_stride;
  VISSM_CHECK_ARG(a->in_ws >= static_cast<int64_t>(d->Lf) * d->Cin || d->n_win == 1,
                  "feat: windows of h0 overlap (in_win_stride < Lf Cin)");
  return VISSM_OK;
}

static Params params(const VissmFeatParams* w) {
  Params p;
  for (int l = 0; l < 4; ++l) {
    p.w[l] = w->w[l];
    p.b[l] = w->b[l];
  }
  p.cw = w->conv_w;
  p.cb = w->conv_b;
  return p;
}

// ---------------------------------------------------------------------------
// Lotka-Volterra's feature branch (lotka_volterra_partial.py:71-82): the first three dense + ELU layers over the
// window's R time-feature rows, H3 = elu(elu(elu(h0 W0 + b0) W1 + b1) W2 + b2), here in fp32 (32 rows per block, the
// dense_elu / wgrad code above); the time-mixing layer D = elu(H3 W3 + b3) ([R][U], U = the conv's time axis) and the
// first conv over D's R channels are matrix-core GEMMs (vissm_gemm_bf16) on the operands packed below.
// ---------------------------------------------------------------------------
constexpr int kLvRows = 32;   // rows per block
constexpr int kLvC = 64;      // columns of H3b: H3, then the ones column (W3b's bias row), then zeros

struct LvArgs {
  int n_win, R, Cin, H;
  int64_t in_ws;   // floats between windows of h0
  int nl;          // dense + ELU layers (LV 3, SV 4)
  int diff;        // SV's first-difference input (SV_dense.py:53)
};

// slab row layout of the layers' gradients: W0 [Cin][H], b0, W1 [H][H], b1, ...
__host__ __device__ inline int lv_off_w(int l, int Cin, int H) { return l == 0 ? 0 : Cin * H + H + (l - 1) * (H * H + H); }
__host__ __device__ inline int lv_n(int Cin, int H, int nl) { return Cin * H + H + (nl - 1) * (H * H + H); }

// the MLP input rows r0 .. r0 + nr - 1 of window w into X [32][ip] (zero rows past nr): h0's rows, or SV's
// [x[r + 1][0 .. Cr), x[r + 1][c] - x[r][c] for c < Cr - 2] of the window's time features x [L][Cr], Cr = (Cin + 2) / 2
__device__ inline void lv_load_in(float* X, int ip, const LvArgs& a, const float* __restrict__ h0, int w, int r0, int nr) {
  const float* hw = h0 + static_cast<int64_t>(w) * a.in_ws;
  const int Cr = (a.Cin + 2) / 2;
  for (int idx = threadIdx.x; idx < kLvRows * a.Cin; idx += kNT) {
    const int r = idx / a.Cin, c = idx % a.Cin;
    float v = 0.f;
    if (r < nr) {
      if (!a.diff) {
        v = hw[static_cast<int64_t>(r0 + r) * a.Cin + c];
      } else {
        const float* x1 = hw + static_cast<int64_t>(r0 + r + 1) * Cr;
        v = c < Cr ? x1[c] : x1[c - Cr] - x1[c - 2 * Cr];
      }
    }
    X[r * ip + c] = v;
  }
}

// forward: grid (ceil(R / 32), n_win); act [nl][n_win][R][H] fp32 (the layer outputs), H3b [n_win][R][64] bf16 (the
// last layer's output, the ones column, zeros) and, when H3lo is not null, its bf16 residual plane
__global__ __launch_bounds__(kNT) void lv_mlp_fwd_kernel(LvArgs a, Params p, const float* __restrict__ h0,
                                                         float* __restrict__ act, __bf16* __restrict__ H3b,
                                                         __bf16* __restrict__ H3lo) {
  const int H = a.H, hp = H + 1, ip = a.Cin + 1;
  __shared__ float hA[kLvRows * 65], hB[kLvRows * 65], Ws[64 * 65];
  const int w = blockIdx.y, r0 = blockIdx.x * kLvRows, nr = min(kLvRows, a.R - r0);
  lv_load_in(hA, ip, a, h0, w, r0, nr);
  const size_t plane = static_cast<size_t>(a.n_win) * a.R * H;
  float* ab = act + (static_cast<size_t>(w) * a.R + r0) * H;
  float* x = hA;
  float* y = hB;
  for (int l = 0; l < a.nl; ++l) {
    const int nin = l == 0 ? a.Cin : H, xp = l == 0 ? ip : hp;
    stage_w(Ws, hp, p.w[l], nin, H);
    __syncthreads();
    dense_elu(x, xp, nin, Ws, hp, p.b[l], y, hp, nr, H, ab + l * plane, nr);
    __syncthreads();
    float* t = x;
    x = y;
    y = t;
  }
  const size_t ofs = (static_cast<size_t>(w) * a.R + r0) * kLvC;
  for (int idx = threadIdx.x; idx < nr * kLvC; idx += kNT) {
    const int r = idx / kLvC, c = idx % kLvC;
    const float v = c < H ? x[r * hp + c] : (c == H ? 1.f : 0.f);
    const __bf16 hi = static_cast<__bf16>(v);
    H3b[ofs + idx] = hi;
    if (H3lo) H3lo[ofs + idx] = static_cast<__bf16>(v - static_cast<float>(hi));
  }
}

// backward: dH3 [n_win][R][ldd] fp32 (columns < H used) -> per-block partials of the three layers' gradients
__global__ __launch_bounds__(kNT) void lv_mlp_bwd_kernel(LvArgs a, Params p, const float* __restrict__ h0,
                                                         const float* __restrict__ act, const float* __restrict__ dH3,
                                                         int ldd, float* __restrict__ slab) {
  const int H = a.H, hp = H + 1, ip = a.Cin + 1;
  __shared__ float Gc_[kLvRows * 65], Gn_[kLvRows * 65], Xs[kLvRows * 65], Ws[64 * 65];
  float* Gc = Gc_;
  float* Gn = Gn_;
  const int w = blockIdx.y, b = blockIdx.x, r0 = b * kLvRows, nr = min(kLvRows, a.R - r0);
  const size_t plane = static_cast<size_t>(a.n_win) * a.R * H;
  float* out = slab + (static_cast<size_t>(w) * gridDim.x + b) * lv_n(a.Cin, H, a.nl);
  const int o = threadIdx.x & 63, rg = threadIdx.x >> 6;
  // dz = dH3 * elu'(H3) of the last layer
  {
    const float* X = act + (a.nl - 1) * plane + (static_cast<size_t>(w) * a.R + r0) * H;
    const float* D = dH3 + (static_cast<size_t>(w) * a.R + r0) * ldd;
    for (int idx = threadIdx.x; idx < kLvRows * hp; idx += kNT) {
      const int r = idx / hp, c = idx % hp;
      Gc[idx] = (r < nr && c < H) ? D[static_cast<size_t>(r) * ldd + c] * elu_d_out(X[static_cast<size_t>(r) * H + c]) : 0.f;
    }
  }
  for (int l = a.nl - 1; l >= 0; --l) {
    const int nin = l == 0 ? a.Cin : H, xp = l == 0 ? ip : hp;
    __syncthreads();
    if (l == 0) {
      lv_load_in(Xs, ip, a, h0, w, r0, nr);
    } else {
      const float* X = act + (l - 1) * plane + (static_cast<size_t>(w) * a.R + r0) * H;
      for (int idx = threadIdx.x; idx < kLvRows * hp; idx += kNT) {
        const int r = idx / hp, c = idx % hp;
        Xs[idx] = (r < nr && c < H) ? X[static_cast<size_t>(r) * H + c] : 0.f;
      }
    }
    if (l > 0) stage_w(Ws, hp, p.w[l], H, H);
    __syncthreads();
    const int ow = lv_off_w(l, a.Cin, H), obias = ow + nin * H;
    wgrad(Xs, xp, nin, Gc, hp, nr, H, out + ow);
    if (rg == 0 && o < H) {
      float sb = 0.f;
      for (int r = 0; r < nr; ++r) sb += Gc[r * hp + o];
      out[obias + o] = sb;
    }
    if (l > 0) {
      const int i = o;
      if (i < H) {
        for (int r0b = rg * 8; r0b < kLvRows; r0b += 32) {
          float acc[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] = 0.f;
          for (int oo = 0; oo < H; ++oo) {
            const float wv = Ws[i * hp + oo];
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[q] = fmaf(Gc[(r0b + q) * hp + oo], wv, acc[q]);
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int r = r0b + q;
            Gn[r * hp + i] = r < nr ? acc[q] * elu_d_out(Xs[r * hp + i]) : 0.f;
          }
        }
      }
      float* t = Gc;
      Gc = Gn;
      Gn = t;
    }
  }
}

__global__ void lv_mlp_scatter_kernel(const float* __restrict__ red, int Cin, int H, int nl, float* gw0, float* gb0,
                                      float* gw1, float* gb1, float* gw2, float* gb2, float* gw3, float* gb3) {
  float* gw[4] = {gw0, gw1, gw2, gw3};
  float* gb[4] = {gb0, gb1, gb2, gb3};
  const int n = lv_n(Cin, H, nl);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int l = nl - 1;
    while (l > 0 && i < lv_off_w(l, Cin, H)) --l;
    const int ow = lv_off_w(l, Cin, H), nin = l == 0 ? Cin : H;
    if (i < ow + nin * H) gw[l][i - ow] = red[i];
    else gb[l][i - ow - nin * H] = red[i];
  }
}

// W3b [64][ldw] bf16: rows < H the time-mixing kernel W3 [H][U], row H its bias, the rest zero; Wc [R][ldc] bf16:
// Wc[r][j H + h] = conv_w[j][1 + r][h] (the conv's feature channels), zero past k H
__global__ void lv_pack_kernel(const float* __restrict__ w3, const float* __restrict__ b3, int H, int U, int ldw,
                               __bf16* __restrict__ W3b, __bf16* __restrict__ W3b_lo, const float* __restrict__ cw,
                               int R, int k, int ldc, __bf16* __restrict__ Wc, __bf16* __restrict__ Wc_lo) {
  const int64_t n1 = static_cast<int64_t>(kLvC) * ldw, n2 = static_cast<int64_t>(R) * ldc;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n1 + n2;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    if (i < n1) {
      const int c = static_cast<int>(i / ldw), u = static_cast<int>(i % ldw);
      const float v = u >= U ? 0.f : c < H ? w3[static_cast<int64_t>(c) * U + u] : c == H ? b3[u] : 0.f;
      const __bf16 hi = static_cast<__bf16>(v);
      W3b[i] = hi;
      if (W3b_lo) W3b_lo[i] = static_cast<__bf16>(v - static_cast<float>(hi));
    } else {
      const int64_t e = i - n1;
      const int r = static_cast<int>(e / ldc), n = static_cast<int>(e % ldc);
      const int j = n / H, h = n % H;
      const float v = j < k ? cw[(static_cast<int64_t>(j) * (1 + R) + 1 + r) * H + h] : 0.f;
      const __bf16 hi = static_cast<__bf16>(v);
      Wc[e] = hi;
      if (Wc_lo) Wc_lo[e] = static_cast<__bf16>(v - static_cast<float>(hi));
    }
  }
}

// C[m][h] = conv_b[h] + sum_{j < k} G[s m + j][j H + h]  (G [U][ldg] fp32)
__global__ void lv_diag_kernel(const float* __restrict__ G, int ldg, const float* __restrict__ cb, int H, int k,
                               int s, int Lh, float* __restrict__ C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Lh * H) return;
  const int m = i / H, h = i % H;
  float v = cb[h];
  for (int j = 0; j < k; ++j) v += G[static_cast<int64_t>(s * m + j) * ldg + j * H + h];
  C[i] = v;
}

// dG[u][j H + h] = dC[(u - j) / s][h] where (u - j) / s is a position (bf16 [U][ldg], zero elsewhere and past k H):
// grid (ceil(ldg / 256), U), 32-bit index arithmetic
__global__ void lv_diag_bwd_kernel(const float* __restrict__ dC, int H, int k, int s, int Lh, int ldg,
                                   __bf16* __restrict__ dG, __bf16* __restrict__ dG_lo) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x, u = blockIdx.y;
  if (c >= ldg) return;
  const int j = c / H, h = c - j * H, t = u - j;
  float v = 0.f;
  if (j < k && t >= 0 && t % s == 0 && t / s < Lh) v = dC[(t / s) * H + h];
  const __bf16 hi = static_cast<__bf16>(v);
  dG[static_cast<int64_t>(u) * ldg + c] = hi;
  if (dG_lo) dG_lo[static_cast<int64_t>(u) * ldg + c] = static_cast<__bf16>(v - static_cast<float>(hi));
}

// db[h] = sum_m dC[m][h]: one block per column, strided partial sums then the fixed-order block sum (deterministic)
__global__ __launch_bounds__(256) void lv_colsum_kernel(const float* __restrict__ dC, int H, int Lh, float* __restrict__ db) {
  __shared__ float red[4];
  const int h = blockIdx.x;
  float v = 0.f;
  for (int m = threadIdx.x; m < Lh; m += 256) v += dC[static_cast<int64_t>(m) * H + h];
  v = block_sum(v, red);
  if (threadIdx.x == 0) db[h] = v;
}

// dconv_w[j][1 + r][h] = dWc[r][j H + h] (channel 0, the flow kernel's w_eps, gets zero)
__global__ void lv_wscatter_kernel(const float* __restrict__ dWc, int ldc, int R, int k, int H, float* __restrict__ gcw) {
  const int64_t n = static_cast<int64_t>(k) * (1 + R) * H;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < n;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int j = static_cast<int>(e / ((1 + R) * static_cast<int64_t>(H)));
    const int c = static_cast<int>((e / H) % (1 + R)), h = static_cast<int>(e % H);
    gcw[e] = c == 0 ? 0.f : dWc[static_cast<int64_t>(c - 1) * ldc + j * H + h];
  }
}

}  // namespace feat
}  // namespace vissm

using namespace vissm;

extern "C" {

size_t vissm_feat_workspace_size(const VissmFeatDesc* d) {
  feat::Args a;
  if (feat::make(d, &a)) return 0;
  const int nb = feat::bwd_blocks(a, feat::pick_kt(a, true));
  const feat::Off of = feat::offsets(a.Cin, a.H, a.k);
  return align_up(static_cast<size_t>(a.n_win) * nb * of.n * sizeof(float)) + align_up(of.n * sizeof(float));
}

int vissm_feat_fwd(const VissmFeatDesc* d, const VissmFeatParams* w, const float* h0, float* C, float* act,
                   void* stream) {
  feat::Args a;
  int rc = feat::make(d, &a);
  if (rc) return rc;
  VISSM_CHECK_ARG(w && h0 && C && act, "feat_fwd: null pointer");
  if (feat::allow_lds()) {
    set_error("feat_fwd: hipFuncSetAttribute failed");
    return VISSM_ELAUNCH;
  }
  const int kt = feat::pick_kt(a, false);
  dim3 grid((a.Lh + kt - 1) / kt, a.n_win);
  if (kt == 8)
    hipLaunchKernelGGL(feat::feat_fwd_kernel<8>, grid, dim3(feat::kNT), feat::fwd_smem(a, 8), as_stream(stream), a,
                       feat::params(w), h0, C, act);
  else if (kt == 16)
    hipLaunchKernelGGL(feat::feat_fwd_kernel<16>, grid, dim3(feat::kNT), feat::fwd_smem(a, 16), as_stream(stream), a,
                       feat::params(w), h0, C, act);
  else
    hipLaunchKernelGGL(feat::feat_fwd_kernel<32>, grid, dim3(feat::kNT), feat::fwd_smem(a, 32), as_stream(stream), a,
                       feat::params(w), h0, C, act);
  VISSM_CHECK_LAUNCH("feat_fwd");
  return VISSM_OK;
}

int vissm_feat_bwd(const VissmFeatDesc* d, const VissmFeatParams* w, const float* h0, const float* act,
                   const float* dC, const VissmFeatGrads* g, void* workspace, size_t ws_bytes, void* stream) {
  feat::Args a;
  int rc = feat::make(d, &a);
  if (rc) return rc;
  VISSM_CHECK_ARG(w && h0 && act && dC && g, "feat_bwd: null pointer");
  VISSM_CHECK_ARG(workspace && ws_bytes >= vissm_feat_workspace_size(d), "feat_bwd: workspace too small");
  if (feat::allow_lds()) {
    set_error("feat_bwd: hipFuncSetAttribute failed");
    return VISSM_ELAUNCH;
  }
  hipStream_t st = as_stream(stream);
  const int kt = feat::pick_kt(a, true);
  const int nb = feat::bwd_blocks(a, kt);
  const feat::Off of = feat::offsets(a.Cin, a.H, a.k);
  float* slab = static_cast<float*>(workspace);
  float* red = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                        align_up(static_cast<size_t>(a.n_win) * nb * of.n * sizeof(float)));
  if (kt == 8)
    hipLaunchKernelGGL(feat::feat_bwd_kernel<8>, dim3(nb, a.n_win), dim3(feat::kNT), feat::bwd_smem(a, 8), st, a,
                       feat::params(w), h0, act, dC, slab);
  else if (kt == 16)
    hipLaunchKernelGGL(feat::feat_bwd_kernel<16>, dim3(nb, a.n_win), dim3(feat::kNT), feat::bwd_smem(a, 16), st, a,
                       feat::params(w), h0, act, dC, slab);
  else
    hipLaunchKernelGGL(feat::feat_bwd_kernel<32>, dim3(nb, a.n_win), dim3(feat::kNT), feat::bwd_smem(a, 32), st, a,
                       feat::params(w), h0, act, dC, slab);
  VISSM_CHECK_LAUNCH("feat_bwd");
  rc = launch_reduce_rows(slab, red, static_cast<int64_t>(a.n_win) * nb, of.n, st);
  if (rc) return rc;
  hipLaunchKernelGGL(feat::feat_scatter_kernel, dim3((of.n + a.k * a.H + 255) / 256), dim3(256), 0, st, red, a.Cin,
                     a.H, a.k, g->w[0], g->b[0], g->w[1], g->b[1], g->w[2], g->b[2], g->w[3], g->b[3], g->conv_w,
                     g->conv_b);
  VISSM_CHECK_LAUNCH("feat_scatter");
  return VISSM_OK;
}

// ---- Lotka-Volterra's feature branch (the three fp32 layers and the GEMM operand packing; lotka_volterra_partial.py:71-82)
static int lv_make(const VissmLvFeatDesc* d, feat::LvArgs* a) {
  VISSM_CHECK_ARG(d && d->n_win >= 1 && d->R >= 1 && d->Cin >= 1 && d->Cin <= feat::kMaxCin && d->H >= 1 && d->H < feat::kLvC,
                  "lv_feat: bad shape (Cin <= %d, H < %d)", feat::kMaxCin, feat::kLvC);
  VISSM_CHECK_ARG(d->n_layers == 0 || d->n_layers == 3 || d->n_layers == 4, "lv_feat: n_layers %d (3 or 4)", d->n_layers);
  VISSM_CHECK_ARG(!d->sv_diff || (d->Cin >= 2 && d->Cin % 2 == 0), "lv_feat: the difference input needs Cin = 2 Cr - 2");
  const int64_t rows = d->sv_diff ? static_cast<int64_t>(d->R + 1) * ((d->Cin + 2) / 2) : static_cast<int64_t>(d->R) * d->Cin;
  VISSM_CHECK_ARG(d->in_win_stride >= rows || d->n_win == 1, "lv_feat: windows of h0 overlap");
  a->n_win = d->n_win; a->R = d->R; a->Cin = d->Cin; a->H = d->H; a->in_ws = d->in_win_stride;
  a->nl = d->n_layers == 0 ? 3 : d->n_layers;
  a->diff = d->sv_diff ? 1 : 0;
  return VISSM_OK;
}

size_t vissm_lv_mlp_workspace_size(const VissmLvFeatDesc* d) {
  feat::LvArgs a;
  if (lv_make(d, &a)) return 0;
  const int nb = (a.R + feat::kLvRows - 1) / feat::kLvRows;
  const int n = feat::lv_n(a.Cin, a.H, a.nl);
  return align_up(static_cast<size_t>(a.n_win) * nb * n * sizeof(float)) + align_up(n * sizeof(float));
}

int vissm_lv_mlp_fwd(const VissmLvFeatDesc* d, const VissmFeatParams* w, const float* h0, float* act, void* H3b,
                     void* H3lo, void* stream) {
  feat::LvArgs a;
  int rc = lv_make(d, &a);
  if (rc) return rc;
  VISSM_CHECK_ARG(w && h0 && act && H3b, "lv_mlp_fwd: null pointer");
  dim3 grid((a.R + feat::kLvRows - 1) / feat::kLvRows, a.n_win);
  hipLaunchKernelGGL(feat::lv_mlp_fwd_kernel, grid, dim3(feat::kNT), 0, as_stream(stream), a, feat::params(w), h0, act,
                     static_cast<__bf16*>(H3b), static_cast<__bf16*>(H3lo));
  VISSM_CHECK_LAUNCH("lv_mlp_fwd");
  return VISSM_OK;
}

int vissm_lv_mlp_bwd(const VissmLvFeatDesc* d, const VissmFeatParams* w, const float* h0, const float* act,
                     const float* dH3, int ld_dH3, const VissmFeatGrads* g, void* workspace, size_t ws_bytes,
                     void* stream) {
  feat::LvArgs a;
  int rc = lv_make(d, &a);
  if (rc) return rc;
  VISSM_CHECK_ARG(w && h0 && act && dH3 && g && ld_dH3 >= d->H, "lv_mlp_bwd: bad argument");
  VISSM_CHECK_ARG(workspace && ws_bytes >= vissm_lv_mlp_workspace_size(d), "lv_mlp_bwd: workspace too small");
  hipStream_t st = as_stream(stream);
  const int nb = (a.R + feat::kLvRows - 1) / feat::kLvRows;
  const int n = feat::lv_n(a.Cin, a.H, a.nl);
  float* slab = static_cast<float*>(workspace);
  float* red = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                        align_up(static_cast<size_t>(a.n_win) * nb * n * sizeof(float)));
  hipLaunchKernelGGL(feat::lv_mlp_bwd_kernel, dim3(nb, a.n_win), dim3(feat::kNT), 0, st, a, feat::params(w), h0, act, dH3,
                     ld_dH3, slab);
  VISSM_CHECK_LAUNCH("lv_mlp_bwd");
  rc = launch_reduce_rows(slab, red, static_cast<int64_t>(a.n_win) * nb, n, st);
  if (rc) return rc;
  VISSM_CHECK_ARG(a.nl < 4 || (g->w[3] && g->b[3]), "lv_mlp_bwd: four layers need the w[3] / b[3] gradients");
  hipLaunchKernelGGL(feat::lv_mlp_scatter_kernel, dim3((n + 255) / 256), dim3(256), 0, st, red, a.Cin, a.H, a.nl,
                     g->w[0], g->b[0], g->w[1], g->b[1], g->w[2], g->b[2], g->w[3], g->b[3]);
  VISSM_CHECK_LAUNCH("lv_mlp_scatter");
  return VISSM_OK;
}

int vissm_lv_pack(const float* w3, const float* b3, int H, int U, int ldw, void* W3b, void* W3b_lo, const float* conv_w,
                  int R, int k, int ldc, void* Wc, void* Wc_lo, void* stream) {
  VISSM_CHECK_ARG((ldw == 0 || (w3 && b3 && W3b && U >= 1 && ldw >= U)) && conv_w && Wc && H >= 1 && H < feat::kLvC &&
                      R >= 1 && k >= 1 && ldc >= k * H,
                  "lv_pack: bad argument");
  const int64_t n = static_cast<int64_t>(feat::kLvC) * ldw + static_cast<int64_t>(R) * ldc;
  hipLaunchKernelGGL(feat::lv_pack_kernel, dim3(static_cast<unsigned>(std::min<int64_t>((n + 255) / 256, 16384))),
                     dim3(256), 0, as_stream(stream), w3, b3, H, U, ldw, static_cast<__bf16*>(W3b),
                     static_cast<__bf16*>(W3b_lo), conv_w, R, k, ldc, static_cast<__bf16*>(Wc), static_cast<__bf16*>(Wc_lo));
  VISSM_CHECK_LAUNCH("lv_pack");
  return VISSM_OK;
}

int vissm_lv_conv_diag(const float* G, int ldg, const float* conv_b, int H, int k, int stride, int Lh, float* C,
                       void* stream) {
  VISSM_CHECK_ARG(G && conv_b && C && H >= 1 && k >= 1 && (stride == 1 || stride == 2) && Lh >= 1 && ldg >= k * H,
                  "lv_conv_diag: bad argument");
  hipLaunchKernelGGL(feat::lv_diag_kernel, dim3((Lh * H + 255) / 256), dim3(256), 0, as_stream(stream), G, ldg, conv_b,
                     H, k, stride, Lh, C);
  VISSM_CHECK_LAUNCH("lv_conv_diag");
  return VISSM_OK;
}

int vissm_lv_conv_diag_bwd(const float* dC, int H, int k, int stride, int Lh, int U, int ldg, void* dG, void* dG_lo,
                           float* dconv_b, void* stream) {
  VISSM_CHECK_ARG(dC && dG && dconv_b && H >= 1 && H <= 256 && k >= 1 && (stride == 1 || stride == 2) && Lh >= 1 &&
                      ldg >= k * H && stride * (Lh - 1) + k <= U,
                  "lv_conv_diag_bwd: bad argument");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(feat::lv_diag_bwd_kernel, dim3((ldg + 255) / 256, U), dim3(256), 0, st, dC, H, k, stride, Lh, ldg,
                     static_cast<__bf16*>(dG), static_cast<__bf16*>(dG_lo));
  VISSM_CHECK_LAUNCH("lv_conv_diag_bwd");
  // the conv bias gradient: column sums of dC over its Lh rows (a single sequential pass per column was 0.65 ms of
  // dependent loads at Lh = 5000)
  hipLaunchKernelGGL(feat::lv_colsum_kernel, dim3(H), dim3(256), 0, st, dC, H, Lh, dconv_b);
  VISSM_CHECK_LAUNCH("lv_conv_diag_bwd colsum");
  return VISSM_OK;
}

int vissm_lv_conv_wscatter(const float* dWc, int ldc, int R, int k, int H, float* dconv_w, void* stream) {
  VISSM_CHECK_ARG(dWc && dconv_w && R >= 1 && k >= 1 && H >= 1 && ldc >= k * H, "lv_conv_wscatter: bad argument");
  const int64_t n = static_cast<int64_t>(k) * (1 + R) * H;
  hipLaunchKernelGGL(feat::lv_wscatter_kernel, dim3(static_cast<unsigned>(std::min<int64_t>((n + 255) / 256, 16384))),
                     dim3(256), 0, as_stream(stream), dWc, ldc, R, k, H, dconv_w);
  VISSM_CHECK_LAUNCH("lv_conv_wscatter");
  return VISSM_OK;
}

}  // extern "C"
