// ELBO log-density kernels, all streaming with one wave per trajectory: the path z is read
// once with 16-byte loads (the backward also writes dz with 16-byte stores), the per-window
// feeds are L2-resident, per-sample constants are hoisted and the per-sample sums are fixed-order
// wave reductions in double (no block barriers).
//
// Reference terms: AR VI_SSM._ELBO (AR.py:168-187); LV Softplus transform and
// _ELBO (lotka_volterra_partial.py:290-297, 234-270); SV dim-one concat and
// _ELBO (SV_dense.py:245-246, 203-232); FHN _ELBO (fitz_nag_NVP.py:232-265).
#include "common.hpp"
#include "elbo_math.hpp"

#include <type_traits>

namespace vissm {
namespace elbo {

struct Args {
  int B, M, n_win;
  float dt, obs_std;
  VissmElboData d;
};

// ---------------------------------------------------------------------------
// LV / SV / FHN streaming path: one wave per trajectory (kSW per 256-thread block), each lane owning
// chunks of kV = 4 consecutive times; a chunk's stored z (LV / FHN: 2 kV interleaved floats, SV: kV)
// and its per-window feed rows (mask / shift / dim_one / obs / obs_bin, L2-resident) are read with
// 16-byte loads, kSU chunks in flight per lane.  The forward evaluates the chunk's kV transitions
// t0 -> t0+1 .. (its states plus the next one); the backward evaluates the kV + 1 transitions touching
// its elements once each (states t0-1 .. t0+kV) and writes the chunk's dz with 16-byte stores.
// Per-lane partials in fp32 over a few dozen chunks, wave reductions in double (fixed order, no
// block barrier).  The first chunk and the tail (t < kV, t >= kV floor(M/kV)) take a per-element path.
// ---------------------------------------------------------------------------
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
// times per chunk (8: slower for every model, LV one-pass 0.48 -> 0.55 ms, profiles/r05/ab_elbo.log)
constexpr int kV = 4;
constexpr int kSU = 2;  // chunks per lane in flight
constexpr int kSW = 4;  // trajectories (waves) per 256-thread block
#ifndef VISSM_ELBO_ONEPASS_NB
#define VISSM_ELBO_ONEPASS_NB 1   // vissm_elbo_fwd_grad's LV / SV / FHN kernel: neighbour exchange (0: chunk-local)
#endif
// waves per trajectory of that kernel by model (stream_onepass_kernel NWV).  One: two or four waves per trajectory
// measured slower for every model (SV 51.8 -> 57.4 / 71.4 us, FHN 75.9 -> 80.6 / 91.4, LV 385 -> 405 / 443 us per
// launch, profiles/r06/ab_r06i.log): the launch already fills the chip, and each range adds its edge states, transition
// and the block barrier
constexpr int kNwvLV = 1, kNwvSV = 1, kNwvFHN = 1;

__device__ __forceinline__ f4u ld4(const float* p) { return *reinterpret_cast<const f4u*>(p); }

// N consecutive floats from p (16-byte loads, then an 8-byte and a 4-byte load for the rest)
template <int N>
__device__ __forceinline__ void ldn(const float* __restrict__ p, float (&o)[N]) {
#pragma unroll
  for (int i = 0; i + 4 <= N; i += 4) {
    const f4u v = ld4(p + i);
    o[i] = v[0]; o[i + 1] = v[1]; o[i + 2] = v[2]; o[i + 3] = v[3];
  }
  constexpr int r = N / 4 * 4;
  if constexpr (N - r >= 2) {
    const f2u v = *reinterpret_cast<const f2u*>(p + r);
    o[r] = v[0]; o[r + 1] = v[1];
  }
  if constexpr ((N - r) % 2 == 1) o[N - 1] = p[N - 1];
}

struct St {
  float x[2];    // state
  float j[2];    // d state / d stored z
  float il[2];   // LV: Softplus ILDJ at the state, and its derivative w.r.t. the stored z
  float dil[2];
};

template <int MODEL>
struct Dev;

// fast transcendentals for the streaming path: hardware exp / log / rcp (v_exp_f32, v_log_f32, v_rcp_f32:
// ~1 ulp), with the small-argument branches that keep log1p / expm1 accurate
// (no denormal range scaling: the arguments here are far from the denormal range, and an
// underflowing e^x flushing to 0 is the right limit)
__device__ __forceinline__ float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float flog(float x) { return __builtin_amdgcn_logf(x) * 0.6931471805599453f; }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
// log1p(e) for e in [0, 1]
__device__ __forceinline__ float flog1p01(float e) { return e > 1e-3f ? flog(1.f + e) : e * (1.f - 0.5f * e); }
// 1 - e^{-y} for y > 0 (= -expm1(-y)); the libm path only where a lane needs it (small y)
__device__ __forceinline__ float one_minus_exp_neg(float y) {
  return y > 0.25f ? 1.f - fexp(-y) : -::expm1f(-y);
}

// LV: x = softplus(z) * mask + shift per coordinate (lotka_volterra_partial.py:290-297), obs N(., 1),
// log q += Softplus ILDJ at x_{t+1}; the Cholesky EM density with exp(theta) hoisted per sample
template <>
struct Dev<VISSM_MODEL_LV> {
  static constexpr int P = 3, ZD = 2, SU = 1;  // (registers: one chunk in flight per lane)
  static constexpr bool kObs = true, kExtra = true;
  static constexpr float kSd = 1.f;
  float E0, E1, E2, c_lp;
  int M;
  const float *mk, *sh, *ob, *bn;  // window rows: mask / shift [2][M+1], obs / obs_bin [2][M]
  __device__ void init(const Args& a, const float* thp, int w) {
    E0 = a.dt * ::expf(thp[0]); E1 = a.dt * ::expf(thp[1]); E2 = a.dt * ::expf(thp[2]);
    c_lp = -em::kLog2Pi_;   // -1/2 log det Sigma is -1/2 log D: dt is inside the rates
    M = a.M;
    mk = a.d.mask + static_cast<size_t>(w) * 2 * (M + 1);
    sh = a.d.shift + static_cast<size_t>(w) * 2 * (M + 1);
    ob = a.d.obs + static_cast<size_t>(w) * 2 * M;
    bn = a.d.obs_bin + static_cast<size_t>(w) * 2 * M;
  }
  // softplus and its derivative from one exp: e = e^{-|z|}, softplus = max(z, 0) + log1p(e).  The ILDJ
  // the reference adds at the transformed path, -log(1 - e^{-x}) (lotka_volterra_partial.py:294-296), is
  // softplus(-z) = max(-z, 0) + log1p(e) where the window's mask is 1 and shift 0 (every position it
  // covers in the reference: x = softplus(z)), with derivative sigmoid(z) - 1: no transcendental beyond
  // the transform's own; any other mask / shift takes the general path.
  __device__ static void tf(float zz, float m, float s, float* x, float* j, float* il, float* dil) {
    const float e = fexp(-::fabsf(zz));
    const float L = flog1p01(e);
    *x = (::fmaxf(zz, 0.f) + L) * m + s;
    const float r = frcp(1.f + e);
    const float sg = zz >= 0.f ? r : e * r;  // sigmoid(z)
    *j = m * sg;
    if (m == 1.f && s == 0.f) {
      *il = L - ::fminf(zz, 0.f);   // max(-z, 0) + L: min(z, 0) shares max(z, 0)'s canonical z
      *dil = sg - 1.f;
    } else {
      float g;
      *il = ildj(*x, &g);
      *dil = g * *j;
    }
  }
  // the transform where the window's mask is 1 and shift 0 (VissmElboData.plain_from): no mask / shift loads
  __device__ static void tf_plain(float zz, float* x, float* j, float* il, float* dil) {
    const float e = fexp(-::fabsf(zz));
    const float L = flog1p01(e);
    *x = ::fmaxf(zz, 0.f) + L;
    const float r = frcp(1.f + e);
    const float sg = zz >= 0.f ? r : e * r;  // sigmoid(z)
    *j = sg;
    *il = L - ::fminf(zz, 0.f);   // max(-z, 0) + L: min(z, 0) shares max(z, 0)'s canonical z
    *dil = sg - 1.f;
  }
  template <int N, bool PLAIN = false>
  __device__ void states(const float* zb, int t0, St (&o)[N]) const {
    if constexpr (PLAIN) {
      float zz[2 * N];
      ldn<2 * N>(zb + 2 * t0, zz);
#pragma unroll
      for (int i = 0; i < N; ++i) {
        tf_plain(zz[2 * i], &o[i].x[0], &o[i].j[0], &o[i].il[0], &o[i].dil[0]);
        tf_plain(zz[2 * i + 1], &o[i].x[1], &o[i].j[1], &o[i].il[1], &o[i].dil[1]);
      }
      return;
    }
    float zz[2 * N], m0[N], m1[N], s0[N], s1[N];
    ldn<2 * N>(zb + 2 * t0, zz);
    ldn<N>(mk + t0, m0);
    ldn<N>(mk + (M + 1) + t0, m1);
    ldn<N>(sh + t0, s0);
    ldn<N>(sh + (M + 1) + t0, s1);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      tf(zz[2 * i], m0[i], s0[i], &o[i].x[0], &o[i].j[0], &o[i].il[0], &o[i].dil[0]);
      tf(zz[2 * i + 1], m1[i], s1[i], &o[i].x[1], &o[i].j[1], &o[i].il[1], &o[i].dil[1]);
    }
  }
  __device__ St state(const float* zb, int t) const {
    St o;
    tf(zb[2 * t], mk[t], sh[t], &o.x[0], &o.j[0], &o.il[0], &o.dil[0]);
    tf(zb[2 * t + 1], mk[M + 1 + t], sh[M + 1 + t], &o.x[1], &o.j[1], &o.il[1], &o.dil[1]);
    return o;
  }
  // em::lv_trans with dt folded into the hoisted rates (E_i = dt e^{theta_i}): the rate terms a = E0 x1, b = E1 x1 x2,
  // c = E2 x2 are the drift components (m = (a - b, b - c)) and the covariance entries (Sigma = [[a + b, -b],
  // [-b, b + c]]) at once; det = a (b + c) + b c (a sum of positive terms: no cancellation), one reciprocal.
  // Gradients through g = Sigma^-1 q: d lp / d Sigma_ij = (g_i g_j - Sigma^-1_ij) / 2, and each rate's theta
  // gradient is (d lp / d rate) rate.
  __device__ em::TG trans(const St& p, const St& q) const {
    em::TG r;
    const float x1 = p.x[0], x2 = p.x[1];
    const float a = E0 * x1, e1x2 = E1 * x2, c = E2 * x2;
    const float b = e1x2 * x1;
    const float A = a + b, C = b + c;
    const float q1 = q.x[0] - x1 - (a - b), q2 = q.x[1] - x2 - (b - c);
    const float D = a * C + b * c;
    const float iD = frcp(D);
    const float g1 = iD * (C * q1 + b * q2), g2 = iD * (b * q1 + A * q2);
    const float quad = q1 * g1 + q2 * g2;
    r.lp = -0.5f * flog(D) - 0.5f * quad + c_lp;
    const float hD = 0.5f * iD;
    const float gA = 0.5f * g1 * g1 - C * hD;        // d lp / d Sigma_11
    const float gC = 0.5f * g2 * g2 - A * hD;        // d lp / d Sigma_22
    const float gb = b * iD - g1 * g2;               // d lp / d b through the off-diagonal entries
    const float Ga = gA + g1, Gc = gC - g2;          // + the drift: d lp / d m = g
    const float Gb = gA + gC + gb - g1 + g2;
    r.gt[0] = -g1;
    r.gt[1] = -g2;
    r.gh[0] = g1 + Ga * E0 + Gb * e1x2;
    r.gh[1] = g2 + Gc * E2 + Gb * (E1 * x1);
    r.gth[0] = Ga * a;
    r.gth[1] = Gb * b;
    r.gth[2] = Gc * c;
    r.gth[3] = r.gth[4] = 0.f;
    return r;
  }
  // Softplus ILDJ at y: -log(1 - e^{-y}), derivative -e^{-y} / (1 - e^{-y}) = 1 - 1 / (1 - e^{-y})
  __device__ static float ildj(float y, float* g) {
    const float v = one_minus_exp_neg(y);
    *g = 1.f - frcp(v);
    return -flog(v);
  }
};

// SV: state (dim_one, z * mask + shift) (SV_dense.py:245-246), no obs term
template <>
struct Dev<VISSM_MODEL_SV> {
  static constexpr int P = 4, ZD = 1, SU = kSU;
  static constexpr bool kObs = false, kExtra = false;
  static constexpr float kSd = 1.f;
  float th[4], dt, sq, e2, s2, is2, c_lp;
  int M;
  const float *mk, *sh, *d1, *ob, *bn;
  __device__ void init(const Args& a, const float* thp, int w) {
    th[0] = thp[0]; th[1] = thp[1]; th[2] = thp[2]; th[3] = thp[3];
    dt = a.dt;
    sq = ::sqrtf(dt);
    e2 = ::expf(th[2]);
    s2 = sq * ::expf(th[3]);
    is2 = 1.f / s2;
    // -log sqrt(dt) (of s1) - log s2 - log 2 pi
    c_lp = -::logf(sq) - ::logf(s2) - em::kLog2Pi_;
    M = a.M;
    mk = a.d.mask + static_cast<size_t>(w) * (M + 1);
    sh = a.d.shift + static_cast<size_t>(w) * (M + 1);
    d1 = a.d.dim_one + static_cast<size_t>(w) * (M + 1);
    ob = bn = nullptr;
  }
  template <int N, bool PLAIN = false>
  __device__ void states(const float* zb, int t0, St (&o)[N]) const {
    float zz[N], m[N], s[N], x1[N];
    ldn<N>(zb + t0, zz);
    if constexpr (!PLAIN) {
      ldn<N>(mk + t0, m);
      ldn<N>(sh + t0, s);
    }
    ldn<N>(d1 + t0, x1);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      o[i].x[0] = x1[i];
      o[i].j[0] = 0.f;
      o[i].x[1] = PLAIN ? zz[i] : zz[i] * m[i] + s[i];
      o[i].j[1] = PLAIN ? 1.f : m[i];
    }
  }
  __device__ St state(const float* zb, int t) const {
    St o;
    o.x[0] = d1[t];
    o.j[0] = 0.f;
    o.x[1] = zb[t] * mk[t] + sh[t];
    o.j[1] = mk[t];
    return o;
  }
  // em::sv_trans with the per-sample terms hoisted and one reciprocal:
  //   s1 = sqrt(dt) x1 e^{x2/2},  log|s1| = log sqrt(dt) + log|x1| + x2 / 2
  __device__ em::TG trans(const St& p, const St& q) const {
    em::TG r;
    const float x1 = p.x[0], x2 = p.x[1];
    const float ex = fexp(0.5f * x2);
    const float s1 = sq * x1 * ex, is1 = frcp(s1);
    const float m1 = dt * th[0] * x1, m2 = dt * (th[1] - e2 * x2);
    const float q1 = q.x[0] - x1 - m1, q2 = q.x[1] - x2 - m2;
    const float z1 = q1 * is1, z2 = q2 * is2;
    r.lp = -0.5f * (z1 * z1 + z2 * z2) - (flog(::fabsf(x1)) + 0.5f * x2) + c_lp;
    const float gq1 = -z1 * is1, gq2 = -z2 * is2;
    const float gs1 = (z1 * z1 - 1.f) * is1, gs2 = (z2 * z2 - 1.f) * is2;
    r.gt[0] = gq1;
    r.gt[1] = gq2;
    float gx1 = -gq1, gx2 = -gq2;
    const float gm1 = -gq1, gm2 = -gq2;
    r.gth[0] = gm1 * dt * x1;
    gx1 += gm1 * dt * th[0];
    r.gth[1] = gm2 * dt;
    r.gth[2] = -gm2 * dt * x2 * e2;
    gx2 += -gm2 * dt * e2;
    gx1 += gs1 * sq * ex;
    gx2 += gs1 * 0.5f * s1;
    r.gth[3] = gs2 * s2;
    r.gth[4] = 0.f;
    r.gh[0] = gx1;
    r.gh[1] = gx2;
    return r;
  }
  __device__ static float ildj(float, float* g) { *g = 0.f; return 0.f; }
};

// FHN: x = z (interleaved), obs N(., 0.1) (fitz_nag_NVP.py:232-234)
template <>
struct Dev<VISSM_MODEL_FHN> {
  static constexpr int P = 5, ZD = 2, SU = kSU;
  static constexpr bool kObs = true, kExtra = false;
  static constexpr float kSd = 0.1f;
  float th[5], dt, E0, is1, is2, c_lp;
  int M;
  const float *ob, *bn;
  __device__ void init(const Args& a, const float* thp, int w) {
#pragma unroll
    for (int i = 0; i < 5; ++i) th[i] = thp[i];
    dt = a.dt;
    E0 = ::expf(th[0]);
    const float sq = ::sqrtf(dt), s1 = sq * ::sqrtf(::expf(th[3])), s2 = sq * ::sqrtf(::expf(th[4]));
    is1 = 1.f / s1;
    is2 = 1.f / s2;
    c_lp = -::logf(s1) - ::logf(s2) - em::kLog2Pi_;
    M = a.M;
    ob = a.d.obs + static_cast<size_t>(w) * 2 * M;
    bn = a.d.obs_bin + static_cast<size_t>(w) * 2 * M;
  }
  template <int N, bool PLAIN = false>
  __device__ void states(const float* zb, int t0, St (&o)[N]) const {
    float zz[2 * N];
    ldn<2 * N>(zb + 2 * t0, zz);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      o[i].x[0] = zz[2 * i];
      o[i].x[1] = zz[2 * i + 1];
      o[i].j[0] = o[i].j[1] = 1.f;
    }
  }
  __device__ St state(const float* zb, int t) const {
    St o;
    o.x[0] = zb[2 * t];
    o.x[1] = zb[2 * t + 1];
    o.j[0] = o.j[1] = 1.f;
    return o;
  }
  // em::fhn_trans with the per-sample scales hoisted (s_i = sqrt(dt e^{th_{3,4}}), their reciprocals
  // and logs): no division per transition
  __device__ em::TG trans(const St& p, const St& q) const {
    em::TG r;
    const float x1 = p.x[0], x2 = p.x[1];
    const float f = x1 - x1 * x1 * x1 - x2 + th[1];
    const float m1 = dt * E0 * f, m2 = dt * (th[2] * x1 - x2 + 1.4f);
    const float q1 = q.x[0] - x1 - m1, q2 = q.x[1] - x2 - m2;
    const float z1 = q1 * is1, z2 = q2 * is2;
    r.lp = -0.5f * (z1 * z1 + z2 * z2) + c_lp;
    const float gq1 = -z1 * is1, gq2 = -z2 * is2;
    r.gt[0] = gq1;
    r.gt[1] = gq2;
    float gx1 = -gq1, gx2 = -gq2;
    const float gm1 = -gq1, gm2 = -gq2;
    r.gth[0] = gm1 * dt * E0 * f;
    const float gf = gm1 * dt * E0;
    gx1 += gf * (1.f - 3.f * x1 * x1);
    gx2 += -gf;
    r.gth[1] = gf;
    r.gth[2] = gm2 * dt * x1;
    gx1 += gm2 * dt * th[2];
    gx2 += -gm2 * dt;
    r.gth[3] = 0.5f * (z1 * z1 - 1.f);   // gs1 s1 / 2 with gs1 = (z1^2 - 1) / s1
    r.gth[4] = 0.5f * (z2 * z2 - 1.f);
    r.gh[0] = gx1;
    r.gh[1] = gx2;
    return r;
  }
  __device__ static float ildj(float, float* g) { *g = 0.f; return 0.f; }
};

template <int MODEL>
__global__ __launch_bounds__(256) void stream_fwd_kernel(Args a, const float* __restrict__ z,
                                                         const float* __restrict__ theta, float* __restrict__ sde,
                                                         float* __restrict__ obs, float* __restrict__ extra) {
  using Dv = Dev<MODEL>;
  constexpr int ZD = Dv::ZD, P = Dv::P;
  const int lane = threadIdx.x & 63;
  const int b = __builtin_amdgcn_readfirstlane(blockIdx.x * kSW + (threadIdx.x >> 6));
  if (b >= a.B) return;  // wave-uniform
  const int M = a.M;
  const int w = a.d.win ? a.d.win[b] : 0;
  Dv m;
  m.init(a, theta + static_cast<size_t>(b) * P, w);
  const float* zb = z + static_cast<size_t>(b) * ZD * (M + 1);
  const float isd = 1.f / Dv::kSd;
  float s_lp = 0.f, s_q = 0.f, s_b = 0.f, s_e = 0.f;
  // transition t: x_t -> x_{t+1}; the obs of row t and the ILDJ observe x_{t+1}
  auto tr = [&](const St& p, const St& q, float y0, float y1, float b0, float b1) {
    s_lp += m.trans(p, q).lp;
    if constexpr (Dv::kObs) {
      const float z0 = (q.x[0] - y0) * isd, z1 = (q.x[1] - y1) * isd;
      s_q += b0 * z0 * z0 + b1 * z1 * z1;
      s_b += b0 + b1;
    }
    if constexpr (Dv::kExtra) s_e += q.il[0] + q.il[1];
  };
  const int nfull = M / kV;  // chunks whose kV transitions all exist
  int c = lane;
  constexpr int SU = Dv::SU;
  for (; c + 64 * (SU - 1) < nfull; c += 64 * SU) {
    St st[SU][kV + 1];
    float y[SU][2][kV], bb[SU][2][kV];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int t0 = kV * (c + 64 * u);
      m.template states<kV + 1>(zb, t0, st[u]);
      if constexpr (Dv::kObs) {
        ldn<kV>(m.ob + t0, y[u][0]);
        ldn<kV>(m.ob + M + t0, y[u][1]);
        ldn<kV>(m.bn + t0, bb[u][0]);
        ldn<kV>(m.bn + M + t0, bb[u][1]);
      }
    }
#pragma unroll
    for (int u = 0; u < SU; ++u)
#pragma unroll
      for (int j = 0; j < kV; ++j)
        tr(st[u][j], st[u][j + 1], Dv::kObs ? y[u][0][j] : 0.f, Dv::kObs ? y[u][1][j] : 0.f,
           Dv::kObs ? bb[u][0][j] : 0.f, Dv::kObs ? bb[u][1][j] : 0.f);
  }
  for (; c < nfull; c += 64) {
    const int t0 = kV * c;
    St st[kV + 1];
    m.template states<kV + 1>(zb, t0, st);
#pragma unroll
    for (int j = 0; j < kV; ++j) {
      const int t = t0 + j;
      tr(st[j], st[j + 1], Dv::kObs ? m.ob[t] : 0.f, Dv::kObs ? m.ob[M + t] : 0.f, Dv::kObs ? m.bn[t] : 0.f,
         Dv::kObs ? m.bn[M + t] : 0.f);
    }
  }
  for (int t = kV * nfull + lane; t < M; t += 64)
    tr(m.state(zb, t), m.state(zb, t + 1), Dv::kObs ? m.ob[t] : 0.f, Dv::kObs ? m.ob[M + t] : 0.f,
       Dv::kObs ? m.bn[t] : 0.f, Dv::kObs ? m.bn[M + t] : 0.f);
  const double r_lp = wave_sum(static_cast<double>(s_lp));
  const double r_q = wave_sum(static_cast<double>(s_q));
  const double r_b = wave_sum(static_cast<double>(s_b));
  const double r_e = wave_sum(static_cast<double>(s_e));
  if (lane == 0) {
    sde[b] = static_cast<float>(r_lp);
    if (obs) obs[b] = Dv::kObs ? static_cast<float>(-0.5 * r_q + r_b * (-std::log(static_cast<double>(Dv::kSd)) -
                                                                     0.5 * kLog2Pi))
                               : 0.f;
    if (extra) extra[b] = static_cast<float>(r_e);
  }
}

// d/dz of gs sde + go obs + ge extra at every stored z entry, d/dtheta of gs sde.  Element e takes the
// head gradient of transition e (e < M) and, for e >= 1, the tail gradient of transition e - 1 and the
// obs / ILDJ terms observing x_e.
// VALS (vissm_elbo_fwd_grad): the same pass also sums the forward values -- each element's head transition, the obs
// row and the ILDJ term observing it are visited exactly once -- so the log-densities, dz and d theta come from one
// read of z when the upstream gradients are known before the forward (the training step: -T/M and -1 per sample)
struct Vals {
  float *sde, *obs, *extra;
};

template <int MODEL, bool VALS = false>
__global__ __launch_bounds__(256) void stream_bwd_kernel(Args a, const float* __restrict__ z,
                                                         const float* __restrict__ theta,
                                                         const float* __restrict__ g_sde,
                                                         const float* __restrict__ g_obs,
                                                         const float* __restrict__ g_ex, float* __restrict__ dz,
                                                         float* __restrict__ dtheta, Vals vo = Vals{}) {
  using Dv = Dev<MODEL>;
  constexpr int ZD = Dv::ZD, P = Dv::P;
  const int lane = threadIdx.x & 63;
  const int b = __builtin_amdgcn_readfirstlane(blockIdx.x * kSW + (threadIdx.x >> 6));
  if (b >= a.B) return;  // wave-uniform
  const int M = a.M;
  const int w = a.d.win ? a.d.win[b] : 0;
  Dv m;
  m.init(a, theta + static_cast<size_t>(b) * P, w);
  const float* zb = z + static_cast<size_t>(b) * ZD * (M + 1);
  float* dzb = dz + static_cast<size_t>(b) * ZD * (M + 1);
  const float gs = g_sde ? g_sde[b] : 0.f;
  const float go = (Dv::kObs && g_obs) ? g_obs[b] : 0.f;
  const float ge = (Dv::kExtra && g_ex) ? g_ex[b] : 0.f;
  const float cgo = -go / (Dv::kSd * Dv::kSd);
  float acc[P];
#pragma unroll
  for (int i = 0; i < P; ++i) acc[i] = 0.f;
  float s_lp = 0.f, s_q = 0.f, s_b = 0.f, s_e = 0.f;  // VALS: the forward's per-sample sums
  constexpr float isd = 1.f / Dv::kSd;
  // the gradient w.r.t. x_e of the terms observing x_e (obs row e - 1, ILDJ), e >= 1
  auto obs_g = [&](const St& s, float y0, float y1, float b0, float b1, float* g) {
    if constexpr (Dv::kObs) {
      const float d0 = s.x[0] - y0, d1 = s.x[1] - y1;
      g[0] += cgo * b0 * d0;
      g[1] += cgo * b1 * d1;
      if constexpr (VALS) {
        s_q += b0 * (d0 * isd) * (d0 * isd) + b1 * (d1 * isd) * (d1 * isd);
        s_b += b0 + b1;
      }
    }
  };
  // the ILDJ term observing x_e (e >= 1), already w.r.t. the stored z
  auto ildj_dz = [&](const St& s, float& o0, float& o1) {
    if constexpr (Dv::kExtra) {
      o0 += ge * s.dil[0];
      o1 += ge * s.dil[1];
      if constexpr (VALS) s_e += s.il[0] + s.il[1];
    }
  };
  auto head = [&](const em::TG& r, float* g) {
    g[0] += gs * r.gh[0];
    g[1] += gs * r.gh[1];
    if constexpr (VALS) s_lp += r.lp;
#pragma unroll
    for (int i = 0; i < P; ++i) acc[i] += r.gth[i];
  };
  auto tail = [&](const em::TG& r, float* g) {
    g[0] += gs * r.gt[0];
    g[1] += gs * r.gt[1];
  };
  // interior chunks c in [1, M / kV): t0 >= 1 and t0 + kV <= M, states t0-1 .. t0+kV exist
  const int ihi = M / kV;
  int c = 1 + lane;
  auto chunk = [&](int t0, const St (&st)[kV + 2], const float (&y)[2][kV], const float (&bb)[2][kV]) {
    // transitions t0-1 .. t0+kV-1 in order, each evaluated once: element t0 + j = st[j + 1] takes the
    // tail of the previous one and the head of the next
    em::TG prev = m.trans(st[0], st[1]);
    float o[ZD * kV];
#pragma unroll
    for (int j = 0; j < kV; ++j) {
      const em::TG cur = m.trans(st[j + 1], st[j + 2]);
      float g[2] = {0.f, 0.f};
      head(cur, g);
      tail(prev, g);
      prev = cur;
      obs_g(st[j + 1], y[0][j], y[1][j], bb[0][j], bb[1][j], g);
      if constexpr (ZD == 2) {
        o[2 * j] = g[0] * st[j + 1].j[0];
        o[2 * j + 1] = g[1] * st[j + 1].j[1];
        ildj_dz(st[j + 1], o[2 * j], o[2 * j + 1]);
      } else {
        o[j] = g[1] * st[j + 1].j[1];
      }
    }
#pragma unroll
    for (int i = 0; i < ZD * kV; i += 4)
      if (dz) *reinterpret_cast<f4u*>(dzb + ZD * t0 + i) = f4u{o[i], o[i + 1], o[i + 2], o[i + 3]};
  };
  constexpr int SU = Dv::SU;
  for (; c + 64 * (SU - 1) < ihi; c += 64 * SU) {
    St st[SU][kV + 2];
    float y[SU][2][kV], bb[SU][2][kV];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int t0 = kV * (c + 64 * u);
      m.template states<kV + 2>(zb, t0 - 1, st[u]);
      if constexpr (Dv::kObs) {  // rows t0-1 .. t0+kV-2 observe x_{t0} .. x_{t0+kV-1}
        ldn<kV>(m.ob + t0 - 1, y[u][0]);
        ldn<kV>(m.ob + M + t0 - 1, y[u][1]);
        ldn<kV>(m.bn + t0 - 1, bb[u][0]);
        ldn<kV>(m.bn + M + t0 - 1, bb[u][1]);
      } else {
#pragma unroll
        for (int j = 0; j < kV; ++j) y[u][0][j] = y[u][1][j] = bb[u][0][j] = bb[u][1][j] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) chunk(kV * (c + 64 * u), st[u], y[u], bb[u]);
  }
  for (; c < ihi; c += 64) {
    const int t0 = kV * c;
    St st[kV + 2];
    float y[2][kV], bb[2][kV];
    m.template states<kV + 2>(zb, t0 - 1, st);
    if constexpr (Dv::kObs) {
      ldn<kV>(m.ob + t0 - 1, y[0]);
      ldn<kV>(m.ob + M + t0 - 1, y[1]);
      ldn<kV>(m.bn + t0 - 1, bb[0]);
      ldn<kV>(m.bn + M + t0 - 1, bb[1]);
    } else {
#pragma unroll
      for (int j = 0; j < kV; ++j) y[0][j] = y[1][j] = bb[0][j] = bb[1][j] = 0.f;
    }
    chunk(t0, st, y, bb);
  }
  // the rest, one element per lane: t in [0, kV) and [kV ihi, M]
  const int lo_end = ihi >= 1 ? kV : M + 1;  // with no interior chunk the first range covers everything
  const int nrest = lo_end + (ihi >= 1 ? (M + 1 - kV * ihi) : 0);
  for (int r = lane; r < nrest; r += 64) {
    const int t = r < lo_end ? r : kV * ihi + (r - lo_end);
    if (t > M || (r >= lo_end && t < lo_end)) continue;
    const St sc = m.state(zb, t);
    float g[2] = {0.f, 0.f};
    if (t < M) head(m.trans(sc, m.state(zb, t + 1)), g);
    if (t >= 1) {
      tail(m.trans(m.state(zb, t - 1), sc), g);
      if constexpr (Dv::kObs)
        obs_g(sc, m.ob[t - 1], m.ob[M + t - 1], m.bn[t - 1], m.bn[M + t - 1], g);
      else
        obs_g(sc, 0.f, 0.f, 0.f, 0.f, g);
    }
    if (!VALS && !dz) continue;
    if constexpr (ZD == 2) {
      float o0 = g[0] * sc.j[0], o1 = g[1] * sc.j[1];
      if (t >= 1) ildj_dz(sc, o0, o1);
      if (dz) {
        dzb[2 * t] = o0;
        dzb[2 * t + 1] = o1;
      }
    } else {
      if (dz) dzb[t] = g[1] * sc.j[1];
    }
  }
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const double s = wave_sum(static_cast<double>(acc[i]));
    if (lane == 0) dtheta[static_cast<size_t>(b) * P + i] = static_cast<float>(gs * s);
  }
  if constexpr (VALS) {
    const double r_lp = wave_sum(static_cast<double>(s_lp));
    const double r_q = wave_sum(static_cast<double>(s_q));
    const double r_b = wave_sum(static_cast<double>(s_b));
    const double r_e = wave_sum(static_cast<double>(s_e));
    if (lane == 0) {
      vo.sde[b] = static_cast<float>(r_lp);
      if (vo.obs)
        vo.obs[b] = Dv::kObs ? static_cast<float>(-0.5 * r_q + r_b * (-std::log(static_cast<double>(Dv::kSd)) -
                                                                      0.5 * kLog2Pi))
                             : 0.f;
      if (vo.extra) vo.extra[b] = static_cast<float>(r_e);
    }
  }
}

// ---------------------------------------------------------------------------
// One pass with neighbour exchange (vissm_elbo_fwd_grad, LV / SV / FHN).  stream_bwd_kernel evaluates kV + 2 states and
// kV + 1 transitions per chunk of kV elements (each chunk recomputes its neighbours' edge states and the transition
// across its left edge); here every state and transition is evaluated exactly once: lane l of iteration i owns chunk
// c = 1 + 64 i + l (elements t0 = kV c .. t0 + kV - 1), evaluates its kV states and the kV transitions ENTERING its
// elements (T_{t0-1} .. T_{t0+kV-2}, T_e: x_e -> x_{e+1}), takes x_{t0-1} from lane l - 1 by a DPP wave shift (lane 0:
// the previous iteration's lane 63, or element kV - 1 before the loop) and the head gradient of its last element --
// T_{t0+kV-1}, lane l + 1's first transition -- by the opposite shift.  The lane whose right neighbour is not in this
// iteration (lane 63, or the last chunk's lane) keeps that element pending: the next iteration's lane 0 (or the
// element-wise tail after the loop) supplies the missing head through v_readlane, then that chunk is stored.  Elements
// [0, kV) and [kV nfull, M] run element-wise as in stream_bwd_kernel, with transition counts chosen so that every
// transition's log-density and theta gradient enters the sums once.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_shr1(float v) {  // lane l <- lane l - 1 (lane 0 keeps v)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                                               0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_shl1(float v) {  // lane l <- lane l + 1 (lane 63 keeps v)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                                               0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane_val(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// OL (VissmElboData.obs_list): the observation term leaves the chunk loop and the element-wise tail (no obs / obs_bin
// row loads there) and is evaluated after them at the window's listed elements only, its dz added to the stored one.
// NWV > 1: NWV waves of the block share one trajectory, each taking a contiguous range of the chunk loop's iterations
// (finer work units than one wave per trajectory: the launch's last round of waves no longer runs on a partly empty
// chip).  A range starts from x of the element before it (one state evaluated) and ends by evaluating the transition
// out of its deferred chunk's last element itself (its head; the transition is counted by the wave that owns it); the
// last wave runs the element-wise tail; the per-sample sums are combined in wave order through LDS after a block
// barrier (fixed order: deterministic).
template <int MODEL, bool OL = false, int NWV = 1>
__global__ __launch_bounds__(256) void stream_onepass_kernel(Args a, const float* __restrict__ z,
                                                             const float* __restrict__ theta,
                                                             const float* __restrict__ g_sde,
                                                             const float* __restrict__ g_obs,
                                                             const float* __restrict__ g_ex, float* __restrict__ dz,
                                                             float* __restrict__ dtheta, Vals vo) {
  using Dv = Dev<MODEL>;
  constexpr int ZD = Dv::ZD, P = Dv::P;
  static_assert(!OL || NWV == 1, "the observation list's post-pass reads the whole row the wave wrote");
  static_assert(kSW % NWV == 0, "whole trajectories per block");
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) % NWV);  // this wave's range of the trajectory
  const int b0 = __builtin_amdgcn_readfirstlane(blockIdx.x * (kSW / NWV) + (threadIdx.x >> 6) / NWV);
  // (NWV > 1: every wave reaches the block barrier below, so one past the batch evaluates the last trajectory and
  //  stores nothing)
  const bool live = b0 < a.B;
  if (NWV == 1 && !live) return;  // wave-uniform
  const int b = live ? b0 : a.B - 1;
  const int M = a.M;
  const int w = a.d.win ? a.d.win[b] : 0;
  Dv m;
  m.init(a, theta + static_cast<size_t>(b) * P, w);
  const float* zb = z + static_cast<size_t>(b) * ZD * (M + 1);
  float* dzb = dz + static_cast<size_t>(b) * ZD * (M + 1);
  const float gs = g_sde ? g_sde[b] : 0.f;
  const float go = (Dv::kObs && g_obs) ? g_obs[b] : 0.f;
  const float ge = (Dv::kExtra && g_ex) ? g_ex[b] : 0.f;
  const float cgo = -go / (Dv::kSd * Dv::kSd);
  constexpr float isd = 1.f / Dv::kSd;
  float acc[P];
#pragma unroll
  for (int i = 0; i < P; ++i) acc[i] = 0.f;
  float s_lp = 0.f, s_q = 0.f, s_b = 0.f, s_e = 0.f;
  // a transition's log-density and theta gradient into the sums (on: a 0 / 1 weight, lanes that own it)
  auto count = [&](const em::TG& r, float on) {
    s_lp += on * r.lp;
#pragma unroll
    for (int i = 0; i < P; ++i) acc[i] += on * r.gth[i];
  };
  // the obs row e - 1 observing x_e (e >= 1): gradient into g, value into the sums
  auto obs_term = [&](const St& s, float y0, float y1, float b0, float b1, float* g, float on) {
    if constexpr (Dv::kObs) {
      const float d0 = s.x[0] - y0, d1 = s.x[1] - y1;
      g[0] += cgo * b0 * d0;
      g[1] += cgo * b1 * d1;
      s_q += on * (b0 * (d0 * isd) * (d0 * isd) + b1 * (d1 * isd) * (d1 * isd));
      s_b += on * (b0 + b1);
    }
  };
  auto obs_g = [&](const St& s, float y0, float y1, float b0, float b1, float* g, float on) {
    if constexpr (!OL) obs_term(s, y0, y1, b0, b1, g, on);
  };
  // dz of element s from its state gradient g (+ the ILDJ term observing it, e >= 1)
  auto dz_of = [&](const St& s, const float* g, bool ildj, float on, float* o) {
    if constexpr (ZD == 2) {
      o[0] = g[0] * s.j[0];
      o[1] = g[1] * s.j[1];
      if constexpr (Dv::kExtra) {
        if (ildj) {
          o[0] += ge * s.dil[0];
          o[1] += ge * s.dil[1];
          s_e += on * (s.il[0] + s.il[1]);
        }
      }
    } else {
      o[0] = g[1] * s.j[1];
    }
  };
  const int nfull = (M + 1) / kV;  // chunks whose kV elements all exist (elements 0 .. M)
  // this wave's iterations of the chunk loop: [it_lo, it_hi) of nit (64 chunks each); the last wave runs the tail
  const int nit = nfull >= 2 ? (nfull - 1 + 63) / 64 : 0;
  const int it_lo = (nit * wv) / NWV, it_hi = (nit * (wv + 1)) / NWV;
  const bool last_wave = wv == NWV - 1;
  // ---- the chunk loop: chunks 1 .. nfull - 1 ----
  float pend[ZD * kV];             // the deferred chunk (meaningful in lane pl only)
  float pg[2] = {0.f, 0.f}, pj[2] = {0.f, 0.f};  // its last element's state gradient (without the head) and d x / d z
  int pl = -1, pt0 = 0;            // the deferring lane and its chunk's first element (wave-uniform)
#pragma unroll
  for (int i = 0; i < ZD * kV; ++i) pend[i] = 0.f;
  float xc0 = 0.f, xc1 = 0.f;      // x of element t0 - 1 for lane 0
  if (it_lo < it_hi) {
    const St s3 = m.state(zb, kV * (1 + 64 * it_lo) - 1);
    xc0 = s3.x[0];
    xc1 = s3.x[1];
  }
  // one iteration, specialised for a plain window span (no mask / shift) and for a full iteration (every lane owns
  // a chunk: no masking of the sums)
  auto iteration = [&](const int c0, auto plain_tag, auto full_tag) {
    constexpr bool PLAIN = decltype(plain_tag)::value, FULL = decltype(full_tag)::value;
    const int c = c0 + lane;
    const bool act = FULL || c < nfull;
    const float on = act ? 1.f : 0.f;
    const int t0 = kV * (act ? c : nfull - 1);   // idle lanes of the last iteration evaluate the last chunk, unused
    St st[kV];
    m.template states<kV, PLAIN>(zb, t0, st);
    float y[2][kV], bb[2][kV];
    if constexpr (Dv::kObs && !OL) {  // rows t0 - 1 .. t0 + kV - 2 observe x_{t0} .. x_{t0+kV-1}
      ldn<kV>(m.ob + t0 - 1, y[0]);
      ldn<kV>(m.ob + M + t0 - 1, y[1]);
      ldn<kV>(m.bn + t0 - 1, bb[0]);
      ldn<kV>(m.bn + M + t0 - 1, bb[1]);
    } else {
#pragma unroll
      for (int j = 0; j < kV; ++j) y[0][j] = y[1][j] = bb[0][j] = bb[1][j] = 0.f;
    }
    // x_{t0-1}: lane l - 1's last state; lane 0: the carry
    St left;
    const float sh0 = wave_shr1(st[kV - 1].x[0]), sh1 = wave_shr1(st[kV - 1].x[1]);  // every lane issues the shift
    left.x[0] = lane == 0 ? xc0 : sh0;
    left.x[1] = lane == 0 ? xc1 : sh1;
    // the transitions entering the chunk's elements
    em::TG tr[kV];
    tr[0] = m.trans(left, st[0]);
#pragma unroll
    for (int j = 1; j < kV; ++j) tr[j] = m.trans(st[j - 1], st[j]);
#pragma unroll
    for (int j = 0; j < kV; ++j) count(tr[j], FULL ? 1.f : on);
    // the head of the chunk's last element: lane l + 1's first transition
    const float hn0 = wave_shl1(tr[0].gh[0]), hn1 = wave_shl1(tr[0].gh[1]);
    // the previous iteration's deferred chunk: its head is this iteration's lane-0 first transition
    if (pl >= 0) {
      const float h0 = lane_val(tr[0].gh[0], 0), h1 = lane_val(tr[0].gh[1], 0);
      if (lane == pl && (NWV == 1 || live)) {
        const float g[2] = {pg[0] + gs * h0, pg[1] + gs * h1};
        if constexpr (ZD == 2) {
          pend[ZD * (kV - 1)] += g[0] * pj[0];
          pend[ZD * (kV - 1) + 1] += g[1] * pj[1];
        } else {
          pend[kV - 1] += g[1] * pj[1];
        }
#pragma unroll
        for (int i = 0; i < ZD * kV; i += 4)
          *reinterpret_cast<f4u*>(dzb + ZD * pt0 + i) = f4u{pend[i], pend[i + 1], pend[i + 2], pend[i + 3]};
      }
    }
    // elements t0 .. t0 + kV - 1
    const int last_c = min(nfull - 1, c0 + 63);
    const int dl = last_c - c0;                   // the lane that defers its last element (wave-uniform)
    float o[ZD * kV];
    float glast[2] = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < kV; ++j) {
      float g[2] = {gs * tr[j].gt[0], gs * tr[j].gt[1]};        // tail: T_{e-1}
      if (j + 1 < kV) {                                            // head: T_e
        g[0] += gs * tr[j + 1].gh[0];
        g[1] += gs * tr[j + 1].gh[1];
      }
      obs_g(st[j], y[0][j], y[1][j], bb[0][j], bb[1][j], g, FULL ? 1.f : on);
      if (j + 1 == kV) {
        glast[0] = g[0];
        glast[1] = g[1];
        if (lane != dl) {
          g[0] += gs * hn0;
          g[1] += gs * hn1;
        }
      }
      dz_of(st[j], g, true, FULL ? 1.f : on, o + ZD * j);
    }
    if (act && lane != dl && (NWV == 1 || live)) {
#pragma unroll
      for (int i = 0; i < ZD * kV; i += 4)
        *reinterpret_cast<f4u*>(dzb + ZD * t0 + i) = f4u{o[i], o[i + 1], o[i + 2], o[i + 3]};
    }
    // defer lane dl's chunk: its dz without the last element's head, that element's state gradient and d x / d z
    if (lane == dl) {
#pragma unroll
      for (int i = 0; i < ZD * kV; ++i) pend[i] = o[i];
      if constexpr (ZD == 2) {
        pend[ZD * (kV - 1)] -= glast[0] * st[kV - 1].j[0];
        pend[ZD * (kV - 1) + 1] -= glast[1] * st[kV - 1].j[1];
      } else {
        pend[kV - 1] -= glast[1] * st[kV - 1].j[1];
      }
      pg[0] = glast[0];
      pg[1] = glast[1];
      pj[0] = st[kV - 1].j[0];
      pj[1] = st[kV - 1].j[1];
    }
    pl = dl;
    pt0 = kV * last_c;
    xc0 = lane_val(st[kV - 1].x[0], 63);
    xc1 = lane_val(st[kV - 1].x[1], 63);
    };
  const int pf = a.d.plain_from ? a.d.plain_from[w] : (1 << 30);   // first element of the plain span
  using T_ = std::true_type;
  using F_ = std::false_type;
  for (int c0 = 1 + 64 * it_lo; c0 < nfull && c0 < 1 + 64 * it_hi; c0 += 64) {
    const bool plain = (MODEL != VISSM_MODEL_FHN) && kV * c0 >= pf;   // the whole iteration lies in the plain span
    const bool full = c0 + 63 < nfull;
    if (plain) {
      if (full) iteration(c0, T_{}, T_{});
      else iteration(c0, T_{}, F_{});
    } else {
      if (full) iteration(c0, F_{}, T_{});
      else iteration(c0, F_{}, F_{});
    }
  }
  // a range other than the last: its deferred chunk's head is the transition out of its last element, which the next
  // range counts (evaluated here by every lane at the same wave-uniform element, applied by the deferring lane)
  if (NWV > 1 && !last_wave && pl >= 0) {
    const em::TG h = m.trans(m.state(zb, pt0 + kV - 1), m.state(zb, pt0 + kV));
    if (lane == pl && live) {
      if constexpr (ZD == 2) {
        pend[ZD * (kV - 1)] += (pg[0] + gs * h.gh[0]) * pj[0];
        pend[ZD * (kV - 1) + 1] += (pg[1] + gs * h.gh[1]) * pj[1];
      } else {
        pend[kV - 1] += (pg[1] + gs * h.gh[1]) * pj[1];
      }
#pragma unroll
      for (int i = 0; i < ZD * kV; i += 4)
        *reinterpret_cast<f4u*>(dzb + ZD * pt0 + i) = f4u{pend[i], pend[i + 1], pend[i + 2], pend[i + 3]};
    }
    pl = -1;
  }
  // ---- element-wise tail: elements [0, kV) and [kV nfull, M] (the last wave) ----
  const int lo_end = nfull >= 1 ? kV : M + 1;
  const int nrest = last_wave ? lo_end + (nfull >= 1 ? (M + 1 - kV * nfull) : 0) : 0;
  float hpend0 = 0.f, hpend1 = 0.f;   // the head of element kV nfull - 1 (the deferred chunk's last element)
  for (int r0 = 0; r0 < nrest; r0 += 64) {
    const int r = r0 + lane;
    const bool on_r = r < nrest;
    const int t = !on_r ? 0 : (r < lo_end ? r : kV * nfull + (r - lo_end));
    const St sc = m.state(zb, t);
    float g[2] = {0.f, 0.f};
    if (on_r && t < M) {
      const em::TG h = m.trans(sc, m.state(zb, t + 1));
      g[0] += gs * h.gh[0];
      g[1] += gs * h.gh[1];
      // counted here unless the chunk loop counted it (T_{kV-1}: chunk 1's first transition)
      if (!(t == kV - 1 && nfull >= 2)) count(h, 1.f);
    }
    if (on_r && t >= 1) {
      const em::TG tl = m.trans(m.state(zb, t - 1), sc);
      g[0] += gs * tl.gt[0];
      g[1] += gs * tl.gt[1];
      if (t == kV * nfull && nfull >= 2) {   // T_{kV nfull - 1}: the deferred element's head, counted once here
        count(tl, 1.f);
        hpend0 = tl.gh[0];
        hpend1 = tl.gh[1];
      }
      if constexpr (Dv::kObs && !OL)
        obs_g(sc, m.ob[t - 1], m.ob[M + t - 1], m.bn[t - 1], m.bn[M + t - 1], g, 1.f);
    }
    float o[ZD];
    dz_of(sc, g, on_r && t >= 1, on_r ? 1.f : 0.f, o);
    if (on_r && (NWV == 1 || live)) {
      if constexpr (ZD == 2) {
        dzb[2 * t] = o[0];
        dzb[2 * t + 1] = o[1];
      } else {
        dzb[t] = o[0];
      }
    }
  }
  // the last deferred chunk: its head from the tail's element kV nfull (lane lo_end), or none (kV nfull - 1 == M)
  if (pl >= 0) {
    float h0 = 0.f, h1 = 0.f;
    if (kV * nfull <= M) {
      h0 = lane_val(hpend0, lo_end % 64);
      h1 = lane_val(hpend1, lo_end % 64);
    }
    if (lane == pl && (NWV == 1 || live)) {
      if constexpr (ZD == 2) {
        pend[ZD * (kV - 1)] += (pg[0] + gs * h0) * pj[0];
        pend[ZD * (kV - 1) + 1] += (pg[1] + gs * h1) * pj[1];
      } else {
        pend[kV - 1] += (pg[1] + gs * h1) * pj[1];
      }
#pragma unroll
      for (int i = 0; i < ZD * kV; i += 4)
        *reinterpret_cast<f4u*>(dzb + ZD * pt0 + i) = f4u{pend[i], pend[i + 1], pend[i + 2], pend[i + 3]};
    }
  }
  if constexpr (Dv::kObs && OL) {
    // the listed observed elements: the obs term's value and its dz, added to the element's stored dz (g enters dz
    // linearly through d x / d z).  This wave wrote every element of its row above: its stores complete first.
    __threadfence_block();
    const int os = a.d.obs_stride;
    const int* ol = a.d.obs_list + static_cast<size_t>(w) * os;
    for (int r0 = 0; r0 < os; r0 += 64) {
      const int e = r0 + lane < os ? ol[r0 + lane] : -1;
      if (e >= 1 && e <= M) {
        const St sc = m.state(zb, e);
        float g[2] = {0.f, 0.f};
        obs_term(sc, m.ob[e - 1], m.ob[M + e - 1], m.bn[e - 1], m.bn[M + e - 1], g, 1.f);
        if constexpr (ZD == 2) {
          float* p2 = dzb + 2 * e;
          const f2u v = *reinterpret_cast<const f2u*>(p2);
          *reinterpret_cast<f2u*>(p2) = f2u{v[0] + g[0] * sc.j[0], v[1] + g[1] * sc.j[1]};
        } else {
          dzb[e] += g[1] * sc.j[1];
        }
      }
    }
  }
  double r[P + 4];
#pragma unroll
  for (int i = 0; i < P; ++i) r[i] = wave_sum(static_cast<double>(acc[i]));
  r[P] = wave_sum(static_cast<double>(s_lp));
  r[P + 1] = wave_sum(static_cast<double>(s_q));
  r[P + 2] = wave_sum(static_cast<double>(s_b));
  r[P + 3] = wave_sum(static_cast<double>(s_e));
  if constexpr (NWV > 1) {
    // the ranges' sums in wave order (the trajectory's first wave writes)
    __shared__ double part[kSW][P + 4];
    const int wi = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < P + 4; ++i) part[wi][i] = r[i];
    __syncthreads();
    if (wv != 0 || !live) return;
#pragma unroll
    for (int i = 0; i < P + 4; ++i) {
      double t = part[wi][i];
      for (int v = 1; v < NWV; ++v) t += part[wi + v][i];
      r[i] = t;
    }
  }
#pragma unroll
  for (int i = 0; i < P; ++i)
    if (lane == 0) dtheta[static_cast<size_t>(b) * P + i] = static_cast<float>(gs * r[i]);
  const double r_lp = r[P], r_q = r[P + 1], r_b = r[P + 2], r_e = r[P + 3];
  if (lane == 0) {
    vo.sde[b] = static_cast<float>(r_lp);
    if (vo.obs)
      vo.obs[b] = Dv::kObs ? static_cast<float>(-0.5 * r_q + r_b * (-std::log(static_cast<double>(Dv::kSd)) -
                                                                    0.5 * kLog2Pi))
                           : 0.f;
    if (vo.extra) vo.extra[b] = static_cast<float>(r_e);
  }
}

// ---------------------------------------------------------------------------
// AR(1) streaming path (the BASELINE configs): the same terms as Model<AR> above, laid out for
// HBM: each thread owns V = 4 consecutive times and reads its z span with one 16-byte load (the
// rows are only dword-aligned: M + 1 floats per sample), the window's obs / obs_bin with one
// 16-byte load each, and the two neighbour values as cached dword loads.  Per-sample constants
// (1/e^th2, 1/obs_std) are hoisted, so a transition costs a handful of FMAs instead of four
// IEEE divisions, and the constant terms of the log-densities are added once per sample:
//   sde = -1/2 sum_t z_t^2 + M (-th2 - log(2 pi)/2),  z_t = (x_{t+1} - th1 x_t - th0) e^{-th2}
//   obs = -1/2 sum_t bin_t zo_t^2 + (sum_t bin_t)(-log sd - log(2 pi)/2),  zo_t = (x_{t+1} - y_t)/sd
// (AR.py:169-176).  One wave per trajectory (kArW per block): the per-sample sums are wave
// reductions in double (fixed order, no block barrier), and each lane keeps kArU chunks of
// loads in flight.  Per-lane partials are fp32 over at most a few dozen chunks.
// ---------------------------------------------------------------------------
constexpr int kArV = 4;  // consecutive times per chunk (one 16-byte load)
#ifndef VISSM_AR_U
#define VISSM_AR_U 8
#endif
#ifndef VISSM_AR_NT
#define VISSM_AR_NT 0  // z read with non-temporal loads (read once)
#endif
constexpr int kArU = VISSM_AR_U;  // chunks per lane in flight
constexpr int kArW = 4;           // trajectories (waves) per 256-thread block

__device__ __forceinline__ f4u ldz4(const float* p) {
  if constexpr (VISSM_AR_NT) return __builtin_nontemporal_load(reinterpret_cast<const f4u*>(p));
  return ld4(p);
}

// TG (vissm_elbo_fwd_theta_grad): the same pass also sums z_t and z_t x_t for d(g_sde sde)/d theta (z constant):
// d/dth0 = g is sum z, d/dth1 = g is sum z x_t, d/dth2 = g (sum z^2 - M) -- the terms ar_elbo_bwd_kernel sums
template <bool TG>
__global__ __launch_bounds__(256) void ar_elbo_fwd_kernel(Args a, const float* __restrict__ z,
                                                          const float* __restrict__ theta, float* __restrict__ sde,
                                                          float* __restrict__ obs, const float* __restrict__ g_sde,
                                                          float* __restrict__ dtheta) {
  const int lane = threadIdx.x & 63;
  const int b = __builtin_amdgcn_readfirstlane(blockIdx.x * kArW + (threadIdx.x >> 6));
  if (b >= a.B) return;  // wave-uniform
  const int M = a.M;
  const int w = a.d.win ? a.d.win[b] : 0;
  const float* zb = z + static_cast<size_t>(b) * (M + 1);
  const float* yb = a.d.obs + static_cast<size_t>(w) * M;
  const float* bb = a.d.obs_bin + static_cast<size_t>(w) * M;
  const float th0 = theta[b * 3 + 0], th1 = theta[b * 3 + 1], th2 = theta[b * 3 + 2];
  const float is = __expf(-th2), io = 1.f / a.obs_std;
  float sq = 0.f, so = 0.f, sb = 0.f, s0 = 0.f, s1 = 0.f;
  auto chunk = [&](const f4u& x, float xn, const f4u& y, const f4u& bn) {
    const float xs[kArV + 1] = {x[0], x[1], x[2], x[3], xn};
#pragma unroll
    for (int j = 0; j < kArV; ++j) {
      const float zt = (xs[j + 1] - th1 * xs[j] - th0) * is;
      const float zo = (xs[j + 1] - y[j]) * io;
      sq += zt * zt;
      so += bn[j] * zo * zo;
      sb += bn[j];
      if constexpr (TG) {
        s0 += zt;
        s1 += zt * xs[j];
      }
    }
  };
  // transitions t -> t+1, t in [0, M): full chunks of V (kArU per lane at a time), then the tail
  const int nfull = M / kArV;
  int i = lane;
  for (; i + 64 * (kArU - 1) < nfull; i += 64 * kArU) {
    f4u x[kArU], y[kArU], bn[kArU];
    float xn[kArU];
#pragma unroll
    for (int q = 0; q < kArU; ++q) {
      const int t0 = kArV * (i + 64 * q);
      x[q] = ldz4(zb + t0);
      xn[q] = zb[t0 + kArV];
      y[q] = ld4(yb + t0);
      bn[q] = ld4(bb + t0);
    }
#pragma unroll
    for (int q = 0; q < kArU; ++q) chunk(x[q], xn[q], y[q], bn[q]);
  }
  for (; i < nfull; i += 64) {
    const int t0 = kArV * i;
    chunk(ldz4(zb + t0), zb[t0 + kArV], ld4(yb + t0), ld4(bb + t0));
  }
  for (int t = kArV * nfull + lane; t < M; t += 64) {
    const float zt = (zb[t + 1] - th1 * zb[t] - th0) * is;
    const float zo = (zb[t + 1] - yb[t]) * io;
    sq += zt * zt;
    so += bb[t] * zo * zo;
    sb += bb[t];
    if constexpr (TG) {
      s0 += zt;
      s1 += zt * zb[t];
    }
  }
  const double rq = wave_sum(static_cast<double>(sq));
  const double ro = wave_sum(static_cast<double>(so));
  const double rb = wave_sum(static_cast<double>(sb));
  if constexpr (TG) {
    const double r0 = wave_sum(static_cast<double>(s0));
    const double r1 = wave_sum(static_cast<double>(s1));
    if (lane == 0) {
      const float gs = g_sde ? g_sde[b] : 0.f;
      dtheta[b * 3 + 0] = static_cast<float>(gs * is * r0);
      dtheta[b * 3 + 1] = static_cast<float>(gs * is * r1);
      dtheta[b * 3 + 2] = static_cast<float>(gs * (rq - M));
    }
  }
  if (lane == 0) {
    sde[b] = static_cast<float>(-0.5 * rq + M * (-static_cast<double>(th2) - 0.5 * kLog2Pi));
    if (obs) obs[b] = static_cast<float>(-0.5 * ro + rb * (-std::log(static_cast<double>(a.obs_std)) - 0.5 * kLog2Pi));
  }
}

// d/dz of gs * sde + go * obs at times t in [0, M], and d/dtheta of gs * sde.  Element t takes the
// head gradient of transition t (t < M) and the tail gradient of transition t - 1 plus its obs
// term (t >= 1); each thread recomputes the transition before its chunk instead of exchanging it.
// VALS (vissm_elbo_fwd_grad): also the forward's sums (sde, obs) in the same pass
template <bool VALS = false>
__global__ __launch_bounds__(256) void ar_elbo_bwd_kernel(Args a, const float* __restrict__ z,
                                                          const float* __restrict__ theta,
                                                          const float* __restrict__ g_sde,
                                                          const float* __restrict__ g_obs, float* __restrict__ dz,
                                                          float* __restrict__ dtheta, Vals vo = Vals{}) {
  const int lane = threadIdx.x & 63;
  const int b = __builtin_amdgcn_readfirstlane(blockIdx.x * kArW + (threadIdx.x >> 6));
  if (b >= a.B) return;  // wave-uniform
  const int M = a.M;
  const int w = a.d.win ? a.d.win[b] : 0;
  const float* zb = z + static_cast<size_t>(b) * (M + 1);
  float* dzb = dz + static_cast<size_t>(b) * (M + 1);
  const float* yb = a.d.obs + static_cast<size_t>(w) * M;
  const float* bb = a.d.obs_bin + static_cast<size_t>(w) * M;
  const float th0 = theta[b * 3 + 0], th1 = theta[b * 3 + 1], th2 = theta[b * 3 + 2];
  const float is = __expf(-th2), io = 1.f / a.obs_std;
  const float gs = g_sde ? g_sde[b] : 0.f, go = g_obs ? g_obs[b] : 0.f;
  const float cgh = gs * is * th1, cgt = -gs * is, cgo = -go * io;  // d/dx_t of the three terms per z / zo
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;  // sum_t of z_t, z_t x_t, z_t^2 - 1 over owned transitions
  float so = 0.f, sb = 0.f;            // VALS: sum_t bin_t zo_t^2, sum_t bin_t
  // element t, given x_{t-1}, x_t, x_{t+1}: transition t (if t < M) and t - 1 (if t >= 1)
  auto elem = [&](int t, float xp, float xc, float xn, float y, float bn) -> float {
    float gx = 0.f;
    if (t < M) {
      const float zt = (xn - th1 * xc - th0) * is;
      gx += cgh * zt;
      a0 += zt;
      a1 += zt * xc;
      a2 += zt * zt - 1.f;
    }
    if (t >= 1) {
      const float zp = (xc - th1 * xp - th0) * is;
      const float zo = (xc - y) * io;
      gx += cgt * zp + cgo * bn * zo;
      if constexpr (VALS) {
        so += bn * zo * zo;
        sb += bn;
      }
    }
    return gx;
  };
  // interior chunks: t0 >= 1 and t0 + V <= M, so x_{t0-1} .. x_{t0+V} and obs[t0-1 .. t0+V-2] exist
  auto chunk = [&](int t0, const f4u& x, float xp, float xn, const f4u& y, const f4u& bn) {
    const float xs[kArV + 2] = {xp, x[0], x[1], x[2], x[3], xn};
    f4u g;
#pragma unroll
    for (int j = 0; j < kArV; ++j) {
      // all four elements are interior: t in [1, M)
      const float zt = (xs[j + 2] - th1 * xs[j + 1] - th0) * is;
      const float zp = (xs[j + 1] - th1 * xs[j] - th0) * is;
      const float zo = (xs[j + 1] - y[j]) * io;
      g[j] = cgh * zt + cgt * zp + cgo * bn[j] * zo;
      a0 += zt;
      a1 += zt * xs[j + 1];
      a2 += zt * zt - 1.f;
      if constexpr (VALS) {
        so += bn[j] * zo * zo;
        sb += bn[j];
      }
    }
    if (dz) *reinterpret_cast<f4u*>(dzb + t0) = g;
  };
  const int ilo = 1, ihi = M / kArV;  // chunks i in [ilo, ihi), kArU per lane at a time
  int i = ilo + lane;
  for (; i + 64 * (kArU - 1) < ihi; i += 64 * kArU) {
    f4u x[kArU], y[kArU], bn[kArU];
    float xp[kArU], xn[kArU];
#pragma unroll
    for (int q = 0; q < kArU; ++q) {
      const int t0 = kArV * (i + 64 * q);
      x[q] = ldz4(zb + t0);
      xp[q] = zb[t0 - 1];
      xn[q] = zb[t0 + kArV];
      y[q] = ld4(yb + t0 - 1);
      bn[q] = ld4(bb + t0 - 1);
    }
#pragma unroll
    for (int q = 0; q < kArU; ++q) chunk(kArV * (i + 64 * q), x[q], xp[q], xn[q], y[q], bn[q]);
  }
  for (; i < ihi; i += 64) {
    const int t0 = kArV * i;
    chunk(t0, ldz4(zb + t0), zb[t0 - 1], zb[t0 + kArV], ld4(yb + t0 - 1), ld4(bb + t0 - 1));
  }
  // the rest: t in [0, V) and [V ihi, M]
  const int nrest = kArV + (M + 1 - kArV * ihi);
  for (int r = lane; r < nrest; r += 64) {
    const int t = r < kArV ? r : kArV * ihi + (r - kArV);
    if (t > M || (r >= kArV && t < kArV)) continue;  // (M < V: the two ranges overlap)
    const float xc = zb[t];
    const float xp = t >= 1 ? zb[t - 1] : 0.f, xn = t < M ? zb[t + 1] : 0.f;
    const float y = t >= 1 ? yb[t - 1] : 0.f, bn = t >= 1 ? bb[t - 1] : 0.f;
    const float gv = elem(t, xp, xc, xn, y, bn);
    if (dz) dzb[t] = gv;
  }
  // dlp/dth0 = sum z/s, dlp/dth1 = sum z x_t / s, dlp/dth2 = sum (z^2 - 1)
  const double r0 = wave_sum(static_cast<double>(a0));
  const double r1 = wave_sum(static_cast<double>(a1));
  const double r2 = wave_sum(static_cast<double>(a2));
  if (lane == 0) {
    dtheta[b * 3 + 0] = static_cast<float>(gs * is * r0);
    dtheta[b * 3 + 1] = static_cast<float>(gs * is * r1);
    dtheta[b * 3 + 2] = static_cast<float>(gs * r2);
  }
  if constexpr (VALS) {
    const double ro = wave_sum(static_cast<double>(so));
    const double rb = wave_sum(static_cast<double>(sb));
    if (lane == 0) {
      // sum z^2 = sum (z^2 - 1) + M
      vo.sde[b] = static_cast<float>(-0.5 * (r2 + M) + M * (-static_cast<double>(th2) - 0.5 * kLog2Pi));
      if (vo.obs)
        vo.obs[b] = static_cast<float>(-0.5 * ro + rb * (-std::log(static_cast<double>(a.obs_std)) - 0.5 * kLog2Pi));
    }
  }
}

static int check(const VissmElboDesc* d, const VissmElboData* data) {
  VISSM_CHECK_ARG(d && data, "elbo: null desc/data");
  VISSM_CHECK_ARG(d->B >= 0 && d->M >= 1 && d->n_win >= 1, "elbo: bad shape B=%d M=%d n_win=%d", d->B, d->M,
                  d->n_win);
  VISSM_CHECK_ARG(d->n_win == 1 || data->win, "elbo: n_win > 1 needs win[]");
  switch (d->model) {
    case VISSM_MODEL_AR:
    case VISSM_MODEL_FHN:
      VISSM_CHECK_ARG(data->obs && data->obs_bin, "elbo: model needs obs/obs_bin");
      break;
    case VISSM_MODEL_LV:
      VISSM_CHECK_ARG(data->obs && data->obs_bin && data->mask && data->shift, "elbo: LV needs obs/bin/mask/shift");
      break;
    case VISSM_MODEL_SV:
      VISSM_CHECK_ARG(data->mask && data->shift && data->dim_one, "elbo: SV needs mask/shift/dim_one");
      break;
    default:
      VISSM_CHECK_ARG(false, "elbo: unknown model %d", d->model);
  }
  return VISSM_OK;
}

static int zlen_of(const VissmElboDesc* d) {
  return (d->model == VISSM_MODEL_LV || d->model == VISSM_MODEL_FHN) ? 2 * (d->M + 1) : d->M + 1;
}
static int theta_len(int model) {
  return model == VISSM_MODEL_SV ? 4 : (model == VISSM_MODEL_FHN ? 5 : 3);
}

static Args make(const VissmElboDesc* d, const VissmElboData* data) {
  Args a;
  a.B = d->B; a.M = d->M; a.n_win = d->n_win; a.dt = d->dt; a.obs_std = d->obs_std; a.d = *data;
  if (d->n_win == 1) a.d.win = nullptr;
  return a;
}

}  // namespace elbo
}  // namespace vissm

using namespace vissm;
using namespace vissm::elbo;

extern "C" {

int vissm_elbo_fwd(const VissmElboDesc* d, const VissmElboData* data, const float* z, const float* theta, float* sde,
                   float* obs, float* extra, void* stream) {
  int rc = check(d, data);
  if (rc) return rc;
  VISSM_CHECK_ARG(z && theta && sde, "elbo_fwd: null pointer");
  if (d->B == 0) return VISSM_OK;
  Args a = make(d, data);
  hipStream_t st = as_stream(stream);
  dim3 grid((d->B + kSW - 1) / kSW), blk(256);
  prof_begin(VISSM_PROF_ELBO_FWD, st);
  switch (d->model) {
    case VISSM_MODEL_AR:
      hipLaunchKernelGGL(ar_elbo_fwd_kernel<false>, dim3((d->B + kArW - 1) / kArW), blk, 0, st, a, z, theta, sde, obs,
                         nullptr, nullptr);
      break;
    case VISSM_MODEL_LV: hipLaunchKernelGGL(stream_fwd_kernel<VISSM_MODEL_LV>, grid, blk, 0, st, a, z, theta, sde, obs, extra); break;
    case VISSM_MODEL_SV: hipLaunchKernelGGL(stream_fwd_kernel<VISSM_MODEL_SV>, grid, blk, 0, st, a, z, theta, sde, obs, extra); break;
    default: hipLaunchKernelGGL(stream_fwd_kernel<VISSM_MODEL_FHN>, grid, blk, 0, st, a, z, theta, sde, obs, extra); break;
  }
  VISSM_CHECK_LAUNCH("elbo_fwd");
  // algorithmic bytes: z read once, theta read, the per-sample sums written (per-window feeds are
  // L2-resident and not counted)
  prof_end(VISSM_PROF_ELBO_FWD, st, 4.0 * d->B * (static_cast<double>(zlen_of(d)) + theta_len(d->model) + 3));
  return VISSM_OK;
}

int vissm_elbo_bwd(const VissmElboDesc* d, const VissmElboData* data, const float* z, const float* theta,
                   const float* g_sde, const float* g_obs, const float* g_extra, float* dz, float* dtheta,
                   void* stream) {
  int rc = check(d, data);
  if (rc) return rc;
  VISSM_CHECK_ARG(z && theta && dtheta, "elbo_bwd: null pointer");
  if (d->B == 0) return VISSM_OK;
  Args a = make(d, data);
  hipStream_t st = as_stream(stream);
  dim3 grid((d->B + kSW - 1) / kSW), blk(256);
  prof_begin(VISSM_PROF_ELBO_BWD, st);
  switch (d->model) {
    case VISSM_MODEL_AR: hipLaunchKernelGGL(ar_elbo_bwd_kernel<false>, dim3((d->B + kArW - 1) / kArW), blk, 0, st, a, z, theta, g_sde, g_obs, dz, dtheta); break;
    case VISSM_MODEL_LV: hipLaunchKernelGGL(stream_bwd_kernel<VISSM_MODEL_LV>, grid, blk, 0, st, a, z, theta, g_sde, g_obs, g_extra, dz, dtheta); break;
    case VISSM_MODEL_SV: hipLaunchKernelGGL(stream_bwd_kernel<VISSM_MODEL_SV>, grid, blk, 0, st, a, z, theta, g_sde, g_obs, g_extra, dz, dtheta); break;
    default: hipLaunchKernelGGL(stream_bwd_kernel<VISSM_MODEL_FHN>, grid, blk, 0, st, a, z, theta, g_sde, g_obs, g_extra, dz, dtheta); break;
  }
  VISSM_CHECK_LAUNCH("elbo_bwd");
  // algorithmic bytes: z read, dz written, theta / dtheta and the upstream gradients
  prof_end(VISSM_PROF_ELBO_BWD, st,
           4.0 * d->B * ((dz ? 2.0 : 1.0) * zlen_of(d) + 2 * theta_len(d->model) + 3));
  return VISSM_OK;
}

}  // extern "C"

// waves per trajectory of vissm_elbo_fwd_grad's LV / SV / FHN kernel (stream_onepass_kernel's NWV): enough work units
// for the launch to fill the chip in whole rounds; VISSM_ELBO_NWV = 1 / 2 / 4 overrides (A/B timing)
static int onepass_waves(const VissmElboDesc* d) {
  static const int env = [] {
    const char* e = std::getenv("VISSM_ELBO_NWV");
    return e ? std::atoi(e) : 0;
  }();
  if (env == 1 || env == 2 || env == 4) return env;
  return d->model == VISSM_MODEL_LV ? kNwvLV : d->model == VISSM_MODEL_SV ? kNwvSV : kNwvFHN;
}

extern "C" {

int vissm_elbo_fwd_grad(const VissmElboDesc* d, const VissmElboData* data, const float* z, const float* theta,
                        const float* g_sde, const float* g_obs, const float* g_extra, float* sde, float* obs,
                        float* extra, float* dz, float* dtheta, void* stream) {
  int rc = check(d, data);
  if (rc) return rc;
  VISSM_CHECK_ARG(z && theta && sde && dz && dtheta, "elbo_fwd_grad: null pointer");
  if (d->B == 0) return VISSM_OK;
  VISSM_CHECK_ARG(!data->obs_list || data->obs_stride > 0, "elbo_fwd_grad: obs_list needs obs_stride > 0");
  Args a = make(d, data);
  hipStream_t st = as_stream(stream);
  dim3 grid((d->B + kSW - 1) / kSW), blk(256);
  const Vals vo{sde, obs, extra};
  const bool ol = data->obs_list != nullptr && (d->model == VISSM_MODEL_LV || d->model == VISSM_MODEL_FHN);
  prof_begin(VISSM_PROF_ELBO_BWD, st);
  switch (d->model) {
    case VISSM_MODEL_AR:
      hipLaunchKernelGGL(ar_elbo_bwd_kernel<true>, dim3((d->B + kArW - 1) / kArW), blk, 0, st, a, z, theta, g_sde,
                         g_obs, dz, dtheta, vo);
      break;
#if VISSM_ELBO_ONEPASS_NB
#define ONEPASS(MODEL_, OL_, NWV_)                                                                                  \
  hipLaunchKernelGGL((stream_onepass_kernel<MODEL_, OL_, NWV_>), dim3((d->B * NWV_ + kSW - 1) / kSW), blk, 0, st, a, \
                     z, theta, g_sde, g_obs, g_extra, dz, dtheta, vo)
#define ONEPASS_NWV(MODEL_)                                                                                       \
  do {                                                                                                           \
    const int nwv_ = onepass_waves(d);                                                                           \
    if (nwv_ == 4) ONEPASS(MODEL_, false, 4);                                                                    \
    else if (nwv_ == 2) ONEPASS(MODEL_, false, 2);                                                               \
    else ONEPASS(MODEL_, false, 1);                                                                              \
  } while (0)
    case VISSM_MODEL_LV:
      if (ol) ONEPASS(VISSM_MODEL_LV, true, 1);
      else ONEPASS_NWV(VISSM_MODEL_LV);
      break;
    case VISSM_MODEL_SV: ONEPASS_NWV(VISSM_MODEL_SV); break;
    default:
      if (ol) ONEPASS(VISSM_MODEL_FHN, true, 1);
      else ONEPASS_NWV(VISSM_MODEL_FHN);
      break;
#undef ONEPASS_NWV
#undef ONEPASS
#else
    case VISSM_MODEL_LV: hipLaunchKernelGGL((stream_bwd_kernel<VISSM_MODEL_LV, true>), grid, blk, 0, st, a, z, theta, g_sde, g_obs, g_extra, dz, dtheta, vo); break;
    case VISSM_MODEL_SV: hipLaunchKernelGGL((stream_bwd_kernel<VISSM_MODEL_SV, true>), grid, blk, 0, st, a, z, theta, g_sde, g_obs, g_extra, dz, dtheta, vo); break;
    default: hipLaunchKernelGGL((stream_bwd_kernel<VISSM_MODEL_FHN, true>), grid, blk, 0, st, a, z, theta, g_sde, g_obs, g_extra, dz, dtheta, vo); break;
#endif
  }
  VISSM_CHECK_LAUNCH("elbo_fwd_grad");
  // algorithmic bytes: z read once, dz written, theta / dtheta, the upstream gradients and the three sums
  prof_end(VISSM_PROF_ELBO_BWD, st, 4.0 * d->B * (2.0 * zlen_of(d) + 2 * theta_len(d->model) + 6));
  return VISSM_OK;
}

int vissm_elbo_fwd_theta_grad(const VissmElboDesc* d, const VissmElboData* data, const float* z, const float* theta,
                              const float* g_sde, const float* g_obs, const float* g_extra, float* sde, float* obs,
                              float* extra, float* dtheta, void* stream) {
  if (!d || d->model != VISSM_MODEL_AR) {
    const int rc = vissm_elbo_fwd(d, data, z, theta, sde, obs, extra, stream);
    return rc ? rc : vissm_elbo_bwd(d, data, z, theta, g_sde, g_obs, g_extra, nullptr, dtheta, stream);
  }
  int rc = check(d, data);
  if (rc) return rc;
  VISSM_CHECK_ARG(z && theta && sde && dtheta, "elbo_fwd_theta_grad: null pointer");
  if (d->B == 0) return VISSM_OK;
  Args a = make(d, data);
  hipStream_t st = as_stream(stream);
  prof_begin(VISSM_PROF_ELBO_FWD, st);
  hipLaunchKernelGGL(ar_elbo_fwd_kernel<true>, dim3((d->B + kArW - 1) / kArW), dim3(256), 0, st, a, z, theta, sde, obs,
                     g_sde, dtheta);
  VISSM_CHECK_LAUNCH("elbo_fwd_theta_grad");
  prof_end(VISSM_PROF_ELBO_FWD, st, 4.0 * d->B * (static_cast<double>(zlen_of(d)) + 2 * theta_len(d->model) + 4));
  return VISSM_OK;
}

}  // extern "C"
