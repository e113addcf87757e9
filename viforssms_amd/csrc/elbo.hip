// ELBO log-density kernels: one 256-thread block per trajectory (LV, SV, FHN) or one
// wave per trajectory (AR, the streaming path below), fixed-order block / wave
// reductions (double accumulation).  Streaming: the path z is read once
// (forward) or once plus its neighbours (backward, which recomputes each
// transition from both of its endpoints instead of exchanging partials).
//
// Reference terms: AR VI_SSM._ELBO (AR.py:168-187); LV Softplus transform and
// _ELBO (lotka_volterra_partial.py:290-297, 234-270); SV dim-one concat and
// _ELBO (SV_dense.py:245-246, 203-232); FHN _ELBO (fitz_nag_NVP.py:232-265).
#include "common.hpp"
#include "elbo_math.hpp"

namespace vissm {
namespace elbo {

struct Args {
  int B, M, n_win;
  float dt, obs_std;
  VissmElboData d;
};

template <int MODEL>
struct Model;

// x at time t for dimension d and its derivative w.r.t. the stored z entry
template <>
struct Model<VISSM_MODEL_AR> {
  static constexpr int D = 1, P = 3;
  __device__ static float x(const Args&, const float* zb, int, int t, int, float* dxdz) {
    *dxdz = 1.f;
    return zb[t];
  }
  __device__ static em::TG trans(const float* xh, const float* xt, const float* th, float) {
    return em::ar_trans(xh[0], xt[0], th);
  }
  __device__ static int zidx(int t, int) { return t; }
};

template <>
struct Model<VISSM_MODEL_LV> {
  static constexpr int D = 2, P = 3;
  __device__ static float x(const Args& a, const float* zb, int w, int t, int d, float* dxdz) {
    const float zz = zb[2 * t + d];
    const size_t mi = (static_cast<size_t>(w) * 2 + d) * (a.M + 1) + t;
    const float mk = a.d.mask[mi];
    *dxdz = mk * em::sigmoid_h(zz);
    return em::softplus_h(zz) * mk + a.d.shift[mi];
  }
  __device__ static em::TG trans(const float* xh, const float* xt, const float* th, float dt) {
    return em::lv_trans(xh, xt, th, dt);
  }
  __device__ static int zidx(int t, int d) { return 2 * t + d; }
};

template <>
struct Model<VISSM_MODEL_SV> {
  static constexpr int D = 2, P = 4;
  __device__ static float x(const Args& a, const float* zb, int w, int t, int d, float* dxdz) {
    const size_t mi = static_cast<size_t>(w) * (a.M + 1) + t;
    if (d == 0) {
      *dxdz = 0.f;
      return a.d.dim_one[mi];
    }
    const float mk = a.d.mask[mi];
    *dxdz = mk;
    return zb[t] * mk + a.d.shift[mi];
  }
  __device__ static em::TG trans(const float* xh, const float* xt, const float* th, float dt) {
    return em::sv_trans(xh, xt, th, dt);
  }
  __device__ static int zidx(int t, int) { return t; }
};

template <>
struct Model<VISSM_MODEL_FHN> {
  static constexpr int D = 2, P = 5;
  __device__ static float x(const Args&, const float* zb, int, int t, int d, float* dxdz) {
    *dxdz = 1.f;
    return zb[2 * t + d];
  }
  __device__ static em::TG trans(const float* xh, const float* xt, const float* th, float dt) {
    return em::fhn_trans(xh, xt, th, dt);
  }
  __device__ static int zidx(int t, int d) { return 2 * t + d; }
};

// number of stored z entries per sample
template <int MODEL>
__device__ __forceinline__ int zlen(const Args& a) {
  return (MODEL == VISSM_MODEL_LV || MODEL == VISSM_MODEL_FHN) ? 2 * (a.M + 1) : (a.M + 1);
}

template <int MODEL>
__device__ __forceinline__ float obs_sd(const Args& a) {
  return MODEL == VISSM_MODEL_AR ? a.obs_std : (MODEL == VISSM_MODEL_FHN ? 0.1f : 1.f);
}
template <int MODEL>
__device__ __forceinline__ constexpr bool has_obs() { return MODEL != VISSM_MODEL_SV; }

template <int MODEL>
__global__ __launch_bounds__(256) void elbo_fwd_kernel(Args a, const float* __restrict__ z,
                                                       const float* __restrict__ theta, float* __restrict__ sde,
                                                       float* __restrict__ obs, float* __restrict__ extra) {
  using Mdl = Model<MODEL>;
  constexpr int D = Mdl::D, P = Mdl::P;
  __shared__ double red[4];
  const int b = blockIdx.x;
  const int w = a.d.win ? a.d.win[b] : 0;
  const float* zb = z + static_cast<size_t>(b) * zlen<MODEL>(a);
  float th[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < P; ++i) th[i] = theta[static_cast<size_t>(b) * P + i];
  const float osd = obs_sd<MODEL>(a);
  double s_sde = 0.0, s_obs = 0.0, s_ex = 0.0;
  for (int t = threadIdx.x; t < a.M; t += blockDim.x) {
    float xh[2], xt[2], dd;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      xh[d] = Mdl::x(a, zb, w, t, d, &dd);
      xt[d] = Mdl::x(a, zb, w, t + 1, d, &dd);
    }
    s_sde += Mdl::trans(xh, xt, th, a.dt).lp;
    if (has_obs<MODEL>()) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const size_t oi = (static_cast<size_t>(w) * D + d) * a.M + t;
        float gx;
        s_obs += em::obs_term(xt[d], a.d.obs[oi], a.d.obs_bin[oi], osd, &gx);
      }
    }
    if (MODEL == VISSM_MODEL_LV) {
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        float gy;
        s_ex += em::sp_ildj(xt[d], &gy);
      }
    }
  }
  const double r0 = block_sum(s_sde, red);
  const double r1 = block_sum(s_obs, red);
  const double r2 = block_sum(s_ex, red);
  if (threadIdx.x == 0) {
    sde[b] = static_cast<float>(r0);
    if (obs) obs[b] = static_cast<float>(r1);
    if (extra) extra[b] = static_cast<float>(r2);
  }
}

template <int MODEL>
__global__ __launch_bounds__(256) void elbo_bwd_kernel(Args a, const float* __restrict__ z,
                                                       const float* __restrict__ theta,
                                                       const float* __restrict__ g_sde,
                                                       const float* __restrict__ g_obs,
                                                       const float* __restrict__ g_ex, float* __restrict__ dz,
                                                       float* __restrict__ dtheta) {
  using Mdl = Model<MODEL>;
  constexpr int D = Mdl::D, P = Mdl::P;
  __shared__ double red[4];
  const int b = blockIdx.x;
  const int w = a.d.win ? a.d.win[b] : 0;
  const float* zb = z + static_cast<size_t>(b) * zlen<MODEL>(a);
  float* dzb = dz + static_cast<size_t>(b) * zlen<MODEL>(a);
  float th[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < P; ++i) th[i] = theta[static_cast<size_t>(b) * P + i];
  const float gs = g_sde ? g_sde[b] : 0.f;
  const float go = (has_obs<MODEL>() && g_obs) ? g_obs[b] : 0.f;
  const float ge = (MODEL == VISSM_MODEL_LV && g_ex) ? g_ex[b] : 0.f;
  const float osd = obs_sd<MODEL>(a);
  double acc[5] = {0, 0, 0, 0, 0};
  for (int t = threadIdx.x; t <= a.M; t += blockDim.x) {
    float xc[2], jac[2], xo[2], dd;
#pragma unroll
    for (int d = 0; d < D; ++d) xc[d] = Mdl::x(a, zb, w, t, d, &jac[d]);
    float gx[2] = {0.f, 0.f};
    if (t < a.M) {
#pragma unroll
      for (int d = 0; d < D; ++d) xo[d] = Mdl::x(a, zb, w, t + 1, d, &dd);
      const em::TG r = Mdl::trans(xc, xo, th, a.dt);
#pragma unroll
      for (int d = 0; d < D; ++d) gx[d] += gs * r.gh[d];
#pragma unroll
      for (int i = 0; i < P; ++i) acc[i] += static_cast<double>(gs) * r.gth[i];
    }
    if (t >= 1) {
#pragma unroll
      for (int d = 0; d < D; ++d) xo[d] = Mdl::x(a, zb, w, t - 1, d, &dd);
      const em::TG r = Mdl::trans(xo, xc, th, a.dt);
#pragma unroll
      for (int d = 0; d < D; ++d) gx[d] += gs * r.gt[d];
      if (has_obs<MODEL>()) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const size_t oi = (static_cast<size_t>(w) * D + d) * a.M + (t - 1);
          float g;
          em::obs_term(xc[d], a.d.obs[oi], a.d.obs_bin[oi], osd, &g);
          gx[d] += go * g;
        }
      }
      if (MODEL == VISSM_MODEL_LV) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          float g;
          em::sp_ildj(xc[d], &g);
          gx[d] += ge * g;
        }
      }
    }
    if (MODEL == VISSM_MODEL_SV) {
      dzb[t] = gx[1] * jac[1];
    } else {
#pragma unroll
      for (int d = 0; d < D; ++d) dzb[Mdl::zidx(t, d)] = gx[d] * jac[d];
    }
  }
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const double s = block_sum(acc[i], red);
    if (threadIdx.x == 0) dtheta[static_cast<size_t>(b) * P + i] = static_cast<float>(s);
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
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
constexpr int kArV = 4;  // consecutive times per chunk (one 16-byte load)
#ifndef VISSM_AR_U
#define VISSM_AR_U 8
#endif
#ifndef VISSM_AR_NT
#define VISSM_AR_NT 0  // z read with non-temporal loads (read once)
#endif
constexpr int kArU = VISSM_AR_U;  // chunks per lane in flight
constexpr int kArW = 4;           // trajectories (waves) per 256-thread block

__device__ __forceinline__ f4u ld4(const float* p) { return *reinterpret_cast<const f4u*>(p); }
__device__ __forceinline__ f4u ldz4(const float* p) {
  if constexpr (VISSM_AR_NT) return __builtin_nontemporal_load(reinterpret_cast<const f4u*>(p));
  return ld4(p);
}

__global__ __launch_bounds__(256) void ar_elbo_fwd_kernel(Args a, const float* __restrict__ z,
                                                          const float* __restrict__ theta, float* __restrict__ sde,
                                                          float* __restrict__ obs) {
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
  float sq = 0.f, so = 0.f, sb = 0.f;
  auto chunk = [&](const f4u& x, float xn, const f4u& y, const f4u& bn) {
    const float xs[kArV + 1] = {x[0], x[1], x[2], x[3], xn};
#pragma unroll
    for (int j = 0; j < kArV; ++j) {
      const float zt = (xs[j + 1] - th1 * xs[j] - th0) * is;
      const float zo = (xs[j + 1] - y[j]) * io;
      sq += zt * zt;
      so += bn[j] * zo * zo;
      sb += bn[j];
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
  }
  const double rq = wave_sum(static_cast<double>(sq));
  const double ro = wave_sum(static_cast<double>(so));
  const double rb = wave_sum(static_cast<double>(sb));
  if (lane == 0) {
    sde[b] = static_cast<float>(-0.5 * rq + M * (-static_cast<double>(th2) - 0.5 * kLog2Pi));
    if (obs) obs[b] = static_cast<float>(-0.5 * ro + rb * (-std::log(static_cast<double>(a.obs_std)) - 0.5 * kLog2Pi));
  }
}

// d/dz of gs * sde + go * obs at times t in [0, M], and d/dtheta of gs * sde.  Element t takes the
// head gradient of transition t (t < M) and the tail gradient of transition t - 1 plus its obs
// term (t >= 1); each thread recomputes the transition before its chunk instead of exchanging it.
__global__ __launch_bounds__(256) void ar_elbo_bwd_kernel(Args a, const float* __restrict__ z,
                                                          const float* __restrict__ theta,
                                                          const float* __restrict__ g_sde,
                                                          const float* __restrict__ g_obs, float* __restrict__ dz,
                                                          float* __restrict__ dtheta) {
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
      gx += cgt * zp + cgo * bn * (xc - y) * io;
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
      g[j] = cgh * zt + cgt * zp + cgo * bn[j] * (xs[j + 1] - y[j]) * io;
      a0 += zt;
      a1 += zt * xs[j + 1];
      a2 += zt * zt - 1.f;
    }
    *reinterpret_cast<f4u*>(dzb + t0) = g;
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
    dzb[t] = elem(t, xp, xc, xn, y, bn);
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
  dim3 grid(d->B), blk(256);
  prof_begin(VISSM_PROF_ELBO_FWD, st);
  switch (d->model) {
    case VISSM_MODEL_AR: hipLaunchKernelGGL(ar_elbo_fwd_kernel, dim3((d->B + kArW - 1) / kArW), blk, 0, st, a, z, theta, sde, obs); break;
    case VISSM_MODEL_LV: hipLaunchKernelGGL(elbo_fwd_kernel<VISSM_MODEL_LV>, grid, blk, 0, st, a, z, theta, sde, obs, extra); break;
    case VISSM_MODEL_SV: hipLaunchKernelGGL(elbo_fwd_kernel<VISSM_MODEL_SV>, grid, blk, 0, st, a, z, theta, sde, obs, extra); break;
    default: hipLaunchKernelGGL(elbo_fwd_kernel<VISSM_MODEL_FHN>, grid, blk, 0, st, a, z, theta, sde, obs, extra); break;
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
  VISSM_CHECK_ARG(z && theta && dz && dtheta, "elbo_bwd: null pointer");
  if (d->B == 0) return VISSM_OK;
  Args a = make(d, data);
  hipStream_t st = as_stream(stream);
  dim3 grid(d->B), blk(256);
  prof_begin(VISSM_PROF_ELBO_BWD, st);
  switch (d->model) {
    case VISSM_MODEL_AR: hipLaunchKernelGGL(ar_elbo_bwd_kernel, dim3((d->B + kArW - 1) / kArW), blk, 0, st, a, z, theta, g_sde, g_obs, dz, dtheta); break;
    case VISSM_MODEL_LV: hipLaunchKernelGGL(elbo_bwd_kernel<VISSM_MODEL_LV>, grid, blk, 0, st, a, z, theta, g_sde, g_obs, g_extra, dz, dtheta); break;
    case VISSM_MODEL_SV: hipLaunchKernelGGL(elbo_bwd_kernel<VISSM_MODEL_SV>, grid, blk, 0, st, a, z, theta, g_sde, g_obs, g_extra, dz, dtheta); break;
    default: hipLaunchKernelGGL(elbo_bwd_kernel<VISSM_MODEL_FHN>, grid, blk, 0, st, a, z, theta, g_sde, g_obs, g_extra, dz, dtheta); break;
  }
  VISSM_CHECK_LAUNCH("elbo_bwd");
  // algorithmic bytes: z read, dz written, theta / dtheta and the upstream gradients
  prof_end(VISSM_PROF_ELBO_BWD, st,
           4.0 * d->B * (2.0 * zlen_of(d) + 2 * theta_len(d->model) + 3));
  return VISSM_OK;
}

}  // extern "C"
