// Per-transition log-densities of the four SDE models and their hand-derived
// gradients.  Shared by the HIP ELBO kernels (elbo.hip) and a host build
// (hostcheck.cpp) that the CPU test-suite checks against the oracle's autograd.
//
//   AR  : N(x_{t+1}; th1 x_t + th0, exp(th2))                       AR.py:172-176
//   LV  : bivariate EM density, chol = sqrt(dt)[[a,0],[b,c]], theta = exp(th)
//                                                  lotka_volterra_partial.py:39-52, 244-261
//   SV  : diag EM, drift (th0 x1, th1 - e^th2 x2), sd sqrt(dt)(x1 e^{x2/2}, e^th3)
//                                                                SV_dense.py:203-223
//   FHN : diag EM, drift (e^th0 (x1 - x1^3 - x2 + th1), th2 x1 - x2 + 1.4),
//         sd sqrt(dt)(sqrt(e^th3), sqrt(e^th4))                  fitz_nag_NVP.py:243-255
#pragma once

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define VHD __host__ __device__ __forceinline__
#else
#include <cmath>
#define VHD inline
#endif

namespace vissm {
namespace em {

#ifdef __HIPCC__
#define VEXP ::expf
#define VLOG ::logf
#define VSQRT ::sqrtf
#define VLOG1P ::log1pf
#define VEXPM1 ::expm1f
#else
#define VEXP std::exp
#define VLOG std::log
#define VSQRT std::sqrt
#define VLOG1P std::log1p
#define VEXPM1 std::expm1
#endif

constexpr float kHalfLog2Pi = 0.91893853320467274f;
constexpr float kLog2Pi_ = 1.8378770664093453f;

// gradient record of one transition: lp, d/dhead[2], d/dtail[2], d/dtheta[5]
struct TG {
  float lp;
  float gh[2];
  float gt[2];
  float gth[5];
};

VHD void tg_zero(TG& r) {
  r.lp = 0.f;
  r.gh[0] = r.gh[1] = r.gt[0] = r.gt[1] = 0.f;
  for (int i = 0; i < 5; ++i) r.gth[i] = 0.f;
}

// ---- AR(1) ----------------------------------------------------------------
VHD TG ar_trans(float x0, float x1, const float* th) {
  TG r;
  tg_zero(r);
  const float s = VEXP(th[2]);
  const float q = x1 - th[1] * x0 - th[0];
  const float z = q / s;
  r.lp = -0.5f * z * z - th[2] - kHalfLog2Pi;
  const float gq = -z / s;          // dlp/dq
  r.gt[0] = gq;
  r.gh[0] = -gq * th[1];
  r.gth[0] = -gq;
  r.gth[1] = -gq * x0;
  r.gth[2] = z * z - 1.f;
  return r;
}

// observation term: bin * log N(x; y, sd); returns lp, writes dlp/dx
VHD float obs_term(float x, float y, float bin, float sd, float* gx) {
  const float z = (x - y) / sd;
  *gx = -bin * z / sd;
  return bin * (-0.5f * z * z - VLOG(sd) - kHalfLog2Pi);
}

// ---- Lotka-Volterra --------------------------------------------------------
VHD TG lv_trans(const float* x, const float* y, const float* th, float dt) {
  TG r;
  tg_zero(r);
  const float e0 = VEXP(th[0]), e1 = VEXP(th[1]), e2 = VEXP(th[2]);
  const float x1 = x[0], x2 = x[1];
  const float p12 = x1 * x2;
  const float Bv = e1 * p12;
  const float A = e0 * x1 + Bv;     // a^2
  const float Cc = Bv + e2 * x2;    // b^2 + c^2
  const float m1 = dt * (e0 * x1 - Bv), m2 = dt * (Bv - e2 * x2);
  const float q1 = y[0] - x1 - m1, q2 = y[1] - x2 - m2;
  const float Dl = A * Cc - Bv * Bv;  // det(Sigma) / dt^2
  const float inv = 1.f / (dt * Dl);
  const float g1 = inv * (Cc * q1 + Bv * q2), g2 = inv * (Bv * q1 + A * q2);  // Sigma^-1 q
  const float quad = q1 * g1 + q2 * g2;
  r.lp = -0.5f * VLOG(dt * dt * Dl) - 0.5f * quad - kLog2Pi_;
  // reverse mode
  const float gq1 = -g1, gq2 = -g2;
  const float iD = 1.f / Dl;
  float gA = -0.5f * Cc * iD - 0.5f * (q2 * q2 * inv - quad * Cc * iD);
  float gC = -0.5f * A * iD - 0.5f * (q1 * q1 * inv - quad * A * iD);
  float gB = Bv * iD - q1 * q2 * inv - quad * Bv * iD;
  r.gt[0] = gq1;
  r.gt[1] = gq2;
  float gx1 = -gq1, gx2 = -gq2;
  const float gm1 = -gq1, gm2 = -gq2;
  float ge0 = gm1 * dt * x1, ge1 = 0.f, ge2 = -gm2 * dt * x2;
  gx1 += gm1 * dt * e0;
  gx2 += -gm2 * dt * e2;
  gB += (gm2 - gm1) * dt;
  // Cc = Bv + e2 x2
  gB += gC;
  ge2 += gC * x2;
  gx2 += gC * e2;
  // A = e0 x1 + Bv
  ge0 += gA * x1;
  gx1 += gA * e0;
  gB += gA;
  // Bv = e1 p12
  ge1 += gB * p12;
  const float gp = gB * e1;
  gx1 += gp * x2;
  gx2 += gp * x1;
  r.gh[0] = gx1;
  r.gh[1] = gx2;
  r.gth[0] = ge0 * e0;
  r.gth[1] = ge1 * e1;
  r.gth[2] = ge2 * e2;
  return r;
}

// diagonal-Gaussian helper: lp of q ~ N(0, s); accumulates dlp/dq and dlp/ds
VHD float diag_term(float q, float s, float* gq, float* gs) {
  const float z = q / s;
  *gq = -z / s;
  *gs = (z * z - 1.f) / s;
  return -0.5f * z * z - VLOG(s < 0.f ? -s : s) - kHalfLog2Pi;
}

// ---- stochastic volatility --------------------------------------------------
VHD TG sv_trans(const float* x, const float* y, const float* th, float dt) {
  TG r;
  tg_zero(r);
  const float x1 = x[0], x2 = x[1];
  const float sq = VSQRT(dt);
  const float e2 = VEXP(th[2]);
  const float m1 = dt * th[0] * x1, m2 = dt * (th[1] - e2 * x2);
  const float s1 = sq * x1 * VEXP(0.5f * x2), s2 = sq * VEXP(th[3]);
  const float q1 = y[0] - x1 - m1, q2 = y[1] - x2 - m2;
  float gq1, gs1, gq2, gs2;
  r.lp = diag_term(q1, s1, &gq1, &gs1) + diag_term(q2, s2, &gq2, &gs2);
  r.gt[0] = gq1;
  r.gt[1] = gq2;
  float gx1 = -gq1, gx2 = -gq2;
  const float gm1 = -gq1, gm2 = -gq2;
  r.gth[0] = gm1 * dt * x1;
  gx1 += gm1 * dt * th[0];
  r.gth[1] = gm2 * dt;
  r.gth[2] = -gm2 * dt * x2 * e2;
  gx2 += -gm2 * dt * e2;
  // s1 = sq x1 e^{x2/2}
  gx1 += gs1 * sq * VEXP(0.5f * x2);
  gx2 += gs1 * 0.5f * s1;
  r.gth[3] = gs2 * s2;
  r.gh[0] = gx1;
  r.gh[1] = gx2;
  return r;
}

// ---- FitzHugh-Nagumo ---------------------------------------------------------
VHD TG fhn_trans(const float* x, const float* y, const float* th, float dt) {
  TG r;
  tg_zero(r);
  const float x1 = x[0], x2 = x[1];
  const float sq = VSQRT(dt);
  const float E0 = VEXP(th[0]);
  const float f = x1 - x1 * x1 * x1 - x2 + th[1];
  const float m1 = dt * E0 * f, m2 = dt * (th[2] * x1 - x2 + 1.4f);
  const float s1 = sq * VSQRT(VEXP(th[3])), s2 = sq * VSQRT(VEXP(th[4]));
  const float q1 = y[0] - x1 - m1, q2 = y[1] - x2 - m2;
  float gq1, gs1, gq2, gs2;
  r.lp = diag_term(q1, s1, &gq1, &gs1) + diag_term(q2, s2, &gq2, &gs2);
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
  r.gth[3] = gs1 * 0.5f * s1;
  r.gth[4] = gs2 * 0.5f * s2;
  r.gh[0] = gx1;
  r.gh[1] = gx2;
  return r;
}

// ---- LV positivity transform (tfb.Softplus), lotka_volterra_partial.py:292-297 ----
VHD float softplus_h(float z) { return z > 0.f ? z + VLOG1P(VEXP(-z)) : VLOG1P(VEXP(z)); }
VHD float sigmoid_h(float z) { return z >= 0.f ? 1.f / (1.f + VEXP(-z)) : VEXP(z) / (1.f + VEXP(z)); }
// Softplus ILDJ at y: -log(-expm1(-y)); derivative -1/expm1(y)
VHD float sp_ildj(float y, float* gy) {
  *gy = -1.f / VEXPM1(y);
  return -VLOG(-VEXPM1(-y));
}

}  // namespace em
}  // namespace vissm
