// C-ABI entry points of the IAF flow (include/vissm.h): argument validation and
// dispatch by precision and shape.  bf16 / bf16x3 run on the bf16 matrix-core kernels
// (flow_v5) where they cover the shape; fp32 runs the exact-fp32 matrix-core kernels:
// flow4 (register-resident weights, latency hiding) for one hidden layer, flow2 for
// deeper heads (LV / SV / FHN), where flow4's register-resident weights do not apply
// and it measured slower (LV-like shape: 64 vs 76 ms bwd).  No process state.
#include "common.hpp"

#include <cstdlib>

namespace vissm {

size_t flow2_workspace_size(const VissmFlowDesc* d, int backward);
size_t flow4_workspace_size(const VissmFlowDesc* d, int backward);
void flow2_geometry(const VissmFlowDesc* d, int backward, int32_t* out);
void flow4_geometry(const VissmFlowDesc* d, int backward, int32_t* out);
void flow5_geometry(const VissmFlowDesc* d, int which, int32_t* out);
void flow5_geometry_nh3(const VissmFlowDesc* d, int which, int32_t* out);
int flow4_fwd(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*, const float*,
              float*, float*, void*, size_t, hipStream_t);
int flow4_bwd(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*, const float*,
              const float*, const float*, float*, float*, float*, const VissmFlowGrads*, void*, size_t, hipStream_t);
int flow2_fwd(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*, const float*,
              float*, float*, void*, size_t, hipStream_t);
int flow2_bwd(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*, const float*,
              const float*, const float*, float*, float*, float*, const VissmFlowGrads*, void*, size_t, hipStream_t);

bool flow5_supports(const VissmFlowDesc* d);
size_t flow5_workspace_size(const VissmFlowDesc* d, int backward);
int flow5_fwd(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*, const float*,
              float*, float*, void*, size_t, hipStream_t);
int flow5_bwd(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*, const float*,
              const float*, const float*, float*, float*, float*, const VissmFlowGrads*, void*, size_t, hipStream_t);

// the same kernels built without the SLP vectorizer (flow_v5n.hip): the three-hidden-layer shapes
bool flow5_supports_nh3(const VissmFlowDesc* d);
size_t flow5_workspace_size_nh3(const VissmFlowDesc* d, int backward);
int flow5_fwd_nh3(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*,
                  const float*, float*, float*, void*, size_t, hipStream_t);
int flow5_bwd_nh3(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*,
                  const float*, const float*, const float*, float*, float*, float*, const VissmFlowGrads*, void*,
                  size_t, hipStream_t);

// and for k > 32 at three hidden layers (flow_v5s.hip)
void flow5_geometry_nh3s(const VissmFlowDesc* d, int which, int32_t* out);
size_t flow5_workspace_size_nh3s(const VissmFlowDesc* d, int backward);
int flow5_fwd_nh3s(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*,
                   const float*, float*, float*, void*, size_t, hipStream_t);
int flow5_bwd_nh3s(const VissmFlowDesc*, const VissmFlowParams*, const float*, const float*, const int32_t*,
                   const float*, const float*, const float*, float*, float*, float*, const VissmFlowGrads*, void*,
                   size_t, hipStream_t);

bool flow5_ar_fused_supports(const VissmFlowDesc* d);
size_t flow5_ar_fused_workspace_size(const VissmFlowDesc* d);
int flow5_ar_fused(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C, const int32_t* win,
                   const float* theta_term, const float* theta, const float* obs, const float* obs_bin, float obs_std,
                   float scale, float* x, float* logsig, float* du, float* dC, float* dtheta_term,
                   const VissmFlowGrads* gr, void* workspace, size_t ws_bytes, hipStream_t st);
// the same, built with the scheduler's register-pressure trackers (flow_v5f.hip): the fused flow's kernels run there
// (VISSM_FUSED_TU=0: the flow_v5.hip build, A/B)
bool flow5_ar_fused_supports_fz(const VissmFlowDesc* d);
size_t flow5_ar_fused_workspace_size_fz(const VissmFlowDesc* d);
int flow5_ar_fused_fz(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C,
                      const int32_t* win, const float* theta_term, const float* theta, const float* obs,
                      const float* obs_bin, float obs_std, float scale, float* x, float* logsig, float* du, float* dC,
                      float* dtheta_term, const VissmFlowGrads* gr, void* workspace, size_t ws_bytes, hipStream_t st);
#ifndef VISSM_FUSED_TU
#define VISSM_FUSED_TU 1
#endif
#if VISSM_FUSED_TU
#define FUSED_API(name) name##_fz
#else
#define FUSED_API(name) name
#endif

static bool use_flow4(const VissmFlowDesc* d) { return d->n_hidden <= 1; }

static int validate(const VissmFlowDesc* d) {
  VISSM_CHECK_ARG(d, "flow: null desc");
  VISSM_CHECK_ARG(d->B >= 1 && d->k >= 1 && d->k <= 64 && d->H >= 1 && d->H <= 64, "flow: bad B/k/H (B=%d k=%d H=%d)",
                  d->B, d->k, d->H);
  VISSM_CHECK_ARG(d->n_hidden >= 0 && d->n_hidden <= 4, "flow: n_hidden=%d not in [0,4]", d->n_hidden);
  VISSM_CHECK_ARG(d->L > d->k, "flow: L=%d must exceed k=%d", d->L, d->k);
  VISSM_CHECK_ARG(!d->stride2 || ((d->L - d->k) % 2 == 0), "flow: stride-2 output length must be even");
  VISSM_CHECK_ARG(!d->swap_out || ((d->L - d->k) % 2 == 0), "flow: swap_out needs an even output length");
  VISSM_CHECK_ARG(d->n_logsig >= 0 && d->n_logsig <= d->L - d->k, "flow: bad n_logsig");
  VISSM_CHECK_ARG(d->n_win >= 1, "flow: n_win must be >= 1");
  VISSM_CHECK_ARG(d->precision == VISSM_PREC_FP32 || d->precision == VISSM_PREC_BF16 ||
                      d->precision == VISSM_PREC_BF16X3 || d->precision == VISSM_PREC_BF16X2 ||
                      d->precision == VISSM_PREC_BF16X2_BF16,
                  "flow: unknown precision %d", d->precision);
  VISSM_CHECK_ARG(d->chunk_tiles >= 0, "flow: chunk_tiles=%d must be >= 0 (0 = automatic)", d->chunk_tiles);
  VISSM_CHECK_ARG(d->u_pitch == 0 || d->u_pitch >= d->L, "flow: u_pitch=%d must be 0 or >= L=%d", d->u_pitch, d->L);
  VISSM_CHECK_ARG(d->out_pitch == 0 || d->out_pitch >= d->L - d->k, "flow: out_pitch=%d must be 0 or >= L - k=%d",
                  d->out_pitch, d->L - d->k);
  return VISSM_OK;
}

// bf16 / bf16x3 requests run on the bf16 matrix-core kernels (flow_v5) where they
// cover the shape; anything else runs the exact-fp32 kernels (never less precise
// than requested).
static bool use_v5(const VissmFlowDesc* d) { return d->precision != VISSM_PREC_FP32 && flow5_supports(d); }
// three hidden layers on one window with the two-sample backward's k (LV, FHN: k <= 24; SV: 32 < k <= 64, stride 1): the
// builds without the SLP vectorizer (LV-cfg backward 18.1 -> 16.8 ms, FHN 3.7 -> 3.5, SV 7.2 -> 6.7 ms per launch),
// k <= 24 in flow_v5n.hip (also VGPR-form MFMAs and AGPR accumulators: LV 16.6 -> 14.6 ms), k > 32 in flow_v5s.hip.
// The one-sample three-layer kernel (several windows) measured slower without the vectorizer (SV: 10.3 -> 10.8 ms).
// VISSM_NH3_DEFAULT_FORM=1 sends the k <= 24 shapes to flow_v5s.hip's build as well (the same source without the
// VGPR-form flag and the asm accumulators): tests/test_gpu_vgpr_form.py checks that flow_v5n.hip's kernels compute what
// that build computes at every shape they ship for -- the flag miscompiled SV's k = 50 du variant
static bool nh3_default_form() {
  const char* e = std::getenv("VISSM_NH3_DEFAULT_FORM");
  return e && e[0] == '1';
}
static bool use_nh3(const VissmFlowDesc* d) {
  return d->n_hidden == 3 && d->n_win == 1 && d->k <= 24 && !nh3_default_form();
}
static bool use_nh3s(const VissmFlowDesc* d) {
  return d->n_hidden == 3 && d->n_win == 1 && d->k <= 64 &&
         ((d->k > 32 && !d->stride2) || (d->k <= 24 && nh3_default_form()));
}

}  // namespace vissm

using namespace vissm;

extern "C" {

size_t vissm_flow_workspace_size(const VissmFlowDesc* d, int32_t backward) {
  if (validate(d) != VISSM_OK) return 0;
  if (use_v5(d))
    return use_nh3(d) ? flow5_workspace_size_nh3(d, backward)
         : use_nh3s(d) ? flow5_workspace_size_nh3s(d, backward) : flow5_workspace_size(d, backward);
  return use_flow4(d) ? flow4_workspace_size(d, backward) : flow2_workspace_size(d, backward);
}

int vissm_flow_geometry(const VissmFlowDesc* d, int32_t which, int32_t* out) {
  int rc = validate(d);
  if (rc) return rc;
  VISSM_CHECK_ARG(out && which >= 0 && which <= 2, "flow_geometry: bad which=%d or null out", which);
  if (which == 2) {
    VISSM_CHECK_ARG(flow5_ar_fused_supports(d), "flow_geometry: the descriptor has no fused AR(1) last flow");
    flow5_geometry(d, 2, out);
  } else if (use_v5(d)) {
    (use_nh3(d) ? flow5_geometry_nh3 : use_nh3s(d) ? flow5_geometry_nh3s : flow5_geometry)(d, which, out);
  } else {
    (use_flow4(d) ? flow4_geometry : flow2_geometry)(d, which, out);
  }
  return VISSM_OK;
}

int vissm_flow_fwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C,
                   const int32_t* win, const float* theta_term, float* u_next, float* logsig, void* workspace,
                   size_t ws_bytes, void* stream) {
  int rc = validate(d);
  if (rc) return rc;
  VISSM_CHECK_ARG(w && u && C && theta_term && u_next && logsig, "flow_fwd: null pointer");
  VISSM_CHECK_ARG(w->w_eps && w->w_head && w->b_head && (d->n_hidden == 0 || (w->w_hid && w->b_hid)),
                  "flow_fwd: null weight pointer");
  VISSM_CHECK_ARG(!d->bn || d->n_hidden == 0 || (w->bn_g && w->bn_b), "flow_fwd: bn needs bn_g/bn_b");
  VISSM_CHECK_ARG(d->n_win == 1 || win, "flow_fwd: n_win > 1 needs win[]");
  VISSM_CHECK_ARG(d->precision != VISSM_PREC_BF16X2_BF16,
                  "flow_fwd: VISSM_PREC_BF16X2_BF16 is a precision of vissm_flow_ar_elbo_fused only");
  hipStream_t st = as_stream(stream);
  if (use_v5(d))
    return (use_nh3(d) ? flow5_fwd_nh3 : use_nh3s(d) ? flow5_fwd_nh3s : flow5_fwd)(d, w, u, C, win, theta_term, u_next,
                                                                                    logsig, workspace, ws_bytes, st);
  if (use_flow4(d)) return flow4_fwd(d, w, u, C, win, theta_term, u_next, logsig, workspace, ws_bytes, st);
  return flow2_fwd(d, w, u, C, win, theta_term, u_next, logsig, workspace, ws_bytes, st);
}

int vissm_flow_bwd(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C,
                   const int32_t* win, const float* theta_term, const float* du_next, const float* dlogsig,
                   float* du, float* dC, float* dtheta_term, const VissmFlowGrads* gr, void* workspace,
                   size_t ws_bytes, void* stream) {
  int rc = validate(d);
  if (rc) return rc;
  VISSM_CHECK_ARG(w && u && C && theta_term && du_next && dlogsig && dC && dtheta_term && gr,
                  "flow_bwd: null pointer");
  VISSM_CHECK_ARG(d->precision != VISSM_PREC_BF16X2_BF16,
                  "flow_bwd: VISSM_PREC_BF16X2_BF16 is a precision of vissm_flow_ar_elbo_fused only");
  VISSM_CHECK_ARG(du || use_v5(d), "flow_bwd: du may be NULL only on the bf16 / bf16x3 kernels");
  VISSM_CHECK_ARG(gr->w_eps && gr->w_head && gr->b_head && (d->n_hidden == 0 || (gr->w_hid && gr->b_hid)),
                  "flow_bwd: null grad pointer");
  VISSM_CHECK_ARG(!d->bn || d->n_hidden == 0 || (gr->bn_g && gr->bn_b && w->bn_g && w->bn_b),
                  "flow_bwd: bn needs bn_g/bn_b pointers");
  VISSM_CHECK_ARG(d->n_win == 1 || win, "flow_bwd: n_win > 1 needs win[]");
  hipStream_t st = as_stream(stream);
  if (use_v5(d))
    return (use_nh3(d) ? flow5_bwd_nh3 : use_nh3s(d) ? flow5_bwd_nh3s : flow5_bwd)(d, w, u, C, win, theta_term,
                                                                                    du_next, dlogsig, du, dC, dtheta_term,
                                                                                    gr, workspace, ws_bytes, st);
  if (use_flow4(d))
    return flow4_bwd(d, w, u, C, win, theta_term, du_next, dlogsig, du, dC, dtheta_term, gr, workspace, ws_bytes, st);
  return flow2_bwd(d, w, u, C, win, theta_term, du_next, dlogsig, du, dC, dtheta_term, gr, workspace, ws_bytes, st);
}

int32_t vissm_flow_kernel_precision(const VissmFlowDesc* d) {
  if (validate(d) != VISSM_OK || d->precision == VISSM_PREC_BF16X2_BF16) return VISSM_EINVAL;
  return use_v5(d) ? d->precision : VISSM_PREC_FP32;
}

int32_t vissm_flow_ar_elbo_fused_supported(const VissmFlowDesc* d) {
  return (validate(d) == VISSM_OK && FUSED_API(flow5_ar_fused_supports)(d)) ? 1 : 0;
}

size_t vissm_flow_ar_elbo_fused_workspace_size(const VissmFlowDesc* d) {
  if (!vissm_flow_ar_elbo_fused_supported(d)) return 0;
  return FUSED_API(flow5_ar_fused_workspace_size)(d);
}

int vissm_flow_ar_elbo_fused(const VissmFlowDesc* d, const VissmFlowParams* w, const float* u, const float* C,
                             const int32_t* win, const float* theta_term, const float* theta, const float* obs,
                             const float* obs_bin, float obs_std, float scale, float* x, float* logsig,
                             float* du, float* dC, float* dtheta_term, const VissmFlowGrads* gr, void* workspace,
                             size_t ws_bytes, void* stream) {
  int rc = validate(d);
  if (rc) return rc;
  VISSM_CHECK_ARG(FUSED_API(flow5_ar_fused_supports)(d),
                  "flow_ar_elbo_fused: needs bf16 / bf16x3 (k <= 32) or bf16x2 / bf16x2_bf16 (k <= 8, one window), one hidden "
                  "layer, no BN, "
                  "stride 1");
  VISSM_CHECK_ARG(w && u && C && theta_term && theta && obs && obs_bin && x && logsig && du && dC && dtheta_term && gr,
                  "flow_ar_elbo_fused: null pointer");
  VISSM_CHECK_ARG(gr->w_eps && gr->w_hid && gr->b_hid && gr->w_head && gr->b_head, "flow_ar_elbo_fused: null grad");
  VISSM_CHECK_ARG(d->n_win == 1 || win, "flow_ar_elbo_fused: n_win > 1 needs win[]");
  VISSM_CHECK_ARG(obs_std > 0.f, "flow_ar_elbo_fused: obs_std must be positive");
  VISSM_CHECK_ARG(d->out_pitch == 0 || d->out_pitch == d->L - d->k, "flow_ar_elbo_fused: x is written dense (out_pitch "
                  "%d must be 0 or L - k)", d->out_pitch);
  return FUSED_API(flow5_ar_fused)(d, w, u, C, win, theta_term, theta, obs, obs_bin, obs_std, scale, x, logsig, du,
                                   dC, dtheta_term, gr, workspace, ws_bytes, as_stream(stream));
}

}  // extern "C"
