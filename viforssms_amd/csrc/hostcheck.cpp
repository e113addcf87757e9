// Host (CPU) build of elbo_math.hpp so the CPU test-suite can check the
// hand-derived transition gradients against the oracle's autograd without a GPU.
// Not part of the product path: libvissm_hostcheck.so is loaded only by tests/.
#include <cstddef>

#include "../../include/vissm.h"
#include "elbo_math.hpp"

extern "C" {

// out = [lp, gh0, gh1, gt0, gt1, gth0..gth4]
void vissm_host_trans(int model, const float* xh, const float* xt, const float* th, float dt, float* out) {
  using namespace vissm::em;
  TG r;
  switch (model) {
    case 0: r = ar_trans(xh[0], xt[0], th); break;
    case 1: r = lv_trans(xh, xt, th, dt); break;
    case 2: r = sv_trans(xh, xt, th, dt); break;
    default: r = fhn_trans(xh, xt, th, dt); break;
  }
  out[0] = r.lp;
  out[1] = r.gh[0]; out[2] = r.gh[1];
  out[3] = r.gt[0]; out[4] = r.gt[1];
  for (int i = 0; i < 5; ++i) out[5 + i] = r.gth[i];
}

float vissm_host_sp_ildj(float y, float* gy) { return vissm::em::sp_ildj(y, gy); }

float vissm_host_obs(float x, float y, float bin, float sd, float* gx) { return vissm::em::obs_term(x, y, bin, sd, gx); }

// the C ABI's struct layouts as the C compiler sees them (the ctypes mirrors in viforssms_amd/_lib.py are
// checked against these): which = 0 VissmFlowDesc, 1 VissmFlowParams, 2 VissmFlowGrads, 3 VissmElboData; out = {size,
// offset of the last field}
void vissm_host_abi_layout(int which, size_t* out) {
  switch (which) {
    case 0: out[0] = sizeof(VissmFlowDesc); out[1] = offsetof(VissmFlowDesc, out_pitch); break;
    case 1: out[0] = sizeof(VissmFlowParams); out[1] = offsetof(VissmFlowParams, theta_rank); break;
    case 2: out[0] = sizeof(VissmFlowGrads); out[1] = offsetof(VissmFlowGrads, b_head); break;
    default: out[0] = sizeof(VissmElboData); out[1] = offsetof(VissmElboData, obs_stride); break;
  }
}

}
