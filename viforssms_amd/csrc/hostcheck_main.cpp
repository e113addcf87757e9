// Sanitizer driver for the host build of elbo_math.hpp (hostcheck.cpp): built with
// -fsanitize=address,undefined into build/hostcheck_san and run by the CPU test-suite
// (tests/test_lib.py::test_hostcheck_sanitized).  Each model's hand-derived transition
// gradient is checked against central finite differences of its own log-density over
// a fixed pseudo-random grid of states and parameters, and the ABI layout query is
// exercised; any sanitizer report aborts the run (-fno-sanitize-recover=all).
// Exit 0 = all checks passed.  Not part of the product path.
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdint>
#include <initializer_list>

extern "C" {
void vissm_host_trans(int model, const float* xh, const float* xt, const float* th, float dt, float* out);
float vissm_host_sp_ildj(float y, float* gy);
float vissm_host_obs(float x, float y, float bin, float sd, float* gx);
void vissm_host_abi_layout(int which, size_t* out);
}

namespace {

uint64_t g_state = 0x9E3779B97F4A7C15ull;
double uniform(double lo, double hi) {  // splitmix64
  uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return lo + (hi - lo) * (static_cast<double>(z >> 11) * 0x1.0p-53);
}

float lp_of(int model, const float* xh, const float* xt, const float* th, float dt) {
  float out[10];
  vissm_host_trans(model, xh, xt, th, dt, out);
  return out[0];
}

// central difference of lp in one input coordinate (which: 0 head, 1 tail, 2 theta)
double fd(int model, float* xh, float* xt, float* th, float dt, int which, int i) {
  float* v = which == 0 ? xh : which == 1 ? xt : th;
  const float x0 = v[i];
  const float h = 1e-2f * std::fmax(1.f, std::fabs(x0));
  v[i] = x0 + h;
  const double lp_p = lp_of(model, xh, xt, th, dt);
  v[i] = x0 - h;
  const double lp_m = lp_of(model, xh, xt, th, dt);
  v[i] = x0;
  return (lp_p - lp_m) / (2.0 * (static_cast<double>(x0 + h) - static_cast<double>(x0)));
}

int check_model(int model, int cases) {
  const int D = model == 0 ? 1 : 2;
  const int P = model == 0 ? 3 : model == 1 ? 3 : model == 2 ? 4 : 5;
  const float dt = model == 0 || model == 2 ? 1.f : 0.1f;
  int bad = 0;
  for (int c = 0; c < cases; ++c) {
    float xh[2] = {0.f, 0.f}, xt[2] = {0.f, 0.f}, th[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int d = 0; d < D; ++d) {
      if (model == 1) {  // LV populations
        xh[d] = static_cast<float>(uniform(20.0, 200.0));
        xt[d] = xh[d] + static_cast<float>(uniform(-3.0, 3.0));
      } else if (model == 2 && d == 0) {  // SV: the sd s1 = sqrt(dt) x1 e^{x2/2} vanishes at x1 = 0; keep |x1| >= 0.5
        xh[d] = static_cast<float>(uniform(0.5, 2.0) * (uniform(0.0, 1.0) < 0.5 ? -1.0 : 1.0));
        xt[d] = xh[d] + static_cast<float>(uniform(-0.5, 0.5));
      } else {
        xh[d] = static_cast<float>(uniform(-2.0, 2.0));
        xt[d] = xh[d] + static_cast<float>(uniform(-0.5, 0.5));
      }
    }
    for (int p = 0; p < P; ++p) th[p] = static_cast<float>(uniform(-1.0, 1.0));
    if (model == 1) {  // LV log-rates near the reference's (log 0.5, log 0.0025, log 0.3)
      th[0] = static_cast<float>(std::log(0.5) + uniform(-0.2, 0.2));
      th[1] = static_cast<float>(std::log(0.0025) + uniform(-0.2, 0.2));
      th[2] = static_cast<float>(std::log(0.3) + uniform(-0.2, 0.2));
    }
    float out[10];
    vissm_host_trans(model, xh, xt, th, dt, out);
    if (!std::isfinite(out[0])) { std::printf("model %d case %d: lp not finite\n", model, c); ++bad; continue; }
    double gmax = 1.0;
    for (int i = 1; i < 10; ++i) gmax = std::fmax(gmax, std::fabs(out[i]));
    struct { int which, n, off; } groups[3] = {{0, D, 1}, {1, D, 3}, {2, P, 5}};
    for (const auto& g : groups)
      for (int i = 0; i < g.n; ++i) {
        const double num = fd(model, xh, xt, th, dt, g.which, i);
        const double ana = out[g.off + i];
        if (!(std::fabs(num - ana) <= 2e-2 * gmax + 2e-2 * std::fabs(num))) {
          std::printf("model %d case %d input %d.%d: analytic %.6g vs finite difference %.6g\n", model, c, g.which, i,
                      ana, num);
          ++bad;
        }
      }
  }
  return bad;
}

}  // namespace

int main() {
  int bad = 0;
  for (int model = 0; model < 4; ++model) bad += check_model(model, 200);
  for (float y : {0.05f, 0.7f, 3.0f, 40.0f}) {
    float g = 0.f;
    const float v = vissm_host_sp_ildj(y, &g);
    const float h = 1e-3f * std::fmax(1.f, y);
    float gp, gm;
    const double num = (vissm_host_sp_ildj(y + h, &gp) - vissm_host_sp_ildj(y - h, &gm)) / (2.0 * h);
    if (!std::isfinite(v) || std::fabs(num - g) > 1e-2 * std::fmax(1.0, std::fabs(num))) {
      std::printf("sp_ildj(%g): %g vs %g\n", y, g, num);
      ++bad;
    }
  }
  float gx = 0.f;
  const float o = vissm_host_obs(1.5f, 1.0f, 1.f, 0.5f, &gx);
  if (!std::isfinite(o) || std::fabs(gx + 2.f) > 1e-5f) { std::printf("obs_term: gx %g\n", gx); ++bad; }
  for (int which = 0; which < 3; ++which) {
    size_t out[2] = {0, 0};
    vissm_host_abi_layout(which, out);
    if (out[0] == 0 || out[1] >= out[0]) { std::printf("abi layout %d: %zu %zu\n", which, out[0], out[1]); ++bad; }
  }
  std::printf("hostcheck_san: %d failures\n", bad);
  return bad ? 1 : 0;
}
