// q(theta): the variational posterior over the SDE parameters (include/vissm.h vissm_theta_*).
//
// Reference: q(theta) = TransformedDistribution(Normal(loc, scale), Chain(reversed([IMAF_0, P_0, ...,
// IMAF_{n-1}]))) (AR.py:376-391; lotka_volterra_partial.py:494-508; SV_dense.py:428-442; fitz_nag_NVP.py:
// 480-494), each IMAF = Invert(MaskedAutoregressiveFlow(masked_autoregressive_default_template([5, 5, 5],
// activation))), whose forward is one parallel pass:
//   [shift | log_scale] = MADE(z),  z' = (z - shift) exp(-clip(log_scale)),  log q += sum clip(log_scale)
// with log_scale clipped to [-5, 3] by a straight-through clip, and Permute between the bijectors.
//
// Layout: the bijectors' variables as the parameter store holds them, bijector after bijector, each
// dense0 kernel [P][5], bias [5], dense1 [5][5], bias [5], dense2 [5][5], bias [5], dense3 [5][2P],
// bias [2P] (NPB = 17 P + 65 floats); the MADE masks in the same layout (ones on the biases).
//
// One thread per sample: the MADE nets are a few hundred FLOPs, so the step's q(theta) (forward and
// backward over B samples) runs as two launches instead of ~150 small tensor kernels.  The weights are
// read with uniform addresses (one fetch serves the wave).  The backward recomputes the forward (the
// bijector inputs stay in registers), sums each parameter's per-sample gradient over the wave, writes one
// row per wave to a slab, and a fixed-order column sum adds the masked result into dw: deterministic.
#include "common.hpp"

namespace vissm {
namespace {

constexpr int HU = 5;  // masked_autoregressive_default_template hidden_layers=[5, 5, 5]

__host__ __device__ constexpr int npb(int P) { return 17 * P + 65; }

struct Net {  // offsets of one bijector's variables
  int w0, b0, w1, b1, w2, b2, w3, b3;
};
__host__ __device__ constexpr Net net_of(int P) {
  return Net{0, 5 * P, 5 * P + 5, 5 * P + 30, 5 * P + 35, 5 * P + 60, 5 * P + 65, 15 * P + 65};
}

__device__ __forceinline__ float act_f(float x, int relu) { return relu ? fmaxf(x, 0.f) : (x > 0.f ? x : expm1f(x)); }
// derivative through the output y = act(x)
__device__ __forceinline__ float act_d(float y, int relu) { return relu ? (y > 0.f ? 1.f : 0.f) : (y > 0.f ? 1.f : y + 1.f); }

// MADE of one bijector: h1..h3 (post-activation), shift / log scale of each coordinate
template <int P>
__device__ __forceinline__ void made(const float* __restrict__ w, const float* __restrict__ m, const float (&z)[P],
                                     int relu, float (&h1)[HU], float (&h2)[HU], float (&h3)[HU], float (&sh)[P],
                                     float (&ls)[P]) {
  constexpr Net n = net_of(P);
#pragma unroll
  for (int o = 0; o < HU; ++o) {
    float a = w[n.b0 + o];
#pragma unroll
    for (int i = 0; i < P; ++i) a = fmaf(z[i], w[n.w0 + i * HU + o] * m[n.w0 + i * HU + o], a);
    h1[o] = act_f(a, relu);
  }
#pragma unroll
  for (int o = 0; o < HU; ++o) {
    float a = w[n.b1 + o];
#pragma unroll
    for (int i = 0; i < HU; ++i) a = fmaf(h1[i], w[n.w1 + i * HU + o] * m[n.w1 + i * HU + o], a);
    h2[o] = act_f(a, relu);
  }
#pragma unroll
  for (int o = 0; o < HU; ++o) {
    float a = w[n.b2 + o];
#pragma unroll
    for (int i = 0; i < HU; ++i) a = fmaf(h2[i], w[n.w2 + i * HU + o] * m[n.w2 + i * HU + o], a);
    h3[o] = act_f(a, relu);
  }
#pragma unroll
  for (int d = 0; d < P; ++d) {
    float s = w[n.b3 + 2 * d], l = w[n.b3 + 2 * d + 1];
#pragma unroll
    for (int i = 0; i < HU; ++i) {
      s = fmaf(h3[i], w[n.w3 + i * 2 * P + 2 * d] * m[n.w3 + i * 2 * P + 2 * d], s);
      l = fmaf(h3[i], w[n.w3 + i * 2 * P + 2 * d + 1] * m[n.w3 + i * 2 * P + 2 * d + 1], l);
    }
    sh[d] = s;
    ls[d] = l;
  }
}

__device__ __forceinline__ float clip_ls(float l) { return fminf(fmaxf(l, -5.f), 3.f); }

template <int P>
__device__ __forceinline__ float base_lp(const float (&x)[P], float loc, float scale) {
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < P; ++d) {
    const float t = (x[d] - loc) / scale;
    s += -0.5f * t * t - logf(scale) - 0.5f * kLog2Pi;
  }
  return s;
}

template <int P>
__device__ __forceinline__ void permute(const VissmThetaDesc& d, int i, float (&z)[P]) {
  float t[P];
#pragma unroll
  for (int q = 0; q < P; ++q) t[q] = z[q];
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const int src = d.perm[i][q];
    float v = t[0];
#pragma unroll
    for (int r = 1; r < P; ++r) v = src == r ? t[r] : v;  // register select, no dynamic indexing
    z[q] = v;
  }
}

template <int P>
__global__ __launch_bounds__(256) void theta_fwd_kernel(VissmThetaDesc d, const float* __restrict__ w,
                                                        const float* __restrict__ m, const float* __restrict__ x0,
                                                        float* __restrict__ theta, float* __restrict__ logq) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  float z[P];
#pragma unroll
  for (int q = 0; q < P; ++q) z[q] = x0[static_cast<size_t>(b) * P + q];
  float lq = base_lp<P>(z, d.base_loc, d.base_scale);
#pragma unroll
  for (int i = 0; i < VISSM_THETA_MAX_BIJ; ++i) {
    if (i >= d.n_bij) break;
    float h1[HU], h2[HU], h3[HU], sh[P], ls[P];
    made<P>(w + i * npb(P), m + i * npb(P), z, d.relu, h1, h2, h3, sh, ls);
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const float l = clip_ls(ls[q]);
      z[q] = (z[q] - sh[q]) * expf(-l);
      lq += l;
    }
    if (i < d.n_bij - 1) permute<P>(d, i, z);
  }
#pragma unroll
  for (int q = 0; q < P; ++q) theta[static_cast<size_t>(b) * P + q] = z[q];
  logq[b] = lq;
}

// x + DPP(x) with row_mask / bank_mask; lanes whose source is outside the row read 0 (bound_ctrl)
template <int CTRL, int RM = 0xf, int BM = 0xf>
__device__ __forceinline__ float add_dpp(float x) {
  return x + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, RM, BM, true));
}
// the wave's sum in lane 63 (fixed order, registers only): row_shr 1, 2, 4, 8 leave each 16-lane row's
// sum in its lane 15; row_bcast:15 adds row 0 into row 1 and row 2 into row 3; row_bcast:31 adds lane 31
// into row 3
__device__ __forceinline__ float wave_sum_l63(float v) {
  v = add_dpp<0x111>(v);
  v = add_dpp<0x112>(v);
  v = add_dpp<0x114>(v);
  v = add_dpp<0x118>(v);
  v = add_dpp<0x142, 0xa>(v);
  v = add_dpp<0x143, 0xc>(v);
  return v;
}
// gradient of one parameter: the wave's sum of its lanes' contributions -> slab row of the wave
__device__ __forceinline__ void put_grad(float* __restrict__ row, int k, float v) {
  v = wave_sum_l63(v);
  if ((threadIdx.x & 63) == 63) row[k] = v;
}

template <int P>
__global__ __launch_bounds__(256) void theta_bwd_kernel(VissmThetaDesc d, const float* __restrict__ w,
                                                        const float* __restrict__ m, const float* __restrict__ x0,
                                                        const float* __restrict__ dtheta,
                                                        const float* __restrict__ dlogq, float* __restrict__ slab) {
  constexpr Net n = net_of(P);
  const int b0 = blockIdx.x * blockDim.x + threadIdx.x;
  if ((b0 & ~63) >= d.B) return;  // a wave with no sample (partial last block): no slab row
  const bool live = b0 < d.B;
  const int b = live ? b0 : d.B - 1;  // idle lanes recompute a real sample and contribute zero
  const int wave = b0 >> 6;
  float* row = slab + static_cast<size_t>(wave) * d.n_bij * npb(P);
  // forward, keeping every bijector's input
  float zs[VISSM_THETA_MAX_BIJ][P];
  float z[P];
#pragma unroll
  for (int q = 0; q < P; ++q) z[q] = x0[static_cast<size_t>(b) * P + q];
#pragma unroll
  for (int i = 0; i < VISSM_THETA_MAX_BIJ; ++i) {
    if (i >= d.n_bij) break;
#pragma unroll
    for (int q = 0; q < P; ++q) zs[i][q] = z[q];
    float h1[HU], h2[HU], h3[HU], sh[P], ls[P];
    made<P>(w + i * npb(P), m + i * npb(P), z, d.relu, h1, h2, h3, sh, ls);
#pragma unroll
    for (int q = 0; q < P; ++q) z[q] = (z[q] - sh[q]) * expf(-clip_ls(ls[q]));
    if (i < d.n_bij - 1) permute<P>(d, i, z);
  }
  // backward: gz = d loss / d z (the bijector's output), gl = d loss / d log q
  float gz[P];
  const float gl = (live && dlogq) ? dlogq[b] : 0.f;
#pragma unroll
  for (int q = 0; q < P; ++q) gz[q] = (live && dtheta) ? dtheta[static_cast<size_t>(b) * P + q] : 0.f;
#pragma unroll
  for (int i = VISSM_THETA_MAX_BIJ - 1; i >= 0; --i) {
    if (i >= d.n_bij) continue;
    if (i < d.n_bij - 1) {  // z_out[q] = z_in[perm[q]]  ->  g_in[perm[q]] += g_out[q]
      float t[P];
#pragma unroll
      for (int q = 0; q < P; ++q) t[q] = 0.f;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const int src = d.perm[i][q];
#pragma unroll
        for (int r = 0; r < P; ++r) t[r] += src == r ? gz[q] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < P; ++q) gz[q] = t[q];
    }
    const float* wi = w + i * npb(P);
    const float* mi = m + i * npb(P);
    float* gi = row + i * npb(P);
    float h1[HU], h2[HU], h3[HU], sh[P], ls[P];
    made<P>(wi, mi, zs[i], d.relu, h1, h2, h3, sh, ls);
    // z' = (z - sh) e^{-l}, log q += l (l = clip(ls), straight-through)
    float dsh[P], dls[P], dz[P];
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const float e = expf(-clip_ls(ls[q]));
      const float zn = (zs[i][q] - sh[q]) * e;
      dz[q] = gz[q] * e;
      dsh[q] = -gz[q] * e;
      dls[q] = -gz[q] * zn + gl;
    }
    // dense3: out[2q] = shift_q, out[2q+1] = log_scale_q
    float dh3[HU];
#pragma unroll
    for (int o = 0; o < HU; ++o) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const int k0 = n.w3 + o * 2 * P + 2 * q;
        s = fmaf(dsh[q], wi[k0] * mi[k0], s);
        s = fmaf(dls[q], wi[k0 + 1] * mi[k0 + 1], s);
        put_grad(gi, k0, h3[o] * dsh[q]);
        put_grad(gi, k0 + 1, h3[o] * dls[q]);
      }
      dh3[o] = s * act_d(h3[o], d.relu);
    }
#pragma unroll
    for (int q = 0; q < P; ++q) {
      put_grad(gi, n.b3 + 2 * q, dsh[q]);
      put_grad(gi, n.b3 + 2 * q + 1, dls[q]);
    }
    // dense2 (input h2), dense1 (input h1)
    float dh2[HU], dh1[HU];
#pragma unroll
    for (int i2 = 0; i2 < HU; ++i2) {
      float s = 0.f;
#pragma unroll
      for (int o = 0; o < HU; ++o) {
        const int k = n.w2 + i2 * HU + o;
        s = fmaf(dh3[o], wi[k] * mi[k], s);
        put_grad(gi, k, h2[i2] * dh3[o]);
      }
      dh2[i2] = s * act_d(h2[i2], d.relu);
    }
#pragma unroll
    for (int o = 0; o < HU; ++o) put_grad(gi, n.b2 + o, dh3[o]);
#pragma unroll
    for (int i1 = 0; i1 < HU; ++i1) {
      float s = 0.f;
#pragma unroll
      for (int o = 0; o < HU; ++o) {
        const int k = n.w1 + i1 * HU + o;
        s = fmaf(dh2[o], wi[k] * mi[k], s);
        put_grad(gi, k, h1[i1] * dh2[o]);
      }
      dh1[i1] = s * act_d(h1[i1], d.relu);
    }
#pragma unroll
    for (int o = 0; o < HU; ++o) put_grad(gi, n.b1 + o, dh2[o]);
    // dense0 (input z)
#pragma unroll
    for (int q = 0; q < P; ++q) {
      float s = dz[q];
#pragma unroll
      for (int o = 0; o < HU; ++o) {
        const int k = n.w0 + q * HU + o;
        s = fmaf(dh1[o], wi[k] * mi[k], s);
        put_grad(gi, k, zs[i][q] * dh1[o]);
      }
      gz[q] = s;
    }
#pragma unroll
    for (int o = 0; o < HU; ++o) put_grad(gi, n.b0 + o, dh1[o]);
  }
}

// dw[k] += mask[k] * tot[k]
__global__ __launch_bounds__(256) void theta_grad_finish_kernel(const float* __restrict__ tot, int N,
                                                                const float* __restrict__ m, float* __restrict__ dw) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < N) dw[k] += tot[k] * m[k];
}

int check_desc(const VissmThetaDesc* d) {
  VISSM_CHECK_ARG(d, "theta: null descriptor");
  VISSM_CHECK_ARG(d->B >= 1 && d->P >= 1 && d->P <= VISSM_THETA_MAX_P && d->n_bij >= 1 &&
                      d->n_bij <= VISSM_THETA_MAX_BIJ && d->base_scale > 0.f,
                  "theta: bad shape (B=%d P=%d n_bij=%d scale=%g)", d->B, d->P, d->n_bij, d->base_scale);
  for (int i = 0; i + 1 < d->n_bij; ++i) {
    int seen = 0;
    for (int q = 0; q < d->P; ++q) {
      const int s = d->perm[i][q];
      VISSM_CHECK_ARG(s >= 0 && s < d->P && !(seen & (1 << s)), "theta: perm %d is not a permutation", i);
      seen |= 1 << s;
    }
  }
  return VISSM_OK;
}

#define THETA_DISPATCH(KERNEL, P, ...)                                   \
  switch (P) {                                                           \
    case 1: hipLaunchKernelGGL((KERNEL<1>), __VA_ARGS__); break;         \
    case 2: hipLaunchKernelGGL((KERNEL<2>), __VA_ARGS__); break;         \
    case 3: hipLaunchKernelGGL((KERNEL<3>), __VA_ARGS__); break;         \
    case 4: hipLaunchKernelGGL((KERNEL<4>), __VA_ARGS__); break;         \
    default: hipLaunchKernelGGL((KERNEL<5>), __VA_ARGS__); break;        \
  }

}  // namespace
}  // namespace vissm

using namespace vissm;

extern "C" {

int32_t vissm_theta_num_params(int32_t P, int32_t n_bij) { return npb(P) * n_bij; }

size_t vissm_theta_workspace_size(const VissmThetaDesc* d) {
  if (!d || d->B < 1 || d->P < 1 || d->P > VISSM_THETA_MAX_P || d->n_bij < 1) return 0;
  const size_t waves = (static_cast<size_t>(d->B) + 63) / 64;
  const size_t N = static_cast<size_t>(npb(d->P)) * d->n_bij;
  return align_up(waves * N * sizeof(float)) + align_up(N * sizeof(float));  // slab, column totals
}

int vissm_theta_fwd(const VissmThetaDesc* d, const float* w, const float* mask, const float* x0, float* theta,
                    float* logq, void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  VISSM_CHECK_ARG(w && mask && x0 && theta && logq, "theta_fwd: null pointer");
  const dim3 grid((d->B + 255) / 256);
  THETA_DISPATCH(theta_fwd_kernel, d->P, grid, dim3(256), 0, as_stream(stream), *d, w, mask, x0, theta, logq);
  VISSM_CHECK_LAUNCH("theta_fwd");
  return VISSM_OK;
}

int vissm_theta_bwd(const VissmThetaDesc* d, const float* w, const float* mask, const float* x0, const float* dtheta,
                    const float* dlogq, float* dw, void* workspace, size_t ws_bytes, void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  VISSM_CHECK_ARG(w && mask && x0 && dw, "theta_bwd: null pointer");
  VISSM_CHECK_ARG(workspace && ws_bytes >= vissm_theta_workspace_size(d), "theta_bwd: workspace too small");
  float* slab = static_cast<float*>(workspace);
  const int waves = (d->B + 63) / 64;
  const int N = npb(d->P) * d->n_bij;
  hipStream_t st = as_stream(stream);
  const dim3 grid((d->B + 255) / 256);
  // (a partial last block: waves past B return at once; the rows of the ceil(B / 64) waves are read)
  THETA_DISPATCH(theta_bwd_kernel, d->P, grid, dim3(256), 0, st, *d, w, mask, x0, dtheta, dlogq, slab);
  VISSM_CHECK_LAUNCH("theta_bwd");
  // column totals in a fixed order (two passes: the slab is tall and narrow), then the masked add
  float* tot = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                        align_up(static_cast<size_t>(waves) * N * sizeof(float)));
  rc = launch_reduce_rows_inplace(slab, tot, waves, N, st);
  if (rc) return rc;
  hipLaunchKernelGGL(theta_grad_finish_kernel, dim3((N + 255) / 256), dim3(256), 0, st, tot, N, mask, dw);
  VISSM_CHECK_LAUNCH("theta_grad_finish");
  return VISSM_OK;
}


// ---------------------------------------------------------------------------
// The flows' theta branch (IAF._create_flow's three linear dense layers on theta, AR.py:63-68):
// theta_term = ((theta W0 + b0) W1 + b1) W2 + b2, with d = d loss / d theta_term [B, H].  Every gradient follows
// from S = theta^T d [P, H], s = sum_b d [H] and dtheta = d (W0 W1 W2)^T [B, P] (nma._ThetaBranch): one pass over d
// (one wave per 32-row slice, lane = column h: S / s partials per block, dtheta rows by wave reductions; each block
// forms W0 W1 W2 from the LDS-staged weights), then one block sums the partials in a fixed order and forms the
// [<= 64]^2 weight gradients.  Two launches instead of the ~14 small library kernels of the torch form.
// ---------------------------------------------------------------------------
}  // extern "C"
namespace vissm {
namespace {
constexpr int kTbMax = 64;   // H, n0, n1 <= 64, P <= 8
constexpr int kTbRows = 32;  // rows of d per wave

// the three weight matrices staged in LDS (W0 [P][n0], W1 [n0][n1], W2 [n1][H], row pitch kTbMax)
struct TbW {
  float W0[8][kTbMax], W1[kTbMax][kTbMax], W2[kTbMax][kTbMax];
};
__device__ void tb_stage(TbW& w, int P, int n0, int n1, int H, const float* __restrict__ W0,
                         const float* __restrict__ W1, const float* __restrict__ W2) {
  for (int i = threadIdx.x; i < P * n0; i += blockDim.x) w.W0[i / n0][i % n0] = W0[i];
  for (int i = threadIdx.x; i < n0 * n1; i += blockDim.x) w.W1[i / n1][i % n1] = W1[i];
  for (int i = threadIdx.x; i < n1 * H; i += blockDim.x) w.W2[i / H][i % H] = W2[i];
}

template <int P>
__global__ __launch_bounds__(256) void theta_branch_pass_kernel(int B, int n0, int n1, int H,
                                                                 const float* __restrict__ theta,
                                                                 const float* __restrict__ d,
                                                                 const float* __restrict__ W0g,
                                                                 const float* __restrict__ W1g,
                                                                 const float* __restrict__ W2g,
                                                                 float* __restrict__ dtheta, float* __restrict__ part) {
  // Wc = W0 W1 W2 [P][H], formed by every block from the LDS-staged weights (no separate launch)
  __shared__ TbW w;
  __shared__ float W01[P][kTbMax], Wc[P][kTbMax];
  tb_stage(w, P, n0, n1, H, W0g, W1g, W2g);
  __syncthreads();
  for (int i = threadIdx.x; i < P * n1; i += 256) {
    const int p = i / n1, jj = i % n1;
    float v = 0.f;
    for (int a = 0; a < n0; ++a) v += w.W0[p][a] * w.W1[a][jj];
    W01[p][jj] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P * H; i += 256) {
    const int p = i / H, h = i % H;
    float v = 0.f;
    for (int jj = 0; jj < n1; ++jj) v += W01[p][jj] * w.W2[jj][h];
    Wc[p][h] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int r0 = wv * kTbRows;
  const bool on = lane < H;
  float wc[P], sacc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    wc[p] = on ? Wc[p][lane] : 0.f;
    sacc[p] = 0.f;
  }
  float ssum = 0.f;
  const int r1 = min(B, r0 + kTbRows);
  constexpr int RB = 8;   // rows whose loads are in flight together
  for (int rb = r0; rb < r1; rb += RB) {
    float v[RB], t[RB][P];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int r = min(rb + i, r1 - 1);   // (rows past r1 are loaded again and not counted)
      v[i] = on ? d[static_cast<size_t>(r) * H + lane] : 0.f;
#pragma unroll
      for (int p = 0; p < P; ++p) t[i][p] = theta[static_cast<size_t>(r) * P + p];
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      if (rb + i >= r1) break;   // wave-uniform
      float q[P];
#pragma unroll
      for (int p = 0; p < P; ++p) {
        sacc[p] += t[i][p] * v[i];
        q[p] = v[i] * wc[p];
      }
      ssum += v[i];
      // dtheta[r][p] = sum_h d[r][h] Wc[p][h]: a fixed-order butterfly over the wave
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int p = 0; p < P; ++p) q[p] += __shfl_xor(q[p], off);
      if (lane < P) {
        float o = q[0];
#pragma unroll
        for (int p = 1; p < P; ++p) o = lane == p ? q[p] : o;
        dtheta[static_cast<size_t>(rb + i) * P + lane] = o;
      }
    }
  }
  // the block's partials (rows p = 0..P-1 of S, row P of s): the four waves' sums in wave order
  __shared__ float wsum[4][P + 1][kTbMax];
  const int wq = threadIdx.x >> 6;
#pragma unroll
  for (int p = 0; p < P; ++p) wsum[wq][p][lane] = sacc[p];
  wsum[wq][P][lane] = ssum;
  __syncthreads();
  float* pb = part + static_cast<size_t>(blockIdx.x) * (P + 1) * kTbMax;
  for (int i = threadIdx.x; i < (P + 1) * kTbMax; i += 256) {
    const int p = i / kTbMax, h = i % kTbMax;
    pb[i] = ((wsum[0][p][h] + wsum[1][p][h]) + wsum[2][p][h]) + wsum[3][p][h];
  }
}

// S, s from the block partials in a fixed order, then the weight gradients (one block of 1024 threads)
__global__ __launch_bounds__(1024) void theta_branch_finish_kernel(int n_rows, int P, int n0, int n1, int H,
                                                                    const float* __restrict__ part,
                                                                    const float* __restrict__ W0g,
                                                                    const float* __restrict__ b0,
                                                                    const float* __restrict__ W1g,
                                                                    const float* __restrict__ b1,
                                                                    const float* __restrict__ W2g,
                                                                    float* __restrict__ dW0, float* __restrict__ db0,
                                                                    float* __restrict__ dW1, float* __restrict__ db1,
                                                                    float* __restrict__ dW2, float* __restrict__ db2) {
  __shared__ TbW w;
  __shared__ float S[9][kTbMax];      // rows 0..P-1: S, row P: s
  __shared__ float SW2[9][kTbMax];    // rows 0..P-1: S W2^T, row P: s W2^T
  __shared__ float W01[8][kTbMax], c1[kTbMax];
  constexpr int NS = 8;               // row slices summed in parallel
  __shared__ float sl[NS][9 * kTbMax];
  const int R = P + 1;
  tb_stage(w, P, n0, n1, H, W0g, W1g, W2g);
  // thread (slice q, column i) sums rows q, q + NS, ... in order (eight loads in flight), then the slices are added
  // in slice order: a fixed order for a given n_rows
  for (int jx = threadIdx.x; jx < NS * R * kTbMax; jx += blockDim.x) {
    const int q = jx / (R * kTbMax), i = jx % (R * kTbMax);
    float v = 0.f;
    int r = q;
    for (; r + 7 * NS < n_rows; r += 8 * NS) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = part[static_cast<size_t>(r + NS * u) * R * kTbMax + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) v += x[u];
    }
    for (; r < n_rows; r += NS) v += part[static_cast<size_t>(r) * R * kTbMax + i];
    sl[q][i] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < R * kTbMax; i += blockDim.x) {
    float v = sl[0][i];
#pragma unroll
    for (int q = 1; q < NS; ++q) v += sl[q][i];
    S[i / kTbMax][i % kTbMax] = v;
  }
  for (int i = threadIdx.x; i < P * n1; i += blockDim.x) {    // W0 W1
    const int p = i / n1, j = i % n1;
    float v = 0.f;
    for (int a = 0; a < n0; ++a) v += w.W0[p][a] * w.W1[a][j];
    W01[p][j] = v;
  }
  for (int j = threadIdx.x; j < n1; j += blockDim.x) {        // b0 W1 + b1
    float v = b1[j];
    for (int a = 0; a < n0; ++a) v += b0[a] * w.W1[a][j];
    c1[j] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < R * n1; i += blockDim.x) {    // [S; s] W2^T
    const int p = i / n1, j = i % n1;
    float v = 0.f;
    for (int h = 0; h < H; ++h) v += S[p][h] * w.W2[j][h];
    SW2[p][j] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n1 * H; i += blockDim.x) {    // dW2 = (W0 W1)^T S + (b0 W1 + b1) s^T
    const int j = i / H, h = i % H;
    float v = c1[j] * S[P][h];
    for (int p = 0; p < P; ++p) v += W01[p][j] * S[p][h];
    dW2[i] = v;
  }
  for (int h = threadIdx.x; h < H; h += blockDim.x) db2[h] = S[P][h];
  for (int j = threadIdx.x; j < n1; j += blockDim.x) db1[j] = SW2[P][j];
  for (int i = threadIdx.x; i < n0 * n1; i += blockDim.x) {   // dW1 = W0^T (S W2^T) + b0 (s W2^T)^T
    const int a = i / n1, j = i % n1;
    float v = b0[a] * SW2[P][j];
    for (int p = 0; p < P; ++p) v += w.W0[p][a] * SW2[p][j];
    dW1[i] = v;
  }
  for (int i = threadIdx.x; i < R * n0; i += blockDim.x) {    // dW0 = (S W2^T) W1^T, db0 = (s W2^T) W1^T
    const int p = i / n0, a = i % n0;
    float v = 0.f;
    for (int j = 0; j < n1; ++j) v += SW2[p][j] * w.W1[a][j];
    if (p < P) dW0[i] = v;
    else db0[a] = v;
  }
}
// the collapsed theta-branch weights (one block): Wc = W0 W1 W2 [P][H], bc = (b0 W1 + b1) W2 + b2 [H]
__global__ __launch_bounds__(256) void theta_branch_fold_kernel(int P, int n0, int n1, int H,
                                                                 const float* __restrict__ W0g,
                                                                 const float* __restrict__ b0,
                                                                 const float* __restrict__ W1g,
                                                                 const float* __restrict__ b1,
                                                                 const float* __restrict__ W2g,
                                                                 const float* __restrict__ b2, float* __restrict__ Wc,
                                                                 float* __restrict__ bc) {
  __shared__ TbW w;
  __shared__ float W01[9][kTbMax];   // rows 0..P-1: W0 W1, row P: b0 W1 + b1
  tb_stage(w, P, n0, n1, H, W0g, W1g, W2g);
  __syncthreads();
  for (int i = threadIdx.x; i < (P + 1) * n1; i += 256) {
    const int p = i / n1, j = i % n1;
    float v = p < P ? 0.f : b1[j];
    for (int a = 0; a < n0; ++a) v += (p < P ? w.W0[p][a] : b0[a]) * w.W1[a][j];
    W01[p][j] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (P + 1) * H; i += 256) {
    const int p = i / H, h = i % H;
    float v = p < P ? 0.f : b2[h];
    for (int j = 0; j < n1; ++j) v += W01[p][j] * w.W2[j][h];
    if (p < P) Wc[p * H + h] = v;
    else bc[h] = v;
  }
}

// theta_term[b][h] = theta[b] Wc[:, h] + bc[h]: lane h, each wave kTermRows rows with their loads in flight together
constexpr int kTermRows = 16;
template <int P>
__global__ __launch_bounds__(256) void theta_branch_term_kernel(int B, int H, const float* __restrict__ theta,
                                                                 const float* __restrict__ Wc,
                                                                 const float* __restrict__ bc,
                                                                 float* __restrict__ out) {
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kTermRows, h = threadIdx.x & 63;
  if (r0 >= B || h >= H) return;
  float wc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) wc[p] = Wc[p * H + h];
  const float c = bc[h];
  float t[kTermRows][P];
#pragma unroll
  for (int i = 0; i < kTermRows; ++i) {
    const int r = min(r0 + i, B - 1);
#pragma unroll
    for (int p = 0; p < P; ++p) t[i][p] = theta[r * P + p];
  }
#pragma unroll
  for (int i = 0; i < kTermRows; ++i) {
    if (r0 + i >= B) break;
    float v = c;
#pragma unroll
    for (int p = 0; p < P; ++p) v += t[i][p] * wc[p];
    out[static_cast<size_t>(r0 + i) * H + h] = v;
  }
}
}  // namespace
}  // namespace vissm

extern "C" {
using namespace vissm;

size_t vissm_theta_branch_bwd_workspace_size(int32_t B, int32_t P) {
  if (B < 1 || P < 1 || P > 8) return 0;
  const size_t waves = (static_cast<size_t>(B) + kTbRows - 1) / kTbRows;
  return align_up(((waves + 3) / 4) * (P + 1) * kTbMax * sizeof(float));
}

int vissm_theta_branch_bwd(int32_t B, int32_t P, int32_t n0, int32_t n1, int32_t H, const float* theta,
                           const float* dterm, const float* W0, const float* b0, const float* W1, const float* b1,
                           const float* W2, float* dtheta, float* dW0, float* db0, float* dW1, float* db1,
                           float* dW2, float* db2, void* workspace, size_t ws_bytes, void* stream) {
  VISSM_CHECK_ARG(B >= 1 && P >= 1 && P <= 8 && n0 >= 1 && n0 <= kTbMax && n1 >= 1 && n1 <= kTbMax && H >= 1 &&
                      H <= kTbMax,
                  "theta_branch_bwd: bad shape (B >= 1, P <= 8, n0 / n1 / H <= %d)", kTbMax);
  VISSM_CHECK_ARG(theta && dterm && W0 && b0 && W1 && b1 && W2 && dtheta && dW0 && db0 && dW1 && db1 && dW2 && db2,
                  "theta_branch_bwd: null pointer");
  VISSM_CHECK_ARG(workspace && ws_bytes >= vissm_theta_branch_bwd_workspace_size(B, P),
                  "theta_branch_bwd: workspace too small");
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  const int waves = (B + kTbRows - 1) / kTbRows;
  const int blocks = (waves + 3) / 4;
  switch (P) {
#define TB_CASE(PP)                                                                                             \
  case PP:                                                                                                      \
    hipLaunchKernelGGL(theta_branch_pass_kernel<PP>, dim3(blocks), dim3(256), 0, st, B, n0, n1, H, theta, dterm, \
                       W0, W1, W2, dtheta, part);                                                              \
    break;
    TB_CASE(1) TB_CASE(2) TB_CASE(3) TB_CASE(4) TB_CASE(5) TB_CASE(6) TB_CASE(7) TB_CASE(8)
#undef TB_CASE
  }
  VISSM_CHECK_LAUNCH("theta_branch_pass");
  // (waves past ceil(B / kTbRows) in the last block add zero partials)
  hipLaunchKernelGGL(theta_branch_finish_kernel, dim3(1), dim3(1024), 0, st, blocks, P, n0, n1, H, part, W0, b0,
                     W1, b1, W2, dW0, db0, dW1, db1, dW2, db2);
  VISSM_CHECK_LAUNCH("theta_branch_finish");
  return VISSM_OK;
}


int vissm_theta_branch_fwd(int32_t B, int32_t P, int32_t n0, int32_t n1, int32_t H, const float* theta,
                           const float* W0, const float* b0, const float* W1, const float* b1, const float* W2,
                           const float* b2, float* Wc, float* bc, float* theta_term, void* stream) {
  VISSM_CHECK_ARG(B >= 0 && P >= 1 && P <= 8 && n0 >= 1 && n0 <= kTbMax && n1 >= 1 && n1 <= kTbMax && H >= 1 &&
                      H <= kTbMax,
                  "theta_branch_fwd: bad shape (B >= 0, P <= 8, n0 / n1 / H <= %d)", kTbMax);
  VISSM_CHECK_ARG(W0 && b0 && W1 && b1 && W2 && b2 && Wc && bc && (B == 0 || !theta_term || theta),
                  "theta_branch_fwd: null pointer");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(theta_branch_fold_kernel, dim3(1), dim3(256), 0, st, P, n0, n1, H, W0, b0, W1, b1, W2, b2, Wc,
                     bc);
  VISSM_CHECK_LAUNCH("theta_branch_fold");
  if (theta_term && B > 0) {
    const dim3 grid(static_cast<unsigned>((B + 4 * kTermRows - 1) / (4 * kTermRows)));
    switch (P) {
#define TT_CASE(PP)                                                                                         \
  case PP:                                                                                                  \
    hipLaunchKernelGGL(theta_branch_term_kernel<PP>, grid, dim3(256), 0, st, B, H, theta, Wc, bc, theta_term); \
    break;
      TT_CASE(1) TT_CASE(2) TT_CASE(3) TT_CASE(4) TT_CASE(5) TT_CASE(6) TT_CASE(7) TT_CASE(8)
#undef TT_CASE
    }
    VISSM_CHECK_LAUNCH("theta_branch_term");
  }
  return VISSM_OK;
}

}  // extern "C"
