/*
 * vissm.h -- C ABI of libvissm.so, the MI355X (gfx950) kernels of the
 * neural-moving-average variational-inference ELBO step.
 *
 * The reference (mehrnazmo/VIforSSMs) is TensorFlow-1.8 Python: it has no FFI.
 * Every entry point below replaces a group of TF ops that the reference builds
 * inside VI_SSM.build_flow() and runs each step through sess.run (AR.py:300-301);
 * the reference interface each one replaces is cited next to it.  The Python
 * host (viforssms_amd/, loaded through ctypes) mirrors the reference's
 * Python API on top of these calls: VI_SSM / Flow_Stack / IAF (AR.py:24-362,
 * lotka_volterra_partial.py, SV_dense.py, fitz_nag_NVP.py) and
 * optimisers.adamax.AdamaxOptimizer (optimisers/adamax.py:11-61).
 *
 * Conventions
 *   - every buffer is a caller-owned DEVICE pointer (fp32 unless stated);
 *     layouts are row-major with the TF variable layouts for weights
 *     (dense [in][out], conv1d [k][C_in][C_out]).
 *   - every call takes the HIP stream to launch on (hipStream_t passed as
 *     void*); there is no implicit device synchronisation, no hipSetDevice and
 *     no allocation on the call path: scratch comes from a caller workspace
 *     sized by the matching *_workspace_size() query.
 *   - return value 0 = OK, negative = error (VISSM_E*); vissm_last_error()
 *     returns a thread-local message for the last failing call.  Nothing
 *     throws across the ABI and nothing exits.
 *   - reductions are fixed-order (partial slabs + ordered tree), so results
 *     are bitwise reproducible run to run; no float atomics.
 */
#ifndef VISSM_H
#define VISSM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VISSM_OK 0
#define VISSM_EINVAL (-1)   /* bad shape / argument */
#define VISSM_ELAUNCH (-2)  /* HIP launch or runtime failure */
#define VISSM_EWORKSPACE (-3)

#define VISSM_PREC_FP32 0     /* exact fp32 arithmetic */
#define VISSM_PREC_BF16 1     /* bf16 MFMA operands, fp32 accumulation */
#define VISSM_PREC_BF16X3 2   /* split-bf16 (hi/lo) MFMA operands: ~fp32 products */
#define VISSM_PREC_BF16X2 3   /* split-bf16 weights, bf16 activations: every product with a weight operand as
                                 w_hi x + w_lo x (two MFMAs), the forward, the backward's recompute and its chain
                                 (W dZ, w_eps dA0, the head backward) alike; the weight-gradient products
                                 (activation x gradient) single bf16.  ELBO within 1e-4 and gradient within 1e-3 of
                                 the float64 oracle at the AR configurations (one hidden layer, k <= 32) */
#define VISSM_PREC_BF16X2_BF16 4  /* vissm_flow_ar_elbo_fused only: the recompute (x, log sigma) on split weights,
                                     the backward products bf16 -- the last flow of a step whose forward runs at
                                     VISSM_PREC_BF16X2 and backward at VISSM_PREC_BF16 (k <= 8, one window) */

const char* vissm_last_error(void);
int vissm_version(void);
/* sha256 (hex) of the sources the library was built from (viforssms_amd/srchash.py); the Python host refuses a
 * library whose hash differs from its source tree.  vissm_build_flags: extra compile flags of an A/B build ("" for
 * the production build). */
const char* vissm_source_hash(void);
const char* vissm_build_flags(void);

/* ---------------------------------------------------------------------------
 * Base noise: init_dist.slp (AR.py:24-35; lotka_volterra_partial.py:25-36).
 * eps[b][j] ~ N(0,1) from counter-based Philox4x32-10 keyed by (seed, offset+b),
 * base_lp[b] = sum_{j >= L - n_last} log N(eps[b][j]; 0, 1).
 * ------------------------------------------------------------------------- */
int vissm_normal_base(uint64_t seed, uint64_t offset, float* eps, float* base_lp,
                      int32_t B, int32_t L, int32_t n_last, void* stream);

/* As vissm_normal_base with the row offset read from device memory (*offset_dev): a captured
 * HIP graph of the training step advances it on the device between replays. */
int vissm_normal_base_dev(uint64_t seed, const uint64_t* offset_dev, float* eps, float* base_lp,
                          int32_t B, int32_t L, int32_t n_last, void* stream);

/* base_lp only, for caller-supplied eps (parity mode). */
int vissm_base_logprob(const float* eps, float* base_lp, int32_t B, int32_t L,
                       int32_t n_last, void* stream);

/* ---------------------------------------------------------------------------
 * One IAF flow of the neural-MA sampler: IAF._create_flow + IAF.slp
 * (AR.py:50-89; lotka_volterra_partial.py:68-108 stride-2/BN variant;
 *  SV_dense.py:50-89; fitz_nag_NVP.py:68-109) with the window-shared part of
 * the first conv (feature branch, conv over features, conv bias) and the theta
 * branch precomputed by the caller:
 *
 *   a0[b,m,:] = C[win[b], m, :] + theta_term[b, :] + sum_j u[b, s*m + j] * w_eps[j, :]
 *   x_0 = elu(a0);  x_{l+1} = bn_l(elu(x_l W_l + b_l))     (l < n_hidden)
 *   (mu, r) = x_nh W_head + b_head;  sigma = softplus(r) + 1e-10
 *   stride 1: u_next[t] = u[t+k] * sigma[t] + mu[t]
 *   stride 2: u_next[2m] = u[2m+k];  u_next[2m+1] = u[2m+1+k] * sigma[m] + mu[m]
 *   logsig[b] = sum of log sigma over the last n_logsig outputs.
 * swap_out != 0 writes u_next with adjacent pairs swapped (the Permute flow of
 * the 2-D models, lotka_volterra_partial.py:137-159, fused into the store).
 * ------------------------------------------------------------------------- */
typedef struct {
  int32_t B;          /* samples (reference p) */
  int32_t L;          /* input length per sample; output length is L - k */
  int32_t k;          /* kernel_len, 1..64 */
  int32_t H;          /* network_dims[i], 1..64 (all equal) */
  int32_t n_hidden;   /* len(network_dims) - 2, 0..4 */
  int32_t bn;         /* batch_normalization(training=False) after each hidden ELU */
  int32_t stride2;    /* 2-D interleaved head (stride 2, (0,1) interleave) */
  int32_t swap_out;   /* fuse the pair-swap permutation into the output store */
  int32_t n_logsig;   /* trailing outputs counted in log q: M (1-D) or 2M (2-D) */
  int32_t n_win;      /* windows in C (1 when every sample shares one window) */
  int32_t precision;  /* VISSM_PREC_* */
  int32_t chunk_tiles; /* 0 = automatic launch geometry; > 0 = head-position tiles per t-chunk of
                          a work item (the kernel's tile size; raised to the halo minimum).  Lets a
                          small batch run the chunk geometry of a large one: a parity test at B = 20
                          walks the ~160-tile chunks the B = 65536 benchmark launch walks. */
  int32_t u_pitch;    /* row stride of u and du in floats (0 = L; else >= L).  A caller that pads rows to
                         16 floats (64 bytes) gets aligned du stores from the t-chunks of the two-sample
                         bf16 backward, which otherwise straddle 32-byte write sectors (+55 % du bytes). */
  int32_t out_pitch;  /* row stride of u_next / du_next in floats (0 = L - k; else >= L - k); the fused
                         AR(1) last flow writes x dense [B][M+1] and takes 0 or L - k */
} VissmFlowDesc;

typedef struct {
  const float* w_eps;   /* [k][H]      conv1d kernel, input channel 0 (the sample) */
  const float* w_hid;   /* [n_hidden][H][H] conv1d k=1 kernels */
  const float* b_hid;   /* [n_hidden][H] */
  const float* bn_g;    /* [n_hidden][H] or NULL (bn == 0) */
  const float* bn_b;    /* [n_hidden][H] or NULL */
  const float* w_head;  /* [H][2]  (col 0 = mu, col 1 = sigma pre-softplus) */
  const float* b_head;  /* [2] */
  /* Optional factorization of the theta branch (AR.py:63-68: three linear dense layers, so
   * theta_term = theta_x w_theta + b_theta exactly).  theta_rank = 0 (or NULL pointers): unused.
   * With 1 <= theta_rank <= 5 the bf16 AR kernels (one hidden layer, k <= 16, one window) form the
   * theta term inside their layer-0 matrix product (split-bf16 theta and w_theta in its unused K
   * rows) and add b_theta to C, instead of reading a [H] theta_term row per sample and unit; every
   * other kernel reads theta_term.  theta_term must still be passed and equal the product. */
  const float* theta_x; /* [B][theta_rank] per-sample theta (the q(theta) draw) */
  const float* w_theta; /* [theta_rank][H] collapsed weight W0 W1 W2 */
  const float* b_theta; /* [H] collapsed bias */
  int32_t theta_rank;
} VissmFlowParams;

typedef struct {        /* outputs of the backward: written, not accumulated */
  float* w_eps; float* w_hid; float* b_hid; float* bn_g; float* bn_b;
  float* w_head; float* b_head;
} VissmFlowGrads;

/* C is [n_win][Lh][H] with Lh = (L-k) (stride 1) or (L-k)/2 (stride 2);
 * win is [B] int32 window index per sample (NULL = all 0). */
size_t vissm_flow_workspace_size(const VissmFlowDesc* d, int32_t backward);

/* The launch geometry the flow kernels pick for d (host-side arithmetic, no GPU call): out[0] = head
 * positions per tile, out[1] = tiles per t-chunk of a work item, out[2] = t-chunks, out[3] = sample
 * groups.  which: 0 vissm_flow_fwd, 1 vissm_flow_bwd, 2 vissm_flow_ar_elbo_fused.  No reference
 * equivalent (TF1 has no launch geometry): the parity tests read it at a benchmark batch and pass
 * out[1] as chunk_tiles at a small one. */
int vissm_flow_geometry(const VissmFlowDesc* d, int32_t which, int32_t* out);

/* The precision vissm_flow_fwd / vissm_flow_bwd compute a descriptor in: its own where the matrix-core kernels cover
 * the shape, VISSM_PREC_FP32 where the call falls back to the exact-fp32 kernels (bf16 / bf16x3 / bf16x2 requests
 * beyond flow5's shapes: never less precise than asked; du must then be non-NULL).  Host arithmetic, no GPU;
 * VISSM_EINVAL for an invalid descriptor or VISSM_PREC_BF16X2_BF16 (a fused-flow precision). */
int32_t vissm_flow_kernel_precision(const VissmFlowDesc* d);

int vissm_flow_fwd(const VissmFlowDesc* d, const VissmFlowParams* w,
                   const float* u, const float* C, const int32_t* win,
                   const float* theta_term, float* u_next, float* logsig,
                   void* workspace, size_t ws_bytes, void* stream);

/* Backward of vissm_flow_fwd for a scalar loss.  du_next = dLoss/du_next (in
 * the stored, possibly swapped layout), dlogsig[b] = dLoss/dlogsig[b].
 * Writes du [B][L], dC [n_win][Lh][H], dtheta_term [B][H] and the weight
 * gradients.  du may be NULL on the bf16 / bf16x3 kernels when the gradient
 * w.r.t. u is not wanted (the first flow: u is the base noise). */
int vissm_flow_bwd(const VissmFlowDesc* d, const VissmFlowParams* w,
                   const float* u, const float* C, const int32_t* win,
                   const float* theta_term, const float* du_next,
                   const float* dlogsig, float* du, float* dC,
                   float* dtheta_term, const VissmFlowGrads* g,
                   void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * The last flow of the AR(1) stack fused with its ELBO terms: forward AND backward of
 * IAF._create_flow / IAF.slp (AR.py:50-89) for the final flow together with VI_SSM._ELBO's
 * AR(1) transition and observation terms (AR.py:168-176), for the loss
 *     loss = -scale * sum_b (sde_b + obs_b + logsig_b)        (scale = T / M, AR.py:184)
 * i.e. the part of -sum_b ELBO_b (AR.py:228-229) that depends on this flow.  The kernel
 * recomputes the flow's output x = u_next itself and evaluates the gradient of the AR(1) terms
 * on the fly, so vissm_flow_fwd for this flow and the ELBO backward's dz are not needed.  theta is
 * the per-sample AR(1) theta [B][3], obs / obs_bin the per-window feeds [n_win][M] (M = L - k - 1).
 * Writes x [B][M+1] (the latent path; the caller takes sde / obs and their theta gradient from it
 * with vissm_elbo_fwd / vissm_elbo_bwd), logsig [B] (the n_logsig counted outputs), du [B][L],
 * dC [n_win][Lh][H], dtheta_term [B][H] and the weight gradients of the loss.
 * Supported: bf16 / bf16x3, one hidden layer, no BN, stride 1, k <= 32. */
int32_t vissm_flow_ar_elbo_fused_supported(const VissmFlowDesc* d);
size_t vissm_flow_ar_elbo_fused_workspace_size(const VissmFlowDesc* d);
int vissm_flow_ar_elbo_fused(const VissmFlowDesc* d, const VissmFlowParams* w,
                             const float* u, const float* C, const int32_t* win,
                             const float* theta_term, const float* theta,
                             const float* obs, const float* obs_bin, float obs_std,
                             float scale, float* x, float* logsig, float* du,
                             float* dC, float* dtheta_term, const VissmFlowGrads* g,
                             void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * ELBO log-densities over a path, one model per id:
 *   AR  : VI_SSM._ELBO obs + AR(1) terms (AR.py:168-176)
 *   LV  : softplus transform + ILDJ (lotka_volterra_partial.py:290-297),
 *         obs N(.,1) and Cholesky EM density (lotka_volterra_partial.py:234-261)
 *   SV  : dim-one concat + mask/shift (SV_dense.py:245-246), diag EM density (SV_dense.py:203-223)
 *   FHN : obs N(.,0.1) and diag EM density (fitz_nag_NVP.py:232-255)
 * z is the flow output [B][D*(M+1)] (2-D models interleaved t-major).
 * Outputs per sample: sde[b], obs[b] (0 for SV) and extra[b] (LV: ILDJ, else 0).
 * ------------------------------------------------------------------------- */
#define VISSM_MODEL_AR 0
#define VISSM_MODEL_LV 1
#define VISSM_MODEL_SV 2
#define VISSM_MODEL_FHN 3

typedef struct {
  int32_t model;
  int32_t B;
  int32_t M;          /* transitions per path (reference batch_dims) */
  int32_t n_win;
  float dt;           /* Euler-Maruyama step (LV/SV/FHN) */
  float obs_std;      /* AR observation sd */
} VissmElboDesc;

typedef struct {
  const int32_t* win;     /* [B] or NULL */
  const float* obs;       /* [n_win][D][M] observation window (AR: [n_win][M]) */
  const float* obs_bin;   /* [n_win][D][M] observation mask */
  const float* mask;      /* LV [n_win][2][M+1]; SV [n_win][M+1]; else NULL */
  const float* shift;     /* same shape as mask */
  const float* dim_one;   /* SV observed coordinate [n_win][M+1]; else NULL */
  const int32_t* plain_from; /* LV / SV, optional [n_win]: from this element on, the window's mask is 1 and its
                                shift 0 (the state is softplus(z) / z itself: the reference's windows pin x_0 only,
                                lotka_volterra_partial.py:381-384, SV_dense.py:322-328); NULL: mask / shift read
                                everywhere.  vissm_elbo_fwd_grad skips their loads and the general transform there. */
  const int32_t* obs_list;   /* LV / FHN, optional [n_win][obs_stride]: the elements e in [1, M] whose observation row
                                e - 1 has a nonzero obs_bin in either coordinate, ascending, padded with -1 (the
                                reference's obs_bin files are sparse: dat/LV_obs_binary.txt, loaded at
                                lotka_volterra_partial.py:481-487, observes every 100th step; fitz_nag_NVP.py:468-473
                                loads its own); NULL: the obs rows are read at every element.  With it
                                vissm_elbo_fwd_grad evaluates the observation term at the listed elements only. */
  int32_t obs_stride;        /* entries per window in obs_list */
} VissmElboData;

int vissm_elbo_fwd(const VissmElboDesc* d, const VissmElboData* data,
                   const float* z, const float* theta, float* sde, float* obs,
                   float* extra, void* stream);

/* dLoss/d(sde, obs, extra) per sample -> dz [B][D*(M+1)], dtheta [B][P_theta].  dz may be NULL
 * (only dtheta wanted, e.g. after vissm_flow_ar_elbo_fused, which differentiates through x itself). */
int vissm_elbo_bwd(const VissmElboDesc* d, const VissmElboData* data,
                   const float* z, const float* theta, const float* g_sde,
                   const float* g_obs, const float* g_extra, float* dz,
                   float* dtheta, void* stream);

/* vissm_elbo_fwd and the theta gradient of vissm_elbo_bwd with dz = NULL, for a path z that is a
 * constant (the training step after vissm_flow_ar_elbo_fused): sde, obs (and extra) per sample and
 * dtheta = d(g_sde . sde + g_obs . obs + g_extra . extra)/dtheta.  AR(1): one pass over z (the two calls
 * would read it twice); other models: the two calls.  Same reference terms as vissm_elbo_fwd. */
int vissm_elbo_fwd_theta_grad(const VissmElboDesc* d, const VissmElboData* data, const float* z,
                              const float* theta, const float* g_sde, const float* g_obs,
                              const float* g_extra, float* sde, float* obs, float* extra,
                              float* dtheta, void* stream);

/* vissm_elbo_fwd and vissm_elbo_bwd in ONE pass over z, for upstream gradients known before the forward (the
 * training step's loss -sum_b ELBO_b: g_sde = -scale, g_obs = -scale, g_extra = +scale per sample): sde, obs,
 * extra (obs / extra may be NULL), dz and dtheta, every element's transition, obs row and ILDJ term evaluated once
 * (the forward values are the backward's own transition records).  Replaces the two launches of the ELBO
 * (AR.py:168-187, lotka_volterra_partial.py:234-297, SV_dense.py:203-232, fitz_nag_NVP.py:232-265 and their
 * tf.gradients) for every model. */
int vissm_elbo_fwd_grad(const VissmElboDesc* d, const VissmElboData* data, const float* z, const float* theta,
                        const float* g_sde, const float* g_obs, const float* g_extra, float* sde, float* obs,
                        float* extra, float* dz, float* dtheta, void* stream);

/* ---------------------------------------------------------------------------
 * Global-norm clip + Adamax over one flat parameter buffer:
 * tf.global_norm / tf.clip_by_global_norm (AR.py:230-232) followed by
 * AdamaxOptimizer._apply_dense (optimisers/adamax.py:42-58):
 *   g <- g * clip * min(1/||g||, 1/clip)   (NaN when ||g|| is not finite)
 *   v <- beta1 v + (1-beta1) g ;  m <- max(beta2 m + eps, |g|) ;  p <- p - lr v/m
 * clip <= 0 disables clipping.  gnorm_out (device, 1 float, may be NULL)
 * receives ||g|| before clipping.
 * ------------------------------------------------------------------------- */
size_t vissm_adamax_workspace_size(int64_t n);
int vissm_adamax_step(float* params, const float* grads, float* v, float* m,
                      int64_t n, float lr, float beta1, float beta2, float eps,
                      float clip, float* gnorm_out, void* workspace,
                      size_t ws_bytes, void* stream);

/* As vissm_adamax_step, with the non-finite guard of the training loop: when ||g||
 * is not finite -- where tf.clip_by_global_norm would write NaN into every variable
 * (AR.py:230-232) -- params, v and m are left untouched and *skipped (device int32, may be NULL)
 * is incremented.  The decision is made on the device: no host synchronisation. */
int vissm_adamax_step_guarded(float* params, const float* grads, float* v, float* m,
                              int64_t n, float lr, float beta1, float beta2, float eps,
                              float clip, float* gnorm_out, int32_t* skipped, void* workspace,
                              size_t ws_bytes, void* stream);

/* Sum of squares of a flat buffer (fixed-order), result to out[0] (device float). */
int vissm_sqnorm(const float* x, int64_t n, float* out, void* workspace,
                 size_t ws_bytes, void* stream);

/* out[c] = sum_r slab[r][c] for r = 0..R-1 in fixed order (deterministic reduce). */
int vissm_reduce_rows(const float* slab, float* out, int64_t R, int64_t N,
                      void* stream);

/* The same over a bf16 slab (each element widened to fp32, rows summed in order r = 0..R-1 in
 * fp32): the flow backward's window-shared dC partials at bf16 products (one row per 16-sample
 * group: 4096 rows at the B = 65536 benchmark), exported for its parity test. */
int vissm_reduce_rows_bf16(const void* slab, float* out, int64_t R, int64_t N, void* stream);

/* x[0..n) = hi + lo (bf16 planes, hi = bf16(x), lo = bf16(x - hi), round to nearest even): the operands of the
 * split-bf16 GEMMs of LV's window-shared conv over its time-mixing features (no reference equivalent: the
 * reference runs that conv in fp32, lotka_volterra_partial.py:78-82).  x 16-byte aligned, hi / lo 8-byte. */
int vissm_split_bf16(const float* x, void* hi, void* lo, int64_t n, void* stream);

/* ---------------------------------------------------------------------------
 * Window-shared feature branch + the first conv's feature channels (AR.py:53-62;
 * SV_dense.py:53-62; fitz_nag_NVP.py:71-79): per window w,
 *   F = elu(elu(elu(elu(h0 W0 + b0) W1 + b1) W2 + b2) W3 + b3)        [Lf][H]
 *   C[w][m][o] = conv_b[o] + sum_{j<k} sum_{i<H} F[s m + j][i] conv_w[j][1 + i][o],  m < Lh
 * (the sample channel conv_w[j][0][:] is the flow kernel's w_eps).  h0: the window's
 * time-feature rows, Lf rows of Cin floats, windows in_win_stride floats apart.
 * fwd writes C [n_win][Lh][H] and the four layer outputs act [4][n_win][Lf][H] (rows
 * s (Lh - 1) + k .. Lf - 1 unused); bwd takes dC and writes (not accumulates) the
 * gradients of W0..W3, b0..b3, conv_w (its sample channel 0) and conv_b.
 * Replaces the four tf.layers.dense and the feature part of tf.layers.conv1d with
 * their gradients.  Cin <= 63, H <= 64, k <= 64, stride 1 | 2; deterministic.
 * ------------------------------------------------------------------------- */
typedef struct {
  int32_t n_win, Lf, Cin, H, k, stride, Lh;
  int64_t in_win_stride;
} VissmFeatDesc;

typedef struct {
  const float* w[4];    /* W0 [Cin][H], W1..W3 [H][H] */
  const float* b[4];    /* [H] */
  const float* conv_w;  /* [k][1 + H][H] */
  const float* conv_b;  /* [H] */
} VissmFeatParams;

typedef struct {
  float* w[4];
  float* b[4];
  float* conv_w;
  float* conv_b;
} VissmFeatGrads;

size_t vissm_feat_workspace_size(const VissmFeatDesc* d);
int vissm_feat_fwd(const VissmFeatDesc* d, const VissmFeatParams* w, const float* h0, float* C, float* act,
                   void* stream);
int vissm_feat_bwd(const VissmFeatDesc* d, const VissmFeatParams* w, const float* h0, const float* act,
                   const float* dC, const VissmFeatGrads* g, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Lotka-Volterra's window-shared feature branch and first conv (lotka_volterra_partial.py:71-82): per window,
 *   H3 = elu(elu(elu(h0 W0 + b0) W1 + b1) W2 + b2)              [R][H]   (R = the window's time-feature rows)
 *   D  = elu(H3 W3 + b3)                                        [R][U]   (the time-mixing dense layer, transposed
 *                                                                         by the reference so that U is the conv's
 *                                                                         time axis and R its channels)
 *   C[m][h] = conv_b[h] + sum_{j<k} sum_{r<R} D[r][s m + j] conv_w[j][1 + r][h]
 * Replaces the four tf.layers.dense, the transpose and the feature part of tf.layers.conv1d with their gradients:
 * the three small layers in fp32 (vissm_lv_mlp_*), the time-mixing layer and the conv as bf16 matrix-core GEMMs
 * (vissm_gemm_bf16) on operands packed by vissm_lv_pack, the conv's diagonal sum and its transpose by
 * vissm_lv_conv_diag[_bwd], the conv weight gradient back to [k][1 + R][H] by vissm_lv_conv_wscatter
 * (viforssms_amd/ops.py LvFeatConvFn chains them).  mlp_fwd writes act [n_layers][n_win][R][H] (fp32 layer outputs)
 * and H3b [n_win][R][64] bf16 (the last layer's output, a ones column at H for W3b's bias row, zeros; H3lo, when not
 * null, the same layout holding the bf16 residual of each element, hi + lo = the fp32 value to ~2^-16); mlp_bwd
 * takes dH3 [n_win][R][ld] (columns < H) and writes the gradients of W0.., b0.. (the conv fields of the grads struct
 * unused).
 *
 * Stochastic volatility's branch (SV_dense.py:50-62: four dense + ELU layers over the window's features with their
 * first differences, then the conv over the 50 feature channels at k = 50) runs through the same entry points:
 * n_layers = 4, sv_diff = 1 (h0 is then the window's time features [L][Cr] and row r of the MLP input is
 * [h0[r + 1][0 .. Cr), h0[r + 1][c] - h0[r][c] for c < Cr - 2], so Cin = 2 Cr - 2 and R = L - 1), the conv as a
 * split-bf16 GEMM (vissm_gemm_bf16x3) on F = H3b / H3lo and the packed conv kernel (vissm_lv_pack with ldw = 0).
 * ------------------------------------------------------------------------- */
typedef struct {
  int32_t n_win, R, Cin, H;
  int64_t in_win_stride;
  int32_t n_layers;   /* dense + ELU layers in the MLP: 0 or 3 (LV), 4 (SV) */
  int32_t sv_diff;    /* 1: SV's first-difference input assembly (above) */
} VissmLvFeatDesc;

size_t vissm_lv_mlp_workspace_size(const VissmLvFeatDesc* d);
int vissm_lv_mlp_fwd(const VissmLvFeatDesc* d, const VissmFeatParams* w, const float* h0, float* act, void* H3b,
                     void* H3lo, void* stream);
int vissm_lv_mlp_bwd(const VissmLvFeatDesc* d, const VissmFeatParams* w, const float* h0, const float* act,
                     const float* dH3, int ld_dH3, const VissmFeatGrads* g, void* workspace, size_t ws_bytes,
                     void* stream);
/* W3b [64][ldw] bf16 (rows < H: w3 [H][U], row H: b3, zeros; columns >= U zero; ldw = 0: none, w3 / b3 / W3b
 * unused) and Wc [R][ldc] bf16 (Wc[r][j H + h] = conv_w[j][1 + r][h], zero for columns >= k H); W3b_lo / Wc_lo,
 * when not null, their bf16 residual planes (the split-bf16 GEMM's operands) */
int vissm_lv_pack(const float* w3, const float* b3, int H, int U, int ldw, void* W3b, void* W3b_lo, const float* conv_w,
                  int R, int k, int ldc, void* Wc, void* Wc_lo, void* stream);
/* C[m][h] = conv_b[h] + sum_{j<k} G[s m + j][j H + h], G [U][ldg] fp32, m < Lh */
int vissm_lv_conv_diag(const float* G, int ldg, const float* conv_b, int H, int k, int stride, int Lh, float* C,
                       void* stream);
/* its transpose: dG[u][j H + h] = dC[(u - j) / s][h] where that is a position (bf16 [U][ldg], zero elsewhere; dG_lo,
 * when not null, the bf16 residual plane), and dconv_b[h] = sum_m dC[m][h] */
int vissm_lv_conv_diag_bwd(const float* dC, int H, int k, int stride, int Lh, int U, int ldg, void* dG, void* dG_lo,
                           float* dconv_b, void* stream);
/* dconv_w[j][1 + r][h] = dWc[r][j H + h]; channel 0 (the flow kernel's w_eps) = 0 */
int vissm_lv_conv_wscatter(const float* dWc, int ldc, int R, int k, int H, float* dconv_w, void* stream);

/* ---------------------------------------------------------------------------
 * bf16 matrix-core GEMM: C[m][n] = sum_k A[m][k] B[k][n], fp32 accumulation (the LV feature branch's products).
 * A: a_kmajor = 0: A[m][k] at A[m lda + k]; 1: at A[k lda + m].  B: b_kmajor = 0: B[k][n] at B[n ldb + k]; 1: at
 * B[k ldb + n].  lda, ldb multiples of 8, A and B 16-byte aligned.  Epilogues: VISSM_GEMM_F32 (fp32 C[m ldc + n]),
 * VISSM_GEMM_ELU_BF16 (bf16 elu(acc)), VISSM_GEMM_DELU_BF16 (bf16 acc * elu'(y), y = aux[m ldc + n] a bf16 ELU
 * output: y < 0 ? y + 1 : 1).  split_k > 1 (fp32 epilogue, ldc == N): per-split partials in the workspace summed in
 * split order (deterministic).
 * ------------------------------------------------------------------------- */
#define VISSM_GEMM_F32 0
#define VISSM_GEMM_ELU_BF16 1
#define VISSM_GEMM_DELU_BF16 2
typedef struct {
  int64_t M, N, K, lda, ldb, ldc;
  int32_t a_kmajor, b_kmajor, epilogue, split_k;
} VissmGemmDesc;

size_t vissm_gemm_workspace_size(const VissmGemmDesc* d);
int vissm_gemm_bf16(const VissmGemmDesc* d, const void* A, const void* B, void* C, const void* aux, void* workspace,
                    size_t ws_bytes, void* stream);
/* The split-bf16 form (fp32-class products: the operands' hi / lo bf16 planes, x = hi + lo to ~2^-16, the same
 * layouts): C = A_hi B_hi + A_hi B_lo + A_lo B_hi, one launch whose K loop runs the three passes (split-K divides
 * the 3 K range).  Every epilogue: the bf16 ones write C as a hi / lo plane pair (the lo plane at C + M ldc) and
 * read aux the same way (y = aux_hi + aux_lo). */
size_t vissm_gemm_bf16x3_workspace_size(const VissmGemmDesc* d);
int vissm_gemm_bf16x3(const VissmGemmDesc* d, const void* A_hi, const void* A_lo, const void* B_hi, const void* B_lo,
                      void* C, const void* aux, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Window gather: the per-step feed assembly of VI_SSM.train (AR.py:267-288;
 * lotka_volterra_partial.py:366-386; SV_dense.py:304-328) from device-resident
 * padded channel tables (built once, AR.py:135-150), keyed by the step's window
 * starts (batch_select):
 *   out[r*os_r + j*os_j + c*os_c] = src[c*c_pitch + stride*starts[r] + offset + j*j_step]
 * for r < n, j < len, c < C.  time_feats [n][kernel_ext][C]: c_pitch = table
 * length, os = (kernel_ext*C, C, 1); per-window feeds [n][D][len] from a [D][..]
 * table: os = (D*len, 1, len).  The caller guarantees every source index lies in
 * the table (the reference's starts come from arange(0, T, M)).
 * ------------------------------------------------------------------------- */
typedef struct {
  int32_t n, len, C;        /* windows, positions per window, channels */
  int32_t stride;           /* start multiplier (2 for the interleaved 2-D series) */
  int64_t offset, j_step, c_pitch;
  int64_t os_r, os_j, os_c; /* output strides (elements) */
} VissmGatherDesc;

int vissm_gather_windows(const VissmGatherDesc* d, const float* src, const int32_t* starts,
                         float* out, void* stream);

/* ---------------------------------------------------------------------------
 * q(theta): the variational posterior over the SDE parameters (AR.py:376-391;
 * lotka_volterra_partial.py:494-508; SV_dense.py:428-442; fitz_nag_NVP.py:480-494):
 * n_bij bijectors Invert(MaskedAutoregressiveFlow(MADE [5, 5, 5], elu | relu)) with
 * Permute between them over a Normal(base_loc, base_scale) base of P dimensions.
 *   fwd: theta [B][P] = chain(x0), logq [B] = log q(theta) (base log-prob + sum of
 *        the clipped log-scales, clip [-5, 3] straight-through).
 *   bwd: dw += d loss / d w for d loss / d theta = dtheta and d loss / d logq = dlogq
 *        (either may be NULL = 0); deterministic (fixed-order sums).
 * w, mask: every bijector's MADE variables in the parameter store's order -- dense0
 * kernel [P][5], bias [5], dense1 [5][5], bias, dense2 [5][5], bias, dense3 [5][2P],
 * bias [2P] -- vissm_theta_num_params(P, n_bij) floats; mask holds the MADE masks in
 * the same layout (1 on the biases).  perm[i][q]: after bijector i, z[q] <- z[perm[i][q]].
 * ------------------------------------------------------------------------- */
#define VISSM_THETA_MAX_P 5
#define VISSM_THETA_MAX_BIJ 8
typedef struct {
  int32_t B, P, n_bij, relu;  /* relu: 0 = elu (AR / LV / FHN), 1 = relu (SV) */
  float base_loc, base_scale;
  int32_t perm[VISSM_THETA_MAX_BIJ - 1][VISSM_THETA_MAX_P];
} VissmThetaDesc;

int32_t vissm_theta_num_params(int32_t P, int32_t n_bij);
size_t vissm_theta_workspace_size(const VissmThetaDesc* d);
int vissm_theta_fwd(const VissmThetaDesc* d, const float* w, const float* mask, const float* x0,
                    float* theta, float* logq, void* stream);
int vissm_theta_bwd(const VissmThetaDesc* d, const float* w, const float* mask, const float* x0,
                    const float* dtheta, const float* dlogq, float* dw, void* workspace,
                    size_t ws_bytes, void* stream);

/* The flows' theta branch backward (IAF._create_flow's three linear dense layers on theta, AR.py:63-68;
 * lotka_volterra_partial.py:84-89): theta_term = ((theta W0 + b0) W1 + b1) W2 + b2 with W0 [P][n0], W1 [n0][n1],
 * W2 [n1][H]; given dterm = d loss / d theta_term [B][H] it writes dtheta [B][P] and the six weight gradients
 * (overwritten, not accumulated).  P <= 8, n0 / n1 / H <= 64; deterministic (fixed-order sums); workspace from
 * vissm_theta_branch_bwd_workspace_size(B, P) (0: bad shape). */
/* its forward: the collapsed weights Wc = W0 W1 W2 [P][H], bc = (b0 W1 + b1) W2 + b2 [H] (the factors the AR flow
 * kernels fold into their layer-0 product, VissmFlowParams.theta_rank) and, when theta_term is not NULL,
 * theta_term = theta Wc + bc [B][H]. */
int vissm_theta_branch_fwd(int32_t B, int32_t P, int32_t n0, int32_t n1, int32_t H, const float* theta,
                           const float* W0, const float* b0, const float* W1, const float* b1, const float* W2,
                           const float* b2, float* Wc, float* bc, float* theta_term, void* stream);
size_t vissm_theta_branch_bwd_workspace_size(int32_t B, int32_t P);
int vissm_theta_branch_bwd(int32_t B, int32_t P, int32_t n0, int32_t n1, int32_t H, const float* theta,
                           const float* dterm, const float* W0, const float* b0, const float* W1, const float* b1,
                           const float* W2, float* dtheta, float* dW0, float* db0, float* dW1, float* db1,
                           float* dW2, float* db2, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Opt-in kernel timing (for bench.py's live roofline): when enabled, the flow
 * entry points bracket their main kernel with hipEvents on the launch stream.
 * kind: VISSM_PROF_FLOW_FWD / VISSM_PROF_FLOW_BWD (flow kernels),
 * VISSM_PROF_ELBO_FWD / VISSM_PROF_ELBO_BWD (log-density kernels), VISSM_PROF_NORMAL
 * (base-noise kernel).  read() synchronises the
 * recorded events and returns the summed milliseconds and the launch count.
 * ------------------------------------------------------------------------- */
#define VISSM_PROF_FLOW_FWD 0
#define VISSM_PROF_FLOW_BWD 1
#define VISSM_PROF_ELBO_FWD 2
#define VISSM_PROF_ELBO_BWD 3
#define VISSM_PROF_NORMAL 4
/* the flow backward launches again, by variant (each launch is also counted in VISSM_PROF_FLOW_BWD):
 * without du (the first flow: its input is the base noise), with du (middle flows), and the last AR(1)
 * flow fused with its ELBO terms (vissm_flow_ar_elbo_fused) */
#define VISSM_PROF_FLOW_BWD_NODU 5
#define VISSM_PROF_FLOW_BWD_DU 6
#define VISSM_PROF_FLOW_FUSED 7
void vissm_profile_enable(int32_t on);
int vissm_profile_read(int32_t kind, double* total_ms, int64_t* count);
void vissm_profile_reset(void);
/* Summed algorithmic HBM bytes of the recorded launches of `kind` (the streaming kernels
 * state theirs: ELBO_FWD / ELBO_BWD / NORMAL; 0 for the flow kernels). */
int vissm_profile_bytes(int32_t kind, double* total_bytes);

#ifdef __cplusplus
}
#endif
#endif /* VISSM_H */
