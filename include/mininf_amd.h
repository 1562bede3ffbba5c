/*
 * mininf_amd.h -- C ABI of the MI355X (gfx950) ELBO hot path.
 *
 * The reference (tillahoffmann/mininf) is pure Python on PyTorch and has no FFI of its own; its
 * "operator API" for the ELBO path is three Python seams:
 *   1. the tracer plugin point  -- mininf/core.py:128-140 (TracerMixin.sample), dispatched from
 *      mininf/core.py:325-328 (sample);
 *   2. the Distribution protocol consumed at mininf/core.py:233-241 (log_prob) and
 *      mininf/nn.py:124-145, 217, 226 (rsample / entropy);
 *   3. the loss module mininf/nn.py:212-228 (EvidenceLowerBoundLoss.forward).
 * Every entry point below replaces the arithmetic behind one of those seams; the comment above each
 * one names the reference line(s) and the torch.distributions code it stands in for.
 *
 * Conventions (all entry points):
 *   - return 0 on success, a negative MI_E* code for an invalid argument, or a positive hipError_t;
 *   - never throw across the ABI, never allocate device memory (workspaces are caller-provided and
 *     sized by the matching *_workspace_bytes query), never synchronise the host;
 *   - asynchronous on the given stream (`stream` is a hipStream_t; NULL = the null stream);
 *   - tensors are device pointers plus int64 element strides over a logical [K, N] space
 *     (K = Monte-Carlo particles, N = flattened elements of one site); a stride of 0 broadcasts;
 *   - floating-point data is IEEE fp32 (the reference's default dtype); accumulation is fp32
 *     within a wavefront and fp64 across wavefronts.
 */
#ifndef MININF_AMD_H
#define MININF_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MI_ABI_VERSION 18

#define MI_MAX_SITES 4
#define MI_MAX_OPERANDS 6
#define MI_MAX_SLOTS 4

/* error codes (negative) */
#define MI_EINVAL (-1)      /* malformed descriptor or size */
#define MI_EWORKSPACE (-2)  /* workspace too small */
#define MI_EUNSUPPORTED (-3)

/* site families (torch.distributions formulas they restate are cited in sites.hip) */
enum mi_family {
  MI_NORMAL = 0,            /* roles: loc, scale, value          torch/distributions/normal.py:88-103 */
  MI_BERNOULLI_LOGITS = 1,  /* roles: logits, -, value            torch/distributions/bernoulli.py:121-125 */
  MI_BERNOULLI_PROBS = 2,   /* roles: probs, -, value (clamped)   bernoulli.py:104-106, utils.py:101-137 */
  MI_BETA = 3,              /* roles: concentration1, concentration0, value  beta.py:88-92, dirichlet.py:90-97 */
  MI_GAMMA = 4,             /* roles: concentration, rate, value  torch/distributions/gamma.py:90-99 */
  MI_POISSON = 5,           /* roles: rate, -, value              torch/distributions/poisson.py:60-65 */
  MI_INVERSE_GAMMA = 6      /* roles: concentration, rate, value  mininf/distributions.py:5-11: Gamma
                               through PowerTransform(-1), transformed_distribution.py:151-170 */
};

/* what to do with d(site total)/d(operand) */
enum mi_grad_mode {
  MI_GRAD_NONE = 0,
  MI_GRAD_DENSE = 1,     /* write g0 * dT_k/dx[k,i] to `grad` (same logical [K,N] space) */
  MI_GRAD_PARTICLE = 2   /* operand is one scalar per particle: reduce dT_k/dx[k] into slot `slot` */
};

/* flag bits reported per site */
/* mi_group.options: the caller has zeroed `flags` (e.g. one buffer for every group of a step),
 * so mi_group_forward does not reset them. */
#define MI_GROUP_FLAGS_ZEROED 1
/* mi_group.options: leave the fused draw's per-particle-block partial sums of dloc / dscale in the
 * workspace (mi_group_draw_partials) instead of reducing them into draw.dloc / draw.dscale -- the
 * ELBO backward reduces them (MI_DRAW_PARTIALS). */
#define MI_GROUP_DRAW_PARTIALS 2

#define MI_FLAG_SUPPORT 1u  /* a (non-masked) value lies outside the family's support */
#define MI_FLAG_PARAM 2u    /* a parameter violates its constraint (e.g. scale <= 0) */
#define MI_FLAG_INTERNAL 0x40000000u  /* an in-kernel completion wait gave up (never expected) */

typedef struct mi_operand {
  const float* data;
  int64_t stride_k;
  int64_t stride_i;
  int32_t grad_mode;     /* enum mi_grad_mode */
  int32_t slot;          /* MI_GRAD_PARTICLE: reduction slot in [0, num_slots) */
  float* grad;           /* MI_GRAD_DENSE: output */
  int64_t grad_stride_k;
  int64_t grad_stride_i;
} mi_operand;

typedef struct mi_site {
  int32_t family;        /* enum mi_family */
  int32_t operand[3];    /* role -> operand index, or -1 to use constant[role] */
  float constant[3];
  int32_t pad0;
  const uint8_t* mask;   /* NULL = all observed; else bool bytes, masked-out elements contribute 0 */
  int64_t mask_stride_k;
  int64_t mask_stride_i;
  double scale;          /* minibatch scale: declared batch numel / observed numel (core.py:267-271) */
} mi_site;

/* A guide draw evaluated inside a site group instead of being read from memory: the operand
 * `operand - 1` of the group is z[k, i] = loc[i] + eps[k, i] * scale[i] with eps the counter-based
 * normals of mi_normal_rsample (same seed, step, stream and particle numbering, so the values are
 * bit-identical). The [K, N] draw and its [K, N] gradient never exist in memory: with
 * compute_grads the group writes
 *   dloc[i]   = sum_k g0 * dT_k / dz[k, i]
 *   dscale[i] = sum_k g0 * dT_k / dz[k, i] * eps[k, i]
 * (the gradients mi_normal_rsample_backward would produce from the dense dz). Requirements: the
 * group's other dense operands are row-major [K, N] with unit element stride, N % 4 == 0 and
 * N >= 512; otherwise mi_group_forward returns MI_EUNSUPPORTED and the caller materialises the
 * draw with mi_normal_rsample. */
typedef struct mi_draw {
  int32_t operand;          /* 1 + index of the operand replaced by the draw; 0 = no draw (so a
                               zero-initialised descriptor has none) */
  uint32_t stream_id;
  const float* loc;
  int64_t loc_stride;       /* element strides (0: one value for all elements) */
  const float* scale;
  int64_t scale_stride;
  uint64_t seed;
  uint64_t step;
  const uint64_t* step_device;  /* may be NULL; added to step */
  int64_t particle_offset;
  float* dloc;              /* [N] outputs (compute_grads) */
  float* dscale;
  /* scale_exp non-NULL: the scale is expf(scale_exp[i * scale_stride]) (a guide's
   * transform_to(positive), nn.py:86-96, as mi_transform_params) and the first particle block
   * writes it to `scale` -- the transform inside the draw's kernel */
  const float* scale_exp;
  /* Global index of element 0 of this draw (a multiple of 4; 0 unless the guide factor is sharded
   * over ranks along its elements, mininf_amd.distributed.DataShard): element i uses the
   * counter block of global element element_offset + i, so the ranks' slices draw exactly what
   * one process drawing all elements would. */
  int64_t element_offset;
} mi_draw;

/* Independent work carried by extra workgroups of a group's launch (see mi_group_side_supported):
 * the per-draw Beta implicit-gradient factors of mi_beta_dgrad for draws x [K, N] (row-major) of
 * Beta(c1, c0), written to out [K, N, 2] (fp64). Their fp64 chains are latency-bound and
 * independent of the group's sites, so they run beside the site kernel's VALU-bound workgroups
 * instead of inside mi_elbo_forward (which then reads them through mi_factor.dgrad).
 * out == NULL: no side job (a zero-initialised descriptor has none). */
typedef struct mi_side {
  const float* x;
  const float* c1;
  int64_t c1_stride;
  const float* c0;
  int64_t c0_stride;
  int64_t K;
  int64_t N;
  double* out;
} mi_side;

/* A one-element-per-particle site folded into a group's launch (replaces the prior site's own launch
 * of the README model, README.md:43-47, `sample("theta", Beta(2, 2))`): its value is operand
 * sites[0].operand[0] of the group -- the per-particle parameter of the group's site, e.g. the
 * coin's theta -- its parameters are constants, and its scale is sites[0].scale. Its log-density
 * joins site 0's value, d log p / d value joins that operand's slot gradient, and its validation
 * bits go to *flags. Only the Bernoulli BCAST kernel carries it
 * (mi_group_prior_supported); mi_group_forward returns MI_EUNSUPPORTED otherwise. */
typedef struct mi_prior {
  int32_t present;       /* 0: no folded prior site */
  int32_t family;        /* MI_BETA (c1, c0), MI_NORMAL (loc, scale) or MI_GAMMA (conc., rate) */
  float constant[2];
  double scale;          /* the prior site's scale (a group's: equal to sites[0].scale) */
  uint32_t* flags;       /* the prior site's validation word (MI_FLAG_*) */
} mi_prior;

/* A group of sites evaluated over one shared [K, N] element space in a single pass, so that an
 * operand read by several sites (e.g. a latent z that is the value of one site and the loc of
 * another) is loaded once and its gradient accumulated in registers. */
typedef struct mi_group {
  int64_t K;
  int64_t N;
  int32_t num_sites;
  int32_t num_operands;
  int32_t num_slots;
  int32_t compute_grads; /* 0: forward values only */
  float grad_scale;      /* g0: upstream dL/dT_k assumed for MI_GRAD_DENSE / PARTICLE outputs */
  int32_t options;       /* MI_GROUP_* bits */
  mi_site sites[MI_MAX_SITES];
  mi_operand operands[MI_MAX_OPERANDS];
  mi_draw draw;          /* draw.operand == 0: no operand is a fused guide draw */
  mi_side side;          /* side.out == NULL: no side job */
  mi_prior prior;        /* prior.present == 0: no folded prior site */
  /* pdraw.operand != 0: operand pdraw.operand - 1 is a per-particle operand (stride_i == 0) that is
   * the guide's draw of a one-element Normal factor (the missing-observations model's mu,
   * FactorizedDistribution.rsample, nn.py:133-145): value_k = loc[0] + eps_k * scale[0] with the
   * eps of mi_normal_rsample for (particle_offset + k, element 0; same seed, step, stream --
   * bit-identical), scale = expf(scale_exp[0]) when scale_exp is non-NULL (then also written to
   * scale). The launch computes the values itself and writes them to the operand's data (column
   * block 0) instead of a mi_normal_rsample launch before it. Fused-draw site programs only
   * (mi_group_pdraw_supported; else MI_EUNSUPPORTED: launch mi_normal_rsample first). */
  mi_draw pdraw;
  /* non-NULL: the main site kernel folds its span into stamps[0] (min over workgroups of the start)
   * and stamps[1] (max of the end), on the device's constant-rate clock (mi_wall_clock_khz);
   * initialise them to (UINT64_MAX, 0). Timing only (bench.py); NULL in production launches. */
  unsigned long long* stamps;
} mi_group;

/* Frequency of the clock the span stamps count (mi_group.stamps), in kHz. */
int mi_wall_clock_khz(int* khz);

/* Library identification: returns MI_ABI_VERSION and writes the offload target ("gfx950"). */
int mi_abi_version(char* target, size_t target_bytes);

/* sizeof(mi_operand), sizeof(mi_site), sizeof(mi_group) as compiled: lets bindings check layout. */
int mi_struct_sizes(size_t* operand, size_t* site, size_t* group);

/* ---- site log-probability accumulation (replaces core.py:211-273 + torch log_prob) ------------ */

/* *supported = 1 when mi_group_forward runs `group`'s side job (the Bernoulli BCAST kernel over
 * unmasked contiguous data carries it), else 0: the caller then computes the factors elsewhere. */
int mi_group_side_supported(const mi_group* group, int* supported);

/* *supported = 1 when mi_group_forward evaluates `group`'s folded prior site (mi_prior), else 0:
 * the caller then launches that site on its own. */
int mi_group_prior_supported(const mi_group* group, int* supported);

/* *supported = 1 when mi_group_forward makes `group`'s per-particle draw (mi_group.pdraw). */
int mi_group_pdraw_supported(const mi_group* group, int* supported);

/* Workspace needed by mi_group_forward for this descriptor. */
int mi_group_workspace_bytes(const mi_group* group, size_t* bytes);

/* Evaluate all sites of `group` for every particle:
 *   total[k]              = sum_s scale_s * sum_i mask_si * log p_s(value_ki | params_ki)  (fp32)
 *   site_lp[s*K + k]      = scale_s * sum_i mask_si * log p_s(...)  (fp64; may be NULL)
 *   slot_grad[j*K + k]    = g0 * dT_k / d x[k] for MI_GRAD_PARTICLE operands in slot j (fp32)
 *   operands[o].grad      = g0 * dT_k / d x[k,i] for MI_GRAD_DENSE operands
 *   flags[s]              = OR of MI_FLAG_* found for site s (zeroed by this call unless
 *                           options has MI_GROUP_FLAGS_ZEROED)
 * Replaces LogProbTracer.sample's dist.log_prob (core.py:241, masked branch core.py:231-239),
 * LogProbTracer.total/contribution (core.py:247-273) and the autograd backward of the same ops. */
int mi_group_forward(const mi_group* group, void* workspace, size_t workspace_bytes, float* total,
                     double* site_lp, float* slot_grad, uint32_t* flags, void* stream);

/* ---- deferred finalize reductions --------------------------------------------------------------
 * A site launch ends with a fixed-order fp64 reduction of its per-(segment, particle) partials
 *   part[(v * nseg + seg) * K + k],  v < num_sites: site log densities, then num_slots slot values
 * into total[k] = sum_v scale[v] * sum_seg part (site_lp[v * K + k] the same per site, when
 * non-NULL) and slot_grad[j * K + k] = slot_scale * sum_seg part[num_sites + j]. The *_deferred
 * forms of the site launches skip that reduction when the segment list is at most
 * MI_REDUCE_MAX_SEG long and describe it in *reduce instead (reduce->part == NULL: the launch
 * reduced itself); mi_elbo_forward then runs it (mi_elbo.reduce) in the same launch as the ELBO's
 * own reduction -- one kernel launch less per site launch. The partials live in the site launch's
 * workspace, which must stay untouched until then. mi_reduce_launch runs a described reduction on
 * its own (a caller that cannot hand it to the ELBO). */
#define MI_MAX_REDUCE 4
#define MI_REDUCE_MAX_SEG 1024
typedef struct mi_reduce {
  const float* part;
  int64_t nseg;
  int64_t K;
  int32_t num_sites;
  int32_t num_slots;
  /* bit v: value v's segment block [nseg * K] holds a rank-one sum instead: u[0 .. nseg) at its
   * start, then f[0 .. K) and e[0 .. K); the value is f[k] * sum_seg u[seg] + e[k] (a per-particle
   * constant times a particle-independent sum, e.g. a Bernoulli site's slot gradient over shared
   * data: w dl_k * sum_i x_i - w dl_k N sigmoid(l_k)) */
  int32_t rank1;
  int32_t pad0;
  double scale[MI_MAX_SITES];
  double slot_scale;
  float* total;          /* [K] */
  double* site_lp;       /* [num_sites, K] or NULL */
  float* slot_grad;      /* [num_slots, K] (num_slots > 0) */
} mi_reduce;

/* mi_group_forward with the finalize handed to the caller through *reduce (see above). When
 * non-NULL, the hipEvent_t `start_event` / `stop_event` are recorded on `stream` immediately before
 * and after the main site kernel (not the flag reset or the finalize reduction), so the caller can
 * time exactly the roofline-bound kernel of an eager launch. Events are eager-only: while `stream`
 * is capturing, a call with either event returns MI_EUNSUPPORTED before enqueuing anything (the
 * capture stays valid); a replayed kernel is timed by `mi_group.stamps` instead. */
int mi_group_forward_deferred(const mi_group* group, void* workspace, size_t workspace_bytes,
                              float* total, double* site_lp, float* slot_grad, uint32_t* flags,
                              void* start_event, void* stop_event, void* stream, mi_reduce* reduce);

/* Run a deferred reduction as its own launch. */
int mi_reduce_launch(const mi_reduce* reduce, void* stream);

/* Where a fused-draw group leaves its partial sums (MI_GROUP_DRAW_PARTIALS): dloc partials are
 * rows [rows, N] at workspace + offset_bytes, dscale partials the next rows * N floats. */
int mi_group_draw_partials(const mi_group* group, size_t* offset_bytes, int64_t* rows);

/* The kernel source the engine specialises for `group` (site families, role kinds and gradient
 * targets compiled in; see mininf_amd/csrc/jit.cpp). Writes at most out_bytes (NUL-terminated) and
 * the full size to *needed. Diagnostic; not on the hot path. */
int mi_group_source(const mi_group* group, char* out, size_t out_bytes, size_t* needed);

/* Compile (hiprtc only; no device needed) the kernel mi_group_source would return. 0 on success,
 * MI_EUNSUPPORTED with the compiler log in `log` otherwise. */
int mi_group_compile_check(const mi_group* group, char* log, size_t log_bytes);

/* Backward rescale of a speculative dense gradient: row k of x is multiplied by g[k] / g0; thread
 * blocks whose rows all have g[k] == g0 return immediately (the common ELBO case). */
int mi_scale_rows(float* x, int64_t stride_k, int64_t stride_i, int64_t K, int64_t N,
                  const float* g, float g0, void* stream);

/* Categorical site (replaces Categorical.__init__'s normalisation, categorical.py:74-78, and
 * log_prob, categorical.py:150-156): logits[k, i, c] raw (or already normalised), value int64:
 *   total[k] = scale * sum_i mask_i * (logits[k, i, value_i] - logsumexp_c logits[k, i, c])
 * and, when dlogits != NULL (same strides as logits), every entry is written:
 *   dlogits[k, i, c] = g0 * scale * mask_i * ([c == value_i] - softmax_c(logits[k, i, :])).
 * A value outside [0, C) of an observed element sets MI_FLAG_SUPPORT in flags[0]. */
int mi_categorical_forward(const float* logits, int64_t stride_k, int64_t stride_i,
                           int64_t stride_c, int64_t K, int64_t N, int64_t C,
                           const int64_t* value, int64_t value_stride_k, int64_t value_stride_i,
                           const uint8_t* mask, int64_t mask_stride_i, double scale, float g0,
                           float* dlogits, void* workspace, size_t workspace_bytes, float* total,
                           uint32_t* flags, void* stream);
int mi_categorical_workspace_bytes(int64_t K, int64_t N, size_t* bytes);

/* MultivariateNormal site (replaces MultivariateNormal.log_prob, multivariate_normal.py:255-262,
 * with _batch_mahalanobis at :80-102; sites such as examples/missing-observations.md:42), float64,
 * row-major contiguous value[b, n], loc[b, n] and lower-triangular scale_tril[b, n, n] (the
 * caller factorises the covariance). Per batch item b, with w = L^-1 (value - loc):
 *   log_prob[b] = -0.5 w.w - sum_i log L_ii - n/2 log(2 pi),
 * and w[b, :], u[b, :] = L^-T w are written for the gradients:
 *   d/dvalue = -u, d/dloc = u, d/dL = tril(u w^T) - diag(1 / L_ii).
 * n <= MI_MVN_MAX_N. */
#define MI_MVN_MAX_N 1024

/* Cholesky factorisation A = L L^T (replaces torch.linalg.cholesky / cholesky_ex, which
 * MultivariateNormal(loc, covariance_matrix) calls in its constructor, multivariate_normal.py:193,
 * for the GP site of examples/missing-observations.md:40-42): batch row-major [n, n] matrices,
 * float32 or float64 in and out (a_bytes / l_bytes = 4 or 8; n > 80 needs a float64 output),
 * float64 arithmetic. Only the lower triangle of A is read; L's upper triangle is written as 0.
 * info[b] (optional) = 0 or j + 1 for the first non-positive pivot (cholesky_ex's convention).
 * Runs on the caller's stream with no host synchronisation, so a captured graph can hold it
 * (rocSOLVER's potrf cannot be captured on this stack). n <= MI_MVN_MAX_N. */
int mi_cholesky(const void* A, int32_t a_bytes, int64_t batch, int64_t n, void* L,
                int32_t l_bytes, int32_t* info, void* stream);
int mi_mvn_tril_forward(const double* value, const double* loc, const double* scale_tril,
                        int64_t batch, int64_t n, double* log_prob, double* w, double* u,
                        void* stream);

/* ---- guide reparameterised sampling (replaces nn.py:133-145 -> Normal/Beta.rsample) ------------ */

/* Counter-based Philox-4x32-7 normals: eps[k, i] is a function of (seed, step, stream_id,
 * particle_offset + k, element_offset + i) only, so the union of draws is independent of how
 * particles (particle_offset) or elements (element_offset, a multiple of 4) are sharded across
 * GPUs. z[k, i] = loc[i] + eps[k, i] * scale[i] (normal.py:83-86). If `eps` is non-NULL it is
 * used instead of the generator (parity mode: injected host noise, row-major [K, N]).
 * The effective step is `step + *step_device` when `step_device` (a device uint64) is non-NULL, so
 * a captured HIP graph advances the generator by incrementing that word on the device. */
int mi_normal_rsample(const float* loc, int64_t loc_stride, const float* scale, int64_t scale_stride,
                      int64_t K, int64_t N, uint64_t seed, uint64_t step,
                      const uint64_t* step_device, uint32_t stream_id, int64_t particle_offset,
                      int64_t element_offset, const float* eps, float* z, void* stream);

/* mi_normal_rsample for a guide whose scale is exp of an unconstrained parameter u
 * (ParameterizedDistribution.forward, nn.py:86-96 -> transform_to(positive)): the draws use
 * expf(u[i * u_stride]) (as mi_transform_params) and the first particle block writes it to
 * scale_out[i * u_stride] -- the transform and the draw in one launch. */
int mi_normal_rsample_exp(const float* loc, int64_t loc_stride, const float* u, int64_t u_stride,
                          float* scale_out, int64_t K, int64_t N, uint64_t seed, uint64_t step,
                          const uint64_t* step_device, uint32_t stream_id, int64_t particle_offset,
                          int64_t element_offset, const float* eps, float* z, void* stream);

/* Backward of mi_normal_rsample: dloc[i] = sum_k dz[k,i], dscale[i] = sum_k dz[k,i] * eps[k,i]
 * with eps regenerated from the counter (or read from `eps`). */
int mi_normal_rsample_backward_workspace_bytes(int64_t K, int64_t N, size_t* bytes);
int mi_normal_rsample_backward(const float* dz, int64_t dz_stride_k, int64_t dz_stride_i,
                               int64_t K, int64_t N, uint64_t seed, uint64_t step,
                               const uint64_t* step_device, uint32_t stream_id,
                               int64_t particle_offset, int64_t element_offset, const float* eps,
                               void* workspace, size_t workspace_bytes, float* dloc, float* dscale,
                               void* stream);

/* Beta(concentration1, concentration0) draws x[k, i] = G1 / (G1 + G0) with Marsaglia-Tsang gamma
 * variates from the same counter-based generator (beta.py:85-86, dirichlet.py:23-36, 85-88). With
 * `x_in` non-NULL the draws are copied from it instead (parity mode). */
int mi_beta_rsample(const float* c1, int64_t c1_stride, const float* c0, int64_t c0_stride,
                    int64_t K, int64_t N, uint64_t seed, uint64_t step,
                    const uint64_t* step_device, uint32_t stream_id,
                    int64_t particle_offset, const float* x_in, float* x, void* stream);

/* mi_beta_rsample for a guide whose concentrations are exp of unconstrained parameters
 * (ParameterizedDistribution.forward, nn.py:86-96 -> transform_to(positive), and Beta.__init__'s
 * stack, beta.py:36-40): every draw computes its concentrations from u1 / u0 (expf, as
 * mi_transform_params) and the k = 0 draws also write them, interleaved, to conc[N, 2] -- the
 * transform and the draw in one launch. */
int mi_beta_rsample_exp(const float* u1, int64_t u1_stride, const float* u0, int64_t u0_stride,
                        float* conc, int64_t K, int64_t N, uint64_t seed, uint64_t step,
                        const uint64_t* step_device, uint32_t stream_id, int64_t particle_offset,
                        const float* x_in, float* x, void* stream);

/* Implicit reparameterisation gradient of the Beta draws (dirichlet.py:17-20 ->
 * torch._dirichlet_grad, ATen/native/Distributions.h dirichlet_grad_one), reduced over particles:
 *   dc1[i * dc1_stride] = sum_k dx[k,i] * dgrad(x, c1, c1+c0) * (1 - x)
 *   dc0[i * dc0_stride] = -sum_k dx[k,i] * dgrad(1 - x, c0, c1+c0) * x
 * (output strides let the gradient land directly in the interleaved [..., 2] concentration layout
 * torch's Beta keeps, beta.py:36-40). */
int mi_beta_rsample_backward_workspace_bytes(int64_t K, int64_t N, size_t* bytes);
int mi_beta_rsample_backward(const float* dx, int64_t dx_stride_k, int64_t dx_stride_i,
                             const float* x, const float* c1, int64_t c1_stride, const float* c0,
                             int64_t c0_stride, int64_t K, int64_t N, void* workspace,
                             size_t workspace_bytes, float* dc1, int64_t dc1_stride, float* dc0,
                             int64_t dc0_stride, void* stream);

/* The upstream-independent factors of mi_beta_rsample_backward, per draw:
 *   out[(k * N + i) * 2 + 0] =  dgrad(x, c1, c1+c0) * (1 - x)
 *   out[(k * N + i) * 2 + 1] = -dgrad(1 - x, c0, c1+c0) * x          (fp64, [K, N, 2])
 * so dc1[i] = sum_k dx[k,i] * out[k,i,0] and dc0[i] = sum_k dx[k,i] * out[k,i,1]. They depend only
 * on the draws, so this can run beside the site kernels; mi_elbo_forward reads them through
 * mi_factor.dgrad. */
int mi_beta_dgrad(const float* x, const float* c1, int64_t c1_stride, const float* c0,
                  int64_t c0_stride, int64_t K, int64_t N, double* out, void* stream);

/* Recovery after a failed hipGraph capture of a training step (mininf_amd.graph.StepGraph): if
 * `stream` is still capturing, end the capture and destroy the partial graph; then clear the
 * thread's last HIP error. *was_capturing (optional) reports whether a capture had to be ended.
 * The host-side counterpart of the reference's exception semantics: an error raised inside a step
 * (mininf/core.py:142-189, nn.py:212-228) leaves the process usable. Not asynchronous: it acts on
 * the stream's capture state, not on its work. */
int mi_capture_abandon(void* stream, int* was_capturing);

/* Start of one ELBO step (EvidenceLowerBoundLoss.forward) in one launch: *snapshot = *counter (the
 * generator step this call's draws and their backward use), *counter += 1, and
 * flags[0 .. nflags) = 0 (the call's validation words, MI_GROUP_FLAGS_ZEROED). */
int mi_step_begin(uint64_t* counter, uint64_t* snapshot, uint32_t* flags, int64_t nflags,
                  void* stream);

/* Gamma(concentration, rate) guide draws (replaces Gamma.rsample, gamma.py:80-88):
 *   g[k, i] = standard Gamma(concentration[i]) draw (Marsaglia-Tsang, same counter scheme as
 *             mi_beta_rsample, sub-stream 2), or g_in[k, i] when g_in != NULL (parity mode);
 *   x[k, i] = max(g[k, i] / rate[i], FLT_MIN).
 * g is the backward's input (torch saves _standard_gamma's result the same way). */
int mi_gamma_rsample(const float* concentration, int64_t concentration_stride, const float* rate,
                     int64_t rate_stride, int64_t K, int64_t N, uint64_t seed, uint64_t step,
                     const uint64_t* step_device, uint32_t stream_id, int64_t particle_offset,
                     const float* g_in, float* g, float* x, void* stream);
/* Backward for upstream dx[k, i] (strided), reduced over particles in fp64:
 *   dconcentration[i] = sum_k dx / rate * standard_gamma_grad(concentration, g)
 *                       (torch _standard_gamma_grad, Distributions.h:310, in double)
 *   drate[i]          = sum_k -dx * g / rate^2 */
int mi_gamma_rsample_backward_workspace_bytes(int64_t K, int64_t N, size_t* bytes);
int mi_gamma_rsample_backward(const float* dx, int64_t dx_stride_k, int64_t dx_stride_i,
                              const float* g, const float* concentration,
                              int64_t concentration_stride, const float* rate,
                              int64_t rate_stride, int64_t K, int64_t N, void* workspace,
                              size_t workspace_bytes, float* dconcentration,
                              int64_t dconcentration_stride, float* drate, int64_t drate_stride,
                              void* stream);

/* Constrained parameters of one guide factor in one launch, interleaved [n, m]:
 *   out[i * m + j] = exp(u[j][i * stride[j]])   (transform[j] MI_TRANSFORM_EXP: transform_to(positive),
 *                                                 torch constraint_registry.py:184-189)
 *                  = u[j][i * stride[j]]        (MI_TRANSFORM_NONE)
 * ParameterizedDistribution.forward (reference nn.py:86-96) for a Beta guide, whose Dirichlet keeps
 * exactly this [..., 2] (concentration1, concentration0) layout (beta.py:36-40). */
#define MI_MAX_PARAMS 4
typedef struct mi_params {
  int32_t m;
  int32_t pad0;
  int64_t n;
  const float* u[MI_MAX_PARAMS];
  int64_t stride[MI_MAX_PARAMS];
  int32_t transform[MI_MAX_PARAMS];
} mi_params;
int mi_transform_params(const mi_params* params, float* out, void* stream);

/* Raw generator output for tests: out[k, i] = standard normal eps of mi_normal_rsample. */
int mi_philox_normal(int64_t K, int64_t N, uint64_t seed, uint64_t step, uint32_t stream_id,
                     int64_t particle_offset, float* out, void* stream);
/* Raw Philox-4x32-10 blocks for known-answer tests: out[4*j .. 4*j+3] = philox(ctr[j], key). */
int mi_philox4x32(const uint32_t* ctr, int64_t count, uint32_t key0, uint32_t key1, uint32_t* out,
                  void* stream);

/* ---- linear-predictor sites (Normal(X @ theta, sigma), Bernoulli(logits = X @ theta)) --------- */

/* A site whose location / logits is the model's own product X @ theta of an observed design matrix
 * X [N, P] and a per-particle coefficient vector theta [K, P] (the reference's regression models:
 * tests/test_mininf.py:13-18, examples/minibatch.md:24-33). The product is evaluated inside the
 * site kernel, so the [K, N] predictor and its gradient never exist in memory:
 *   total[k]        = site_scale * sum_i mask_i * log p(value_i | (X theta_k)_i, sigma_k)
 *   dslots[j*K + k] = g0 * d total[k] / d theta[k, j]   for j < P (slot-major: row j holds all k)
 *   dslots[P*K + k] = g0 * d total[k] / d sigma_k       (Normal with per-particle sigma only)
 *   flags[0]        = OR of MI_FLAG_* (value support; sigma > 0; finite predictor)
 * family: MI_NORMAL (sigma = scale[k * scale_stride_k], or scale_constant when scale == NULL) or
 * MI_BERNOULLI_LOGITS (scale unused). P <= MI_LINEAR_MAX_P. */
#define MI_LINEAR_MAX_P 64
/* options bit: run the VALU kernel even where the matrix-core (v_mfma_f32_32x32x2_f32) kernel
 * applies (contiguous 16-byte aligned rows of X, P % 4 == 0); for cross-checks. */
#define MI_LINEAR_VALU 2

/* The rows of the next minibatch drawn by the kernel that reads them (instead of a separate
 * mi_minibatch_rows launch): counter, n, batch, batches_per_epoch, shuffle and seed have
 * mi_minibatch_rows's meaning; the kernel reads the batch number counter[0], draws its rows, writes
 * them to `out` (when non-NULL, for later readers of the batch) and advances counter[0] once all
 * of its blocks have read it (counter[1]: completion count, zero between launches).
 * DataLoader(TensorDataset(X, y), batch_size, shuffle=True) of examples/minibatch.md:78. */
typedef struct mi_rows {
  uint64_t* counter;      /* NULL: no rows drawn here */
  int64_t n;
  int64_t batch;
  int64_t batches;
  uint64_t seed;
  int32_t shuffle;
  int32_t pad0;
  int32_t* out;
} mi_rows;

typedef struct mi_linear {
  int64_t K;
  int64_t N;
  int64_t P;
  int32_t family;
  int32_t options;        /* MI_GROUP_FLAGS_ZEROED | MI_LINEAR_VALU */
  const float* x;         /* X[i, j] at x[i * x_stride_i + j * x_stride_j] */
  int64_t x_stride_i;
  int64_t x_stride_j;
  const float* theta;     /* theta[k, j] at theta[k * theta_stride_k + j * theta_stride_j] */
  int64_t theta_stride_k;
  int64_t theta_stride_j;
  const float* value;     /* value[i * value_stride_i] */
  int64_t value_stride_i;
  const uint8_t* mask;    /* NULL or mask[i * mask_stride_i] */
  int64_t mask_stride_i;
  const float* scale;     /* Normal sigma per particle, or NULL */
  int64_t scale_stride_k;
  float scale_constant;
  float grad_scale;       /* g0 */
  double site_scale;      /* minibatch scale (core.py:267-271) */
  int32_t compute_grads;  /* write dtheta (and dsigma when `scale` is non-NULL) */
  int32_t pad0;
  const int32_t* row_index; /* NULL, or row i of the site reads row row_index[i] of x, value and
                               mask (a device-resident minibatch, mi_minibatch_rows) */
  mi_rows rows;           /* rows.counter non-NULL (row_index NULL): the site draws its batch's
                             rows itself; only the matrix-core kernel with one row stage per
                             block does (else MI_EUNSUPPORTED: launch mi_minibatch_rows first) */
  mi_prior prior;         /* prior.present: a site over theta itself ([K, P], every element; the
                             regression's `theta ~ Normal(0, 1)`, examples/minibatch.md:45-50)
                             evaluated by this launch: its log density joins the site's total,
                             d log p / d theta joins dslots (mi_linear_prior_supported) */
  mi_draw draw;           /* draw.operand != 0: theta is the guide's Normal draw, made by this launch
                             instead of a mi_normal_rsample launch before it (FactorizedDistribution
                             .rsample, nn.py:133-145): theta[k, j] = loc[j] + eps * scale[j] with the
                             eps of mi_normal_rsample (same seed, step, stream, particle_offset + k,
                             element_offset + j; bit-identical values), scale = expf(scale_exp[j])
                             when scale_exp is non-NULL (then also written to scale, as
                             mi_normal_rsample_exp). `theta` is not read; every element of it is
                             written by the launch. dloc / dscale unused. Matrix-core kernel only,
                             P % 4 == 0 (else MI_EUNSUPPORTED: launch mi_normal_rsample first). */
  unsigned long long* stamps; /* as mi_group.stamps: the site kernel's span (timing only) */
} mi_linear;

/* *supported = 1 when mi_linear_forward evaluates `site`'s folded prior (the matrix-core kernel). */
int mi_linear_prior_supported(const mi_linear* site, int* supported);

int mi_linear_workspace_bytes(const mi_linear* site, size_t* bytes);
int mi_linear_forward(const mi_linear* site, void* workspace, size_t workspace_bytes, float* total,
                      float* dslots, uint32_t* flags, void* stream);
int mi_linear_struct_size(size_t* bytes);
/* mi_linear_forward with the finalize handed to the caller through *reduce (see mi_reduce); the
 * events as for mi_group_forward_deferred. */
int mi_linear_forward_deferred(const mi_linear* site, void* workspace, size_t workspace_bytes,
                               float* total, float* dslots, uint32_t* flags, void* start_event,
                               void* stop_event, void* stream, mi_reduce* reduce);

/* ---- device-resident minibatches (replaces examples/minibatch.md:78-88, the host DataLoader) ---- */

/* Row indices of the next minibatch of an n-row dataset: with c = counter[0] (then counter[0] =
 * c + 1, in the same launch; counter[1] is the launch's completion count and must be zero
 * initially -- every launch leaves it at zero), epoch e = c / batches_per_epoch and batch
 * b = c % batches_per_epoch,
 *   rows[j] = perm_e(b * batch + j)  (shuffle)   or   b * batch + j,   j < count,
 * where perm_e is a keyed Feistel permutation of [0, n) (seed, e): a fresh random order every
 * epoch, like DataLoader(..., shuffle=True) (dataloader.py RandomSampler), computed on the device.
 * count is batch, or the shorter last batch of an epoch (batch b * batch + count <= n; positions
 * past the data are not permuted). batches_per_epoch is ceil or floor of n / batch. n < 2^31. */
int mi_minibatch_rows(uint64_t* counter, int64_t n, int64_t batch, int64_t batches_per_epoch,
                      int32_t shuffle, uint64_t seed, int32_t* rows, int64_t count, void* stream);

/* out[j] = base[rows[j]]: count rows of row_bytes bytes (multiples of 4) -- a minibatch
 * materialised for uses other than the site kernels that read rows through the index. */
int mi_gather_rows(const void* base, int64_t base_stride_bytes, int64_t row_bytes,
                   const int32_t* rows, int64_t count, void* out, int64_t out_stride_bytes,
                   void* stream);

/* ---- optimizer step (replaces torch.optim.Adam.step of the training loop, README.md:66-69) ----- */

/* One Adam step for up to MI_ADAM_MAX_TENSORS fp32 parameters in one launch, arithmetic of torch's
 * fused Adam (fused_adam_utils.cuh adam_math: ADAM_MODE::ORIGINAL, no AMSGrad):
 *   s = *step + 1;  g = (maximize ? -grad : grad) + weight_decay * param
 *   m = beta1 m + (1 - beta1) g;  v = beta2 v + (1 - beta2) g^2
 *   param -= lr / (1 - beta1^s) * m / (sqrt(v) / sqrt(1 - beta2^s) + eps);  *step = s
 * per tensor (its own step word, fp32 as torch keeps it). `counters`: MI_ADAM_COUNTER_WORDS uint32
 * words, zero before first use, owned by one caller's launches on one stream: the completion
 * counters (every launch leaves them zero), then a cache of the next step's bias corrections per
 * tensor slot (ABI 16; a slot that does not match the step and betas is recomputed). */
#define MI_ADAM_MAX_TENSORS 8
#define MI_ADAM_COUNTER_WORDS (MI_ADAM_MAX_TENSORS * 33 + MI_ADAM_MAX_TENSORS * 16)
typedef struct mi_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  float* step;
  int64_t numel;          /* contiguous */
} mi_adam_tensor;
typedef struct mi_adam {
  int32_t num;
  int32_t maximize;
  double lr;
  double beta1;
  double beta2;
  double eps;
  double weight_decay;
  mi_adam_tensor tensors[MI_ADAM_MAX_TENSORS];
} mi_adam;
int mi_adam_step(const mi_adam* adam, uint32_t* counters, void* stream);

/* ---- one-shot peer-write all-reduce (replaces the sharded step's small-bucket
 * dist.all_reduce / ncclAllReduce, distributed.GradientBucket) -------------------------------------
 * Each rank allocates one region (mi_peer_region_bytes for the largest bucket, mi_peer_alloc:
 * fine-grained device memory, zeroed, and its IPC handle, MI_PEER_HANDLE_BYTES), exchanges the
 * handles over its process group and maps the peers' regions (mi_peer_open). mi_peer_allreduce
 * then sums a float bucket over the ranks in ONE kernel on the caller's stream (capturable): the
 * bucket is written into a slot of every peer's region with system-scope stores, a flag carrying
 * the call number follows, the caller waits for every peer's flag in its own region and adds the
 * slots in rank order (two ranks: the same sum as any SUM all-reduce). A peer that never arrives
 * ends the wait after about a second: the call sets bit 0 of *error (device-visible memory, e.g.
 * pinned host memory the host can poll; never cleared by the library), fills `out` with NaN and
 * does not advance the call counter. A call that finds *error set at entry does the same without
 * writing into any peer's region (sticky failure: the communicator is unusable afterwards). Every
 * rank must call it the same number of times, with buckets of the same length. */
#define MI_PEER_MAX_RANKS 8
#define MI_PEER_MAX_FLOATS 4096
#define MI_PEER_HANDLE_BYTES 64
typedef struct mi_peer {
  int32_t rank;
  int32_t world;
  int64_t max_floats;                    /* the regions' slot length */
  void* regions[MI_PEER_MAX_RANKS];      /* [rank]: this rank's region; others: the mapped peers' */
} mi_peer;
int mi_peer_region_bytes(int64_t max_floats, size_t* bytes);
int mi_peer_alloc(size_t bytes, void** region, void* handle);
int mi_peer_open(const void* handle, void** region);
int mi_peer_close(void* region);
int mi_peer_free(void* region);
int mi_peer_allreduce(const mi_peer* peer, const float* in, float* out, int64_t n,
                      uint32_t* error, void* stream);
/* Diagnostics (synchronous): the number of calls this rank's region has completed. */
int mi_peer_call_count(const mi_peer* peer, uint64_t* count);

/* ---- ELBO tail (replaces nn.py:224-228 + FactorizedDistribution.entropy, nn.py:121-131) -------- */

#define MI_MAX_TERMS 8
#define MI_MAX_FACTORS 8
#define MI_MAX_BUFFERS 16

/* One mean-field guide factor whose entropy enters the ELBO, viewed as n elements:
 *   MI_NORMAL: param[0] = loc (read only with an absorbed draw), param[1] = scale
 *   MI_BETA:   param[0] = concentration1, param[1] = concentration0
 *   MI_GAMMA:  param[0] = concentration, param[1] = rate (gamma.py:101-107; draw_kind NONE only)
 * Parameters are fp32 with element stride `stride` (0 only when n == 1). mi_elbo_backward writes
 *   grad[j][i * grad_stride[j]] = d loss / d param_j(i)                  (transform[j] NONE)
 *                               = d loss / d u_j(i) = (d loss / d param_j) * param_j
 *                                                       (transform[j] EXP: param_j = exp(u_j))
 * for every non-NULL grad[j]. The transforms restate ParameterizedDistribution's
 * transform_to(constraint) (nn.py:86-96): EXP is transform_to(positive) = exp.
 *
 * Absorbed guide draw (draw_kind != MI_DRAW_NONE). The factor's K draws z (Normal: z = loc +
 * eps * scale, normal.py:83-86; Beta: implicit reparameterisation, dirichlet.py:17-20) feed only
 * site kernels of this ELBO, so d loss / d param also carries the draws' backward (what
 * mi_normal_rsample_backward / mi_beta_rsample_backward and autograd's accumulation would add):
 *   MI_DRAW_SOURCES:  dz[k, i] = sum_s source[s].ptr[k * stride_k + i * stride_i]  (pre-scaled by
 *                     g0, like every speculative site gradient); Normal: eps from the generator
 *                     (seed, step, step_device, stream_id, particle_offset) or `eps` [K, n];
 *                     Beta: `draws` holds x [K, n] row-major.
 *   MI_DRAW_PARTIALS: Normal draws fused into a site group (mi_draw): partial[0] / partial[1] hold
 *                     partial_rows rows [rows, n] of sum_k g0 dT/dz and sum_k g0 dT/dz * eps. */
#define MI_TRANSFORM_NONE 0
#define MI_TRANSFORM_EXP 1
#define MI_DRAW_NONE 0
#define MI_DRAW_SOURCES 1
#define MI_DRAW_PARTIALS 2
#define MI_MAX_SOURCES 4

typedef struct mi_source {
  const float* ptr;
  int64_t stride_k;
  int64_t stride_i;
} mi_source;

typedef struct mi_factor {
  int32_t family;
  int32_t draw_kind;            /* MI_DRAW_* */
  int64_t n;
  const float* param[2];
  int64_t stride[2];
  float* grad[2];
  int64_t grad_stride[2];
  int32_t transform[2];         /* MI_TRANSFORM_* per parameter */
  int32_t num_sources;
  uint32_t stream_id;
  mi_source source[MI_MAX_SOURCES];
  const float* draws;           /* Beta draws x [K, n] */
  const float* eps;             /* Normal: injected noise [K, n], or NULL to regenerate */
  uint64_t seed;
  uint64_t step;
  const uint64_t* step_device;  /* may be NULL; added to step */
  int64_t particle_offset;
  const float* partial[2];      /* MI_DRAW_PARTIALS */
  int64_t partial_rows;
  const double* dgrad;          /* Beta, MI_DRAW_SOURCES: mi_beta_dgrad output [K, n, 2], or NULL
                                   to evaluate the implicit gradients in mi_elbo_forward */
  double* saved;                /* Beta, MI_DRAW_SOURCES: [n, 4] fp64 sums mi_elbo_forward writes
                                   and mi_elbo_backward of the same evaluation reads (required).
                                   Owned by the caller per evaluation, so evaluations sharing a
                                   workspace may interleave (loss1 + loss2, then backward). */
  int64_t element_offset;       /* Normal, regenerated eps: the draw's mi_draw.element_offset */
  double weight;                /* this factor's entropy enters as entropy_scale * weight * H_f:
                                   1 for a factor every rank holds whole or owns a slice of, 1/W
                                   for one replicated on W data-sharded ranks; > 0 (a zeroed
                                   descriptor is rejected) */
} mi_factor;

/* loss = g0 * sum_t sum_k terms[t][k] - entropy_scale * sum_f weight_f * sum_i H_f(i)
 * terms: per-particle log joints [K] (site-group totals, categorical totals, torch-evaluated sites);
 * g0 = -1/K_total (fp32); entropy_scale = 1/world when particles are sharded over ranks.
 * buffers: the speculative gradients of the site groups (computed for upstream g0), rescaled by
 * mi_elbo_backward when the loss's upstream gradient is not exactly 1. */
typedef struct mi_elbo {
  int64_t K;
  int32_t num_terms;
  int32_t num_factors;
  int32_t num_buffers;
  int32_t num_reduce;
  float g0;
  int32_t options;       /* MI_ELBO_* bits */
  double entropy_scale;
  const float* terms[MI_MAX_TERMS];
  mi_factor factors[MI_MAX_FACTORS];
  float* buffers[MI_MAX_BUFFERS];
  int64_t buffer_len[MI_MAX_BUFFERS];
  /* deferred site finalize reductions (same K): mi_elbo_forward writes their outputs and adds
   * g0 * sum_k total[k] of each to the loss (their totals are not listed in `terms`). Forward-
   * absorbed Beta factors (MI_DRAW_SOURCES) must then have `dgrad`: their sums over the particles
   * (which read slot gradients the reductions write) move to mi_elbo_backward. */
  mi_reduce reduce[MI_MAX_REDUCE];
  /* step_counter != NULL: after everything else, the launch's last block sets
   * *step_snapshot = *step_counter and *step_counter += 1 (the generator step of this ELBO
   * evaluation's draws -- read from step_counter in the forward, from step_snapshot afterwards). */
  uint64_t* step_counter;
  uint64_t* step_snapshot;
  /* flags_mirror != NULL: the last block copies flags[0 .. nflags) there (e.g. host-mapped memory:
   * the validation words of this evaluation without a separate device-to-host copy). */
  const uint32_t* flags;
  uint32_t* flags_mirror;
  int64_t nflags;
} mi_elbo;


/* mi_elbo.options: the forward's last block also writes the final gradients (`grad` of every
 * factor) for an upstream gradient of exactly 1 -- loss.backward() of the training loop,
 * README.md:66-69 -- when mi_elbo_final_grads reports the forward complete; the caller then need not
 * launch mi_elbo_backward for that upstream (any other upstream: launch it, it rewrites them). */
#define MI_ELBO_FINAL_GRADS 1

/* *complete = 1 when mi_elbo_forward with MI_ELBO_FINAL_GRADS leaves nothing for mi_elbo_backward
 * at an upstream of 1: every factor is a one-element forward-absorbed Beta factor whose sums the
 * forward finishes (the README model's theta, with deferred site reductions). */
int mi_elbo_final_grads(const mi_elbo* elbo, int* complete);

/* sizeof(mi_factor), sizeof(mi_elbo) as compiled. */
int mi_elbo_struct_sizes(size_t* factor, size_t* elbo);

/* Workspace of mi_elbo_forward and mi_elbo_backward. Its first MI_ELBO_COUNTER_BYTES hold
 * completion counters that must be zero before first use (mi_elbo_workspace_init) and that every
 * launch leaves at zero, so one workspace serves every step (and captured HIP graphs) on one
 * stream. */
#define MI_ELBO_COUNTER_BYTES 16640
int mi_elbo_workspace_bytes(const mi_elbo* elbo, size_t* bytes);
int mi_elbo_workspace_init(void* workspace, size_t workspace_bytes, void* stream);

/* Writes the scalar loss (fp32, reduced in fp64 in a fixed order). MI_EUNSUPPORTED when num_reduce
 * > 0 and a forward-absorbed Beta factor has no dgrad (see mi_elbo.reduce). */
int mi_elbo_forward(const mi_elbo* elbo, void* workspace, size_t workspace_bytes, float* loss,
                    void* stream);

/* The optimizer step of the factors an ELBO forward finishes (ABI 14). With MI_ELBO_FINAL_GRADS
 * the forward's last block writes the gradients of one-element Beta tails and of the Normal tail
 * (nt) for an upstream of 1; mi_elbo_forward_adam also runs Adam there, on the unconstrained tensor
 * behind factor `factor`'s parameter `param` (mi_factor.grad[param] is its gradient), with
 * mi_adam_step's arithmetic (torch's fused Adam): the update, the moments and the step count, by
 * the thread that writes the gradient -- no optimizer launch for the step. `adam` is a DEVICE
 * pointer (the descriptor is read by the kernel; it may be reused across launches); NULL: as
 * mi_elbo_forward. mi_elbo_adam_supported checks a HOST copy against the launch: every slot's
 * factor finished by the last block, numel = the factor's n, the gradient written, no
 * (factor, param) twice; a fused-draw factor's slots are declined (mi_adam_step streams them at
 * full occupancy). Replaces optimizer.step() (README.md:66-69) for those parameters. */
#define MI_ELBO_ADAM_SLOTS 4
typedef struct mi_elbo_adam_slot {
  int32_t factor;
  int32_t param;
  float* value;           /* the optimised tensor (contiguous, numel = the factor's n) */
  float* exp_avg;
  float* exp_avg_sq;
  float* step;            /* one float */
  int64_t numel;
} mi_elbo_adam_slot;
typedef struct mi_elbo_adam {
  int32_t num;
  int32_t maximize;
  double lr;
  double beta1;
  double beta2;
  double eps;
  double weight_decay;
  mi_elbo_adam_slot slots[MI_ELBO_ADAM_SLOTS];
} mi_elbo_adam;
int mi_elbo_adam_supported(const mi_elbo* elbo, const mi_elbo_adam* adam, int* supported);
int mi_elbo_forward_adam(const mi_elbo* elbo, void* workspace, size_t workspace_bytes,
                         float* loss, const mi_elbo_adam* adam, void* stream);

/* With u = *upstream (device scalar, d out / d loss): dterm[0] = u * g0 (the gradient of every
 * term element); factors[f].grad[j] = the gradient of -u * entropy_scale * H_f (plus u times the
 * absorbed draw's backward, and the transform's chain rule; see mi_factor); every buffer is
 * multiplied by u unless u == 1. One launch; `workspace` is the mi_elbo_forward workspace. */
int mi_elbo_backward(const mi_elbo* elbo, const float* upstream, float* dterm, void* workspace,
                     size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MININF_AMD_H */
