/*
 * dbsde.h -- C ABI of the MI355X-native deep-BSDE training step.
 *
 * This is the drop-in boundary for the reference's FBSNN solver surface
 * (nd_BSPDE_case.py:126-500, DeepBSDE.py:140-323, with_corr...py:132-540,
 * heston_dnnpde.py:519-699).  Every entry point below replaces one reference
 * method; the Python binding that a maintainer adds to a reference-style script
 * is the ctypes class in
 * deep-neural-network-solutions-for-partial-differential-equations_amd/fbsnn.py
 * (see INTEGRATION.md).
 *
 * Conventions
 *   - Every function returns 0 on success and a negative DBSDE_E* code on
 *     failure; dbsde_last_error() then holds a message.
 *   - Pointers documented as "device" are HIP device pointers on the
 *     context's device (e.g. torch.Tensor.data_ptr() of a cuda tensor).
 *   - Parameters, gradients and optimizer moments are FLAT fp32 vectors in
 *     the reference module's state_dict() order (nd_BSPDE_case.py:445-456
 *     save format), so torch checkpoints interoperate.
 *   - Work is enqueued on the stream set by dbsde_set_stream (default: the
 *     legacy null stream) and is asynchronous: results are valid once the
 *     stream has been synchronised.  Setting a different stream orders it
 *     after the work already queued on the previous one (the context's
 *     workspace is shared by its calls), so a caller may switch streams
 *     between calls without synchronising.  The context keeps no caller pointer
 *     after a call returns.  A context is not thread safe.
 */
#ifndef DBSDE_H
#define DBSDE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DBSDE_ABI_VERSION 3

/* error codes */
#define DBSDE_OK 0
#define DBSDE_EINVAL -1   /* bad configuration or argument (Python: ValueError)   */
#define DBSDE_EHIP -2     /* HIP runtime failure             (Python: RuntimeError) */
#define DBSDE_ENOMEM -3   /* device allocation failed        (Python: MemoryError)  */

/* network modes: DeepBSDE.py:166-178, nd_BSPDE_case.py:159-172 */
#define DBSDE_MODE_FC 0        /* "FC"       nn.Sequential of Linear/act            */
#define DBSDE_MODE_NAIS_NET 1  /* "NAIS-Net" Resnet(stable=True), DeepBSDE.py:23-65 */
#define DBSDE_MODE_RESNET 2    /* "Resnet"   Resnet(stable=False)                   */
#define DBSDE_MODE_NAISNET 3   /* "Naisnet"  Functions/naisnet.py:6-96              */

/* activations: Functions/Sine.py, nn.ReLU, nn.Tanh */
#define DBSDE_ACT_SINE 0
#define DBSDE_ACT_RELU 1
#define DBSDE_ACT_TANH 2

/* terminal conditions g(X) over the leading g_cols state columns */
#define DBSDE_G_SUMSQ 0       /* sum X^2                 DeepBSDE.py:333-335          */
#define DBSDE_G_CALL_SUM 1    /* max(sum X - K, 0)       nd_BSPDE_case.py:521-522     */
#define DBSDE_G_CALL_MEAN 2   /* max(mean X - K, 0)      with_corr...py:577-579,
                                                         heston_dnnpde.py:550 (k = 1)  */
#define DBSDE_G_LOG 3         /* log(1/2 + 1/2 sum X^2)  hjb_implement.py:597-598     */
#define DBSDE_G_SMOOTH_CALL 4 /* a / (1 + exp(-alpha a)), a = mean X - K
                                                         heston_dnnpde.py:551-556     */

/* problem kinds */
#define DBSDE_PROB_DIAG 0     /* mu = mu_a X, sigma = diag(sig_a X + sig_b)          */
#define DBSDE_PROB_HESTON 1   /* k-asset Heston (heston_dnnpde.py:519-659), state
                                 [S_1..S_k, v_1..v_k], one Brownian motion per asset */

/*
 * Problem coefficients (one FBSNN subclass = one filled struct):
 *   kind DIAG:
 *     mu(X)    = mu_a * X                                (diagonal drift)
 *     sigma(X) = diag(sig_a * X + sig_b)                 (the reference's
 *                                                          dense diag_embed sigma)
 *   kind HESTON (heston_dnnpde.py:587-605), per asset i, sv = sqrt(max(v_i, 1e-8)):
 *     mu       = clamp([mu_a S_i, h_kappa (h_theta - v_i)], -100, 100)
 *     Sigma_i  = clamp([[sv S_i, h_rho h_sigma sv], [h_rho sv S_i, h_sigma sv]], -100, 100)
 *     driven by the asset's scalar dW_i (the reference's FBSNN dimension is 1;
 *     its einsum broadcasts dW over both state components)
 *   phi      = phi_r * (Y - phi_c * X.Z) + phi_zz * |Z|^2
 *   g        = g_kind over the first g_cols state columns (0 = all), strike,
 *              g_alpha (DBSDE_G_SMOOTH_CALL); the terminal |Z - grad g|^2 term
 *              runs over the same columns (heston_dnnpde.py:654: dU/dS only)
 *   u_clamp  = 1: u = max(net(t, X), 0) (heston_dnnpde.py:568)
 *   q3       = 1: for D == 1 reproduce the reference's squeeze() broadcast in
 *              the Y-tilde term (1d_BSPDE_case.py:271-273)
 */
typedef struct dbsde_problem {
  int kind;
  float mu_a, sig_a, sig_b;
  float phi_r, phi_c, phi_zz;
  int g_kind;
  float strike;
  int q3;
  int g_cols;
  float g_alpha;
  int u_clamp;
  float h_kappa, h_theta, h_sigma, h_rho;
} dbsde_problem;

typedef struct dbsde_config {
  int mode;          /* DBSDE_MODE_*                                   */
  int activation;    /* DBSDE_ACT_*                                    */
  int n_layers;      /* len(layers), 4..9                              */
  int layers[16];    /* [D+1, W1, ..., Wk, 1]                          */
  dbsde_problem problem;
  float T;           /* terminal time                                  */
  int device;        /* HIP device ordinal                             */
} dbsde_config;

typedef struct dbsde_ctx dbsde_ctx;

/* FBSNN.__init__ (network/problem construction; weights are caller-owned) */
int dbsde_create(const dbsde_config* cfg, dbsde_ctx** out);
void dbsde_destroy(dbsde_ctx* ctx);
const char* dbsde_last_error(const dbsde_ctx* ctx); /* ctx may be NULL */
int dbsde_abi_version(void);
int dbsde_set_stream(dbsde_ctx* ctx, void* hip_stream);

/* No reference counterpart (the reference has one stream).  The context
 * orders its internal streams with stream value operations (a wait spins
 * until the writer's queue has run the write); under anything that runs one
 * kernel at a time that wait would never end, so a context created in such an
 * environment orders them with events.  Returns 1 when the current process
 * environment selects events: DBSDE_STREAM_ORDER=events, AMD_SERIALIZE_KERNEL,
 * HIP_LAUNCH_BLOCKING, ROCPROF_COUNTER_COLLECTION, ROCPROF_COUNTERS,
 * HSA_TOOLS_LIB, an LD_PRELOAD naming rocprof, or any ROCPROFILER_* / ROCP_*
 * variable (DBSDE_STREAM_ORDER=values overrides all of them); 0 otherwise.
 * env: a NULL-terminated "NAME=VALUE" block to evaluate instead of the
 * process environment (NULL = the process environment).  The first context
 * of a process names its choice on stderr (DBSDE_QUIET=1 silences it).  Any
 * other serialising tool needs DBSDE_STREAM_ORDER=events. */
int dbsde_stream_order_by_events(const char* const* env);

/* size of the flat parameter vector = sum of state_dict numels */
long long dbsde_param_count(const dbsde_ctx* ctx);
/* host mask[i] = 1 if parameter element i receives a gradient (SURVEY Q6:
 * Resnet(stable) input_layers[-1] is never used and stays grad=None) */
int dbsde_param_used_mask(const dbsde_ctx* ctx, unsigned char* mask, long long n);

/* matrix-core form of this network's kernels (no reference counterpart:
 * reporting only).  Bit 0: the fused phase kernels, bit 1: the weight-gradient
 * kernel (wave-owned tiles, or the chain layouts' 128x128 tiles), bit 2: the
 * per-layer chain GEMMs (FC / Resnet layouts without a
 * fused variant) run fp32 operands as exact split-bf16 triples (six bf16 MFMAs
 * per product block, fp32 accumulation, error at or below the fp32-input
 * MFMA's); 0 = fp32-input MFMA (v_mfma_f32_16x16x4_f32) throughout.  Set at
 * create time (DBSDE_X3=0 / DBSDE_TNW_X3=0 select the fp32 forms). */
int dbsde_matrix_form(const dbsde_ctx* ctx);

/* Brownian dimension nb of a batch's W [M, N+1, nb]: D, or D/2 for Heston */
int dbsde_brownian_dim(const dbsde_ctx* ctx);

/*
 * Cholesky factor of the increments' correlation matrix for the DEVICE mode
 * (with_corr_high_dimension_pde.py:339-341: dW = L (sqrt(dt) z)).  L is a host
 * [n, n] row-major lower-triangular fp32 matrix, n = dbsde_brownian_dim <= 128;
 * the context keeps a device copy (staged in LDS by the path kernel).  L ==
 * NULL clears it.  Parity-mode batches (W != NULL) already carry correlated W
 * and ignore L.  DIAG problems only.
 */
int dbsde_set_corr(dbsde_ctx* ctx, const float* L, int n);

/*
 * One minibatch (FBSNN.fetch_minibatch output, DeepBSDE.py:247-262).
 *   W != NULL : parity mode, t [M,N+1] and W [M,N+1,nb] device fp32 exactly as
 *               the reference builds them (cumsum in fp64, cast).
 *   W == NULL : device mode, Brownian increments sqrt(dt)*N(0,1) drawn by an
 *               in-kernel Philox4x32-10 keyed by (seed, offset, global path,
 *               step, Brownian coordinate), correlated by L when set;
 *               t == NULL means the reference's grid fp32(cumsum_fp64(T/N)).
 *               A rank holding paths [path0, path0+M) of a larger batch draws
 *               exactly the increments a single device would draw for them.
 *   Xi         : device [xi_rows, D] initial state (Heston: [S_1..S_k, v_1..v_k]).
 */
typedef struct dbsde_batch {
  int M, N;
  const float* t;
  const float* W;
  unsigned long long seed, offset;
  long long path0;   /* global index of local path 0 (Philox stream of a rank's shard) */
  const float* Xi;   /* device [xi_rows, D], xi_rows in {1, M} */
  int xi_rows;
} dbsde_batch;

typedef struct dbsde_outputs {
  float* loss;   /* device scalar, nullable        */
  float* X;      /* device [M, N+1, D], nullable   */
  float* Y;      /* device [M, N+1], nullable      */
  float* Z;      /* device [M, N+1, D], nullable   */
} dbsde_outputs;

/*
 * Device FBSNN.fetch_minibatch (DeepBSDE.py:247-262, with_corr...py:316-353)
 * for a device-mode batch (batch->W must be NULL, batch->t NULL): writes t
 * [M, N+1] and, with increments == 0, W [M, N+1, nb] = fp32(fp64 cumsum of dW)
 * (the reference's layout), or with increments == 1 the raw dW
 * [M, N, nb] the device-mode rollout consumes (correlated when
 * dbsde_set_corr was called).
 */
int dbsde_brownian(dbsde_ctx* ctx, const dbsde_batch* batch, float* t, float* W, int increments);

/*
 * Roll out a device-mode batch ahead of the dbsde_loss_grad that consumes it
 * (the reference's next fetch_minibatch, DeepBSDE.py:247-262, drawn while the
 * current iteration runs: train() draws each iteration's batch independently
 * of the model, nd_BSPDE_case.py:371).  The batch is held back for the next
 * dbsde_loss_grad / dbsde_train_step: if that step runs the two-stream phase
 * pipeline, the rollout runs on its second stream after its weight-gradient
 * work, ordered before the following step; otherwise (or at any other call
 * that selects path buffers) it is issued then on an internal stream ordered
 * after the work queued on the context's stream, and work queued later
 * overlaps it.  A later
 * dbsde_loss_grad whose batch descriptor is identical (M, N, seed, offset,
 * path0, Xi pointer and rows; t = W = NULL) uses the prefetched paths instead
 * of rolling out; any other batch rolls out as usual.  At most two batches
 * are pending.  Xi is read when the rollout runs: it must not change after
 * this call until the batch is consumed or cancelled.  dbsde_set_corr drops
 * pending prefetches.
 */
int dbsde_prefetch(dbsde_ctx* ctx, const dbsde_batch* next);
/* Forget every pending prefetch (e.g. the caller is about to rewrite the Xi
 * buffer a prefetch read); later batches roll out as usual.  The context stream
 * is ordered after the pending rollouts, so their buffers are reused safely. */
int dbsde_prefetch_cancel(dbsde_ctx* ctx);

/*
 * FBSNN.loss_function + loss.backward (DeepBSDE.py:202-245, 279).
 * grad (device, flat, param_count) receives d loss / d params (overwritten,
 * 0 for unused parameters); grad == NULL runs the forward only (predict,
 * nd_BSPDE_case.py:412-443).
 */
int dbsde_loss_grad(dbsde_ctx* ctx, const float* params, const dbsde_batch* batch,
                    float* grad, const dbsde_outputs* out);

/* FBSNN.net_u (DeepBSDE.py:189-194): u [R] and Du [R,D] at R points
 * (Heston: the clamped u and its masked gradient, heston_dnnpde.py:560-579). */
int dbsde_net_u(dbsde_ctx* ctx, const float* params, int R, const float* t,
                const float* X, float* u, float* Du);

/* The vector-Jacobian product of net_u: the gradient the reference's autograd
 * graph of (u, Du) delivers (nd_BSPDE_case.py:191-221, create_graph=True),
 *   grad = d/dparams [ sum_r ubar[r] u[r] + sum_{r,d} zbar[r,d] Du[r,d] ]
 * at the R points (t [R], X [R,D]); ubar [R], zbar [R,D], grad (flat,
 * param_count) are device buffers (grad overwritten).  Not the gradient with
 * respect to X. */
int dbsde_net_u_vjp(dbsde_ctx* ctx, const float* params, int R, const float* t,
                    const float* X, const float* ubar, const float* zbar, float* grad);

/* optimizers (nd_BSPDE_case.py:331-350), torch.optim single-tensor formula order */
#define DBSDE_OPT_ADAM 0
#define DBSDE_OPT_ADAMW 1
#define DBSDE_OPT_SGD 2
#define DBSDE_OPT_RMSPROP 3   /* state: v = square_avg                 */
#define DBSDE_OPT_ADAGRAD 4   /* state: v = state_sum                  */
#define DBSDE_OPT_ADAMAX 5    /* state: m = exp_avg, v = exp_inf       */
#define DBSDE_OPT_ADADELTA 6  /* state: v = square_avg, m = acc_delta  */
#define DBSDE_OPT_ASGD 7      /* state: m = ax (averaged parameters)   */

typedef struct dbsde_optim {
  int kind;
  float lr, beta1, beta2, eps, weight_decay;
  float max_norm;    /* clip_grad_norm_(max_norm) before the step; <= 0: no clip */
  long long step;    /* 1-based step count of THIS update (bias correction) */
  float alpha;       /* RMSprop smoothing constant (torch default 0.99) */
  float rho;         /* Adadelta rho (0.9) */
  float lr_decay;    /* Adagrad lr_decay (0) */
  float lambd;       /* ASGD lambd (1e-4) */
  float asgd_eta;    /* ASGD eta and mu of THIS step: torch keeps them as fp32 */
  float asgd_mu;     /* state; the caller runs that recursion                   */
  const float* loss; /* nullable device scalar: skip the update when it is not
                        finite (heston_dnnpde.py:409-411 NaN skip)              */
  /* nullable device double[2]: the optimizer's step count kept on the device,
     so that a skipped update does not advance it (the reference `continue`s
     before optimizer.step(), heston_dnnpde.py:409-411).  When set, the update
     reads the completed step count from step_state[step_parity], runs update
     number count + 1 (bias corrections, Adagrad's clr, ASGD's eta / mu derived
     on the device from it; `step`, asgd_eta and asgd_mu are ignored) and writes
     the new count -- the old one when skipped -- to step_state[1 - step_parity].
     Successive calls alternate step_parity. */
  double* step_state;
  int step_parity;
} dbsde_optim;

/* clip_grad_norm_ + optimizer.step() (nd_BSPDE_case.py:383-384); m, v device
 * flat state owned by the caller (zero-initialised for a fresh optimizer). */
int dbsde_optimizer_step(dbsde_ctx* ctx, float* params, float* grad, float* m, float* v,
                         const dbsde_optim* opt);

/*
 * One training iteration of one process: dbsde_loss_grad followed by
 * dbsde_optimizer_step (nd_BSPDE_case.py:376-384: loss.backward(),
 * clip_grad_norm_, optimizer.step()).  When the update needs nothing but each
 * element's own gradient -- no clipping (max_norm <= 0), no NaN skip (loss ==
 * NULL) and a device step counter (step_state) -- it is applied inside the
 * gradient finalize kernels, element by element as each gradient is formed
 * (one launch fewer per step; grad is still written).  Otherwise the two calls
 * run in sequence.  Data-parallel callers, whose all-reduce sits between the
 * gradient and the update, use the two calls instead.
 */
int dbsde_train_step(dbsde_ctx* ctx, float* params, const dbsde_batch* batch, float* grad, float* m, float* v,
                     const dbsde_optim* opt, const dbsde_outputs* out);

/*
 * L-BFGS (torch.optim.LBFGS(params, lr) as nd_BSPDE_case.py:347-348 and
 * with_corr...py:386-387 build it; train() calls optimizer.step(closure) with a
 * closure that re-runs loss_function + backward on the same batch, without
 * clipping: nd_BSPDE_case.py:357-361,380-381).  The closure is dbsde_loss_grad;
 * the host runs torch's step logic (fbsnn.py) on these device-vector
 * primitives.  Vectors are device fp32 of n elements (the flat parameter
 * order); reductions are fixed-order fp64, returned to the host (they
 * synchronise the context stream).
 */
#define DBSDE_VEC_DOT 0    /* sum_i a_i b_i */
#define DBSDE_VEC_ASUM 1   /* sum_i |a_i|   (b unused) */
#define DBSDE_VEC_AMAX 2   /* max_i |a_i|   (b unused) */
int dbsde_vec_reduce(dbsde_ctx* ctx, int op, const float* a, const float* b, long long n, double* result);
/* z = alpha x + beta y in fp32 (z may alias x or y; y may be NULL when beta == 0) */
int dbsde_vec_axpby(dbsde_ctx* ctx, float* z, const float* x, const float* y, long long n, float alpha, float beta);
/* The L-BFGS two-loop recursion (torch's LBFGS.step direction), one launch:
 *   q = -g; for i = num-1..0: al_i = (s_i.q) ro_i, q -= al_i y_i;
 *   d = q h_diag; for i = 0..num-1: be_i = (y_i.d) ro_i, d += (al_i - be_i) s_i
 * s_i / y_i = rows slot[i] of the device [*, ld] history matrices S / Y (oldest
 * first, num <= 128); slot and ro are host arrays. */
int dbsde_lbfgs_direction(dbsde_ctx* ctx, const float* g, const float* S, const float* Y, long long ld, long long n,
                          const int* slot, const float* ro, int num, float h_diag, float* d);

/*
 * Exact / comparator solutions on the device (the references' evaluators):
 *   DBSDE_EXACT_BSB          u = exp((r + s^2)(T - t)) |x|^2    DeepBSDE.py:345-349
 *                            (r, s = p[0], p[1])
 *   DBSDE_EXACT_BS_CALL      Black-Scholes call price / delta of every coordinate
 *                            (nd_BSPDE_case.py:587-618; r, sigma, K = p[0..2])
 *   DBSDE_EXACT_BASKET_AVG   call on mean(x) with sigma / sqrt(D)
 *                            (with_corr...py:663-700; r, sigma, K = p[0..2])
 *   DBSDE_EXACT_BASKET_MEAN  mean over coordinates of the per-asset BS call
 *                            (with_corr...py:621-660; r, sigma, K = p[0..2])
 * t [R], x [R, D] device fp32; price and delta (nullable) [R * ncol],
 * ncol = D for BS_CALL, 1 otherwise.  At t >= T the payoff and its 0 / 1/2 / 1
 * delta are returned, as the references do.  Computed in fp64.
 */
#define DBSDE_EXACT_BSB 0
#define DBSDE_EXACT_BS_CALL 1
#define DBSDE_EXACT_BASKET_AVG 2
#define DBSDE_EXACT_BASKET_MEAN 3
int dbsde_exact(int kind, const float* t, const float* x, long long R, int D, float T, const double* params,
                float* price, float* delta, void* hip_stream);

/*
 * HJB Monte-Carlo comparator (hjb_implement.py:1088-1095):
 *   u(t, x) = -log( mean_k exp(-g(x + sqrt(2 |T - t|) z_k)) ),  g = log(1/2 + |y|^2/2)
 * over mc Philox draws z_k keyed by (seed, point index); t [P], x [P, D],
 * u [P] device.  Deterministic (fixed-order fp64 reduction).
 */
int dbsde_hjb_mc(const float* t, const float* x, int P, int D, float T, long long mc, unsigned long long seed,
                 float* u, void* hip_stream);

/* Per-kernel timing with HIP events on the context stream (bench/profiling). */
int dbsde_profile_enable(dbsde_ctx* ctx, int enable);
int dbsde_profile_count(dbsde_ctx* ctx);
int dbsde_profile_read(dbsde_ctx* ctx, int idx, char* name, int name_len, double* total_ms,
                       double* alg_flops, double* alg_bytes, long long* launches);
int dbsde_profile_reset(dbsde_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* DBSDE_H */
