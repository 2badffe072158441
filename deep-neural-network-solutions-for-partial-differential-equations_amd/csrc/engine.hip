// engine.hip -- context, buffers and launch sequence of the deep-BSDE step,
// exported through the C ABI of include/dbsde.h.
//
// One dbsde_loss_grad call = FBSNN.loss_function + loss.backward of the
// reference (DeepBSDE.py:202-245, 279) restated time-parallel:
//   prep      NAIS projection A_j (Q4), weight packing       (once per call)
//   rollout   Euler-Maruyama X path, sigma*dW                 (HBM-bound)
//   forward   x-stack GEMM + K block GEMMs, u                 (MFMA fp32)
//   input-grad K block GEMMs + Z GEMM with the residual epilogue
//   tangent   forward-mode along zbar                         (MFMA fp32)
//   reverse   K block GEMMs                                   (MFMA fp32)
//   weight-grad split-K TN GEMMs into slabs, fixed-order slab sums, NAIS adjoint
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <strings.h>
#include <vector>

#include "../../include/dbsde.h"

// the events that order the context's streams need no system-scope fence
// (device work only; kernels carry their own device-scope release / acquire):
// 0.4625 vs 0.4663 ms/step, M = 128 0.1448 vs 0.1474 (profiles/r5_ab_streams.txt)
#ifndef DBSDE_EVF
#define DBSDE_EVF (hipEventDisableTiming | hipEventDisableSystemFence)
#endif
// a prefetched rollout runs on the next chunked step's second stream
#ifndef DBSDE_DEFER_PF
#define DBSDE_DEFER_PF 1
#endif
// device-mode diagonal rollout: in-step by default the two-pass form (parallel
// draws into the sdw rows, then the Euler chains: rollout_draw_kernel +
// rollout_chain_kernel, ctx rollout2; DBSDE_ROLLOUT2=0 turns it off: M = 128
// 0.146 vs 0.156 ms/step, profiles/r6_ab_rollout.txt 4); prefetched, and else, the
// draws spread over the time steps (rollout_steps_kernel, DBSDE_RS = 1) or one
// thread per (path, column group) for all steps (rollout4_kernel, 0).  The prefetched rollout is off the step's
// critical path either way (0.4472 vs 0.4445 ms/step at M = 1024, 0.140 vs
// 0.140 at M = 128), but beside the phase section of a profiled step the
// step-parallel kernel's 4-wave, 32 KB-LDS workgroups slow the section by
// ~13 us: off (profiles/r6_ab_phase.txt 4).
#ifndef DBSDE_RS
#define DBSDE_RS 0
#endif
// chunk fork / join through stream memory operations (stream_order)
#ifndef DBSDE_MEMOPS
#define DBSDE_MEMOPS 1
#endif
#include "kernels.hpp"
#include "paths.hpp"
#include "phase.hpp"
#include "phase2.hpp"
#include "phasecs.hpp"

// minimum rows per weight-gradient row split of the chain layouts: 448 keeps
// HJB's 43,008 rows at the 96-split capacity (1.222-1.232 ms/step against
// 1.244-1.250 with 84 splits) and gives config 1's 13,056 rows 30 splits
// (0.457-0.465 against 0.483-0.494 ms with 96: a third of the finalize reads),
// profiles/r4_ab_tn_splits.txt
#ifndef DBSDE_TN_SPLIT_ROWS
#define DBSDE_TN_SPLIT_ROWS 448
#endif
#include "chainx3.hpp"
#include "tnx3.hpp"
#include "tnw.hpp"
#include "vec.hpp"

using namespace dbsde;

namespace {

thread_local std::string g_last_error;


inline int pad16(int x) { return (x + 15) / 16 * 16; }
inline int padw(int x) { return x <= 128 ? pad16(x) : (x + 127) / 128 * 128; }
inline int nt_for(int w) { return w <= 128 ? w / 16 : 8; }

struct Lin {
  long long w = -1, b = -1;
  int out = 0, in = 0;
};

struct ProfAgg {
  std::string name;
  double ms = 0, flops = 0, bytes = 0;
  long long n = 0;
};
struct ProfRec {
  int id;
  hipEvent_t e0, e1;
  double flops, bytes;
};

}  // namespace

struct dbsde_ctx {
  dbsde_config cfg{};
  std::string err;
  hipStream_t stream = nullptr;
  int device = 0;
  // path buffers (xin, sdw) x 2: a device-mode rollout can be prefetched into
  // the buffer the queued work no longer reads (dbsde_prefetch) on pf_stream
  float* xin_b[2] = {nullptr, nullptr};
  float* sdw_b[2] = {nullptr, nullptr};
  struct Pending {
    bool valid = false;
    dbsde_batch b{};
    hipEvent_t ready = nullptr;
    unsigned long long ready_v = 0;   // its order_mark token
    // joined_to is already ordered after this rollout (the second chunk stream
    // waited for it before its join into joined_to), so a consumer on that
    // stream need not wait; a consumer on any other stream (dbsde_set_stream
    // may have swapped it) waits for the ready mark
    bool joined = false;
    hipStream_t joined_to = nullptr;
    unsigned long long seq = 0;   // issue order: the older pending slot is the one replaced / reused
  } pend[2];
  unsigned long long pf_seq = 0;
  // a prefetch held back for the next chunked step, which runs the rollout on
  // its second stream after that stream's weight-gradient slices (the stream
  // finishes ahead of the main one); other steps issue it on pf_stream
  bool deferred = false;
  dbsde_batch defer_b{};
  hipStream_t pf_stream = nullptr;
  hipEvent_t ev_pf_order = nullptr;
  hipEvent_t ev_switch = nullptr;   // dbsde_set_stream: the new stream after the old one
  // path-chunked phase pipeline: chunk i runs phase A then phase C on stream
  // (main, pipe2)[i % 2], so one chunk's phase C fills the other's phase-A tail.
  // The context creates only the streams it uses (pipe2, pf_stream): a process
  // gets GPU_MAX_HW_QUEUES (4) hardware queues, and streams beyond that share
  // one, where a stream's event wait also holds the other streams' work queued
  // behind it (the prefetch stream shared the second chunk's queue, so the
  // second chunk's phase A started after the prefetched rollout)
  hipStream_t pipe2 = nullptr;
  hipEvent_t ev_pipe[2] = {nullptr, nullptr};
  // the fork / join of the two chunk streams as stream memory operations
  // (a value written by one stream, waited for by the other) instead of
  // events, when the device supports them: per step 36 us less queue time in
  // the stream model of tools/ubench/stream_gaps.hip (events 467, no-fence
  // events 458, value write / wait 431 us per step)
  bool memops = false;
  unsigned long long* d_order = nullptr;   // [slot] = last epoch written (ORD_* slots)
  unsigned long long order_epoch[8] = {};
  hipEvent_t ev_prof[2] = {nullptr, nullptr};
  // 0 = by size: two chunks only when one phase launch has more workgroups
  // than the chip has slots (below that the chunks only serialize: A0, C0 || A1,
  // C1 is three workgroup lifetimes against A, C's two); DBSDE_CHUNKS=n forces n
  int chunks = 0;
  int cus = 256;   // compute units of the device
  int fv_slots[64] = {0};   // resident workgroups of the chip per phase variant (lazily queried)
  int fv_cs = -1;           // the column-split variant of fv (phasecs.hpp), or -1
  int cs_mode = 2;          // 0 off, 1 always, 2 by batch size
  bool side_pending[2] = {false, false};

  // ---- network description
  int mode = 0, act = 0, K = 0, D = 0;
  int nb = 0;                 // Brownian dimension (D; D/2 for Heston)
  int gcols = 0;              // state columns entering g and the terminal Z loss
  bool heston = false, u_clamp = false;
  float* Lt = nullptr;        // correlated device mode: L^T [nb][nb] (dbsde_set_corr)
  std::vector<int> L;
  bool has_v = false, proj = false;
  float rho = 0.f;
  Lin in, out;
  std::vector<Lin> B, V;  // B[j-1], V[j-1] for block j = 1..K
  long long nparams = 0;
  std::vector<unsigned char> used;

  // ---- padded geometry
  int Dp = 0, Stot = 0, Stot_x = 0, Wmax = 0;
  std::vector<int> Wp, col;  // per level j = 0..K

  // ---- weight buffers (fixed)
  float *BtIn = nullptr, *BtZ = nullptr, *wout = nullptr, *bout = nullptr;
  std::vector<float*> Bf, Bb, beta, rtr, abar;
  double* norms = nullptr;
  long long* d_woffs = nullptr;   // NAIS: W_j offsets in the flat params
  float** d_rtr = nullptr;
  float** d_abar = nullptr;
  float** d_wsnap = nullptr;      // NAIS: W_j as of rtr_params_kernel (read by the projection adjoint)
  double* proj_part = nullptr;
  double* dot_part = nullptr;     // <Abar_j, R_j> partials from the gradient finalize (one per 64 elements)
  int dot_nblk = 0;               // partials slots per block (stride)
  int dot_nused = 0;              // partials the finalize writes (tilefin: one per 256 tile elements)
  unsigned char* d_used = nullptr;
  PackDesc* d_prep = nullptr;
  int n_prep = 0;

  int prep_blocks = 1;   // pack_tagged_kernel grid.x: one element per thread
  PackDesc* d_fin = nullptr;
  int n_fin = 0;
  TileFinTable* d_fintab = nullptr;   // tilefin_kernel: d_fin's windows grouped by problem tile
  std::vector<float*> slab;  // TN problem slabs (0 = x-stack, j = block j)
  std::vector<int> slab_mt, slab_nt, slab_mv, slab_nv;
  double* opt_part = nullptr;
  int opt_nparts = 0;
  double* vec_part = nullptr;     // L-BFGS reductions: VEC_RED_BLOCKS partials + the result

  // ---- row buffers (grow with Rp)
  int cap_rows = 0, cap_n = 0;
  float *xin = nullptr, *sdw = nullptr, *zbar = nullptr, *zfull = nullptr;
  float *Abuf = nullptr, *Adot = nullptr, *Delta = nullptr, *Alpha = nullptr, *H = nullptr, *Hdot = nullptr,
        *G = nullptr;
  float* Pbuf[2] = {nullptr, nullptr};
  float *u = nullptr, *rres = nullptr, *lossrow = nullptr, *ubar = nullptr, *q3S = nullptr, *umask = nullptr;
  float *u16 = nullptr, *o16 = nullptr;  // [Rp,16]: col 0 = ubar / 1 (output-layer TN operands)
  double* loss_part = nullptr;
  float* loss_tmp = nullptr;

  std::vector<void*> allocs;      // fixed-size buffers
  std::vector<void*> row_allocs;  // buffers sized by the row count (regrown)

  float* rowsum = nullptr;        // [Rp, 8] residual row sums (fused path)
  bool fused = false;             // wave-level fused phase kernels usable for this net
  bool x3 = false;                // ... in their split-bf16 form (phase.hpp)
  int fv = -1;                    // the fused variant (kFused index) or -1
  bool x3chain = false;           // per-layer chain GEMMs in split-bf16 form (chainx3.hpp)
  bool tnx3 = false;              // the split-K weight-gradient tiles in split-bf16 form (tnx3.hpp; !tnw layouts)
  // fragment images (phase.hpp) of every operand matrix: X_j = [W_in|b] / [V_j|b_j+c_j]
  // (out W, in Dp), Z_j = its transpose (out Dp, in W), F_j = B_j, Bk_j = B_j^T
  std::vector<float*> imgX, imgZ, imgF, imgB;
  int tn_splits = 96;              // weight-gradient GEMM row splits (A/B: 64..128 best on MI355X): slab capacity
  int tn_splits_cur = 96;          // the splits of the last weight-gradient launch (<= tn_splits)
  // wave-owned weight-gradient tiles (tnw.hpp): NAIS layouts with Dp == Wp
  bool tnw = false;
  int tnw_nb = 0, tnw_P = 0, tnw_S = 128;  // P * S = 1024 waves = one per SIMD at K = 3
  int tnw_Smax = 128;                       // slab capacity; tnw_S is set per batch (tnw_slices)
  bool tnw_x3 = false;                     // split-bf16 weight-gradient kernel (tnwx3.hip)
  bool rollout2 = true;                    // two-pass device-mode diagonal rollout (paths.hpp)
  float* slabW = nullptr;
  int fin_blocks = 1;             // slabsum grid.x

  // ---- profiling
  bool prof = false;
  std::vector<ProfAgg> agg;
  std::map<std::string, int> agg_idx;
  std::vector<ProfRec> pending;
  std::vector<hipEvent_t> ev_pool;
};

namespace {

int fail(dbsde_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  g_last_error = msg;
  return code;
}

#define HIPC(ctx, expr)                                                                         \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return fail(ctx, DBSDE_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));          \
  } while (0)

int dalloc(dbsde_ctx* c, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return fail(c, DBSDE_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  e = hipMemset(*p, 0, bytes);
  if (e != hipSuccess) return fail(c, DBSDE_EHIP, std::string("hipMemset: ") + hipGetErrorString(e));
  c->allocs.push_back(*p);
  return DBSDE_OK;
}
template <typename T>
int dalloc_t(dbsde_ctx* c, T** p, size_t n) {
  return dalloc(c, (void**)p, n * sizeof(T));
}

// A value wait is a kernel that spins until the value arrives, so it needs
// the writer's queue to make progress beside it: anything that runs one kernel
// at a time (kernel serialisation, launch blocking, rocprofv3 counter
// collection) would never run the write.  Those environments, any profiler /
// tool library the runtime loads (HSA_TOOLS_LIB, a preloaded rocprof library,
// ROCPROFILER_* / ROCP_* settings) and DBSDE_STREAM_ORDER=events order the
// streams with events instead; DBSDE_STREAM_ORDER=values forces value ops.
// Returns the reason (nullptr: value operations).
// (env: a NULL-terminated NAME=VALUE block, nullptr = the process environment)
const char* env_get(const char* const* env, const char* n) {
  if (!env) return getenv(n);
  const size_t k = strlen(n);
  for (; *env; ++env)
    if (!strncmp(*env, n, k) && (*env)[k] == '=') return *env + k + 1;
  return nullptr;
}
bool env_set(const char* n, const char* const* env = nullptr) {
  const char* v = env_get(env, n);
  return v && v[0] && strcmp(v, "0") != 0 && strcasecmp(v, "false") != 0;
}
extern "C" char** environ;
const char* events_reason(const char* const* env = nullptr) {
  if (const char* v = env_get(env, "DBSDE_STREAM_ORDER")) {
    if (strcmp(v, "events") == 0) return "DBSDE_STREAM_ORDER=events";
    if (strcmp(v, "values") == 0) return nullptr;
  }
  static const char* const serial[] = {"AMD_SERIALIZE_KERNEL", "HIP_LAUNCH_BLOCKING", "ROCPROF_COUNTER_COLLECTION",
                                       "ROCPROF_COUNTERS", "HSA_TOOLS_LIB"};
  for (const char* n : serial)
    if (env_set(n, env)) return n;
  if (const char* p = env_get(env, "LD_PRELOAD"))
    if (strstr(p, "rocprof")) return "LD_PRELOAD (rocprof)";
  for (const char* const* e = env ? env : environ; e && *e; ++e)
    if (!strncmp(*e, "ROCPROFILER_", 12) || !strncmp(*e, "ROCP_", 5)) return "ROCPROFILER_* / ROCP_* setting";
  return nullptr;
}
bool order_by_events() { return events_reason() != nullptr; }
// stderr line naming the ordering the first context chose (once per process)
void log_ordering(bool memops) {
  static bool done = false;
  if (done || env_set("DBSDE_QUIET")) return;
  done = true;
  const char* why = events_reason();
  fprintf(stderr, "dbsde: cross-stream order by %s%s%s\n", memops ? "stream value operations" : "events",
          why ? " -- " : (memops ? "" : " -- value waits unsupported by the device"), why ? why : "");
}

// Cross-stream order points: order_mark(slot, from) marks `from`'s current
// queue position and returns its token; order_wait(slot, token, to) holds
// `to` until `from` has passed that mark.  A wait takes the token of a mark
// already enqueued, so it never lacks its write.  Slots: the chunk fork and
// join, the prefetch stream after the caller's stream and back, the two
// prefetch buffers' rollouts.
enum { ORD_FORK = 0, ORD_JOIN = 1, ORD_PF_AFTER_MAIN = 2, ORD_MAIN_AFTER_PF = 3, ORD_PEND0 = 4, ORD_SWITCH = 6 };
hipEvent_t order_event(dbsde_ctx* c, int slot) {
  switch (slot) {
    case ORD_FORK: return c->ev_pipe[0];
    case ORD_JOIN: return c->ev_pipe[1];
    case ORD_PF_AFTER_MAIN:
    case ORD_MAIN_AFTER_PF: return c->ev_pf_order;
    case ORD_SWITCH: return c->ev_switch;
    default: return c->pend[slot - ORD_PEND0].ready;
  }
}
int order_mark(dbsde_ctx* c, int slot, hipStream_t from, unsigned long long& token) {
  if (c->memops) {
    token = ++c->order_epoch[slot];
    HIPC(c, hipStreamWriteValue64(from, c->d_order + slot, token, 0));
  } else {
    token = 0;
    HIPC(c, hipEventRecord(order_event(c, slot), from));
  }
  return DBSDE_OK;
}
int order_wait(dbsde_ctx* c, int slot, unsigned long long token, hipStream_t to) {
  if (c->memops)
    HIPC(c, hipStreamWaitValue64(to, c->d_order + slot, token, hipStreamWaitValueGte, ~0ull));
  else
    HIPC(c, hipStreamWaitEvent(to, order_event(c, slot), 0));
  return DBSDE_OK;
}
// `to` waits until `from` has reached this point of its queue
int stream_order(dbsde_ctx* c, hipStream_t from, hipStream_t to, int slot) {
  unsigned long long v = 0;
  int rc = order_mark(c, slot, from, v);
  return rc ? rc : order_wait(c, slot, v, to);
}

hipEvent_t get_event(dbsde_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

int prof_id(dbsde_ctx* c, const std::string& name) {
  auto it = c->agg_idx.find(name);
  if (it != c->agg_idx.end()) return it->second;
  int id = (int)c->agg.size();
  c->agg.push_back(ProfAgg{name});
  c->agg_idx[name] = id;
  return id;
}

// Launch wrapper: per-kernel HIP events when profiling is on.
template <typename F>
int run(dbsde_ctx* c, const char* name, double flops, double bytes, F&& launch) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->prof) {
    e0 = get_event(c);
    e1 = get_event(c);
    if (e0) (void)hipEventRecord(e0, c->stream);
  }
  launch();
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(c, DBSDE_EHIP, std::string(name) + ": " + hipGetErrorString(e));
  if (c->prof && e0 && e1) {
    (void)hipEventRecord(e1, c->stream);
    c->pending.push_back(ProfRec{prof_id(c, name), e0, e1, flops, bytes});
  }
  return DBSDE_OK;
}

#define RUN(ctx, name, fl, by, ...)                        \
  do {                                                     \
    int rc_ = run(ctx, name, fl, by, [&]() { __VA_ARGS__; }); \
    if (rc_) return rc_;                                   \
  } while (0)


// ---------------------------------------------------------------------------
// fused phase-kernel instantiations: (level tiles T, D tiles TD, blocks K)
struct FusedVariant {
  int T, TD, K, act, hv, x3;
  int rows;     // rows per workgroup: 64 (phase.hpp, or phase2 with one tile per wave) or 128 (phase2, two)
  int adot;     // phase C keeps adot_j in memory (phase2 ADOT)
  int xfirst;   // phase C image order: every x-stack image first (X0, X1..XK, F1..FK, B_K..B1)
  void (*A)(FusedArgs);
  void (*C)(FusedArgs);
};
// HV: the network has the NAIS x-stack (V_j); a template flag, so each kernel
// carries only its own code path (smaller straight-line kernels).  X3: the
// split-bf16 matrix-core form (phase.hpp), at width 110/112; the fp32-input
// MFMA form stays selectable (DBSDE_X3=0) and serves width 16.  phase2.hpp:
// the width-112 networks with two tiles per wave (DBSDE_NT=2; DBSDE_ADOT=1 the
// adot-in-memory phase C) and config 4's FC width 256.
#define FV(T, TD, K, ACT, HV, X3)                                                                      \
  {T, TD, K, ACT, HV, X3, P3_ROWS, 0, (X3) && (HV), phaseA_kernel<T, TD, K, ACT, HV, X3>, \
   phaseC_kernel<T, TD, K, ACT, HV, X3>}
#define FV2(T, TD, K, ACT, X3) FV(T, TD, K, ACT, true, X3), FV(T, TD, K, ACT, false, X3)
#define FQ(T, TD, K, ACT, HV, NT, NBUF, ADOT)                                                              \
  {T, TD, K, ACT, HV, 1, 64 * NT, ADOT, (HV) && !(ADOT), phaseA2_kernel<T, TD, K, ACT, HV, NT, NBUF, ADOT>, \
   phaseC2_kernel<T, TD, K, ACT, HV, NT, NBUF, ADOT>},
// column-split kernels (phasecs.hpp): 16 rows per workgroup, the small-M form
#define FCS(T, TD, K, ACT, HV) \
  {T, TD, K, ACT, HV, 1, CS_ROWS, 0, (HV), phaseAcs_kernel<T, TD, K, ACT, HV>, phaseCcs_kernel<T, TD, K, ACT, HV>},
const FusedVariant kFused[] = {
    DBSDE_PHASE2_INSTANCES(FQ)
    DBSDE_PHASECS_INSTANCES(FCS)
    FV2(7, 7, 3, 0, 1), FV2(7, 7, 3, 1, 1), FV2(7, 7, 3, 2, 1), FV2(7, 7, 3, 0, 0), FV2(7, 7, 3, 1, 0),
    FV2(7, 7, 3, 2, 0), FV2(1, 1, 1, 0, 0), FV2(1, 1, 1, 1, 0), FV2(1, 1, 1, 2, 0), FV2(1, 1, 2, 0, 0),
    FV2(1, 1, 2, 1, 0), FV2(1, 1, 2, 2, 0), FV2(1, 1, 3, 0, 0), FV2(1, 1, 3, 1, 0), FV2(1, 1, 3, 2, 0),
};
#undef FQ
#undef FCS
#undef FV2
#undef FV
constexpr int kNumFused = (int)(sizeof(kFused) / sizeof(kFused[0]));
static_assert(kNumFused <= 64, "dbsde_ctx::fv_slots");
// the variant for a network (each (T, TD, K, act, hv, x3) has at most one
// 64-row and one column-split instance)
// (DBSDE_W256=0 leaves the width-256 FC networks to the per-layer chain)
// (cs: the column-split variant, which the launch picks for small batches)
int fused_variant(int T, int TD, int K, int act, bool hv, bool x3, bool cs = false) {
  const char* ew = getenv("DBSDE_W256");
  const bool wide = !(ew && ew[0] == '0');
  for (int i = 0; i < kNumFused; ++i)
    if ((wide || kFused[i].T <= 8) && kFused[i].T == T && kFused[i].TD == TD && kFused[i].K == K &&
        kFused[i].act == act && kFused[i].hv == hv && kFused[i].x3 == (int)x3 && (kFused[i].rows == CS_ROWS) == cs)
      return i;
  return -1;
}

// ---------------------------------------------------------------------------
// network layout (state_dict order; oracle/timeparallel.param_layout mirrors it)
// ---------------------------------------------------------------------------
int build_net(dbsde_ctx* c) {
  const dbsde_config& g = c->cfg;
  if (g.n_layers < 4 || g.n_layers > 16) return fail(c, DBSDE_EINVAL, "len(layers) must be in [4, 16]");
  c->L.assign(g.layers, g.layers + g.n_layers);
  for (int v : c->L)
    if (v <= 0) return fail(c, DBSDE_EINVAL, "layer widths must be positive");
  const int n = g.n_layers;
  c->D = c->L[0] - 1;
  if (c->L.back() != 1) return fail(c, DBSDE_EINVAL, "last layer width must be 1 (u is a scalar)");
  if (c->D < 1) return fail(c, DBSDE_EINVAL, "layers[0] must be D+1 >= 2");
  c->K = n - 3;
  if (c->K > 6) return fail(c, DBSDE_EINVAL, "at most 6 hidden blocks (len(layers) <= 9) are supported");
  c->mode = g.mode;
  c->act = g.activation;
  if (c->act < 0 || c->act > 2) return fail(c, DBSDE_EINVAL, "unknown activation");
  long long off = 0;
  auto lin = [&](int o, int i) {
    Lin l;
    l.out = o;
    l.in = i;
    l.w = off;
    off += (long long)o * i;
    l.b = off;
    off += o;
    return l;
  };
  c->B.clear();
  c->V.clear();
  const auto& L = c->L;
  if (g.mode == DBSDE_MODE_FC) {
    c->has_v = false;
    c->proj = false;
    c->rho = 0.f;
    c->in = lin(L[1], L[0]);
    for (int j = 1; j <= c->K; ++j) c->B.push_back(lin(L[j + 1], L[j]));
    c->out = lin(L[n - 1], L[n - 2]);
  } else if (g.mode == DBSDE_MODE_NAIS_NET || g.mode == DBSDE_MODE_RESNET) {
    const bool st = g.mode == DBSDE_MODE_NAIS_NET;
    c->has_v = st;
    c->proj = st;
    c->rho = 1.f;
    c->in = lin(L[1], L[0]);
    for (int j = 1; j <= c->K; ++j) c->B.push_back(lin(L[j + 1], L[j]));
    c->out = lin(L[n - 1], L[n - 2]);
    if (st)
      for (int i = 1; i <= n - 2; ++i) {
        Lin v = lin(L[i], L[0]);
        if (i <= c->K) c->V.push_back(v);  // input_layers[K] is never used (Q6)
      }
  } else if (g.mode == DBSDE_MODE_NAISNET) {
    if (n < 4 || n > 6) return fail(c, DBSDE_EINVAL, "Naisnet supports len(layers) in {4,5,6}");
    c->has_v = true;
    c->proj = true;
    c->rho = 1.f;
    c->in = lin(L[1], L[0]);
    for (int j = 1; j <= c->K; ++j) {
      c->B.push_back(lin(L[j + 1], L[j]));
      c->V.push_back(lin(L[j + 1], L[0]));
    }
    c->out = lin(L[n - 1], L[n - 2]);
  } else {
    return fail(c, DBSDE_EINVAL, "unknown mode");
  }
  if (c->rho != 0.f)
    for (int j = 2; j < n - 1; ++j)
      if (L[j] != L[1]) return fail(c, DBSDE_EINVAL, "residual modes need equal hidden widths");
  if (c->proj && L[1] > NAIS_LMAX) return fail(c, DBSDE_EINVAL, "NAIS projection supports hidden width <= 128");
  c->nparams = off;
  c->used.assign(off, 1);
  if (g.mode == DBSDE_MODE_NAIS_NET) {
    // input_layers[K] occupies the tail of the flat vector
    const long long tail = (long long)L[n - 2] * L[0] + L[n - 2];
    std::fill(c->used.end() - tail, c->used.end(), 0);
  }
  // padded geometry
  c->Dp = pad16(c->D + 2);
  if (c->Dp > 128) return fail(c, DBSDE_EINVAL, "D > 126 is not supported by this build (Z epilogue tile)");
  c->Wp.resize(c->K + 1);
  c->col.resize(c->K + 1);
  c->Stot = 0;
  c->Wmax = 0;
  for (int j = 0; j <= c->K; ++j) {
    c->Wp[j] = padw(L[j + 1]);
    c->col[j] = c->Stot;
    c->Stot += c->Wp[j];
    c->Wmax = std::max(c->Wmax, c->Wp[j]);
  }
  c->Stot_x = c->has_v ? c->Stot : c->Wp[0];
  bool uniform = true;
  for (int j = 1; j <= c->K; ++j) uniform = uniform && c->Wp[j] == c->Wp[0];
  const char* env = getenv("DBSDE_FUSED");
  const bool allow = !(env && env[0] == '0');
  const char* ex3 = getenv("DBSDE_X3");
  const bool want_x3 = !(ex3 && ex3[0] == '0');
  c->x3 = want_x3 && fused_variant(c->Wp[0] / 16, c->Dp / 16, c->K, c->act, c->has_v, true) >= 0;
  c->fused = allow && uniform && fused_variant(c->Wp[0] / 16, c->Dp / 16, c->K, c->act, c->has_v, c->x3) >= 0;
  c->x3 = c->x3 && c->fused;
  c->fv = c->fused ? fused_variant(c->Wp[0] / 16, c->Dp / 16, c->K, c->act, c->has_v, c->x3) : -1;
  // the column-split form for small batches (DBSDE_CS=0 never, =1 always,
  // default when the 64-row kernels would fill at most half the chip's slots)
  {
    const char* ecs = getenv("DBSDE_CS");
    c->cs_mode = !ecs ? 2 : (ecs[0] == '0' ? 0 : 1);
    c->fv_cs = (c->fv >= 0 && c->cs_mode && kFused[c->fv].rows == P3_ROWS && c->x3)
                   ? fused_variant(c->Wp[0] / 16, c->Dp / 16, c->K, c->act, c->has_v, true, true)
                   : -1;
  }
  // FC / Resnet layouts the fused kernels do not cover: split-bf16 chain GEMMs
  // (uniform hidden width, output blocks a multiple of the column tile)
  // (the same layouts' weight-gradient tiles run split-bf16 behind the fused
  // phase kernels too: tnx3)
  c->tnx3 = want_x3 && !c->has_v && uniform && c->Dp <= 128;
  for (int j = 0; j <= c->K && c->tnx3; ++j) c->tnx3 = (c->Wp[j] / 16) % nt_for(c->Wp[j]) == 0;
  c->x3chain = c->tnx3 && !c->fused;
  // problem kind: Brownian dimension, g columns, u clamp
  const dbsde_problem& pr = g.problem;
  if (pr.kind != DBSDE_PROB_DIAG && pr.kind != DBSDE_PROB_HESTON) return fail(c, DBSDE_EINVAL, "unknown problem kind");
  if (pr.g_kind < 0 || pr.g_kind > 4) return fail(c, DBSDE_EINVAL, "unknown terminal condition");
  c->heston = pr.kind == DBSDE_PROB_HESTON;
  if (c->heston && c->D % 2 != 0)
    return fail(c, DBSDE_EINVAL, "Heston state is [S_1..S_k, v_1..v_k]: layers[0] - 1 must be even");
  c->nb = c->heston ? c->D / 2 : c->D;
  c->gcols = pr.g_cols > 0 ? pr.g_cols : c->D;
  if (c->gcols > c->D) return fail(c, DBSDE_EINVAL, "g_cols exceeds the state dimension");
  c->u_clamp = pr.u_clamp != 0;
  return DBSDE_OK;
}

PackDesc mk_desc(const float* src, int src_ld, float* dst, int dst_ld, int rows, int cols, int transpose,
                 int mode, float scale = 1.f) {
  PackDesc d{};
  d.src = src;
  d.src_ld = src_ld;
  d.dst = dst;
  d.dst_ld = dst_ld;
  d.rows = rows;
  d.cols = cols;
  d.transpose = transpose;
  d.mode = mode;
  d.scale = scale;
  return d;
}

// Pack descriptors use "relative" pointers: a src/dst value < 2^40 with bit
// flags is awkward, so instead we encode param/grad-relative addresses as
// offsets from a null base and fix them up per call (see fixup_descs).
constexpr uintptr_t kParamTag = (uintptr_t)1 << 62;
constexpr uintptr_t kGradTag = (uintptr_t)1 << 61;
inline float* ptag(long long off) { return (float*)(kParamTag | (uintptr_t)(off * 4)); }
inline float* gtag(long long off) { return (float*)(kGradTag | (uintptr_t)(off * 4)); }

int build_buffers(dbsde_ctx* c) {
  const int K = c->K, D = c->D, Dp = c->Dp;
  int rc;
  if ((rc = dalloc_t(c, &c->BtIn, (size_t)c->Stot_x * Dp))) return rc;
  if ((rc = dalloc_t(c, &c->BtZ, (size_t)Dp * c->Stot_x))) return rc;
  if ((rc = dalloc_t(c, &c->wout, (size_t)c->Wp[K]))) return rc;
  if ((rc = dalloc_t(c, &c->bout, 16))) return rc;
  c->Bf.assign(K + 1, nullptr);
  c->Bb.assign(K + 1, nullptr);
  c->beta.assign(K + 1, nullptr);
  c->rtr.assign(K + 1, nullptr);
  c->abar.assign(K + 1, nullptr);
  for (int j = 1; j <= K; ++j) {
    if ((rc = dalloc_t(c, &c->Bf[j], (size_t)c->Wp[j] * c->Wp[j - 1]))) return rc;
    if ((rc = dalloc_t(c, &c->Bb[j], (size_t)c->Wp[j - 1] * c->Wp[j]))) return rc;
    if ((rc = dalloc_t(c, &c->beta[j], (size_t)c->Wp[j]))) return rc;
  }
  const int LW = c->L[1];
  if (c->proj) {
    if ((rc = dalloc_t(c, &c->norms, (size_t)K + 1))) return rc;
    std::vector<float*> hr(K), ha(K), hs(K);
    std::vector<long long> hw(K);
    for (int j = 1; j <= K; ++j) {
      if ((rc = dalloc_t(c, &c->rtr[j], (size_t)LW * LW))) return rc;
      if ((rc = dalloc_t(c, &c->abar[j], (size_t)LW * LW))) return rc;
      if ((rc = dalloc_t(c, &hs[j - 1], (size_t)LW * LW))) return rc;
      hr[j - 1] = c->rtr[j];
      ha[j - 1] = c->abar[j];
      hw[j - 1] = c->B[j - 1].w;
    }
    if ((rc = dalloc_t(c, &c->proj_part, (size_t)K * std::max((LW * LW + 255) / 256, ((LW + 15) / 16) * ((LW + 15) / 16)))))
      return rc;
    c->dot_nblk = (LW * LW + 63) / 64;
    c->dot_nused = c->dot_nblk;   // tnw layouts override below
    if ((rc = dalloc_t(c, &c->dot_part, (size_t)K * c->dot_nblk))) return rc;
    if ((rc = dalloc_t(c, &c->d_rtr, K))) return rc;
    if ((rc = dalloc_t(c, &c->d_abar, K))) return rc;
    if ((rc = dalloc_t(c, &c->d_wsnap, K))) return rc;
    if ((rc = dalloc_t(c, &c->d_woffs, K))) return rc;
    HIPC(c, hipMemcpy(c->d_rtr, hr.data(), K * sizeof(float*), hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(c->d_abar, ha.data(), K * sizeof(float*), hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(c->d_wsnap, hs.data(), K * sizeof(float*), hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(c->d_woffs, hw.data(), K * sizeof(long long), hipMemcpyHostToDevice));
  }
  if ((rc = dalloc_t(c, &c->d_used, (size_t)c->nparams))) return rc;
  HIPC(c, hipMemcpy(c->d_used, c->used.data(), c->nparams, hipMemcpyHostToDevice));
  c->opt_nparts = 256;
  if ((rc = dalloc_t(c, &c->opt_part, c->opt_nparts))) return rc;

  // ---- fragment images for the phase kernels (phase.hpp)
  const int TW = c->Wp[0] / 16, TDp = Dp / 16;
  c->imgX.assign(K + 1, nullptr);
  c->imgZ.assign(K + 1, nullptr);
  c->imgF.assign(K + 1, nullptr);
  c->imgB.assign(K + 1, nullptr);
  // floats of an image with tout output / tin input blocks of 16: fp32
  // fragments (1 KiB each), or split-bf16 fragments (3 KiB per 32-wide block)
  const bool img_x3 = c->x3 || c->x3chain;
  auto img_floats = [&](int tout, int tin) -> size_t {
    return img_x3 ? (size_t)tout * ((tin + 1) / 2) * 768 : (size_t)tout * tin * 256;
  };
  if (c->fused || c->x3chain) {
    for (int j = 0; j <= (c->has_v ? K : 0); ++j) {
      if ((rc = dalloc_t(c, &c->imgX[j], img_floats(TW, TDp)))) return rc;
      if ((rc = dalloc_t(c, &c->imgZ[j], img_floats(TDp, TW)))) return rc;
    }
    for (int j = 1; j <= K; ++j) {
      if ((rc = dalloc_t(c, &c->imgF[j], img_floats(TW, TW)))) return rc;
      if ((rc = dalloc_t(c, &c->imgB[j], img_floats(TW, TW)))) return rc;
    }
  }
  const int fsplit = img_x3 ? 1 : 0;
  // the fused phase kernels read only the fragment images: their contexts skip
  // the fp32 copies the per-layer chain GEMMs use (half the pack writes, and
  // all of its transposed ones)
  const bool images_only = c->fused;
  auto frag = [fsplit, images_only](PackDesc d, float* img, int tin, int tout, int row0, int col0) {
    if (images_only) d.dst = nullptr;
    d.fdst = img;
    d.ftin = tin;
    d.ftout = tout;
    d.frow0 = row0;
    d.fcol0 = col0;
    d.fsplit = fsplit;
    return d;
  };

  // ---- prep descriptors: flat params -> packed weight buffers
  std::vector<PackDesc> P;
  auto add_x_level = [&](int j, const Lin& w, const Lin* b2) {
    float* dst = c->BtIn + (size_t)c->col[j] * Dp;
    P.push_back(frag(mk_desc(ptag(w.w), D + 1, dst, Dp, w.out, D + 1, 0, PK_COPY), c->imgX[j], TDp, TW, 0, 0));
    if (b2) {
      PackDesc d = mk_desc(ptag(w.b), 1, dst + D + 1, Dp, w.out, 1, 0, PK_ADD2);
      d.src2 = ptag(b2->b);
      d.src2_ld = 1;
      P.push_back(frag(d, c->imgX[j], TDp, TW, 0, D + 1));
    } else {
      P.push_back(frag(mk_desc(ptag(w.b), 1, dst + D + 1, Dp, w.out, 1, 0, PK_COPY), c->imgX[j], TDp, TW, 0, D + 1));
    }
    P.push_back(frag(mk_desc(ptag(w.w), D + 1, c->BtZ + c->col[j], c->Stot_x, w.out, D + 1, 1, PK_COPY), c->imgZ[j],
                     TW, TDp, 0, 0));
  };
  add_x_level(0, c->in, nullptr);
  if (c->has_v)
    for (int j = 1; j <= K; ++j) add_x_level(j, c->V[j - 1], &c->B[j - 1]);
  for (int j = 1; j <= K; ++j) {
    const Lin& b = c->B[j - 1];
    if (c->proj) {
      const int nblk = ((LW + 15) / 16) * ((LW + 15) / 16);
      PackDesc d = mk_desc(c->rtr[j], LW, c->Bf[j], c->Wp[j - 1], LW, LW, 0, PK_NEGPROJ);
      d.proj = c->proj_part + (size_t)(j - 1) * nblk;
      d.proj_n = nblk;
      d.proj_norm = c->norms + (j - 1);
      P.push_back(frag(d, c->imgF[j], TW, TW, 0, 0));
      d = mk_desc(c->rtr[j], LW, c->Bb[j], c->Wp[j], LW, LW, 1, PK_NEGPROJ);
      d.proj = c->proj_part + (size_t)(j - 1) * nblk;
      d.proj_n = nblk;
      d.proj_norm = nullptr;
      P.push_back(frag(d, c->imgB[j], TW, TW, 0, 0));
    } else {
      P.push_back(frag(mk_desc(ptag(b.w), b.in, c->Bf[j], c->Wp[j - 1], b.out, b.in, 0, PK_COPY), c->imgF[j], TW,
                       TW, 0, 0));
      P.push_back(frag(mk_desc(ptag(b.w), b.in, c->Bb[j], c->Wp[j], b.out, b.in, 1, PK_COPY), c->imgB[j], TW, TW, 0,
                       0));
      P.push_back(mk_desc(ptag(b.b), 1, c->beta[j], 1, b.out, 1, 0, PK_COPY));
    }
  }
  P.push_back(mk_desc(ptag(c->out.w), 1, c->wout, 1, c->out.in, 1, 0, PK_COPY));
  P.push_back(mk_desc(ptag(c->out.b), 1, c->bout, 1, 1, 1, 0, PK_COPY));
  c->n_prep = (int)P.size();
  c->prep_blocks = 1;
  for (const PackDesc& d : P) c->prep_blocks = std::max(c->prep_blocks, (d.rows * d.cols + 255) / 256);

  // ---- gradient slabs and finalize descriptors
  bool uniformW = true;
  for (int j = 0; j <= K; ++j) uniformW = uniformW && c->Wp[j] == c->Wp[0];
  // P = 2K + 2 problems in 4-wave workgroups: K odd
  c->tnw = c->has_v && uniformW && c->Wp[0] == Dp && Dp <= 128 && K <= 6 && (2 * K + 2) % 4 == 0;
  if (const char* e = getenv("DBSDE_TNW")) c->tnw = c->tnw && atoi(e) != 0;
  if (const char* e = getenv("DBSDE_ROLLOUT2")) c->rollout2 = atoi(e) != 0;
  std::vector<PackDesc> F;
  if (c->tnw) {
    const int T = Dp, P = 2 * K + 2, S = c->tnw_Smax;
    c->tnw_nb = T / 16;
    c->tnw_P = P;
    const char* ex = getenv("DBSDE_TNW_X3");
    c->tnw_x3 = c->x3 && c->tnw_nb == 7 && !(ex && ex[0] == '0');
    if (c->proj) {
      c->dot_nused = (T * T + TF_ELEMS - 1) / TF_ELEMS;
      if (c->dot_nused > c->dot_nblk) return fail(c, DBSDE_EINVAL, "internal: dot partials");
    }
    if ((rc = dalloc_t(c, &c->slabW, (size_t)S * P * T * T))) return rc;
    auto wsum = [&](int p, int r0, int c0, int rows, int cols, float* dst, int dst_ld, float scale) {
      PackDesc d = mk_desc(c->slabW + (size_t)p * T * T + (size_t)r0 * T + c0, T, dst, dst_ld, rows, cols, 0,
                           PK_SLABSUM, scale);
      d.nslab = S;
      d.slab_stride = (long long)P * T * T;
      d.sp = p;
      d.sr0 = r0;
      d.sc0 = c0;
      F.push_back(d);
    };
    // x-stack problems p = j (input layer, V_j), block problems p = K + j (B_j)
    wsum(0, 0, 0, c->in.out, D + 1, gtag(c->in.w), D + 1, 1.f);
    wsum(0, 0, D + 1, c->in.out, 1, gtag(c->in.b), 1, 1.f);
    for (int j = 1; j <= K; ++j) {
      const Lin& v = c->V[j - 1];
      wsum(j, 0, 0, v.out, D + 1, gtag(v.w), D + 1, 1.f);
      wsum(j, 0, D + 1, v.out, 1, gtag(v.b), 1, 1.f);
      wsum(j, 0, D + 1, v.out, 1, gtag(c->B[j - 1].b), 1, 1.f);
      const Lin& b = c->B[j - 1];
      wsum(K + j, 0, 0, b.out, b.in, c->abar[j], LW, -1.f);  // Abar = -Bbar
      F.back().dotR = c->rtr[j];
      F.back().dot_part = c->dot_part + (size_t)(j - 1) * c->dot_nblk;
    }
    // output layer: row 0 of problem 2K+1 is w_out, element (1, 0) is b_out
    wsum(2 * K + 1, 0, 0, 1, c->out.in, gtag(c->out.w), 1, 1.f);
    wsum(2 * K + 1, 1, 0, 1, 1, gtag(c->out.b), 1, 1.f);
  } else {
    c->slab.assign(K + 1, nullptr);
    c->slab_mt.assign(K + 1, 0);
    c->slab_nt.assign(K + 1, 0);
    c->slab_mv.assign(K + 2, 0);
    c->slab_nv.assign(K + 2, 0);
    auto mkslab = [&](int j, int m, int n) -> int {
      c->slab_mv[j] = m;
      c->slab_nv[j] = n;
      c->slab_mt[j] = (m + 63) / 64;
      c->slab_nt[j] = (n + 63) / 64;
      return dalloc_t(c, &c->slab[j], (size_t)c->tn_splits * c->slab_mt[j] * 64 * c->slab_nt[j] * 64);
    };
    c->slab.resize(K + 2, nullptr);
    c->slab_mt.resize(K + 2, 0);
    c->slab_nt.resize(K + 2, 0);
    c->slab_mv.resize(K + 2, 0);
    c->slab_nv.resize(K + 2, 0);
    if ((rc = mkslab(0, c->Stot_x, Dp))) return rc;
    for (int j = 1; j <= K; ++j)
      if ((rc = mkslab(j, c->Wp[j], c->Wp[j - 1] + (c->has_v ? 0 : 1)))) return rc;
    if ((rc = mkslab(K + 1, 16, c->Wp[K] + 1))) return rc;  // output layer: [w_out | b_out]

    auto slabsum = [&](int j, int r0, int c0, int rows, int cols, float* dst, int dst_ld, float scale) {
      const int ld = c->slab_nt[j] * 64;
      PackDesc d = mk_desc(c->slab[j] + (size_t)r0 * ld + c0, ld, dst, dst_ld, rows, cols, 0, PK_SLABSUM, scale);
      d.nslab = c->tn_splits;
      d.slab_stride = (long long)c->slab_mt[j] * 64 * ld;
      F.push_back(d);
    };
    slabsum(0, 0, 0, c->in.out, D + 1, gtag(c->in.w), D + 1, 1.f);
    slabsum(0, 0, D + 1, c->in.out, 1, gtag(c->in.b), 1, 1.f);
    if (c->has_v)
      for (int j = 1; j <= K; ++j) {
        const Lin& v = c->V[j - 1];
        slabsum(0, c->col[j], 0, v.out, D + 1, gtag(v.w), D + 1, 1.f);
        slabsum(0, c->col[j], D + 1, v.out, 1, gtag(v.b), 1, 1.f);
        slabsum(0, c->col[j], D + 1, v.out, 1, gtag(c->B[j - 1].b), 1, 1.f);
      }
    for (int j = 1; j <= K; ++j) {
      const Lin& b = c->B[j - 1];
      if (c->proj) {
        slabsum(j, 0, 0, b.out, b.in, c->abar[j], LW, -1.f);  // Abar = -Bbar
        F.back().dotR = c->rtr[j];
        F.back().dot_part = c->dot_part + (size_t)(j - 1) * c->dot_nblk;
      } else {
        slabsum(j, 0, 0, b.out, b.in, gtag(b.w), b.in, 1.f);
        slabsum(j, 0, c->Wp[j - 1], b.out, 1, gtag(b.b), 1, 1.f);
      }
    }
    slabsum(K + 1, 0, 0, 1, c->out.in, gtag(c->out.w), 1, 1.f);
    slabsum(K + 1, 0, c->Wp[K], 1, 1, gtag(c->out.b), 1, 1.f);
  }
  if (c->mode == DBSDE_MODE_NAIS_NET) {
    // Q6: input_layers[K] never receives a gradient; its slots are written as
    // zeros here so the gradient buffer needs no clearing memset
    const long long tail = (long long)c->L[c->cfg.n_layers - 2] * c->L[0] + c->L[c->cfg.n_layers - 2];
    PackDesc d = mk_desc(gtag(c->nparams - tail), 1, gtag(c->nparams - tail), (int)tail, 1, (int)tail, 0,
                         PK_SLABSUM, 1.f);
    d.nslab = 0;
    F.push_back(d);
  }
  c->n_fin = (int)F.size();
  c->fin_blocks = 1;
  for (const PackDesc& d : F) c->fin_blocks = std::max(c->fin_blocks, (d.rows * d.cols + 63) / 64);
  if (c->tnw) {
    // the windows of each problem tile (and, row P, the zero windows)
    TileFinTable tab{};
    const int Pn = c->tnw_P;
    if (Pn > TNW_PMAX_FIN) return fail(c, DBSDE_EINVAL, "internal: finalize table");
    for (const PackDesc& d : F) {
      const int row = d.nslab != 0 ? d.sp : Pn;
      if (row < 0 || row > Pn || tab.n[row] >= TF_WMAX) return fail(c, DBSDE_EINVAL, "internal: finalize windows");
      tab.w[row][tab.n[row]++] = d;
    }
    if ((rc = dalloc_t(c, &c->d_fintab, 1))) return rc;
    HIPC(c, hipMemcpy(c->d_fintab, &tab, sizeof(tab), hipMemcpyHostToDevice));
  }
  if ((rc = dalloc_t(c, &c->d_prep, P.size()))) return rc;
  if ((rc = dalloc_t(c, &c->d_fin, F.size()))) return rc;
  // descriptors are stored with tagged pointers; the kernel arguments carry the
  // real params/grad bases (pack_kernel_tagged below).
  HIPC(c, hipMemcpy(c->d_prep, P.data(), P.size() * sizeof(PackDesc), hipMemcpyHostToDevice));
  HIPC(c, hipMemcpy(c->d_fin, F.data(), F.size() * sizeof(PackDesc), hipMemcpyHostToDevice));
  return DBSDE_OK;
}

int ensure_rows(dbsde_ctx* c, int Rp, int N) {
  if (Rp <= c->cap_rows && N <= c->cap_n) return DBSDE_OK;
  const int nr = std::max(Rp, c->cap_rows), nn = std::max(N, c->cap_n);
  if (!c->row_allocs.empty()) {
    HIPC(c, hipStreamSynchronize(c->stream));
    if (c->pf_stream) HIPC(c, hipStreamSynchronize(c->pf_stream));
    if (c->pipe2) HIPC(c, hipStreamSynchronize(c->pipe2));
    c->pend[0].valid = c->pend[1].valid = false;
    c->deferred = false;
    for (void* p : c->row_allocs) {
      (void)hipFree(p);
      c->allocs.erase(std::find(c->allocs.begin(), c->allocs.end(), p));
    }
    c->row_allocs.clear();
  }
  const size_t first = c->allocs.size();
  const size_t R = nr;
  int rc;
  const int ldx = c->Dp, S = c->Stot;
  for (int i = 0; i < 2; ++i) {
    if ((rc = dalloc_t(c, &c->xin_b[i], R * ldx))) return rc;
    if ((rc = dalloc_t(c, &c->sdw_b[i], R * ldx))) return rc;
  }
  c->xin = c->xin_b[0];
  c->sdw = c->sdw_b[0];
  if ((rc = dalloc_t(c, &c->zbar, R * ldx))) return rc;
  if ((rc = dalloc_t(c, &c->zfull, R * ldx))) return rc;
  if ((rc = dalloc_t(c, &c->Abuf, R * S))) return rc;
  if ((rc = dalloc_t(c, &c->Adot, R * S))) return rc;
  if ((rc = dalloc_t(c, &c->Delta, R * S))) return rc;
  if ((rc = dalloc_t(c, &c->Alpha, R * S))) return rc;
  if ((rc = dalloc_t(c, &c->H, R * S))) return rc;
  if ((rc = dalloc_t(c, &c->Hdot, R * S))) return rc;
  if ((rc = dalloc_t(c, &c->G, R * S))) return rc;
  if ((rc = dalloc_t(c, &c->Pbuf[0], R * c->Wmax))) return rc;
  if ((rc = dalloc_t(c, &c->Pbuf[1], R * c->Wmax))) return rc;
  if ((rc = dalloc_t(c, &c->u, R + 64))) return rc;
  if ((rc = dalloc_t(c, &c->rres, R))) return rc;
  if ((rc = dalloc_t(c, &c->lossrow, R))) return rc;
  if ((rc = dalloc_t(c, &c->ubar, R))) return rc;
  if ((rc = dalloc_t(c, &c->umask, R))) return rc;
  if ((rc = dalloc_t(c, &c->u16, R * 16))) return rc;
  if ((rc = dalloc_t(c, &c->o16, R * 16))) return rc;
  fill_col0_kernel<<<(unsigned)((R + 255) / 256), 256, 0, c->stream>>>(c->o16, 16, (long long)R, 1.f);
  HIPC(c, hipGetLastError());
  if ((rc = dalloc_t(c, &c->loss_part, R / 16 + 2))) return rc;
  if ((rc = dalloc_t(c, &c->rowsum, R * 8))) return rc;
  if ((rc = dalloc_t(c, &c->loss_tmp, 16))) return rc;
  if ((rc = dalloc_t(c, &c->q3S, (size_t)nn + 1))) return rc;
  c->row_allocs.assign(c->allocs.begin() + first, c->allocs.end());
  c->cap_rows = nr;
  c->cap_n = nn;
  return DBSDE_OK;
}

// ---------------------------------------------------------------------------
// chain GEMM dispatch
// ---------------------------------------------------------------------------
template <int EPI>
int chain(dbsde_ctx* c, const char* name, ChainArgs& a, int Rp, int NP, int NT, double flops, double bytes) {
  dim3 grid(Rp / CH_BM, NP / (16 * NT));
  if (NP % (16 * NT) != 0) return fail(c, DBSDE_EINVAL, "internal: column tiling mismatch");
  if (a.K % CH_KC != 0) return fail(c, DBSDE_EINVAL, "internal: K not a multiple of 16");
  hipStream_t s = c->stream;
  // split-bf16 form (the weight image must hold this launch's output columns);
  // tile widths without an X3 instantiation (e.g. the Z GEMM at Dp = 32) run the
  // fp32 chain on the fp32 weights the packer writes alongside the images
  if (a.x3_img && (NT == 7 || NT == 8)) {
    if (a.x3_tout < NP / 16 || a.x3_ti * 16 < a.K) return fail(c, DBSDE_EINVAL, "internal: x3 chain image geometry");
    switch (NT) {
      case 7:
        RUN(c, name, flops, bytes, (chain_gemm_kernel<7, EPI, true><<<grid, 256, 0, s>>>(a)));
        return DBSDE_OK;
      case 8:
        RUN(c, name, flops, bytes, (chain_gemm_kernel<8, EPI, true><<<grid, 256, 0, s>>>(a)));
        return DBSDE_OK;
      default:
        return fail(c, DBSDE_EINVAL, "internal: x3 chain tile");
    }
  }
#define CASE_NT(X) \
  case X:          \
    RUN(c, name, flops, bytes, chain_gemm_kernel<X, EPI><<<grid, 256, 0, s>>>(a)); \
    break;
  switch (NT) {
    CASE_NT(1)
    CASE_NT(2)
    CASE_NT(3)
    CASE_NT(4)
    CASE_NT(5)
    CASE_NT(6)
    CASE_NT(7)
    CASE_NT(8)
    default:
      return fail(c, DBSDE_EINVAL, "internal: bad NT");
  }
#undef CASE_NT
  return DBSDE_OK;
}

ChainArgs base_args(dbsde_ctx* c) {
  ChainArgs a;
  memset(&a, 0, sizeof(a));
  a.rho = c->rho;
  a.act = c->act;
  return a;
}
// the split-bf16 chain form of a launch: weight image img with tout output /
// ti input 16-blocks (no-op for the fp32 chain)
void x3_weights(dbsde_ctx* c, ChainArgs& a, const float* img, int tout, int ti) {
  if (!c->x3chain) return;
  a.x3_img = (const unsigned short*)img;
  a.x3_tout = tout;
  a.x3_ti = ti;
}

// rows per 64-row phase-kernel workgroup (a multiple of the chain-GEMM tile,
// 64, and of the column-split workgroup, 16)
constexpr int ROW_PAD = P3_ROWS;
static_assert(ROW_PAD % CS_ROWS == 0, "row padding");

RolloutArgs rollout_args(dbsde_ctx* c, const dbsde_batch* b) {
  const dbsde_problem& pr = c->cfg.problem;
  RolloutArgs ra{};
  ra.M = b->M;
  ra.N = b->N;
  ra.D = c->D;
  ra.ldx = c->Dp;
  ra.nb = c->nb;
  ra.t = b->t;
  ra.W = b->W;
  ra.Xi = b->Xi;
  ra.xi_rows = b->xi_rows;
  ra.T = c->cfg.T;
  ra.seed = b->seed;
  ra.offset = b->offset;
  ra.path0 = b->path0;
  ra.mu_a = pr.mu_a;
  ra.sig_a = pr.sig_a;
  ra.sig_b = pr.sig_b;
  ra.kappa = pr.h_kappa;
  ra.theta = pr.h_theta;
  ra.hsig = pr.h_sigma;
  ra.rho = pr.h_rho;
  ra.Lt = c->Lt;
  ra.xin = c->xin;
  ra.sdw = c->sdw;
  return ra;
}

// the correlated path kernel for ceil(nb / 16) output blocks
void launch_corr(const RolloutArgs& ra, hipStream_t s) {
  const dim3 g((ra.M + CP_PATHS - 1) / CP_PATHS);
  switch ((ra.nb + 15) / 16) {
    case 1: rollout_corr_kernel<1><<<g, CP_THREADS, 0, s>>>(ra); break;
    case 2: rollout_corr_kernel<2><<<g, CP_THREADS, 0, s>>>(ra); break;
    case 3: rollout_corr_kernel<3><<<g, CP_THREADS, 0, s>>>(ra); break;
    case 4: rollout_corr_kernel<4><<<g, CP_THREADS, 0, s>>>(ra); break;
    case 5: rollout_corr_kernel<5><<<g, CP_THREADS, 0, s>>>(ra); break;
    case 6: rollout_corr_kernel<6><<<g, CP_THREADS, 0, s>>>(ra); break;
    case 7: rollout_corr_kernel<7><<<g, CP_THREADS, 0, s>>>(ra); break;
    default: rollout_corr_kernel<8><<<g, CP_THREADS, 0, s>>>(ra); break;
  }
}

// Euler-Maruyama paths (ra.out == PATH_ROLLOUT) or the device fetch_minibatch
// (PATH_FETCH_*): Heston, Cholesky-correlated device mode, or diagonal
// side: a prefetched rollout running beside other work (the two-pass form's
// 1456-workgroup draw pass floods the CUs the phase section runs on: 0.451 vs
// 0.443 ms/step prefetched at M = 1024, so it serves in-step rollouts only)
int launch_paths(dbsde_ctx* c, RolloutArgs& ra, bool side = false) {
  hipStream_t s = c->stream;
  const char* name = ra.out == PATH_ROLLOUT ? "rollout" : "brownian";
  const double steps = (double)ra.M * ra.N;
  const double bytes = ra.out == PATH_ROLLOUT ? 4.0 * steps * (2.0 * ra.D + (ra.W ? ra.nb : 0)) : 4.0 * steps * ra.nb;
  if (c->heston) {
    const int nthr = ra.M * ra.nb;
    RUN(c, name, 0.0, bytes, rollout_heston_kernel<<<(nthr + 255) / 256, 256, 0, s>>>(ra));
  } else if (c->Lt && !ra.W) {
    if (ra.ldx > cp_srow((ra.nb + 15) / 16) || ra.ldx % 4 != 0)
      return fail(c, DBSDE_EINVAL, "internal: correlated rollout row staging");
    RUN(c, name, 2.0 * steps * ra.nb * ra.nb / 2, bytes,
        launch_corr(ra, s));
  } else if (c->rollout2 && !side && ra.out == PATH_ROLLOUT && !ra.W && !ra.t && ra.ldx % 4 == 0) {
    // device-mode increments: parallel draws, then the Euler chains (paths.hpp)
    const long long draws = (long long)ra.M * ((ra.N + 3) / 4) * (ra.ldx / 4);
    const int chains = ra.M * (ra.ldx / 4);
    RUN(c, name, 0.0, bytes,
        rollout_draw_kernel<<<(unsigned)((draws + 255) / 256), 256, 0, s>>>(ra);
        rollout_chain_kernel<<<(unsigned)((chains + RC_THREADS - 1) / RC_THREADS), RC_THREADS, 0, s>>>(ra));
  } else if (DBSDE_RS && ra.out == PATH_ROLLOUT && !ra.W && ra.ldx % 4 == 0) {
    // device-mode increments: draws spread over the time steps (paths.hpp)
    const long long pairs = (long long)ra.M * (ra.ldx / 4);
    RUN(c, name, 0.0, bytes, rollout_steps_kernel<<<(unsigned)((pairs + RS_PAIRS - 1) / RS_PAIRS), RS_THREADS, 0, s>>>(ra));
  } else if (ra.out == PATH_ROLLOUT && ra.ldx % 4 == 0) {
    const int nthr = ra.M * (ra.ldx / 4);   // whole-row float4 stores
    RUN(c, name, 0.0, bytes, rollout4_kernel<<<(nthr + 255) / 256, 256, 0, s>>>(ra));
  } else {
    const int nthr = ra.M * ra.D;
    RUN(c, name, 0.0, bytes, rollout_kernel<<<(nthr + 255) / 256, 256, 0, s>>>(ra));
  }
  return DBSDE_OK;
}

bool same_batch(const dbsde_batch& a, const dbsde_batch& b) {
  return a.M == b.M && a.N == b.N && a.t == b.t && a.W == b.W && a.seed == b.seed && a.offset == b.offset &&
         a.path0 == b.path0 && a.Xi == b.Xi && a.xi_rows == b.xi_rows;
}
// dbsde_prefetch's rollout on pf_stream, ordered after everything queued so
// far on the caller's stream
int issue_prefetch(dbsde_ctx* c, const dbsde_batch* next, const float* avoid = nullptr) {
  int rc;
  const int M = next->M, N = next->N, R = M * (N + 1), Rp = (R + ROW_PAD - 1) / ROW_PAD * ROW_PAD;
  // a buffer no pending prefetch holds (else the older one's is replaced: its
  // rollout is earlier on the same stream), never `avoid`
  int j = !c->pend[0].valid ? 0 : (!c->pend[1].valid ? 1 : (c->pend[0].seq <= c->pend[1].seq ? 0 : 1));
  if (c->xin_b[j] == avoid) j = 1 - j;
  // after everything queued so far on the caller's stream (Xi ready, the
  // buffer's previous readers done); work queued later overlaps this
  if ((rc = stream_order(c, c->stream, c->pf_stream, ORD_PF_AFTER_MAIN))) return rc;
  hipStream_t main_stream = c->stream;
  float *xin0 = c->xin, *sdw0 = c->sdw;
  c->stream = c->pf_stream;
  c->xin = c->xin_b[j];
  c->sdw = c->sdw_b[j];
  hipError_t e = hipSuccess;
  if (Rp > R) e = hipMemsetAsync(c->xin + (size_t)R * c->Dp, 0, (size_t)(Rp - R) * c->Dp * 4, c->stream);
  if (e == hipSuccess) {
    RolloutArgs ra = rollout_args(c, next);
    ra.out = PATH_ROLLOUT;
    rc = launch_paths(c, ra, true);
  }
  c->stream = main_stream;
  c->xin = xin0;
  c->sdw = sdw0;
  if (e != hipSuccess) return fail(c, DBSDE_EHIP, std::string("prefetch: ") + hipGetErrorString(e));
  if (rc) return rc;
  if ((rc = order_mark(c, ORD_PEND0 + j, c->pf_stream, c->pend[j].ready_v))) return rc;
  c->pend[j].valid = true;
  c->pend[j].joined = false;
  c->pend[j].b = *next;
  c->pend[j].seq = ++c->pf_seq;
  return DBSDE_OK;
}
// issue a held-back prefetch on pf_stream now; avoid = the path buffer of a
// step whose kernels are already queued (mid-step), which it must not overwrite
int flush_deferred(dbsde_ctx* c, const float* avoid = nullptr) {
  if (!c->deferred) return DBSDE_OK;
  c->deferred = false;
  const dbsde_batch b = c->defer_b;
  return issue_prefetch(c, &b, avoid);
}
// the held-back prefetch on stream st (the chunked step's second stream, after
// its weight-gradient slices and its join into the main stream), into the path
// buffer the current step does not use: it runs beside the step's tail
// (finalize, projection adjoint, repack: a few latency-bound workgroups) and
// only the next step's phase A waits for it (its ready mark, wait_pending).
// Falls back to pf_stream when no buffer is free.
int launch_deferred_on(dbsde_ctx* c, hipStream_t st) {
  if (!c->deferred) return DBSDE_OK;
  int j = -1;
  for (int i = 0; i < 2 && j < 0; ++i)
    if (c->xin_b[i] != c->xin && !c->pend[i].valid) j = i;
  // no free buffer: issue it on pf_stream, never into the buffer this step's
  // queued kernels read (the older pending buffer is replaced instead)
  if (j < 0) return flush_deferred(c, c->xin);
  c->deferred = false;
  const dbsde_batch nb = c->defer_b;
  const int R = nb.M * (nb.N + 1), Rp = (R + ROW_PAD - 1) / ROW_PAD * ROW_PAD;
  hipStream_t main_stream = c->stream;
  float *xin0 = c->xin, *sdw0 = c->sdw;
  c->stream = st;
  c->xin = c->xin_b[j];
  c->sdw = c->sdw_b[j];
  hipError_t e = hipSuccess;
  int rc = DBSDE_OK;
  if (Rp > R) e = hipMemsetAsync(c->xin + (size_t)R * c->Dp, 0, (size_t)(Rp - R) * c->Dp * 4, st);
  if (e == hipSuccess) {
    RolloutArgs ra = rollout_args(c, &nb);
    ra.out = PATH_ROLLOUT;
    rc = launch_paths(c, ra, true);
  }
  c->stream = main_stream;
  c->xin = xin0;
  c->sdw = sdw0;
  if (e != hipSuccess) return fail(c, DBSDE_EHIP, std::string("prefetch: ") + hipGetErrorString(e));
  if (rc) return rc;
  if ((rc = order_mark(c, ORD_PEND0 + j, st, c->pend[j].ready_v))) return rc;
  c->pend[j].valid = true;
  c->pend[j].joined = false;
  c->pend[j].b = nb;
  c->pend[j].seq = ++c->pf_seq;
  return DBSDE_OK;
}

// order the context stream after pending rollout i: its ready mark, or, for a
// rollout joined into another stream (dbsde_set_stream changed it since), the
// latest chunk join (written on pipe2 after the rollout was ordered there)
int wait_pending(dbsde_ctx* c, int i) {
  const auto& p = c->pend[i];
  if (!p.joined) return order_wait(c, ORD_PEND0 + i, p.ready_v, c->stream);
  if (p.joined_to == c->stream) return DBSDE_OK;
  return order_wait(c, ORD_JOIN, c->order_epoch[ORD_JOIN], c->stream);
}

// Point c->xin / c->sdw at the path buffer this call uses.  A device-mode
// batch that dbsde_prefetch already rolled out takes that buffer (the main
// stream waits for the prefetch; from_pf = true); anything else takes a
// buffer no pending prefetch writes.
int select_paths(dbsde_ctx* c, const dbsde_batch* b, bool& from_pf) {
  from_pf = false;
  int use = -1;
  if (b && !b->W)
    for (int i = 0; i < 2 && use < 0; ++i)
      if (c->pend[i].valid && same_batch(c->pend[i].b, *b)) {
        use = i;
        from_pf = true;
      }
  if (use < 0) {
    // a buffer no prefetch holds; both pending and neither is this batch: the
    // older one's buffer is reused once its rollout is done
    use = !c->pend[0].valid ? 0 : (!c->pend[1].valid ? 1 : (c->pend[0].seq <= c->pend[1].seq ? 0 : 1));
    if (c->pend[use].valid) {
      const int rc = wait_pending(c, use);
      if (rc) return rc;
    }
  } else {
    const int rc = wait_pending(c, use);
    if (rc) return rc;
  }
  c->pend[use].valid = false;
  c->xin = c->xin_b[use];
  c->sdw = c->sdw_b[use];
  return DBSDE_OK;
}

int prep_weights(dbsde_ctx* c, const float* params);
int finalize_grads(dbsde_ctx* c, const float* params, float* grad, const double* loss_part = nullptr, int nloss = 0,
                   float* loss = nullptr, const FusedOpt* fo = nullptr);

}  // namespace

// tagged-pointer fixup happens inside a thin wrapper kernel
namespace dbsde {
__device__ __forceinline__ const float* untag(const float* p, const float* params, const float* grad) {
  uintptr_t v = (uintptr_t)p;
  if (v & ((uintptr_t)1 << 62)) return params + ((v & (((uintptr_t)1 << 61) - 1)) >> 2);
  if (v & ((uintptr_t)1 << 61)) return grad + ((v & (((uintptr_t)1 << 61) - 1)) >> 2);
  return p;
}
__device__ __forceinline__ void pack_block(const PackDesc* descs, int di, const float* params, float* grad) {
  PackDesc d = descs[di];
  d.src = untag(d.src, params, grad);
  d.src2 = untag(d.src2, params, grad);
  d.dst = (float*)untag(d.dst, params, grad);
  const int total = d.rows * d.cols;
  if ((int)blockIdx.x * 256 >= total) return;
  // the first element's source value in the round of the norm partials below
  const int i0 = blockIdx.x * 256 + threadIdx.x;
  const float rv0 = (d.mode == PK_NEGPROJ && i0 < total) ? d.src[(size_t)(i0 / d.cols) * d.src_ld + i0 % d.cols] : 0.f;
  // NAIS projection: |RtR|_F from rtr_params_kernel's partials (fixed order)
  __shared__ float nrm_s;
  if (d.mode == PK_NEGPROJ) {
    if (threadIdx.x < 64) {   // wave 0: lane b holds partials b, b + 64, ... ; fixed-order butterfly
      double sq = 0.0;
      for (int b = threadIdx.x; b < d.proj_n; b += 64) sq += d.proj[b];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
      if (threadIdx.x == 0) {
        const double n = sqrt(sq);
        nrm_s = (float)n;
        if (blockIdx.x == 0 && d.proj_norm) *d.proj_norm = n;
      }
    }
    __syncthreads();
  }
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int r = i / d.cols, cc = i - r * d.cols;
    float v;
    if (d.mode == PK_COPY) {
      v = d.scale * d.src[(size_t)r * d.src_ld + cc];
    } else if (d.mode == PK_ADD2) {
      v = d.src[(size_t)r * d.src_ld + cc] + d.src2[(size_t)r * d.src2_ld + cc];
    } else if (d.mode == PK_NEGPROJ) {
      const float rv = i == i0 ? rv0 : d.src[(size_t)r * d.src_ld + cc];
      const float nrm = nrm_s;
      float a = rv;
      if (nrm > 0.98f) a = ((float)0.98994949366116658 * rv) / sqrtf(nrm);
      a = a + (r == cc ? 0.01f : 0.f);
      v = -a;
    } else {
      const float* src = d.src + (size_t)r * d.src_ld + cc;
      double sa[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      int k = 0;
      for (; k + 8 <= d.nslab; k += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) sa[u] += src[(size_t)(k + u) * d.slab_stride];
      }
      for (; k < d.nslab; ++k) sa[0] += src[(size_t)k * d.slab_stride];
      const double s0 = (sa[0] + sa[1]) + (sa[2] + sa[3]), s1 = (sa[4] + sa[5]) + (sa[6] + sa[7]);
      const double s2 = 0.0, s3 = 0.0;
      v = d.scale * (float)((s0 + s1) + (s2 + s3));
    }
    if (d.dst) {
      if (d.transpose)
        d.dst[(size_t)cc * d.dst_ld + r] = v;
      else
        d.dst[(size_t)r * d.dst_ld + cc] = v;
    }
    if (d.fdst) {
      const int dr = (d.transpose ? cc : r) + d.frow0, dc = (d.transpose ? r : cc) + d.fcol0;
      if (d.fsplit) {
        // v = hi + mid + lo exactly: hi, mid rounded to nearest even, lo the
        // remainder (phase.hpp split_two)
        unsigned short* img = (unsigned short*)d.fdst + x3_off(dr, dc, d.ftout);
        const __bf16 h = (__bf16)v;
        const float r1 = v - (float)h;
        const __bf16 m = (__bf16)r1;
        const float r2 = r1 - (float)m;
        img[0] = __builtin_bit_cast(unsigned short, h);
        img[512] = __builtin_bit_cast(unsigned short, m);
        img[1024] = (unsigned short)(__float_as_uint(r2) >> 16);
      } else {
        d.fdst[frag_off(dr, dc, d.ftin, d.ftout)] = v;
      }
    }
  }
}
__global__ void __launch_bounds__(256) pack_tagged_kernel(const PackDesc* descs, const float* params, float* grad) {
  pack_block(descs, blockIdx.y, params, grad);
}
// RtR_j = W_j^T W_j (Functions/naisnet.py:33) and per-tile partial sums of
// squares for the Frobenius norm (fixed order).  One 16x16 output tile per
// 256-thread workgroup; the whole 16 x L and L x 16 operand strips (L <= 128)
// are staged in LDS with one round of independent loads (a K-tiled loop would
// chain L/16 dependent global-load latencies).
__device__ __forceinline__ void rtr_tile(const float* params, const long long* woffs, int L, float* const* rtr,
                                         float* const* wsnap, double* part, int nblk, int j, int tile) {
  __shared__ float As[16][NAIS_LMAX + 1];   // As[r][k] = W[k][16 ti + r]
  __shared__ float Bs[NAIS_LMAX][17];       // Bs[k][c] = W[k][16 tj + c]
  const int nt = (L + 15) / 16;
  const int ti = tile / nt, tj = tile % nt;
  const float* W = params + woffs[j];
  // every operand load in one round (a strided loop waited for each load
  // before the next: ~7 dependent global round trips)
  constexpr int PER = NAIS_LMAX * 16 / 256;
  float av[PER], bv[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int k = e >> 4, q = e & 15;
    const int ra = 16 * ti + q, cb = 16 * tj + q;
    av[u] = (k < L && ra < L) ? W[k * L + ra] : 0.f;
    bv[u] = (k < L && cb < L) ? W[k * L + cb] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int k = e >> 4, q = e & 15;
    if (k < L) {
      As[q][k] = av[u];
      Bs[k][q] = bv[u];
    }
  }
  __syncthreads();
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float v = 0.f;
  for (int k = 0; k < L; ++k) v += As[ty][k] * Bs[k][tx];
  const int row = ti * 16 + ty, col = tj * 16 + tx;
  // snapshot of W_j before this step's update (one 16 x 16 tile per block):
  // the fused optimizer update rewrites params while proj_backward_kernel's
  // other blocks still read W_j
  if (row < L && col < L) wsnap[j][row * L + col] = W[row * L + col];
  double sq = 0.0;
  if (row < L && col < L) {
    rtr[j][row * L + col] = v;
    sq = (double)v * (double)v;
  }
  __shared__ double red[256];
  red[threadIdx.x] = sq;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[j * nblk + tile] = red[0];
}
__global__ void __launch_bounds__(256) rtr_params_kernel(const float* params, const long long* woffs, int L,
                                                         float* const* rtr, float* const* wsnap, double* part, int nblk) {
  rtr_tile(params, woffs, L, rtr, wsnap, part, nblk, blockIdx.y, blockIdx.x);
}
// NAIS projection adjoint (Functions/naisnet.py:30-39 reversed), one kernel:
//   Abar_j = dL/dA_j (slab sums), R_j = W_j^T W_j, n = |R_j|_F
//   Rbar   = c n^-1/2 (Abar - 1/2 <Abar, R> R / n^2)  (Q4 branch taken, c = sqrt 0.98)
//          = Abar                                     (not taken)
//   Wbar_j = W_j (Rbar + Rbar^T)  -> grad
// Every block recomputes <Abar_j, R_j> in the same fixed order (L^2 products,
// cheap), so no separate reduction launch is needed; S = Rbar + Rbar^T is
// formed on the fly in the B tile of the LDS-tiled GEMM.
__global__ void __launch_bounds__(256) proj_backward_kernel(const float* const* wsnap, const long long* woffs,
                                                            float* const* abar, float* const* rtr, int L,
                                                            const double* proj_part, int proj_n, const double* dot_part,
                                                            int dot_nblk, int dot_nused, float* grad, FusedOpt fo,
                                                            int fuse) {
  __shared__ float As[16][NAIS_LMAX + 1];   // As[r][k] = W[16 ti + r][k]
  __shared__ float Bs[NAIS_LMAX][17];       // Bs[k][c] = S[k][16 tj + c], S = Rbar + Rbar^T
  __shared__ double dot_s, nrm_s;
  const int j = blockIdx.y, nt = (L + 15) / 16;
  const int ti = blockIdx.x / nt, tj = blockIdx.x % nt;
  const float* Ab = abar[j];
  const float* R = rtr[j];
  // W_j from the snapshot rtr_params_kernel took: with the fused update, the
  // blocks (ti, tj') of this launch rewrite params' W_j rows in place while
  // this block still reads them
  const float* W = wsnap[j];
  // every operand load in one round, before the scalars are known
  constexpr int PER = NAIS_LMAX * 16 / 256;
  float wv[PER], abs_[PER], rs[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int k = e >> 4, q = e & 15;
    const int ra = 16 * ti + q, cb = 16 * tj + q;
    const bool in = k < L;
    wv[u] = (in && ra < L) ? W[ra * L + k] : 0.f;
    const bool ok = in && cb < L;
    abs_[u] = ok ? Ab[k * L + cb] + Ab[cb * L + k] : 0.f;
    rs[u] = ok ? R[k * L + cb] + R[cb * L + k] : 0.f;
  }
  // this thread's parameter / moments for the fused update, in the same round
  const int row = ti * 16 + (threadIdx.x >> 4), col = tj * 16 + (threadIdx.x & 15);
  const bool own = row < L && col < L;
  const long long gi_idx = own ? woffs[j] + row * L + col : 0;
  OptVals pv{};
  if (fuse && own) pv = opt_load(gi_idx, fo.prm, fo.m, fo.v);
  // the optimizer scalars while the operand loads are in flight
  if (fuse) fused_opt_prologue(fo, false);
  if (threadIdx.x < 64) {   // <Abar_j, R_j> from the finalize partials, fixed-order butterfly
    double dsum = 0.0;
    for (int b = threadIdx.x; b < dot_nused; b += 64) dsum += dot_part[(size_t)j * dot_nblk + b];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dsum += __shfl_xor(dsum, o);
    // |R_j|_F from the rtr partials (proj_n <= 64), the phase kernels' order
    const double nrm = nais_norm_from(threadIdx.x < proj_n ? proj_part[(size_t)j * proj_n + threadIdx.x] : 0.0);
    if (threadIdx.x == 0) {
      dot_s = dsum;
      nrm_s = nrm;
    }
  }
  __syncthreads();
  const double dot = dot_s;
  const double n = nrm_s;
  const bool taken = (float)n > 0.98f;
  const float cA = taken ? (float)(0.98994949366116658 / sqrt(n)) : 1.f;
  const float cR = taken ? (float)(0.98994949366116658 / sqrt(n) * 0.5 * dot / (n * n)) : 0.f;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int k = e >> 4, q = e & 15;
    if (k < L) {
      As[q][k] = wv[u];
      Bs[k][q] = cA * abs_[u] - cR * rs[u];
    }
  }
  __syncthreads();
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc = 0.f;
  for (int k = 0; k < L; ++k) acc += As[ty][k] * Bs[k][tx];
  if (own) {
    grad[gi_idx] = acc;
    if (fuse) opt_apply(fo.a, gi_idx, acc, pv, fo.prm, fo.m, fo.v);
  }
}
}  // namespace dbsde

namespace {

int prep_weights(dbsde_ctx* c, const float* params) {
  hipStream_t s = c->stream;
  const int LW = c->L[1];
  if (c->proj) {
    const double fl = 2.0 * c->K * LW * (double)LW * LW;
    const int nblk = ((LW + 15) / 16) * ((LW + 15) / 16);
    RUN(c, "rtr", fl, 0.0,
        rtr_params_kernel<<<dim3(nblk, c->K), 256, 0, s>>>(params, c->d_woffs, LW, c->d_rtr, c->d_wsnap,
                                                            c->proj_part, nblk));
  }
  RUN(c, "pack_weights", 0.0, 0.0, pack_tagged_kernel<<<dim3(c->prep_blocks, c->n_prep), 256, 0, s>>>(c->d_prep, params, nullptr));
  return DBSDE_OK;
}

// Weight-gradient contraction, wave-owned tiles (tnw.hpp).  Problem p = j:
// x-stack level j (alpha_j^T x + delta_j^T zbar); p = K + j: block B_j
// (alpha_j^T h_{j-1} + delta_j^T hdot_{j-1}); plus the output-layer column sums.
// Slices [s0, s0 + sn) (sn < 0: all), on stream st without profiling records
// (st == nullptr: the context stream, profiled).
int launch_tnw(dbsde_ctx* c, int R, int Rp, int s0 = 0, int sn = -1, hipStream_t st = nullptr) {
  const int K = c->K, S = c->Stot, T = c->Dp;
  TNWArgs a;
  memset(&a, 0, sizeof(a));
  for (int j = 0; j <= K; ++j) {
    TNWProb& p = a.prob[j];
    p.A1 = c->Alpha + c->col[j];
    p.lda1 = S;
    p.B1 = c->xin;
    p.ldb1 = c->Dp;
    p.A2 = c->Delta + c->col[j];
    p.lda2 = S;
    p.B2 = c->zbar;
    p.ldb2 = c->Dp;
  }
  for (int j = 1; j <= K; ++j) {
    TNWProb& p = a.prob[K + j];
    p.A1 = c->Alpha + c->col[j];
    p.lda1 = S;
    p.B1 = c->H + c->col[j - 1];
    p.ldb1 = S;
    p.A2 = c->Delta + c->col[j];
    p.lda2 = S;
    p.B2 = c->Hdot + c->col[j - 1];
    p.ldb2 = S;
  }
  a.P = c->tnw_P;
  a.S = c->tnw_S;
  // the four waves of a workgroup (one CU, one slice, in step) share operand
  // rows through the CU's cache: group 0 = {x-stack 0, x-stack 1, block 1,
  // output}, group g = {x-stack 2g, 2g + 1, blocks 2g, 2g + 1} -- x / zbar
  // twice and alpha_j / delta_j of each block with its x-stack level
  for (int g = 0; g < a.P / 4; ++g) {
    int* o = a.order + 4 * g;
    if (g == 0) {
      o[0] = 0; o[1] = 1; o[2] = K + 1; o[3] = a.P - 1;
    } else {
      o[0] = 2 * g; o[1] = 2 * g + 1; o[2] = K + 2 * g; o[3] = K + 2 * g + 1;
    }
  }
  if (const char* e = getenv("DBSDE_TNW_ORDER"))   // A/B: 0 = problems in index order
    if (e[0] == '0')
      for (int q = 0; q < a.P; ++q) a.order[q] = q;
  a.s0 = s0;
  a.sn = sn < 0 ? a.S : sn;
  a.nchunk = Rp / 16;
  a.slab = c->slabW;
  a.ubar = c->ubar;
  a.Hk = c->H + c->col[K];
  a.Hdk = c->Hdot + c->col[K];
  a.ldh = S;
  a.R = R;
  if (Rp % 16 != 0 || c->Wp[K] != T || a.S % 8 != 0 || a.P != 2 * K + 2 || a.P % 4 != 0 || a.sn % 8 != 0 ||
      a.s0 < 0 || a.s0 + a.sn > a.S)
    return fail(c, DBSDE_EINVAL, "internal: tnw geometry");
  const double fl = 2.0 * 2.0 * (double)R * (K + 1) * c->L[1] * (c->D + 2) + 2.0 * 2.0 * (double)R * K * c->L[1] * c->L[1] +
                    4.0 * (double)R * c->L[K + 1];
  const unsigned grid = (unsigned)(a.S * a.P);
  hipStream_t s = c->stream;
  (void)grid;
  if (c->tnw_nb < 1 || c->tnw_nb > 8) return fail(c, DBSDE_EINVAL, "internal: tnw tile");
  if (st) {   // a slice range inside the phase pipeline (loss_grad_impl)
    const int lr = c->tnw_x3 ? (Rp % 32 != 0 ? -1 : tnw_x3_launch(c->tnw_nb, a, st)) : tnw_launch(c->tnw_nb, a, st);
    if (lr) return fail(c, DBSDE_EINVAL, "internal: tnw launch geometry");
    HIPC(c, hipGetLastError());
    return DBSDE_OK;
  }
  if (c->tnw_x3) {
    if (Rp % 32 != 0) return fail(c, DBSDE_EINVAL, "internal: tnw x3 geometry");
    int lr = 0;
    RUN(c, "tn_weight_grad", fl, 0.0, lr = tnw_x3_launch(c->tnw_nb, a, s));
    if (lr) return fail(c, DBSDE_EINVAL, "internal: tnw x3 launch geometry");
  } else {
    int lr = 0;
    RUN(c, "tn_weight_grad", fl, 0.0, lr = tnw_launch(c->tnw_nb, a, s));
    if (lr) return fail(c, DBSDE_EINVAL, "internal: tnw launch geometry");
  }
  return DBSDE_OK;
}

int finalize_grads(dbsde_ctx* c, const float* params, float* grad, const double* loss_part, int nloss, float* loss,
                   const FusedOpt* fo) {
  hipStream_t s = c->stream;
  FusedOpt fz{};
  const FusedOpt& f = fo ? *fo : fz;
  const int fuse = fo ? 1 : 0;
  if (fo && !c->tnw) return fail(c, DBSDE_EINVAL, "internal: fused update needs the tile finalize");
  if (c->tnw) {
    const int T = c->Dp;
    RUN(c, fuse ? "grad_finalize_update" : "grad_finalize", 0.0, 0.0,
        tilefin_kernel<<<dim3((T * T + TF_ELEMS - 1) / TF_ELEMS, c->tnw_P + 1), 256, 0, s>>>(
            c->d_fintab, c->slabW, c->tnw_S, c->tnw_P, T, grad, loss_part, nloss, loss, f, fuse));
  } else {
    RUN(c, "grad_finalize", 0.0, 0.0,
        slabsum_kernel<<<dim3(c->fin_blocks, c->n_fin), 256, 0, s>>>(c->d_fin, grad, c->tn_splits_cur, loss_part,
                                                                      nloss, loss));
  }
  if (c->proj) {
    const int LW = c->L[1];
    const int ntile = ((LW + 15) / 16) * ((LW + 15) / 16);
    RUN(c, "proj_backward", 2.0 * c->K * LW * (double)LW * LW, 0.0,
        proj_backward_kernel<<<dim3(ntile, c->K), 256, 0, s>>>(c->d_wsnap, c->d_woffs, c->d_abar, c->d_rtr, LW,
                                                               c->proj_part, ntile, c->dot_part, c->dot_nblk,
                                                               c->dot_nused, grad, f, fuse));
  }
  return DBSDE_OK;
}

// forward + input gradient for rows already in xin; leaves u, Abuf, H, Delta, G.
int forward_and_inputgrad(dbsde_ctx* c, int R, int Rp, bool need_u_only_and_z_store) {
  (void)need_u_only_and_z_store;
  const int K = c->K, S = c->Stot, D = c->D;
  const auto& L = c->L;
  // x-stack GEMM (a_0 and, for NAIS, the x V_j^T + beta_j parts of every level)
  {
    ChainArgs a = base_args(c);
    a.A = c->xin;
    a.lda = c->Dp;
    a.Bt = c->BtIn;
    x3_weights(c, a, c->imgX[0], c->Wp[0] / 16, c->Dp / 16);
    a.ldb = c->Dp;
    a.K = c->Dp;
    a.out[0] = c->Abuf;
    a.ldo[0] = S;
    a.out[1] = c->H;
    a.ldo[1] = S;
    a.lvl0_cols = c->Wp[0];
    int nv = 0;
    for (int j = 0; j <= (c->has_v ? K : 0); ++j) nv += L[j + 1];
    const double fl = 2.0 * R * (D + 1) * nv;
    int rc = chain<EPI_FWD0>(c, "gemm_xstack_fwd", a, Rp, c->Stot_x, nt_for(c->Wp[0]), fl,
                             4.0 * R * ((D + 1) + nv + L[1]));
    if (rc) return rc;
  }
  for (int j = 1; j <= K; ++j) {
    ChainArgs a = base_args(c);
    a.A = c->H + c->col[j - 1];
    a.lda = S;
    a.Bt = c->Bf[j];
    x3_weights(c, a, c->imgF[j], c->Wp[j] / 16, c->Wp[j - 1] / 16);
    a.ldb = c->Wp[j - 1];
    a.K = c->Wp[j - 1];
    a.in[0] = c->has_v ? c->Abuf + c->col[j] : nullptr;
    a.ldi[0] = S;
    a.vec[0] = c->beta[j];
    a.in[1] = c->H + c->col[j - 1];
    a.ldi[1] = S;
    a.out[0] = c->Abuf + c->col[j];
    a.ldo[0] = S;
    a.out[1] = c->H + c->col[j];
    a.ldo[1] = S;
    a.last = j == K;
    a.out[2] = c->Delta + c->col[K];
    a.ldo[2] = S;
    a.vec[1] = c->wout;
    const double fl = 2.0 * R * L[j] * L[j + 1];
    int rc = chain<EPI_FWD>(c, "gemm_block_fwd", a, Rp, c->Wp[j], nt_for(c->Wp[j]), fl,
                            4.0 * R * (L[j] + 4.0 * L[j + 1]));
    if (rc) return rc;
  }
  RUN(c, "rowdot_u", 2.0 * R * L[K + 1], 4.0 * R * L[K + 1],
      rowdot_kernel<<<Rp / 16, 256, 0, c->stream>>>(c->H + c->col[K], S, c->Wp[K], c->wout, c->bout, c->u, Rp,
                                                   c->u_clamp ? c->umask : nullptr));
  for (int j = K; j >= 1; --j) {
    ChainArgs a = base_args(c);
    a.A = c->Delta + c->col[j];
    a.lda = S;
    a.Bt = c->Bb[j];
    x3_weights(c, a, c->imgB[j], c->Wp[j - 1] / 16, c->Wp[j] / 16);
    a.ldb = c->Wp[j];
    a.K = c->Wp[j];
    a.in[0] = j == K ? nullptr : c->G + c->col[j];
    a.ldi[0] = S;
    a.vec[0] = c->wout;
    a.in[1] = c->Abuf + c->col[j - 1];
    a.ldi[1] = S;
    a.out[0] = c->G + c->col[j - 1];
    a.ldo[0] = S;
    a.out[1] = c->Delta + c->col[j - 1];
    a.ldo[1] = S;
    const double fl = 2.0 * R * L[j] * L[j + 1];
    int rc = chain<EPI_BWD>(c, "gemm_block_inputgrad", a, Rp, c->Wp[j - 1], nt_for(c->Wp[j - 1]), fl,
                            4.0 * R * (L[j + 1] + 4.0 * L[j]));
    if (rc) return rc;
  }
  return DBSDE_OK;
}

int zgemm_args(dbsde_ctx* c, ChainArgs& a) {
  a.A = c->Delta;
  a.lda = c->Stot;
  a.Bt = c->BtZ;
  x3_weights(c, a, c->imgZ[0], c->Dp / 16, c->Wp[0] / 16);
  a.ldb = c->Stot_x;
  a.K = c->Stot_x;
  a.out[0] = c->zfull;
  a.ldo[0] = c->Dp;
  return DBSDE_OK;
}

double zgemm_flops(dbsde_ctx* c, int R) {
  int nv = 0;
  for (int j = 0; j <= (c->has_v ? c->K : 0); ++j) nv += c->L[j + 1];
  return 2.0 * R * nv * c->D;
}

int validate_batch(dbsde_ctx* c, const dbsde_batch* b) {
  if (!b) return fail(c, DBSDE_EINVAL, "batch is NULL");
  if (b->M < 1 || b->N < 1) return fail(c, DBSDE_EINVAL, "M and N must be >= 1");
  if ((long long)b->M * (b->N + 1) > (1LL << 30)) return fail(c, DBSDE_EINVAL, "M*(N+1) too large");
  if (!b->Xi) return fail(c, DBSDE_EINVAL, "Xi is NULL");
  if (b->xi_rows != 1 && b->xi_rows != b->M) return fail(c, DBSDE_EINVAL, "Xi must have 1 or M rows");
  if (b->W && !b->t) return fail(c, DBSDE_EINVAL, "t is required with W");
  if (b->path0 < 0 || b->path0 + b->M > (1LL << 32)) return fail(c, DBSDE_EINVAL, "path0 out of range");
  return DBSDE_OK;
}

int nv_x(dbsde_ctx* c) {
  int nv = 0;
  for (int j = 0; j <= (c->has_v ? c->K : 0); ++j) nv += c->L[j + 1];
  return nv;
}

CotanParams cotan_params(dbsde_ctx* c, int R, int Rp, int N1, bool q3) {
  const dbsde_problem& pr = c->cfg.problem;
  CotanParams p{};
  p.R = R;
  p.Rp = Rp;
  p.N1 = N1;
  p.D = c->D;
  p.Dp = c->Dp;
  p.gcols = c->gcols;
  p.xin = c->xin;
  p.sdw = c->sdw;
  p.zfull = c->zfull;
  p.u = c->u;
  p.rowsum = c->rowsum;
  p.q3S = q3 ? c->q3S : nullptr;
  p.phi_r = pr.phi_r;
  p.phi_c = pr.phi_c;
  p.phi_zz = pr.phi_zz;
  p.strike = pr.strike;
  p.g_alpha = pr.g_alpha;
  p.g_kind = pr.g_kind;
  return p;
}

FusedArgs fused_args(dbsde_ctx* c, int R, int Rp, int N1, bool q3) {
  FusedArgs a;
  memset(&a, 0, sizeof(a));
  a.R = R;
  a.N1 = N1;
  a.D = c->D;
  a.gcols = c->gcols;
  a.u_clamp = c->u_clamp;
  a.Dp = c->Dp;
  a.W = c->Wp[0];
  a.S = c->Stot;
  a.has_v = c->has_v;
  a.act = c->act;
  a.rho = c->rho;
  a.xin = c->xin;
  for (int j = 1; j <= c->K; ++j) a.beta[j - 1] = c->beta[j];
  a.wout = c->wout;
  a.bout = c->bout;
  a.Abuf = c->Abuf;
  a.H = c->H;
  a.G = c->G;
  a.Delta = c->Delta;
  a.u = c->u;
  a.zfull = c->zfull;
  a.rowsum = c->rowsum;
  a.sdw = c->sdw;
  a.cp = cotan_params(c, R, Rp, N1, q3);
  a.zbar = c->zbar;
  a.ubar = c->ubar;
  a.u16 = c->tnw ? nullptr : c->u16;
  a.loss_part = c->loss_part;
  a.Hdot = c->Hdot;
  a.Alpha = c->Alpha;
  a.Adot = c->Adot;

  // stage sequences (phase.hpp): every image streamed as two pieces, input
  // blocks [0, H) and [H, TI)
  const int TW = c->Wp[0] / 16, TDp = c->Dp / 16, K = c->K;
  auto add = [&](const float** imgs, int* nfs, int& n, const float* img, int TO, int TI) {
    if (c->x3) {   // one piece per 32-wide input block: TO fragments of 3 chunks
      for (int kb = 0; kb < (TI + 1) / 2; ++kb) {
        imgs[n] = img + (size_t)kb * TO * 768;
        nfs[n++] = 3 * TO;
      }
      return;
    }
    if (TI < 2) {
      imgs[n] = img;
      nfs[n++] = TO * TI;
      return;
    }
    const int H = (TI + 1) / 2;
    imgs[n] = img;
    nfs[n++] = H * TO;
    imgs[n] = img + (size_t)H * TO * 256;
    nfs[n++] = (TI - H) * TO;
  };
  auto addA = [&](const float* img, int TO, int TI) { add(a.simgA, a.snfA, a.nA, img, TO, TI); };
  auto addC = [&](const float* img, int TO, int TI) { add(a.simgC, a.snfC, a.nC, img, TO, TI); };
  addA(c->imgX[0], TW, TDp);
  addC(c->imgX[0], TW, TDp);
  const bool xfirst = c->fv >= 0 && kFused[c->fv].xfirst;   // phase C's X-first stage order (phase.hpp)
  if (xfirst)
    for (int j = 1; j <= K; ++j) addC(c->imgX[j], TW, TDp);
  for (int j = 1; j <= K; ++j) {
    addA(c->imgF[j], TW, TW);
    addC(c->imgF[j], TW, TW);
    if (c->has_v) {
      addA(c->imgX[j], TW, TDp);
      if (!xfirst) addC(c->imgX[j], TW, TDp);
    }
  }
  for (int j = K; j >= 1; --j) {
    if (c->has_v) addA(c->imgZ[j], TDp, TW);
    addA(c->imgB[j], TW, TW);
    addC(c->imgB[j], TW, TW);
  }
  addA(c->imgZ[0], TDp, TW);
  return a;
}

// the split-bf16 phase kernels (T == TD) hold their piece counts at compile
// time (phase.hpp PieceStager NP) and the piece pointers in one VGPR's lanes
bool fused_piece_counts_ok(dbsde_ctx* c, const FusedArgs& a) {
  const int TW = c->Wp[0] / 16, TDp = c->Dp / 16, K = c->K, hv = c->has_v ? 1 : 0;
  if (!c->x3 || TW != TDp) return a.nA <= 64 && a.nC <= 64;
  const int nkb = (TW + 1) / 2;
  return a.nA == nkb * (2 + 2 * K * (1 + hv)) && a.nC == nkb * (1 + K * (2 + hv)) && a.nA <= 64 && a.nC <= 64;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int dbsde_abi_version(void) { return DBSDE_ABI_VERSION; }

int dbsde_matrix_form(const dbsde_ctx* c) {
  if (!c) return 0;
  // bit 1: the wave-tile weight-gradient kernel in split-bf16 form, or the
  // chain layouts' weight-gradient tiles (tnx3.hpp, split-bf16 with x3chain)
  const bool tn_x3 = c->tnw ? c->tnw_x3 : c->tnx3;
  return (c->x3 ? 1 : 0) | (tn_x3 ? 2 : 0) | (c->x3chain ? 4 : 0);
}

const char* dbsde_last_error(const dbsde_ctx* ctx) {
  if (ctx && !ctx->err.empty()) return ctx->err.c_str();
  return g_last_error.c_str();
}

int dbsde_create(const dbsde_config* cfg, dbsde_ctx** out) {
  if (!cfg || !out) return fail(nullptr, DBSDE_EINVAL, "cfg/out is NULL");
  *out = nullptr;
  dbsde_ctx* c = new dbsde_ctx();
  c->cfg = *cfg;
  c->device = cfg->device;
  int rc = build_net(c);
  if (!rc) {
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) rc = fail(c, DBSDE_EHIP, "no HIP device available");
    else if (cfg->device < 0 || cfg->device >= ndev) rc = fail(c, DBSDE_EINVAL, "bad device ordinal");
    else if ((e = hipSetDevice(cfg->device)) != hipSuccess) rc = fail(c, DBSDE_EHIP, hipGetErrorString(e));
    else if ((e = hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, cfg->device)) != hipSuccess)
      rc = fail(c, DBSDE_EHIP, hipGetErrorString(e));
    if (const char* ec = getenv("DBSDE_CHUNKS")) c->chunks = std::max(0, atoi(ec));
  }
  if (!rc) rc = build_buffers(c);
  if (!rc) {
    hipError_t e = hipStreamCreateWithFlags(&c->pipe2, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
      e = hipEventCreateWithFlags(&c->ev_pipe[i], DBSDE_EVF);
      if (e == hipSuccess) e = hipEventCreate(&c->ev_prof[i]);
    }
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->pf_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_pf_order, DBSDE_EVF);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_switch, DBSDE_EVF);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->pend[i].ready, DBSDE_EVF);
    if (e != hipSuccess) rc = fail(c, DBSDE_EHIP, std::string("side stream: ") + hipGetErrorString(e));
    int wv = 0;
    if (!rc && DBSDE_MEMOPS && !order_by_events() &&
        hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, c->device) == hipSuccess && wv)
      c->memops = (rc = dalloc_t(c, &c->d_order, 8)) == DBSDE_OK;
    if (!rc) log_ordering(c->memops);
  }
  if (rc) {
    g_last_error = c->err;
    dbsde_destroy(c);
    return rc;
  }
  *out = c;
  return DBSDE_OK;
}

void dbsde_destroy(dbsde_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->pipe2) (void)hipStreamSynchronize(c->pipe2);
  if (c->pf_stream) {
    (void)hipStreamSynchronize(c->pf_stream);
    (void)hipStreamDestroy(c->pf_stream);
  }
  if (c->ev_pf_order) (void)hipEventDestroy(c->ev_pf_order);
  if (c->ev_switch) (void)hipEventDestroy(c->ev_switch);
  for (int i = 0; i < 2; ++i) {
    if (c->pend[i].ready) (void)hipEventDestroy(c->pend[i].ready);
    if (c->ev_pipe[i]) (void)hipEventDestroy(c->ev_pipe[i]);
    if (c->ev_prof[i]) (void)hipEventDestroy(c->ev_prof[i]);
  }
  if (c->pipe2) (void)hipStreamDestroy(c->pipe2);
  for (auto& r : c->pending) {
    c->ev_pool.push_back(r.e0);
    c->ev_pool.push_back(r.e1);
  }
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  for (void* p : c->allocs) (void)hipFree(p);
  delete c;
}

int dbsde_set_stream(dbsde_ctx* c, void* s) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  const hipStream_t ns = (hipStream_t)s;
  if (ns != c->stream && c->ev_switch) {
    // the context's workspace (row buffers, pending rollouts, slabs) is
    // written by the work already queued on the old stream: the new stream
    // starts after it, so a caller may switch streams between calls without
    // ordering them itself (no cost while the stream stays the same)
    HIPC(c, hipSetDevice(c->device));
    const int rc = stream_order(c, c->stream, ns, ORD_SWITCH);
    if (rc) return rc;
  }
  c->stream = ns;
  return DBSDE_OK;
}

int dbsde_stream_order_by_events(const char* const* env) { return events_reason(env) ? 1 : 0; }

long long dbsde_param_count(const dbsde_ctx* c) { return c ? c->nparams : -1; }

int dbsde_param_used_mask(const dbsde_ctx* c, unsigned char* mask, long long n) {
  if (!c || !mask || n != c->nparams) return fail(nullptr, DBSDE_EINVAL, "bad mask buffer");
  memcpy(mask, c->used.data(), (size_t)n);
  return DBSDE_OK;
}

}  // extern "C"

namespace {
// dbsde_loss_grad, and dbsde_train_step's fused form (fo != NULL: the
// optimizer update is applied inside the gradient finalize)
// Everything after the cotangents: for the per-layer (chain) form the forward
// tangent along zbar and the reverse, then the weight-gradient contraction and
// the finalize (+ the fused optimizer update).  Shared by loss_grad_impl and
// the net_u VJP.
// The chain layouts' weight-gradient problems over S_ row splits (split-bf16
// tiles + the output-layer GEMV, or the fp32 split-K GEMM): arguments and
// launch geometry, shared by the launch after the phase section and the
// per-chunk launches inside the two-stream pipeline
struct TNGeom {
  int S_ = 0, maxt = 0, maxt3 = 0, rps32 = 0;
  double tfl = 0.0;
  float* oslab = nullptr;
  long long sstride = 0;
};
// align > 0 (split-bf16 form): the row count of the first path chunk, which
// must then end on a split boundary -- when the default split does not, the
// largest 32-row multiple no longer than it that divides align is taken
int tn_setup(dbsde_ctx* c, int R, int Rp, TNArgs& ta, TNGeom& g, long long align = 0) {
  const auto& L = c->L;
  const int K = c->K, S = c->Stot, D = c->D;
  memset(&ta, 0, sizeof(ta));
  // row splits for this batch: at least DBSDE_TN_SPLIT_ROWS rows each, at
  // most the slab capacity; every kernel below covers all S_ splits, empty
  // ones writing zeros, and the finalize sums exactly S_ of them
  int S_ = std::min(c->tn_splits, std::max(8, (Rp + DBSDE_TN_SPLIT_ROWS - 1) / DBSDE_TN_SPLIT_ROWS));
  if (align > 0 && c->tnx3) {
    int r32 = ((Rp + S_ - 1) / S_ + 31) / 32 * 32;
    if (align % r32 != 0) {
      for (r32 -= 32; r32 >= 32 && align % r32 != 0; r32 -= 32) {
      }
      if (r32 >= 32 && (Rp + r32 - 1) / r32 <= c->tn_splits) S_ = (Rp + r32 - 1) / r32;
    }
  }
  g.S_ = c->tn_splits_cur = S_;
  const int rps = ((Rp + S_ - 1) / S_ + TN_KC - 1) / TN_KC * TN_KC;
  ta.rows_per_split = rps;
  ta.Rp = Rp;
  double& tfl = g.tfl;
  tfl = 0.0;
  {
    TNProb& p0 = ta.prob[0];
    p0.A[0] = c->Alpha;
    p0.lda[0] = S;
    p0.nA[0] = c->Stot_x;
    p0.B[0] = c->xin;
    p0.ldb[0] = c->Dp;
    p0.nB[0] = c->Dp;
    p0.A[1] = c->Delta;
    p0.lda[1] = S;
    p0.nA[1] = c->Stot_x;
    p0.B[1] = c->zbar;
    p0.ldb[1] = c->Dp;
    p0.nB[1] = c->Dp;
    p0.npairs = 2;
    p0.ones_col = -1;
    p0.mv = c->slab_mv[0];
    p0.nv = c->slab_nv[0];
    p0.mt = c->slab_mt[0];
    p0.nt = c->slab_nt[0];
    p0.slab = c->slab[0];
    int nv = 0;
    for (int j = 0; j <= (c->has_v ? K : 0); ++j) nv += L[j + 1];
    tfl += 2.0 * 2.0 * R * nv * (D + 2);
  }
  int& maxt = g.maxt;
  maxt = ta.prob[0].mt * ta.prob[0].nt;
  for (int j = 1; j <= K; ++j) {
    TNProb& pj = ta.prob[j];
    pj.A[0] = c->Alpha + c->col[j];
    pj.lda[0] = S;
    pj.nA[0] = c->Wp[j];
    pj.B[0] = c->H + c->col[j - 1];
    pj.ldb[0] = S;
    pj.nB[0] = c->Wp[j - 1];
    pj.A[1] = c->Delta + c->col[j];
    pj.lda[1] = S;
    pj.nA[1] = c->Wp[j];
    pj.B[1] = c->Hdot + c->col[j - 1];
    pj.ldb[1] = S;
    pj.nB[1] = c->Wp[j - 1];
    pj.npairs = 2;
    pj.ones_col = c->has_v ? -1 : c->Wp[j - 1];
    pj.mv = c->slab_mv[j];
    pj.nv = c->slab_nv[j];
    pj.mt = c->slab_mt[j];
    pj.nt = c->slab_nt[j];
    pj.slab = c->slab[j];
    maxt = std::max(maxt, pj.mt * pj.nt);
    tfl += 2.0 * 2.0 * R * L[j] * (L[j + 1] + (c->has_v ? 0 : 1));
  }
  {
    // output layer: [w_out | b_out] = sum_r ubar_r [h_{K+1} | 1] + hdot_{K+1}
    TNProb& po = ta.prob[K + 1];
    po.A[0] = c->u16;
    po.lda[0] = 16;
    po.nA[0] = 16;
    po.B[0] = c->H + c->col[K];
    po.ldb[0] = S;
    po.nB[0] = c->Wp[K];
    po.A[1] = c->o16;
    po.lda[1] = 16;
    po.nA[1] = 16;
    po.B[1] = c->Hdot + c->col[K];
    po.ldb[1] = S;
    po.nB[1] = c->Wp[K];
    po.npairs = 2;
    po.ones_col = c->Wp[K];
    po.mv = 1;
    po.nv = c->slab_nv[K + 1];
    po.mt = c->slab_mt[K + 1];
    po.nt = c->slab_nt[K + 1];
    po.slab = c->slab[K + 1];
    maxt = std::max(maxt, po.mt * po.nt);
    tfl += 2.0 * 2.0 * R * (L[K + 1] + 1);
  }
  if (K + 2 > 8) return fail(c, DBSDE_EINVAL, "internal: too many TN problems");
  if (c->tnx3) {
    for (int j = 0; j <= K; ++j)
      g.maxt3 = std::max(g.maxt3, ((ta.prob[j].nA[0] + TX_TILE - 1) / TX_TILE) * ((ta.prob[j].nB[0] + TX_TILE - 1) / TX_TILE));
    g.rps32 = ((Rp + S_ - 1) / S_ + 31) / 32 * 32;
    // tn_out_kernel's float4 loads at H + col[K] + r S: 16-byte aligned rows and column
    if (Rp % 32 != 0 || c->Wp[K] % 4 != 0 || c->col[K] % 4 != 0 || S % 4 != 0)
      return fail(c, DBSDE_EINVAL, "internal: tn x3 geometry");
    const TNProb& po = ta.prob[K + 1];
    g.oslab = po.slab;
    g.sstride = (long long)po.mt * 64 * po.nt * 64;
  }
  return DBSDE_OK;
}
// split-bf16 chain weight gradients of row splits [s0, s0 + sn) on stream st
int tn_launch_splits(dbsde_ctx* c, int R, TNArgs ta, const TNGeom& g, int s0, int sn, hipStream_t st) {
  const int K = c->K, S = c->Stot;
  ta.split0 = s0;
  tn_x3_kernel<<<dim3(g.maxt3, sn, K + 1), 256, 0, st>>>(ta, g.rps32);
  tn_out_kernel<<<dim3(sn, (c->Wp[K] + 255) / 256), 1024, 0, st>>>(c->u16, c->H + c->col[K], c->Hdot + c->col[K], S,
                                                                    c->Wp[K], R, g.rps32, g.oslab, g.sstride, s0);
  HIPC(c, hipGetLastError());
  return DBSDE_OK;
}

int backward_tail(dbsde_ctx* c, const float* params, int R, int Rp, int fv, float* grad, const double* loss_part,
                  int nloss_parts, float* loss_dst, const FusedOpt* fo, bool tnw_piped, bool tn_piped) {
  int rc;
  hipStream_t s = c->stream;
  const auto& L = c->L;
  const int K = c->K, S = c->Stot, D = c->D;
  if (fv < 0) {
    // ---- forward tangent along zbar
    {
      ChainArgs a = base_args(c);
      a.A = c->zbar;
      a.lda = c->Dp;
      a.Bt = c->BtIn;
      x3_weights(c, a, c->imgX[0], c->Wp[0] / 16, c->Dp / 16);
      a.ldb = c->Dp;
      a.K = c->Dp;
      a.in[0] = c->Abuf;
      a.ldi[0] = S;
      a.out[0] = c->Adot;
      a.ldo[0] = S;
      a.out[1] = c->Hdot;
      a.ldo[1] = S;
      a.lvl0_cols = c->Wp[0];
      int nv = 0;
      for (int j = 0; j <= (c->has_v ? K : 0); ++j) nv += L[j + 1];
      if ((rc = chain<EPI_TAN0>(c, "gemm_xstack_tangent", a, Rp, c->Stot_x, nt_for(c->Wp[0]),
                                2.0 * R * D * nv, 4.0 * R * (D + 2.0 * nv + L[1]))))
        return rc;
    }
    for (int j = 1; j <= K; ++j) {
      ChainArgs a = base_args(c);
      a.A = c->Hdot + c->col[j - 1];
      a.lda = S;
      a.Bt = c->Bf[j];
      x3_weights(c, a, c->imgF[j], c->Wp[j] / 16, c->Wp[j - 1] / 16);
      a.ldb = c->Wp[j - 1];
      a.K = c->Wp[j - 1];
      a.in[0] = c->has_v ? c->Adot + c->col[j] : nullptr;
      a.ldi[0] = S;
      a.in[1] = c->Hdot + c->col[j - 1];
      a.ldi[1] = S;
      a.in[2] = c->Abuf + c->col[j];
      a.ldi[2] = S;
      a.out[0] = c->Adot + c->col[j];
      a.ldo[0] = S;
      a.out[1] = c->Hdot + c->col[j];
      a.ldo[1] = S;
      a.last = j == K;
      a.out[2] = c->Alpha + c->col[K];
      a.ldo[2] = S;
      a.vec[0] = c->wout;
      a.ubar = c->ubar;
      if ((rc = chain<EPI_TAN>(c, "gemm_block_tangent", a, Rp, c->Wp[j], nt_for(c->Wp[j]),
                               2.0 * R * L[j] * L[j + 1], 4.0 * R * (L[j] + 6.0 * L[j + 1]))))
        return rc;
    }
    // ---- reverse over (primal, tangent)
    for (int j = K; j >= 1; --j) {
      ChainArgs a = base_args(c);
      a.A = c->Alpha + c->col[j];
      a.lda = S;
      a.Bt = c->Bb[j];
      x3_weights(c, a, c->imgB[j], c->Wp[j - 1] / 16, c->Wp[j] / 16);
      a.ldb = c->Wp[j];
      a.K = c->Wp[j];
      a.in[0] = j == K ? nullptr : c->Pbuf[(j + 1) & 1];
      a.ldi[0] = c->Wmax;
      a.ubar = c->ubar;
      a.vec[0] = c->wout;
      a.in[1] = c->Abuf + c->col[j - 1];
      a.ldi[1] = S;
      a.in[2] = c->G + c->col[j - 1];
      a.ldi[2] = S;
      a.in[3] = c->Adot + c->col[j - 1];
      a.ldi[3] = S;
      a.out[0] = c->Pbuf[j & 1];
      a.ldo[0] = c->Wmax;
      a.out[1] = c->Alpha + c->col[j - 1];
      a.ldo[1] = S;
      if ((rc = chain<EPI_REV>(c, "gemm_block_reverse", a, Rp, c->Wp[j - 1], nt_for(c->Wp[j - 1]),
                               2.0 * R * L[j] * L[j + 1], 4.0 * R * (L[j + 1] + 6.0 * L[j]))))
        return rc;
    }
  }
  // ---- parameter gradients
  if (c->tnw) {
    if (!tnw_piped && (rc = launch_tnw(c, R, Rp))) return rc;
    if ((rc = finalize_grads(c, params, grad, loss_part, nloss_parts, loss_dst, fo))) return rc;
  } else {
  if (!tn_piped) {
    TNArgs ta;
    TNGeom g;
    if ((rc = tn_setup(c, R, Rp, ta, g))) return rc;
    hipStream_t s = c->stream;
    if (c->tnx3) {
      const int S_ = g.S_, rps32 = g.rps32;
      RUN(c, "tn_weight_grad", g.tfl, 0.0,
          tn_x3_kernel<<<dim3(g.maxt3, S_, K + 1), 256, 0, s>>>(ta, rps32);
          tn_out_kernel<<<dim3(S_, (c->Wp[K] + 255) / 256), 1024, 0, s>>>(c->u16, c->H + c->col[K], c->Hdot + c->col[K],
                                                                           S, c->Wp[K], R, rps32, g.oslab, g.sstride, 0));
    } else {
      RUN(c, "tn_weight_grad", g.tfl, 0.0, tn_gemm_kernel<<<dim3(g.maxt, g.S_, K + 2), 256, 0, s>>>(ta));
    }
  }
  if ((rc = finalize_grads(c, params, grad, loss_part, nloss_parts, loss_dst, fo))) return rc;
  }
  return DBSDE_OK;
}

// weight-gradient row slices for a batch of Rp rows.  Always the slab
// capacity: fewer, longer slices at small batches (48 at M = 128, four 32-row
// steps each) cut the finalize's slab reads (23.9 -> 22.4 us) but leave the
// weight-gradient kernel with a third of the waves (33 -> 49 us,
// profiles/r4_ab_column_split.txt)
int tnw_slices(const dbsde_ctx* c, int Rp) {
  (void)Rp;
  return c->tnw_Smax;
}

// resident workgroups of the chip for a phase variant (two per CU for the
// 64-row and column-split kernels, one for the 512-register ones), queried once
int variant_slots(dbsde_ctx* c, int fv) {
  if (c->fv_slots[fv] == 0) {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kFused[fv].A, 64 * P3_WAVES, 0) != hipSuccess) per = 1;
    c->fv_slots[fv] = std::max(1, per) * c->cus;
  }
  return c->fv_slots[fv];
}

int loss_grad_impl(dbsde_ctx* c, const float* params, const dbsde_batch* b, float* grad, const dbsde_outputs* out,
                   const FusedOpt* fo) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  if (!params) return fail(c, DBSDE_EINVAL, "params is NULL");
  int rc = validate_batch(c, b);
  if (rc) return rc;
  HIPC(c, hipSetDevice(c->device));
  const int M = b->M, N = b->N, N1 = N + 1, D = c->D, K = c->K, S = c->Stot;
  const int R = M * N1, Rp = (R + ROW_PAD - 1) / ROW_PAD * ROW_PAD;
  if ((rc = ensure_rows(c, Rp, N))) return rc;
  hipStream_t s = c->stream;
  const auto& L = c->L;
  const dbsde_problem& pr = c->cfg.problem;

  // a held-back prefetch of this very batch: issue it now (its consumer)
  if (c->deferred && same_batch(c->defer_b, *b) && (rc = flush_deferred(c))) return rc;
  // weight repack (projection, norms, fragment images) overlaps the rollout
  if ((rc = prep_weights(c, params))) return rc;

  // ---- rollout (network-independent: mu/sigma never read Y, Z), unless
  // dbsde_prefetch already produced this batch's paths
  bool from_pf = false;
  if ((rc = select_paths(c, b, from_pf))) return rc;
  if (!from_pf) {
    if (Rp > R) HIPC(c, hipMemsetAsync(c->xin + (size_t)R * c->Dp, 0, (size_t)(Rp - R) * c->Dp * 4, s));
    RolloutArgs ra = rollout_args(c, b);
    ra.out = PATH_ROLLOUT;
    if ((rc = launch_paths(c, ra))) return rc;
  }
  const bool q3 = pr.q3 && D == 1;
  if (q3) RUN(c, "q3_sum", 0.0, 4.0 * M * N, q3_sum_kernel<<<N, 256, 0, s>>>(c->sdw, c->Dp, M, N, c->q3S));

  int nloss_parts;
  bool tnw_piped = false, tn_piped = false;
  TNArgs tn_a;
  TNGeom tn_g;
  FusedArgs fa;
  c->tnw_S = tnw_slices(c, Rp);
  int fv = c->fv;
  // small batches: the column-split kernels when all their 16-row workgroups
  // are resident at once (M <= 128 per GPU at the north star); past that their
  // 4x workgroup count costs more than the shorter chains save (M = 256:
  // 0.235 vs 0.209 ms/step, profiles/r4_ab_column_split.txt)
  if (fv >= 0 && c->fv_cs >= 0 &&
      (c->cs_mode == 1 || (c->cs_mode == 2 && Rp / CS_ROWS <= variant_slots(c, c->fv_cs))))
    fv = c->fv_cs;
  if (fv >= 0) {
    fa = fused_args(c, R, Rp, N1, q3);
    if (!fused_piece_counts_ok(c, fa)) return fail(c, DBSDE_EINVAL, "internal: fused kernel piece counts");
    const int nv = nv_x(c);
    const double flA = 2.0 * R * ((D + 1.0) * nv + 2.0 * K * L[1] * (double)L[1] + (double)nv * D);
    const double byA = 4.0 * R * (c->Dp + 4.0 * S + 8.0);
    const double flC = 2.0 * R * ((double)nv * D + 2.0 * K * L[1] * (double)L[1]);
    const double byC = 4.0 * R * (4.0 * c->Dp + 5.0 * S);
    // chunks of whole paths and whole WR-row tiles (WR paths = WR (N+1) rows =
    // N+1 tiles), WR = the variant's rows per workgroup
    const int WR = kFused[fv].rows;
    // workgroup slots of the chip for this variant (two per CU for the
    // 64-row kernels, one for the 512-register ones)
    const int slots = variant_slots(c, fv);
    int nch = !grad ? 1 : (c->chunks > 0 ? c->chunks : (Rp / WR > slots ? 2 : 1));
    while (nch > 1 && (M % WR != 0 || (M / WR) % nch != 0)) --nch;
    if (nch <= 1) {
      if ((rc = flush_deferred(c, c->xin))) return rc;
      RUN(c, "fused_fwd_inputgrad", flA, byA, kFused[fv].A<<<Rp / WR, 64 * P3_WAVES, 0, s>>>(fa));
    } else {
      // phase A / phase C of chunk i on stream (i even ? main : pipe2); the
      // two phases are timed as one pipelined segment
      // equal chunks in units of WR paths
      const int units = M / WR, utile = N1;   // WR paths = N1 tiles
      std::vector<int> cu(nch, units / nch);
      if (c->prof) HIPC(c, hipEventRecord(c->ev_prof[0], s));
      const int np = std::min(2, nch);
      // Unprofiled steps run each chunk's weight-gradient row slices on the
      // chunk's stream right after its phase C (the slices of the first chunk
      // overlap the second chunk's phases; slice s covers 32-row steps
      // [s n32 / S, (s + 1) n32 / S), so the chunk boundary must be a slice
      // boundary).  Profiled steps keep them after the section, so the section
      // and the weight-gradient kernel are timed on their own.
      // sb[i]: the first slice of chunk i (sb[nch] = S); every chunk boundary
      // must be a slice boundary that is a multiple of 8 (the kernel's
      // slice groups)
      std::vector<int> sb(nch + 1, 0);
      {
        const int S = c->tnw_S, n32 = Rp / 32;
        bool ok = Rp % 32 == 0;
        long long crow = 0;
        sb[nch] = S;
        for (int i = 1; i < nch && ok; ++i) {
          crow += (long long)cu[i - 1] * utile * WR;
          for (int k = sb[i - 1] + 8; k < S && !sb[i]; k += 8)
            if (32LL * ((long long)k * n32 / S) == crow) sb[i] = k;
          ok = sb[i] > 0;
        }
        // (two chunks only: with more, a chunk's slices sit in front of the
        // next chunk's phase A on the same stream -- 4 chunks 0.607 vs 0.495
        // ms/step, profiles/r4_ab_chunks_piped.txt)
        tnw_piped = grad && c->tnw && !c->prof && np == 2 && nch == 2 && ok;
      }
      // the chain layouts' split-bf16 weight gradients the same way: row
      // splits of chunk 0 after its phase C on the main stream, the rest after
      // chunk 1's on the second (the chunk boundary must be a split boundary)
      int tn_s0 = 0;
      if (grad && !c->tnw && c->tnx3 && !c->prof && np == 2 && nch == 2) {
        const long long crow = (long long)cu[0] * utile * WR;
        if ((rc = tn_setup(c, R, Rp, tn_a, tn_g, crow))) return rc;
        if (tn_g.rps32 > 0 && crow % tn_g.rps32 == 0 && crow / tn_g.rps32 < tn_g.S_) {
          tn_s0 = (int)(crow / tn_g.rps32);
          tn_piped = true;
        }
      }
      if (!tnw_piped && !tn_piped && (rc = flush_deferred(c, c->xin))) return rc;
      hipStream_t ps[2] = {s, c->pipe2};
      if (np > 1 && (rc = stream_order(c, s, c->pipe2, ORD_FORK))) return rc;
      int t0 = 0;
      for (int i = 0; i < nch; ++i) {
        hipStream_t st = ps[i % np];
        FusedArgs fc = fa;
        fc.tile0 = t0;
        // the last chunk also runs the padding tiles past R (Rp > R when the
        // workgroup is 16 rows and R is not a multiple of the 64-row padding):
        // the loss partials and the weight-gradient rows of every tile up to
        // Rp / WR are then written by this step
        const int tiles = i + 1 < nch ? cu[i] * utile : Rp / WR - t0;
        kFused[fv].A<<<tiles, 64 * P3_WAVES, 0, st>>>(fc);
        kFused[fv].C<<<tiles, 64 * P3_WAVES, 0, st>>>(fc);
        if (tnw_piped && (rc = launch_tnw(c, R, Rp, sb[i], sb[i + 1] - sb[i], st))) return rc;
        if (tn_piped && (rc = tn_launch_splits(c, R, tn_a, tn_g, i == 0 ? 0 : tn_s0,
                                               i == 0 ? tn_s0 : tn_g.S_ - tn_s0, st)))
          return rc;
        t0 += tiles;
      }
      HIPC(c, hipGetLastError());
      // the pending prefetched rollouts (this step's other buffer, started a
      // step ago) are waited for on the second chunk stream, so the join orders
      // the main stream after them too
      for (int i = 0; i < 2; ++i)
        if (c->pend[i].valid) {
          // (a rollout joined before is already behind pipe2: the join below
          // orders this step's stream after it)
          if (!c->pend[i].joined && (rc = order_wait(c, ORD_PEND0 + i, c->pend[i].ready_v, c->pipe2))) return rc;
          c->pend[i].joined = true;
          c->pend[i].joined_to = s;
        }
      if ((rc = stream_order(c, c->pipe2, s, ORD_JOIN))) return rc;
      // the held-back batch after the join: beside this step's tail, not in
      // front of it (profiles/r6_ab_rollout.txt 6)
      if ((tnw_piped || tn_piped) && (rc = launch_deferred_on(c, c->pipe2))) return rc;
      if (c->prof) {
        HIPC(c, hipEventRecord(c->ev_prof[1], s));
        HIPC(c, hipEventSynchronize(c->ev_prof[1]));
        float ms = 0.f;
        HIPC(c, hipEventElapsedTime(&ms, c->ev_prof[0], c->ev_prof[1]));
        ProfAgg& ag = c->agg[prof_id(c, "fused_phases_pipelined")];
        ag.ms += ms;
        ag.flops += flA + flC;
        ag.bytes += byA + byC;
        ag.n += 1;
      }
    }
    if (grad) {
      if (nch <= 1)
        RUN(c, "fused_tangent_reverse", flC, byC, kFused[fv].C<<<Rp / WR, 64 * P3_WAVES, 0, s>>>(fa));
      nloss_parts = Rp / WR;
    } else {
      RUN(c, "loss_rows", 0.0, 4.0 * R * 3.0 * D,
          cotan_kernel<<<Rp / 16, 256, 0, s>>>(cotan_params(c, R, Rp, N1, q3), c->loss_part));
      nloss_parts = Rp / 16;
    }
  } else {
    if ((rc = flush_deferred(c, c->xin))) return rc;
    if ((rc = forward_and_inputgrad(c, R, Rp, false))) return rc;

    // ---- Z GEMM + residuals / cotangents / loss rows
    {
      ChainArgs a = base_args(c);
      zgemm_args(c, a);
      a.R = R;
      a.N1 = N1;
      a.D = D;
      a.xin = c->xin;
      a.sdw = c->sdw;
      a.ldx = c->Dp;
      a.u = c->u;
      a.q3S = q3 ? c->q3S : nullptr;
      a.umask = c->u_clamp ? c->umask : nullptr;
      a.phi_r = pr.phi_r;
      a.phi_c = pr.phi_c;
      a.phi_zz = pr.phi_zz;
      a.strike = pr.strike;
      a.g_alpha = pr.g_alpha;
      a.g_kind = pr.g_kind;
      a.gcols = c->gcols;
      a.zbar = c->zbar;
      a.rres = c->rres;
      a.lossrow = c->lossrow;
      if ((rc = chain<EPI_COTAN>(c, "gemm_z_cotangent", a, Rp, c->Dp, c->Dp / 16, zgemm_flops(c, R),
                                 4.0 * R * (c->Stot_x + 5.0 * D))))
        return rc;
    }
    RUN(c, "ubar_loss", 0.0, 16.0 * R,
        ubar_kernel<<<Rp / 256 + 1, 256, 0, s>>>(c->rres, c->xin, c->Dp, R, Rp, N1, pr.phi_r, c->lossrow, c->ubar,
                                                 c->u16, c->loss_part, c->u_clamp ? c->umask : nullptr));
    nloss_parts = Rp / 256 + 1;
  }
  float* loss_dst = (out && out->loss) ? out->loss : c->loss_tmp;
  // the loss sum: inside the gradient finalize (tilefin_kernel or
  // slabsum_kernel), else (no gradient) its own launch
  const bool loss_in_fin = grad;
  if (!loss_in_fin)
    RUN(c, "loss_final", 0.0, 0.0, loss_final_kernel<<<1, 256, 0, s>>>(c->loss_part, nloss_parts, loss_dst));

  if (grad && (rc = backward_tail(c, params, R, Rp, fv, grad, c->loss_part, nloss_parts, loss_dst, fo, tnw_piped,
                                  tn_piped)))
    return rc;
  if ((rc = flush_deferred(c, c->xin))) return rc;   // (every path above has issued it already)

  if (out && (out->X || out->Y || out->Z)) {
    const long long n = (long long)R * D;
    RUN(c, "export", 0.0, 0.0,
        export_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(c->xin, c->zfull, c->Dp, c->u, R, D, out->X,
                                                                  out->Y, out->Z, nullptr));
  }
  return DBSDE_OK;
}

// dbsde_optim -> the kernel's OptArgs (scalar factors in double, as
// torch.optim computes them in Python floats)
int make_optargs(dbsde_ctx* c, const dbsde_optim* o, OptArgs& a) {
  if (o->kind < DBSDE_OPT_ADAM || o->kind > DBSDE_OPT_ASGD) return fail(c, DBSDE_EINVAL, "unknown optimizer kind");
  if (o->step < 1) return fail(c, DBSDE_EINVAL, "step must be >= 1");
  a = OptArgs{};
  a.kind = o->kind;
  a.lr = o->lr;
  a.beta2 = o->beta2;
  a.eps = o->eps;
  a.wd = o->weight_decay;
  a.max_norm = o->max_norm;
  a.omb1 = (float)(1.0 - (double)o->beta1);
  a.omb2 = (float)(1.0 - (double)o->beta2);
  const double t = (double)o->step;
  const double bc1 = 1.0 - std::pow((double)o->beta1, t);
  const double bc2 = 1.0 - std::pow((double)o->beta2, t);
  a.step_size = (float)((double)o->lr / bc1);
  a.bc2_sqrt = (float)std::sqrt(bc2);
  a.alpha = o->alpha;
  a.rho = o->rho;
  if (o->kind == DBSDE_OPT_RMSPROP) a.omb2 = (float)(1.0 - (double)o->alpha);
  if (o->kind == DBSDE_OPT_ADADELTA) a.omb2 = (float)(1.0 - (double)o->rho);
  if (o->kind == DBSDE_OPT_ADAGRAD) a.step_size = (float)((double)o->lr / (1.0 + (t - 1.0) * (double)o->lr_decay));
  if (o->kind == DBSDE_OPT_ASGD) {
    a.asgd_eta = o->asgd_eta;
    a.asgd_decay = (float)(1.0 - (double)o->lambd * (double)o->asgd_eta);
    a.asgd_mu = o->asgd_mu;
    a.asgd_copy = o->asgd_mu == 1.f;
  }
  a.loss = o->loss;
  a.nparts = c->opt_nparts;
  if (o->step_state) {
    if (o->step_parity != 0 && o->step_parity != 1) return fail(c, DBSDE_EINVAL, "step_parity must be 0 or 1");
    a.state = o->step_state;
    a.parity = o->step_parity;
    a.lr_d = o->lr;
    a.beta1_d = o->beta1;
    a.beta2_d = o->beta2;
    a.lr_decay_d = o->lr_decay;
    a.lambd_d = o->lambd;
    a.asgd_alpha_d = 0.75;   // torch.optim.ASGD defaults (alpha, t0)
    a.asgd_t0_d = 1e6;
  }
  return DBSDE_OK;
}
}  // namespace

extern "C" {

int dbsde_loss_grad(dbsde_ctx* c, const float* params, const dbsde_batch* b, float* grad,
                    const dbsde_outputs* out) {
  return loss_grad_impl(c, params, b, grad, out, nullptr);
}

int dbsde_train_step(dbsde_ctx* c, float* params, const dbsde_batch* b, float* grad, float* m, float* v,
                     const dbsde_optim* o, const dbsde_outputs* out) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  if (!params || !grad || !o) return fail(c, DBSDE_EINVAL, "bad train_step arguments");
  // the update can ride in the gradient finalize when nothing needs the whole
  // gradient first: no clip (global norm), no NaN skip (the loss), a device
  // step counter, and the tile finalize (wave-owned weight-gradient layouts)
  const bool fuse = c->tnw && o->max_norm <= 0.f && !o->loss && o->step_state;
  if (!fuse) {
    int rc = loss_grad_impl(c, params, b, grad, out, nullptr);
    if (rc) return rc;
    return dbsde_optimizer_step(c, params, grad, m, v, o);
  }
  const bool needs_m = o->kind == DBSDE_OPT_ADAM || o->kind == DBSDE_OPT_ADAMW || o->kind == DBSDE_OPT_ADAMAX ||
                       o->kind == DBSDE_OPT_ADADELTA || o->kind == DBSDE_OPT_ASGD;
  const bool needs_v = o->kind != DBSDE_OPT_SGD && o->kind != DBSDE_OPT_ASGD;
  if ((needs_m && !m) || (needs_v && !v)) return fail(c, DBSDE_EINVAL, "optimizer state buffer is NULL");
  FusedOpt fo{};
  int rc = make_optargs(c, o, fo.a);
  if (rc) return rc;
  fo.prm = params;
  fo.m = m;
  fo.v = v;
  return loss_grad_impl(c, params, b, grad, out, &fo);
}

int dbsde_net_u(dbsde_ctx* c, const float* params, int R, const float* t, const float* X, float* u, float* Du) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  if (!params || !t || !X || R < 1) return fail(c, DBSDE_EINVAL, "bad net_u arguments");
  HIPC(c, hipSetDevice(c->device));
  const int Rp = (R + ROW_PAD - 1) / ROW_PAD * ROW_PAD, D = c->D;
  int rc;
  if ((rc = ensure_rows(c, Rp, 1))) return rc;
  hipStream_t s = c->stream;
  if ((rc = prep_weights(c, params))) return rc;
  const long long n = (long long)Rp * c->Dp;
  bool from_pf;
  if ((rc = flush_deferred(c))) return rc;
  if ((rc = select_paths(c, nullptr, from_pf))) return rc;
  RUN(c, "netu_input", 0.0, 0.0,
      netu_input_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(t, X, R, D, c->Dp, c->xin));
  if (Rp > R) HIPC(c, hipMemsetAsync(c->xin + (size_t)R * c->Dp, 0, (size_t)(Rp - R) * c->Dp * 4, s));
  if (c->fv >= 0) {
    // the fused forward + input-gradient kernel writes u and Z (its residual
    // row sums read sdw, unused here)
    FusedArgs fa = fused_args(c, R, Rp, 1, false);
    if (!fused_piece_counts_ok(c, fa)) return fail(c, DBSDE_EINVAL, "internal: fused kernel piece counts");
    const int WR = kFused[c->fv].rows;
    RUN(c, "fused_fwd_inputgrad", 0.0, 0.0, kFused[c->fv].A<<<Rp / WR, 64 * P3_WAVES, 0, s>>>(fa));
  } else {
    if ((rc = forward_and_inputgrad(c, R, Rp, true))) return rc;
    ChainArgs a = base_args(c);
    zgemm_args(c, a);
    if ((rc = chain<EPI_STORE>(c, "gemm_z", a, Rp, c->Dp, c->Dp / 16, zgemm_flops(c, R), 0.0))) return rc;
  }
  const long long m = (long long)R * D;
  RUN(c, "export", 0.0, 0.0,
      export_kernel<<<(unsigned)((m + 255) / 256), 256, 0, s>>>(c->xin, c->zfull, c->Dp, c->u, R, D, nullptr, u,
                                                                Du, (c->fv < 0 && c->u_clamp) ? c->umask : nullptr));
  return DBSDE_OK;
}

// net_u's VJP (loss.backward through the reference's net_u outputs,
// nd_BSPDE_case.py:191-221 with create_graph=True): grad = d/dparams of
// sum_r ubar_r u_r + zbar_r . Du_r at the points (t, X).  The same backward as
// dbsde_loss_grad with the caller's cotangents in place of the BSDE residual
// ones: the fused phase kernels take them in phase C's prologue, the per-layer
// form in its ubar / zbar buffers.
int dbsde_net_u_vjp(dbsde_ctx* c, const float* params, int R, const float* t, const float* X, const float* ubar,
                    const float* zbar, float* grad) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  if (!params || !t || !X || !ubar || !zbar || !grad || R < 1) return fail(c, DBSDE_EINVAL, "bad net_u_vjp arguments");
  HIPC(c, hipSetDevice(c->device));
  const int Rp = (R + ROW_PAD - 1) / ROW_PAD * ROW_PAD, D = c->D;
  int rc;
  if ((rc = ensure_rows(c, Rp, 1))) return rc;
  hipStream_t s = c->stream;
  if ((rc = prep_weights(c, params))) return rc;
  bool from_pf;
  if ((rc = flush_deferred(c))) return rc;
  if ((rc = select_paths(c, nullptr, from_pf))) return rc;
  const long long n = (long long)Rp * c->Dp;
  const unsigned nb = (unsigned)((n + 255) / 256);
  RUN(c, "netu_input", 0.0, 0.0, netu_input_kernel<<<nb, 256, 0, s>>>(t, X, R, D, c->Dp, c->xin));
  if (Rp > R) HIPC(c, hipMemsetAsync(c->xin + (size_t)R * c->Dp, 0, (size_t)(Rp - R) * c->Dp * 4, s));
  const int fv = c->fv;
  if (fv >= 0) {
    // ubar -> rres rows, zbar -> the sdw rows phase C reads (phase A's use of
    // sdw only feeds the residual row sums, unused here)
    RUN(c, "vjp_cotangents", 0.0, 0.0,
        ext_cotan_kernel<<<nb, 256, 0, s>>>(ubar, zbar, R, Rp, D, c->Dp, nullptr, c->rres, c->sdw, nullptr));
    FusedArgs fa = fused_args(c, R, Rp, 1, false);
    if (!fused_piece_counts_ok(c, fa)) return fail(c, DBSDE_EINVAL, "internal: fused kernel piece counts");
    fa.cp.ext = 1;
    fa.cp.ext_ub = c->rres;
    const int WR = kFused[fv].rows;
    RUN(c, "fused_fwd_inputgrad", 0.0, 0.0, kFused[fv].A<<<Rp / WR, 64 * P3_WAVES, 0, s>>>(fa));
    RUN(c, "fused_tangent_reverse", 0.0, 0.0, kFused[fv].C<<<Rp / WR, 64 * P3_WAVES, 0, s>>>(fa));
  } else {
    if ((rc = flush_deferred(c, c->xin))) return rc;
    if ((rc = forward_and_inputgrad(c, R, Rp, false))) return rc;
    RUN(c, "vjp_cotangents", 0.0, 0.0,
        ext_cotan_kernel<<<nb, 256, 0, s>>>(ubar, zbar, R, Rp, D, c->Dp, c->u_clamp ? c->umask : nullptr, c->ubar,
                                            c->zbar, c->u16));
  }
  c->tnw_S = tnw_slices(c, Rp);
  return backward_tail(c, params, R, Rp, fv, grad, nullptr, 0, nullptr, nullptr, false, false);
}

int dbsde_optimizer_step(dbsde_ctx* c, float* params, float* grad, float* m, float* v, const dbsde_optim* o) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  if (!params || !grad || !o) return fail(c, DBSDE_EINVAL, "bad optimizer arguments");
  const bool needs_m = o->kind == DBSDE_OPT_ADAM || o->kind == DBSDE_OPT_ADAMW || o->kind == DBSDE_OPT_ADAMAX ||
                       o->kind == DBSDE_OPT_ADADELTA || o->kind == DBSDE_OPT_ASGD;
  const bool needs_v = o->kind != DBSDE_OPT_SGD && o->kind != DBSDE_OPT_ASGD;
  if ((needs_m && !m) || (needs_v && !v)) return fail(c, DBSDE_EINVAL, "optimizer state buffer is NULL");
  OptArgs a;
  int rc = make_optargs(c, o, a);
  if (rc) return rc;
  HIPC(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const long long n = c->nparams;
  if (o->max_norm > 0.f)
    RUN(c, "grad_sqnorm", 2.0 * n, 4.0 * n, sqnorm_kernel<<<c->opt_nparts, 256, 0, s>>>(grad, c->d_used, n, c->opt_part));
  RUN(c, "optimizer", 10.0 * n, 24.0 * n,
      optim_kernel<<<256, 256, 0, s>>>(params, grad, m, v, c->d_used, n, c->opt_part, a));
  return DBSDE_OK;
}

int dbsde_vec_reduce(dbsde_ctx* c, int op, const float* a, const float* b, long long n, double* result) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  if (op < DBSDE_VEC_DOT || op > DBSDE_VEC_AMAX || !a || (op == DBSDE_VEC_DOT && !b) || n < 1 || !result)
    return fail(c, DBSDE_EINVAL, "bad dbsde_vec_reduce arguments");
  HIPC(c, hipSetDevice(c->device));
  int rc;
  if (!c->vec_part && (rc = dalloc_t(c, &c->vec_part, VEC_RED_BLOCKS + 1))) return rc;
  hipStream_t s = c->stream;
  RUN(c, "vec_reduce", 2.0 * n, 8.0 * n, vec_reduce_kernel<<<VEC_RED_BLOCKS, 256, 0, s>>>(op, a, b, n, c->vec_part));
  RUN(c, "vec_reduce", 0.0, 0.0,
      vec_reduce_final_kernel<<<1, 256, 0, s>>>(op, c->vec_part, VEC_RED_BLOCKS, c->vec_part + VEC_RED_BLOCKS));
  HIPC(c, hipMemcpyAsync(result, c->vec_part + VEC_RED_BLOCKS, sizeof(double), hipMemcpyDeviceToHost, s));
  HIPC(c, hipStreamSynchronize(s));
  return DBSDE_OK;
}

int dbsde_vec_axpby(dbsde_ctx* c, float* z, const float* x, const float* y, long long n, float alpha, float beta) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  if (!z || !x || n < 1 || (!y && beta != 0.f)) return fail(c, DBSDE_EINVAL, "bad dbsde_vec_axpby arguments");
  HIPC(c, hipSetDevice(c->device));
  const unsigned blocks = (unsigned)std::min<long long>((n + 255) / 256, 1024);
  RUN(c, "vec_axpby", 3.0 * n, 12.0 * n, vec_axpby_kernel<<<blocks, 256, 0, c->stream>>>(z, x, y, n, alpha, beta));
  return DBSDE_OK;
}

int dbsde_lbfgs_direction(dbsde_ctx* c, const float* g, const float* S, const float* Y, long long ld, long long n,
                          const int* slot, const float* ro, int num, float h_diag, float* d) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  if (!g || !d || n < 1 || num < 0 || num > LBFGS_HMAX || (num > 0 && (!S || !Y || !slot || !ro || ld < n)))
    return fail(c, DBSDE_EINVAL, "bad dbsde_lbfgs_direction arguments (at most 128 history entries)");
  HIPC(c, hipSetDevice(c->device));
  LbfgsArgs a{};
  a.g = g;
  a.S = S;
  a.Y = Y;
  a.ld = ld;
  a.n = n;
  a.d = d;
  a.num = num;
  a.h_diag = h_diag;
  for (int i = 0; i < num; ++i) {
    if (slot[i] < 0) return fail(c, DBSDE_EINVAL, "negative history slot");
    a.slot[i] = slot[i];
    a.ro[i] = ro[i];
  }
  RUN(c, "lbfgs_direction", 8.0 * n * num, 16.0 * n * num, lbfgs_direction_kernel<<<1, 1024, 0, c->stream>>>(a));
  return DBSDE_OK;
}

int dbsde_brownian_dim(const dbsde_ctx* c) { return c ? c->nb : -1; }

int dbsde_set_corr(dbsde_ctx* c, const float* L, int n) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  HIPC(c, hipSetDevice(c->device));
  // a prefetched rollout read the old factor: drop it (and let it finish)
  if (c->pf_stream) HIPC(c, hipStreamSynchronize(c->pf_stream));
  c->pend[0].valid = c->pend[1].valid = false;
  c->deferred = false;
  if (!L) {
    if (c->Lt) {
      HIPC(c, hipStreamSynchronize(c->stream));
      (void)hipFree(c->Lt);
      c->allocs.erase(std::find(c->allocs.begin(), c->allocs.end(), (void*)c->Lt));
      c->Lt = nullptr;
    }
    return DBSDE_OK;
  }
  if (c->heston) return fail(c, DBSDE_EINVAL, "dbsde_set_corr: correlated increments are for DIAG problems");
  if (n != c->nb) return fail(c, DBSDE_EINVAL, "dbsde_set_corr: L must be [nb, nb], nb = the Brownian dimension");
  if (n > CP_NBMAX) return fail(c, DBSDE_EINVAL, "dbsde_set_corr: Brownian dimension > 128 is not supported");
  std::vector<float> lt((size_t)n * n, 0.f);
  for (int d = 0; d < n; ++d)
    for (int k = 0; k <= d; ++k) lt[(size_t)k * n + d] = L[(size_t)d * n + k];   // L^T, lower part of L only
  int rc;
  if (!c->Lt && (rc = dalloc_t(c, &c->Lt, (size_t)n * n))) return rc;
  HIPC(c, hipStreamSynchronize(c->stream));
  HIPC(c, hipMemcpy(c->Lt, lt.data(), lt.size() * sizeof(float), hipMemcpyHostToDevice));
  return DBSDE_OK;
}

int dbsde_prefetch(dbsde_ctx* c, const dbsde_batch* next) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  int rc = validate_batch(c, next);
  if (rc) return rc;
  if (next->W || next->t) return fail(c, DBSDE_EINVAL, "dbsde_prefetch: device-mode batches only (t and W NULL)");
  HIPC(c, hipSetDevice(c->device));
  const int M = next->M, N = next->N, R = M * (N + 1), Rp = (R + ROW_PAD - 1) / ROW_PAD * ROW_PAD;
  if ((rc = ensure_rows(c, Rp, N))) return rc;
  for (int i = 0; i < 2; ++i)
    if (c->pend[i].valid && same_batch(c->pend[i].b, *next)) return DBSDE_OK;   // already queued
  if (c->deferred && same_batch(c->defer_b, *next)) return DBSDE_OK;
  if ((rc = flush_deferred(c))) return rc;
  if (DBSDE_DEFER_PF && c->pipe2) {
    c->deferred = true;
    c->defer_b = *next;
    return DBSDE_OK;
  }
  return issue_prefetch(c, next);
}


int dbsde_prefetch_cancel(dbsde_ctx* c) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  HIPC(c, hipSetDevice(c->device));
  // the pending rollouts still run to completion; their buffers are just not
  // matched any more (and are not rewritten before they are done: the stream
  // that reuses a buffer waits for the prefetch stream)
  if (c->pf_stream) {
    const int rc = stream_order(c, c->pf_stream, c->stream, ORD_MAIN_AFTER_PF);
    if (rc) return rc;
  }
  // (rollouts on the chunk stream are ordered by its join, into the stream
  // they were joined to; another stream waits for the latest join)
  for (int i = 0; i < 2; ++i)
    if (c->pend[i].valid && c->pend[i].joined) {
      const int rc = wait_pending(c, i);
      if (rc) return rc;
    }
  c->pend[0].valid = c->pend[1].valid = false;
  c->deferred = false;   // a held-back prefetch has issued no work
  return DBSDE_OK;
}

int dbsde_brownian(dbsde_ctx* c, const dbsde_batch* b, float* t, float* W, int increments) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  int rc = validate_batch(c, b);
  if (rc) return rc;
  if (b->W || b->t) return fail(c, DBSDE_EINVAL, "dbsde_brownian draws a device-mode batch (W and t must be NULL)");
  if (!t || !W) return fail(c, DBSDE_EINVAL, "t and W outputs are required");
  HIPC(c, hipSetDevice(c->device));
  RolloutArgs ra = rollout_args(c, b);
  ra.out = increments ? PATH_FETCH_DW : PATH_FETCH_W;
  ra.t_out = t;
  ra.W_out = W;
  return launch_paths(c, ra);
}

int dbsde_profile_enable(dbsde_ctx* c, int enable) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  c->prof = enable != 0;
  return DBSDE_OK;
}

static int collect(dbsde_ctx* c) {
  if (c->pending.empty()) return DBSDE_OK;
  HIPC(c, hipStreamSynchronize(c->stream));
  for (auto& r : c->pending) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, r.e0, r.e1);
    ProfAgg& a = c->agg[r.id];
    a.ms += ms;
    a.flops += r.flops;
    a.bytes += r.bytes;
    a.n += 1;
    c->ev_pool.push_back(r.e0);
    c->ev_pool.push_back(r.e1);
  }
  c->pending.clear();
  return DBSDE_OK;
}

int dbsde_profile_count(dbsde_ctx* c) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  int rc = collect(c);
  if (rc) return rc;
  return (int)c->agg.size();
}

int dbsde_profile_read(dbsde_ctx* c, int idx, char* name, int name_len, double* total_ms, double* flops,
                       double* bytes, long long* launches) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  int rc = collect(c);
  if (rc) return rc;
  if (idx < 0 || idx >= (int)c->agg.size()) return fail(c, DBSDE_EINVAL, "profile index out of range");
  const ProfAgg& a = c->agg[idx];
  if (name && name_len > 0) {
    strncpy(name, a.name.c_str(), name_len - 1);
    name[name_len - 1] = 0;
  }
  if (total_ms) *total_ms = a.ms;
  if (flops) *flops = a.flops;
  if (bytes) *bytes = a.bytes;
  if (launches) *launches = a.n;
  return DBSDE_OK;
}

int dbsde_profile_reset(dbsde_ctx* c) {
  if (!c) return fail(nullptr, DBSDE_EINVAL, "ctx is NULL");
  int rc = collect(c);
  if (rc) return rc;
  for (auto& a : c->agg) {
    a.ms = a.flops = a.bytes = 0;
    a.n = 0;
  }
  return DBSDE_OK;
}

}  // extern "C"
