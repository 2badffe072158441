// paths.hpp -- Brownian increments and the Euler-Maruyama path step (gfx950).
//
// FBSNN.fetch_minibatch (DeepBSDE.py:247-262, with_corr...py:316-353) and the
// X recursion of loss_function (DeepBSDE.py:218-222, heston_dnnpde.py:629-642)
// as HIP kernels.  mu and sigma never read Y or Z, so the whole X path is
// computed before the network runs; every kernel here writes the
// network input rows xin[r] = [t, X_1..X_D, 1, 0..] and sdw[r] = sigma(X_n) dW_n
// (the vector the Y-tilde term contracts with Z), r = m (N+1) + n.
//
// Increments come either from the caller (parity mode: W [M, N+1, nb] exactly
// as the reference builds it, dW = W1 - W0 in fp32) or from an
// in-kernel Philox4x32-10 (device mode), keyed by the GLOBAL path index so a
// rank holding paths [path0, path0 + M) draws what one device would draw.
// The device-mode time grid is the reference's: t_n = fp32(fp64 cumsum of
// T/N) (DeepBSDE.py:250-258).
//
// HIP contracts a*b + c into an FMA by default (-ffp-contract=fast), and its
// __fmul_rn/__fadd_rn are plain operators whose contract flag comes from the
// header that defines them, so a pragma at the call site does not stop the
// fusion.  The path kernels use rn_mul/rn_add/rn_sub below, whose operations
// carry no contract flag: the reference (torch CPU) rounds each product and
// sum, and X is bit-exact against it.
#pragma once
#include "philox.hpp"

namespace dbsde {

__device__ __forceinline__ float rn_mul(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float rn_add(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float rn_sub(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}

enum PathOut { PATH_ROLLOUT = 0, PATH_FETCH_W = 1, PATH_FETCH_DW = 2 };

struct RolloutArgs {
  int M, N, D, ldx;
  int nb;                // Brownian dimension (D; D/2 for Heston)
  const float* t;        // [M, N+1] or null (device grid)
  const float* W;        // [M, N+1, nb] or null (Philox)
  const float* Xi;       // [xi_rows, D]
  int xi_rows;
  float T;
  unsigned long long seed, offset;
  long long path0;
  float mu_a, sig_a, sig_b;                // diagonal problems
  float kappa, theta, hsig, rho;           // Heston
  const float* Lt;       // correlated device mode: L^T [nb][nb] (upper part of L^T zero)
  float* xin;            // [Rp, ldx]
  float* sdw;            // [Rp, ldx]
  int out;               // PathOut
  float* t_out;          // fetch: [M, N+1]
  float* W_out;          // fetch: [M, N+1, nb] (W) or [M, N, nb] (dW)
};

// increments of steps n0+1 .. n0+4 of coordinate d of local path m: host W
// differences (fp32, the reference's W1 - W0) or sqrt(dt) * Philox normals;
// t1[k] is the time of step n0+k+1 (clamped to N), tacc the fp64 grid sum
__device__ __forceinline__ void step_block(const RolloutArgs& p, int m, int d, int n0, float& w0, double& tacc,
                                           double dt64, float sqdt, float dw[4], float t1[4]) {
  const int N1 = p.N + 1;
  if (p.W) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int n = min(n0 + k + 1, p.N);
      const float w1 = p.W[((size_t)m * N1 + n) * p.nb + d];
      t1[k] = p.t[(size_t)m * N1 + n];
      dw[k] = rn_sub(w1, w0);
      w0 = w1;
    }
  } else {
    float z[4];
    philox_normal4(p.seed, p.offset, (uint32_t)(p.path0 + m), (uint32_t)(n0 >> 2), (uint32_t)d, z);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      dw[k] = sqdt * z[k];
      if (n0 + k + 1 <= p.N) tacc += dt64;
      const int n = min(n0 + k + 1, p.N);
      t1[k] = p.t ? p.t[(size_t)m * N1 + n] : (float)tacc;
    }
  }
}

// fetch_minibatch output of one coordinate: t (d == 0) and W = fp32(fp64
// cumsum of dW), or the raw increments
struct FetchAcc {
  double wsum = 0.0;
  __device__ __forceinline__ void put(const RolloutArgs& p, int m, int d, int n, float tn, float dwn) {
    const int N1 = p.N + 1;
    if (n == 0) {
      if (p.out == PATH_FETCH_W) p.W_out[((size_t)m * N1) * p.nb + d] = 0.f;
      if (d == 0) p.t_out[(size_t)m * N1] = tn;
      return;
    }
    wsum += (double)dwn;
    if (p.out == PATH_FETCH_W)
      p.W_out[((size_t)m * N1 + n) * p.nb + d] = (float)wsum;
    else
      p.W_out[((size_t)m * p.N + n - 1) * p.nb + d] = dwn;
    if (d == 0) p.t_out[(size_t)m * N1 + n] = tn;
  }
};

// --------------------------------------------------------------------------
// diagonal problems: thread per (path m, dim d), sequential over n
//   X1 = (X0 + (mu_a X0) dt) + (sig_a X0 + sig_b) dW   (reference op order,
//   no contraction; sigma (x) dW is bit-identical to the dense bmm)
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) rollout_kernel(RolloutArgs p) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= p.M * p.D) return;
  const int m = gid / p.D, d = gid - m * p.D;
  const int N1 = p.N + 1;
  float x = p.Xi[(p.xi_rows == 1 ? 0 : m) * p.D + d];
  const double dt64 = (double)p.T / (double)p.N;
  const float sqdt = sqrtf(p.T / (float)p.N);
  double tacc = 0.0;
  float t0 = p.t ? p.t[(size_t)m * N1] : 0.0f;
  float w0 = p.W ? p.W[(size_t)m * N1 * p.nb + d] : 0.0f;
  size_t r = (size_t)m * N1;
  FetchAcc fa;
  if (p.out != PATH_ROLLOUT) fa.put(p, m, d, 0, t0, 0.f);
  for (int n0 = 0; n0 < p.N; n0 += 4) {
    float dw[4], t1[4];
    step_block(p, m, d, n0, w0, tacc, dt64, sqdt, dw, t1);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (n0 + k >= p.N) break;
      if (p.out != PATH_ROLLOUT) {
        fa.put(p, m, d, n0 + k + 1, t1[k], dw[k]);
        continue;
      }
      float* xr = p.xin + r * p.ldx;
      xr[1 + d] = x;
      if (d == 0) {
        xr[0] = t0;
        xr[p.D + 1] = 1.0f;
      }
      const float dt = rn_sub(t1[k], t0);
      const float sg = rn_add(rn_mul(p.sig_a, x), p.sig_b);
      const float s = rn_mul(sg, dw[k]);
      p.sdw[r * p.ldx + 1 + d] = s;
      x = rn_add(rn_add(x, rn_mul(rn_mul(p.mu_a, x), dt)), s);
      t0 = t1[k];
      ++r;
    }
  }
  if (p.out != PATH_ROLLOUT) return;
  float* xr = p.xin + r * p.ldx;  // n = N
  xr[1 + d] = x;
  p.sdw[r * p.ldx + 1 + d] = 0.0f;
  if (d == 0) {
    xr[0] = t0;
    xr[p.D + 1] = 1.0f;
  }
}

// The same rollout with whole-row float4 stores: thread per (path m, 16-byte
// column group c of the xin / sdw rows), columns 4c .. 4c + 3 = t (column 0),
// X_d (column 1 + d), 1 (column D + 1) and zero padding.  Every row is written
// whole, 16 bytes per lane: the thread-per-dimension form leaves the padding
// columns and the misaligned row ends to partial-line writes (the L2 then reads
// the rest of each line back: 23 MB of reads for a kernel with no inputs,
// profiles/r3_pmc_fetch).  Per dimension the arithmetic is rollout_kernel's,
// so X is bit-identical.
__global__ void __launch_bounds__(256) rollout4_kernel(RolloutArgs p) {
  const int C = p.ldx >> 2;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= p.M * C) return;
  const int m = gid / C, c = gid - m * C;
  const int N1 = p.N + 1;
  float x[4], w0[4];
  bool live[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int d = 4 * c + k - 1;
    live[k] = d >= 0 && d < p.D;
    const int dd = live[k] ? d : 0;
    x[k] = live[k] ? p.Xi[(p.xi_rows == 1 ? 0 : m) * p.D + dd] : 0.f;
    w0[k] = (live[k] && p.W) ? p.W[(size_t)m * N1 * p.nb + dd] : 0.f;
  }
  const double dt64 = (double)p.T / (double)p.N;
  const float sqdt = sqrtf(p.T / (float)p.N);
  double tacc = 0.0;
  float t0 = p.t ? p.t[(size_t)m * N1] : 0.0f;
  size_t r = (size_t)m * N1;
  for (int n0 = 0; n0 < p.N; n0 += 4) {
    // increments of the live dimensions; every call sees the same grid sum, so
    // t1 (the times of steps n0 + 1 .. n0 + 4) is the same from each
    float dw[4][4], t1[4] = {0.f, 0.f, 0.f, 0.f};
    double tn = tacc;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dw[k][i] = 0.f;
      if (live[k]) {
        tn = tacc;
        step_block(p, m, 4 * c + k - 1, n0, w0[k], tn, dt64, sqdt, dw[k], t1);
      }
    }
    tacc = tn;   // unchanged for a thread without live dimensions: its rows hold no t
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (n0 + i >= p.N) break;
      const float dt = rn_sub(t1[i], t0);
      floatx4 xo, so;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int col = 4 * c + k;
        float sv = 0.f;
        if (live[k]) {
          const float sg = rn_add(rn_mul(p.sig_a, x[k]), p.sig_b);
          sv = rn_mul(sg, dw[k][i]);
        }
        xo[k] = col == 0 ? t0 : (col == p.D + 1 ? 1.f : x[k]);
        so[k] = sv;
        if (live[k]) x[k] = rn_add(rn_add(x[k], rn_mul(rn_mul(p.mu_a, x[k]), dt)), sv);
      }
      *(floatx4*)(p.xin + r * p.ldx + 4 * c) = xo;
      *(floatx4*)(p.sdw + r * p.ldx + 4 * c) = so;
      t0 = t1[i];
      ++r;
    }
  }
  floatx4 xo, so;
#pragma unroll
  for (int k = 0; k < 4; ++k) {   // n = N
    const int col = 4 * c + k;
    xo[k] = col == 0 ? t0 : (col == p.D + 1 ? 1.f : x[k]);
    so[k] = 0.f;
  }
  *(floatx4*)(p.xin + r * p.ldx + 4 * c) = xo;
  *(floatx4*)(p.sdw + r * p.ldx + 4 * c) = so;
}

// --------------------------------------------------------------------------
// Device-mode diagonal rollout with the draws spread over the time steps.
// rollout4_kernel gives each (path, column group) pair one thread that draws
// and steps all N steps in sequence: 28 x M threads, a 50-step chain of Philox
// + Box-Muller + Euler per thread (latency-bound, 33 us at M = 1024 and at
// M = 128).  Here a 256-thread workgroup owns 64 pairs: the Philox draws of a
// 16-step window (64 pairs x 4 four-step blocks = 256 tasks, each the 4 live
// dimensions of one block) go to an LDS buffer, and while waves 1-3 draw the
// next window into the other buffer, wave 0 -- one lane per pair -- runs the
// Euler recursion of the current window out of LDS and writes the whole xin /
// sdw rows.  Per dimension every value is rollout4_kernel's (same Philox key,
// same sqrt(dt) z, same non-contracted step, the same sequential fp64 time
// grid), so X is bit-identical.
// LDS: dw[buf][step in window][pair] as float4 (the pair's 4 columns):
// lane-linear 16-byte reads, 2 x 16 KB.
// --------------------------------------------------------------------------
constexpr int RS_PAIRS = 64;
constexpr int RS_THREADS = 256;
constexpr int RS_WIN = 16;                       // steps per window (4 Philox blocks)

__device__ __forceinline__ void rs_draw(const RolloutArgs& p, int g0, int C, int blk0, float sqdt, floatx4* buf,
                                        int task) {
  const int pr = task & (RS_PAIRS - 1), bw = task >> 6;   // pair, block within the window
  const int g = g0 + pr, m = g / C, c = g - m * C;
  const int b = blk0 + bw;
  if (m >= p.M || 4 * b >= p.N) return;
  float dw[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int d = 4 * c + k - 1;
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    if (d >= 0 && d < p.D) philox_normal4(p.seed, p.offset, (uint32_t)(p.path0 + m), (uint32_t)b, (uint32_t)d, z);
#pragma unroll
    for (int s = 0; s < 4; ++s) dw[k][s] = sqdt * z[s];
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) buf[(4 * bw + s) * RS_PAIRS + pr] = floatx4{dw[0][s], dw[1][s], dw[2][s], dw[3][s]};
}

__global__ void __launch_bounds__(RS_THREADS) rollout_steps_kernel(RolloutArgs p) {
  __shared__ floatx4 dws[2 * RS_WIN * RS_PAIRS];
  const int C = p.ldx >> 2;
  const int g0 = blockIdx.x * RS_PAIRS;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int N1 = p.N + 1, nsb = (p.N + 3) / 4, nw = (nsb + 3) / 4;
  const float sqdt = sqrtf(p.T / (float)p.N);
  const double dt64 = (double)p.T / (double)p.N;
  // window 0: every thread draws one task
  rs_draw(p, g0, C, 0, sqdt, dws, threadIdx.x);
  __syncthreads();
  // the chain lane's state (wave 0)
  const int g = g0 + lane, m = g / C, c = g - m * C;
  const bool ok = wave == 0 && m < p.M;
  float x[4];
  bool live[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int d = 4 * c + k - 1;
    live[k] = d >= 0 && d < p.D;
    x[k] = (ok && live[k]) ? p.Xi[(p.xi_rows == 1 ? 0 : m) * p.D + d] : 0.f;
  }
  double tacc = 0.0;
  float t0 = (ok && p.t) ? p.t[(size_t)m * N1] : 0.0f;
  for (int w = 0; w < nw; ++w) {
    if (wave != 0) {
      // the next window's 256 tasks over the 192 drawing threads
      if (w + 1 < nw)
        for (int task = threadIdx.x - 64; task < RS_WIN / 4 * RS_PAIRS; task += RS_THREADS - 64)
          rs_draw(p, g0, C, 4 * (w + 1), sqdt, dws + ((w + 1) & 1) * RS_WIN * RS_PAIRS, task);
    } else if (ok) {
      const floatx4* buf = dws + (w & 1) * RS_WIN * RS_PAIRS;
      for (int i = 0; i < RS_WIN; ++i) {
        const int n = RS_WIN * w + i;
        if (n >= p.N) break;
        tacc += dt64;
        const float t1 = p.t ? p.t[(size_t)m * N1 + n + 1] : (float)tacc;
        const floatx4 dw = buf[i * RS_PAIRS + lane];
        const float dt = rn_sub(t1, t0);
        floatx4 xo, so;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int col = 4 * c + k;
          float sv = 0.f;
          if (live[k]) {
            const float sg = rn_add(rn_mul(p.sig_a, x[k]), p.sig_b);
            sv = rn_mul(sg, dw[k]);
          }
          xo[k] = col == 0 ? t0 : (col == p.D + 1 ? 1.f : x[k]);
          so[k] = sv;
          if (live[k]) x[k] = rn_add(rn_add(x[k], rn_mul(rn_mul(p.mu_a, x[k]), dt)), sv);
        }
        const size_t r = (size_t)m * N1 + n;
        *(floatx4*)(p.xin + r * p.ldx + 4 * c) = xo;
        *(floatx4*)(p.sdw + r * p.ldx + 4 * c) = so;
        t0 = t1;
      }
    }
    __syncthreads();
  }
  if (!ok) return;
  floatx4 xo, so;
#pragma unroll
  for (int k = 0; k < 4; ++k) {   // n = N
    const int col = 4 * c + k;
    xo[k] = col == 0 ? t0 : (col == p.D + 1 ? 1.f : x[k]);
    so[k] = 0.f;
  }
  const size_t r = (size_t)m * N1 + p.N;
  *(floatx4*)(p.xin + r * p.ldx + 4 * c) = xo;
  *(floatx4*)(p.sdw + r * p.ldx + 4 * c) = so;
}

// --------------------------------------------------------------------------
// Device-mode diagonal rollout in two passes (the default for device-mode
// diagonal problems).  rollout4_kernel's 28 M threads each run Philox +
// Box-Muller + Euler for all N steps in sequence, so the draws sit on the
// chain and only M / 9 workgroups exist (33 us at M = 128 as at M = 1024).
//   pass 1 (rollout_draw_kernel): every (path, 4-step Philox block, 16-byte
//     column group) draws in parallel and writes the raw increments
//     sqrt(dt) z into the sdw rows (columns of dims outside [0, D) are 0);
//   pass 2 (rollout_chain_kernel): thread per (path, column group), 64-thread
//     workgroups (spread over every CU: the row stores are bound by each CU's
//     store issue), runs the Euler recursion reading its increments 8 steps
//     ahead and overwrites each sdw row in place with sigma(X) dW.
// Per dimension every value is rollout4_kernel's (same Philox key, same
// sqrt(dt) z, same non-contracted step, the same sequential fp64 time grid),
// so X is bit-identical; sdw is read once more and written once more (2 x
// 4 M N Dp bytes).
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) rollout_draw_kernel(RolloutArgs p) {
  const int C = p.ldx >> 2, nsb = (p.N + 3) >> 2;
  const long long gid = blockIdx.x * 256LL + threadIdx.x;
  if (gid >= (long long)p.M * nsb * C) return;
  const int c = (int)(gid % C);
  const long long rest = gid / C;
  const int b = (int)(rest % nsb), m = (int)(rest / nsb);
  const float sqdt = sqrtf(p.T / (float)p.N);
  float dw[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int d = 4 * c + k - 1;
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    if (d >= 0 && d < p.D) philox_normal4(p.seed, p.offset, (uint32_t)(p.path0 + m), (uint32_t)b, (uint32_t)d, z);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) dw[k][s2] = (d >= 0 && d < p.D) ? sqdt * z[s2] : 0.f;
  }
  const size_t r0 = (size_t)m * (p.N + 1) + 4 * b;
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2)
    if (4 * b + s2 < p.N)
      *(floatx4*)(p.sdw + (r0 + s2) * p.ldx + 4 * c) = floatx4{dw[0][s2], dw[1][s2], dw[2][s2], dw[3][s2]};
}

constexpr int RC_THREADS = 64;
constexpr int RC_AHEAD = 8;   // increments loaded ahead of the chain
__global__ void __launch_bounds__(RC_THREADS) rollout_chain_kernel(RolloutArgs p) {
  const int C = p.ldx >> 2;
  const int gid = blockIdx.x * RC_THREADS + threadIdx.x;
  if (gid >= p.M * C) return;
  const int m = gid / C, c = gid - m * C;
  const int N1 = p.N + 1;
  float x[4];
  bool live[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int d = 4 * c + k - 1;
    live[k] = d >= 0 && d < p.D;
    x[k] = live[k] ? p.Xi[(p.xi_rows == 1 ? 0 : m) * p.D + d] : 0.f;
  }
  const double dt64 = (double)p.T / (double)p.N;
  double tacc = 0.0;
  float t0 = 0.0f;
  const size_t r0 = (size_t)m * N1;
  for (int n0 = 0; n0 < p.N; n0 += RC_AHEAD) {
    floatx4 dw[RC_AHEAD];
#pragma unroll
    for (int i = 0; i < RC_AHEAD; ++i)
      dw[i] = n0 + i < p.N ? *(const floatx4*)(p.sdw + (r0 + n0 + i) * p.ldx + 4 * c) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < RC_AHEAD; ++i) {
      const int n = n0 + i;
      if (n >= p.N) break;
      tacc += dt64;
      const float t1 = (float)tacc;
      const float dt = rn_sub(t1, t0);
      floatx4 xo, so;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int col = 4 * c + k;
        float sv = 0.f;
        if (live[k]) {
          const float sg = rn_add(rn_mul(p.sig_a, x[k]), p.sig_b);
          sv = rn_mul(sg, dw[i][k]);
        }
        xo[k] = col == 0 ? t0 : (col == p.D + 1 ? 1.f : x[k]);
        so[k] = sv;
        if (live[k]) x[k] = rn_add(rn_add(x[k], rn_mul(rn_mul(p.mu_a, x[k]), dt)), sv);
      }
      *(floatx4*)(p.xin + (r0 + n) * p.ldx + 4 * c) = xo;
      *(floatx4*)(p.sdw + (r0 + n) * p.ldx + 4 * c) = so;
      t0 = t1;
    }
  }
  floatx4 xo, so;
#pragma unroll
  for (int k = 0; k < 4; ++k) {   // n = N
    const int col = 4 * c + k;
    xo[k] = col == 0 ? t0 : (col == p.D + 1 ? 1.f : x[k]);
    so[k] = 0.f;
  }
  *(floatx4*)(p.xin + (r0 + p.N) * p.ldx + 4 * c) = xo;
  *(floatx4*)(p.sdw + (r0 + p.N) * p.ldx + 4 * c) = so;
}

// --------------------------------------------------------------------------
// Cholesky-correlated device mode (with_corr...py:339-341: dW = L (sqrt(dt) z))
// with the correlation product on the matrix cores: per step n the increments
// of a 16-path group are dW^T = L . xi^T, one v_mfma_f32_16x16x4_f32 per
// (16-dim output block o, 4-dim input step t) -- A = L (constant, held in
// registers for the whole rollout), B = xi (this step's uncorrelated
// sqrt(dt) z of the 16 paths, staged in LDS).  L is lower triangular, so block
// o stops at t < 4 o + 4.  The MFMA output layout (lane (cl, q): path cl, dims
// 16 o + 4 q + r) is the layout the Euler step and the xin / sdw rows need, so
// the step runs straight out of the accumulators.
// Workgroup = 16 paths, 8 waves (two per SIMD); wave w < nblk owns output
// block w, with its K-sum in two independent accumulation chains (the
// dependent-accumulator latency bounds a step, not the issue rate).  The
// Philox draws of the next 4-step block (4 normals per (path, dim) call) are
// made by all 512 threads into the other LDS buffer.  nb <= 128.
// LDS: xi[buf][k][q][p][t] (dim 4 t + q of path p at step 4 blk + k), t
// padded to TS = 28 (nb <= 112) or 36 floats: the 16 paths of one q read
// 16-byte slots 28 / 36 floats apart = distinct 4-bank groups (conflict-free
// ds_read_b128).
// --------------------------------------------------------------------------
// Timing-only ablations of the correlated rollout (results wrong by
// construction, never built into the library): bit 0 no row stores, bit 1 no
// draws after the first block, bit 2 no MFMA chain, bit 3 no per-step barrier.
#ifndef DBSDE_AB_CORR
#define DBSDE_AB_CORR 0
#endif
constexpr int CP_NBMAX = 128;
constexpr int CP_PATHS = 16;
constexpr int CP_THREADS = 512;                     // 8 waves: one per output block, the rest draw
// each step's xin / sdw rows are staged in LDS and written as whole float4
// rows (the MFMA layout gives each lane 4 dims of one path, one column off the
// 16-byte grid): [xin, sdw][path][SROW] (SROW = 16 nblk + 20 >= Dp).  Two
// stage buffers: step n's rows are copied out while step n + 1 is computed
// (one barrier per step; the row stores, bound by the CU's store issue, no
// longer wait for the MFMA chain and the Euler step, nor they for them).  At
// nb <= 112 the workgroup's LDS stays at 91 KB, so a phase-kernel workgroup
// (63 KB) still fits beside a prefetched rollout on a CU.
__host__ __device__ constexpr int cp_srow(int nblk) { return 16 * nblk + 20; }
template <int NBLK>
struct CPGeom {
  static constexpr int TS = NBLK <= 7 ? 28 : 36;
  static constexpr int BUF = 4 * 4 * CP_PATHS * TS;     // floats per 4-step draw buffer
  static constexpr int SROW = cp_srow(NBLK);
  static constexpr int STAGE = 2 * CP_PATHS * SROW;     // floats per stage buffer
};

typedef float cpf4 __attribute__((ext_vector_type(4)));

// the uncorrelated sqrt(dt) z of step block sb (steps 4 sb .. 4 sb + 3) of the
// workgroup's 16 paths into one LDS buffer: item (path, dim) -> 4 steps
template <int TS>
__device__ __forceinline__ void corr_draw(const RolloutArgs& p, int m0, int nt4, float sqdt, int sb, float* xb) {
  for (int it = threadIdx.x; it < CP_PATHS * 4 * nt4; it += CP_THREADS) {
    const int pp = it & (CP_PATHS - 1), d = it >> 4;
    const int m = m0 + pp;
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    if (d < p.nb && m < p.M) philox_normal4(p.seed, p.offset, (uint32_t)(p.path0 + m), (uint32_t)sb, (uint32_t)d, z);
    const int qq = d & 3, t = d >> 2;
#pragma unroll
    for (int k = 0; k < 4; ++k) xb[((k * 4 + qq) * CP_PATHS + pp) * TS + t] = sqdt * z[k];
  }
}

// rows of step n (stage buffer sg) -> xin / sdw: every thread of the
// workgroup, whole float4 columns
template <int SROW>
__device__ __forceinline__ void corr_rows_out(const RolloutArgs& p, const float* sg, int m0, int n, int N1) {
  if constexpr (DBSDE_AB_CORR & 1) return;
  const int c4 = p.ldx / 4;
  for (int it = threadIdx.x; it < 2 * CP_PATHS * c4; it += CP_THREADS) {
    const int c = it % c4, rest = it / c4, pp = rest % CP_PATHS, arr = rest / CP_PATHS;
    const int mm = m0 + pp;
    if (mm >= p.M) continue;
    const size_t r2 = (size_t)mm * N1 + n;
    float* dst = arr ? p.sdw : p.xin;
    *(cpf4*)(dst + r2 * p.ldx + 4 * c) = *(const cpf4*)(sg + (arr * CP_PATHS + pp) * SROW + 4 * c);
  }
}

// one wave's share: output blocks O1 and O2 (O2 < 0: none; O1 < 0: the wave
// only draws), K-steps t < 4 O + 4 (the lower triangle; L is zero-padded past
// nb), everything compile-time so the L fragments stay in registers
template <int NBLK, int O1, int O2>
__device__ __forceinline__ void corr_wave(const RolloutArgs& p, float* xs, float* stg) {
  using G = CPGeom<NBLK>;
  constexpr int NO = (O1 >= 0) + (O2 >= 0);
  constexpr int T1 = O1 >= 0 ? 4 * O1 + 4 : 0, T2 = O2 >= 0 ? 4 * O2 + 4 : 0;
  constexpr int TM = T1 > T2 ? T1 : T2;
  const int nb = p.nb, nt4 = (nb + 3) / 4;
  const int lane = threadIdx.x & 63, cl = lane & 15, q = lane >> 4;
  const int m0 = blockIdx.x * CP_PATHS;
  const int N1 = p.N + 1, nsb = (p.N + 3) / 4;
  const float sqdt = sqrtf(p.T / (float)p.N);
  const double dt64 = (double)p.T / (double)p.N;
  const int ob[2] = {O1, O2};
  // A fragments: L[16 o + cl][4 t + q] (zero outside the lower triangle / nb)
  float la1[T1 > 0 ? T1 : 1], la2[T2 > 0 ? T2 : 1];
#pragma unroll
  for (int t = 0; t < T1; ++t) {
    const int d = 16 * O1 + cl, k = 4 * t + q;
    la1[t] = (d < nb && k <= d && k < nb) ? p.Lt[(size_t)k * nb + d] : 0.f;
  }
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const int d = 16 * O2 + cl, k = 4 * t + q;
    la2[t] = (d < nb && k <= d && k < nb) ? p.Lt[(size_t)k * nb + d] : 0.f;
  }
  const int m = m0 + cl;
  const bool ok = m < p.M;
  float x[2][4];
  FetchAcc fa[2][4];
  float t0 = (p.t && ok) ? p.t[(size_t)m * N1] : 0.f;
#pragma unroll
  for (int oc = 0; oc < NO; ++oc)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = 16 * ob[oc] + 4 * q + r;
      const bool own = d < nb && ok;
      x[oc][r] = own ? p.Xi[(p.xi_rows == 1 ? 0 : m) * p.D + d] : 0.f;
      if (own && p.out != PATH_ROLLOUT) fa[oc][r].put(p, m, d, 0, t0, 0.f);
    }
  const bool writes_t = O1 == 0 && q == 0 && ok;   // columns 0 (t) and D + 1 (1)
  double tacc = 0.0;
  // the K-steps past nb (t >= nt4 up to 4 O + 4) read slots no draw writes:
  // zero both buffers once (0 * stale LDS could be NaN)
  for (int i = threadIdx.x; i < 2 * G::BUF; i += CP_THREADS) xs[i] = 0.f;
  for (int i = threadIdx.x; i < 2 * G::STAGE; i += CP_THREADS) stg[i] = 0.f;   // columns never written stay 0
  __syncthreads();
  corr_draw<G::TS>(p, m0, nt4, sqdt, 0, xs);
  __syncthreads();
  for (int sb = 0; sb < nsb; ++sb) {
    if (!(DBSDE_AB_CORR & 2) && sb + 1 < nsb) corr_draw<G::TS>(p, m0, nt4, sqdt, sb + 1, xs + ((sb + 1) & 1) * G::BUF);
    const float* xb = xs + (sb & 1) * G::BUF;
    for (int k = 0; k < 4; ++k) {
      const int n = 4 * sb + k;
      if (n >= p.N) break;
      tacc += dt64;
      const float t1 = (p.t && ok) ? p.t[(size_t)m * N1 + n + 1] : (float)tacc;
      if constexpr (NO > 0) {
        const float* xr = xb + ((k * 4 + q) * CP_PATHS + cl) * G::TS;
        // two independent accumulation chains per block (even / odd K-steps):
        // the dependent-accumulator latency, not the issue rate, bounds a step
        cpf4 acc[2], acc2[2];
#pragma unroll
        for (int oc = 0; oc < 2; ++oc) acc[oc] = acc2[oc] = cpf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < TM / 4; ++s4) {
          const cpf4 bz = *(const cpf4*)(xr + 4 * s4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int t = 4 * s4 + j;
            cpf4& a1 = (j & 1) ? acc2[0] : acc[0];
            cpf4& a2 = (j & 1) ? acc2[1] : acc[1];
            if constexpr (DBSDE_AB_CORR & 4) {
              if (t == 0) a1[0] += bz[j];
              continue;
            }
            if (t < T1) a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(la1[t < T1 ? t : 0], bz[j], a1, 0, 0, 0);
            if (t < T2) a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(la2[t < T2 ? t : 0], bz[j], a2, 0, 0, 0);
          }
        }
#pragma unroll
        for (int oc = 0; oc < 2; ++oc) acc[oc] += acc2[oc];
        const size_t row = (size_t)m * N1 + n;
        const float dt = rn_sub(t1, t0);
#pragma unroll
        for (int oc = 0; oc < NO; ++oc)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int d = 16 * ob[oc] + 4 * q + r;
            if (d >= nb || !ok) continue;
            const float dw = acc[oc][r];
            if (p.out != PATH_ROLLOUT) {
              fa[oc][r].put(p, m, d, n + 1, t1, dw);
              continue;
            }
            float* sr = stg + (n & 1) * G::STAGE + cl * G::SROW;
            sr[1 + d] = x[oc][r];
            const float sg = rn_add(rn_mul(p.sig_a, x[oc][r]), p.sig_b);
            const float sv = rn_mul(sg, dw);
            sr[CP_PATHS * G::SROW + 1 + d] = sv;
            x[oc][r] = rn_add(rn_add(x[oc][r], rn_mul(rn_mul(p.mu_a, x[oc][r]), dt)), sv);
          }
        if (writes_t && p.out == PATH_ROLLOUT) {
          float* sr = stg + (n & 1) * G::STAGE + cl * G::SROW;
          sr[0] = t0;
          sr[p.D + 1] = 1.0f;
        }
        (void)row;
      }
      if (p.out == PATH_ROLLOUT) {
        // the previous step's rows (its stage buffer completed before the last
        // barrier) while this step's stage fills; the barrier then orders this
        // step's stage before its copy and the copy before the buffer's reuse
        if (n > 0) corr_rows_out<G::SROW>(p, stg + ((n - 1) & 1) * G::STAGE, m0, n - 1, N1);
        if constexpr (!(DBSDE_AB_CORR & 8)) __syncthreads();
      }
      t0 = t1;
    }
    __syncthreads();
  }
  // the last step's rows
  if (p.out == PATH_ROLLOUT && p.N > 0) corr_rows_out<G::SROW>(p, stg + ((p.N - 1) & 1) * G::STAGE, m0, p.N - 1, N1);
  if constexpr (NO > 0) {
    if (p.out != PATH_ROLLOUT || !ok) return;
    const size_t row = (size_t)m * N1 + p.N;
#pragma unroll
    for (int oc = 0; oc < NO; ++oc)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = 16 * ob[oc] + 4 * q + r;
        if (d >= nb) continue;
        p.xin[row * p.ldx + 1 + d] = x[oc][r];
        p.sdw[row * p.ldx + 1 + d] = 0.0f;
      }
    if (writes_t) {
      p.xin[row * p.ldx] = t0;
      p.xin[row * p.ldx + p.D + 1] = 1.0f;
    }
  }
}

// The output block of wave w (-1: it only draws).  Block o costs 4 o + 4
// MFMAs per step (the lower triangle), and waves w and w + 4 share a SIMD, so
// the blocks go in pairs (7 - s, s) of an 8-block triangle to SIMD s (the
// NBLK blocks are its last NBLK): at NBLK = 7 the SIMDs issue 28 MFMAs per
// step each instead of 24 / 32 / 40 / 16 with block w on wave w.
template <int NBLK>
constexpr int corr_block_of_wave(int w) {
  const int s = w & 3, v = (w >> 2) ? s : 7 - s, b = v - (8 - NBLK);
  return b >= 0 ? b : -1;
}
// all 8 waves draw
template <int NBLK>
__global__ void __launch_bounds__(CP_THREADS) rollout_corr_kernel(RolloutArgs p) {
  __shared__ __attribute__((aligned(16))) float xs[2 * CPGeom<NBLK>::BUF];
  __shared__ __attribute__((aligned(16))) float stg[2 * CPGeom<NBLK>::STAGE];
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: corr_wave<NBLK, corr_block_of_wave<NBLK>(0), -1>(p, xs, stg); break;
    case 1: corr_wave<NBLK, corr_block_of_wave<NBLK>(1), -1>(p, xs, stg); break;
    case 2: corr_wave<NBLK, corr_block_of_wave<NBLK>(2), -1>(p, xs, stg); break;
    case 3: corr_wave<NBLK, corr_block_of_wave<NBLK>(3), -1>(p, xs, stg); break;
    case 4: corr_wave<NBLK, corr_block_of_wave<NBLK>(4), -1>(p, xs, stg); break;
    case 5: corr_wave<NBLK, corr_block_of_wave<NBLK>(5), -1>(p, xs, stg); break;
    case 6: corr_wave<NBLK, corr_block_of_wave<NBLK>(6), -1>(p, xs, stg); break;
    default: corr_wave<NBLK, corr_block_of_wave<NBLK>(7), -1>(p, xs, stg); break;
  }
}

// --------------------------------------------------------------------------
// k-asset Heston (heston_dnnpde.py:587-605, 629-642), state [S_1..S_k,
// v_1..v_k], one scalar Brownian motion per asset that drives both S and v
// (the reference's FBSNN dimension is 1 and einsum broadcasts dW over the two
// state components).  Thread per (path m, asset i):
//   mu    = clamp([0.05 S, kappa (theta - v)], +-100)
//   sv    = sqrt(max(v, 1e-8));  Sig = clamp([[sv S, rho sig sv], [rho sv S, sig sv]], +-100)
//   X1    = (X0 + mu dt) + (Sig_i0 + Sig_i1) dW     (einsum sums over j first)
//   sdw_i = Sig_i0 dW + Sig_i1 dW                   (the Y-tilde term, :641-642)
// --------------------------------------------------------------------------
__device__ __forceinline__ float clamp100(float v) { return fminf(fmaxf(v, -100.f), 100.f); }

__global__ void __launch_bounds__(256) rollout_heston_kernel(RolloutArgs p) {
  const int k = p.nb;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= p.M * k) return;
  const int m = gid / k, i = gid - m * k;
  const int N1 = p.N + 1;
  const float* xi = p.Xi + (size_t)(p.xi_rows == 1 ? 0 : m) * p.D;
  float S = xi[i], v = xi[k + i];
  const double dt64 = (double)p.T / (double)p.N;
  const float sqdt = sqrtf(p.T / (float)p.N);
  double tacc = 0.0;
  float t0 = p.t ? p.t[(size_t)m * N1] : 0.0f;
  float w0 = p.W ? p.W[(size_t)m * N1 * p.nb + i] : 0.0f;
  size_t r = (size_t)m * N1;
  FetchAcc fa;
  if (p.out != PATH_ROLLOUT) fa.put(p, m, i, 0, t0, 0.f);
  for (int n0 = 0; n0 < p.N; n0 += 4) {
    float dw[4], t1[4];
    step_block(p, m, i, n0, w0, tacc, dt64, sqdt, dw, t1);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (n0 + kk >= p.N) break;
      if (p.out != PATH_ROLLOUT) {
        fa.put(p, m, i, n0 + kk + 1, t1[kk], dw[kk]);
        continue;
      }
      float* xr = p.xin + r * p.ldx;
      xr[1 + i] = S;
      xr[1 + k + i] = v;
      if (i == 0) {
        xr[0] = t0;
        xr[p.D + 1] = 1.0f;
      }
      const float dt = rn_sub(t1[kk], t0);
      const float muS = clamp100(rn_mul(p.mu_a, S));
      const float muV = clamp100(rn_mul(p.kappa, rn_sub(p.theta, v)));
      const float sv = sqrtf(fmaxf(v, 1e-8f));   // correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt)
      const float sigS = rn_mul(sv, S), sigV = rn_mul(p.hsig, sv);
      const float d00 = clamp100(sigS), d11 = clamp100(sigV);
      const float d01 = clamp100(rn_mul(p.rho, sigV)), d10 = clamp100(rn_mul(p.rho, sigS));
      const float w = dw[kk];
      p.sdw[r * p.ldx + 1 + i] = rn_add(rn_mul(d00, w), rn_mul(d01, w));
      p.sdw[r * p.ldx + 1 + k + i] = rn_add(rn_mul(d10, w), rn_mul(d11, w));
      S = rn_add(rn_add(S, rn_mul(muS, dt)), rn_mul(rn_add(d00, d01), w));
      v = rn_add(rn_add(v, rn_mul(muV, dt)), rn_mul(rn_add(d10, d11), w));
      t0 = t1[kk];
      ++r;
    }
  }
  if (p.out != PATH_ROLLOUT) return;
  float* xr = p.xin + r * p.ldx;
  xr[1 + i] = S;
  xr[1 + k + i] = v;
  p.sdw[r * p.ldx + 1 + i] = 0.0f;
  p.sdw[r * p.ldx + 1 + k + i] = 0.0f;
  if (i == 0) {
    xr[0] = t0;
    xr[p.D + 1] = 1.0f;
  }
}

// Q3 (D == 1): S_n = sum over paths of sdw[m, n]   (1d_BSPDE_case.py:271-273)
__global__ void __launch_bounds__(256) q3_sum_kernel(const float* sdw, int ldx, int M, int N, float* S) {
  const int n = blockIdx.x;
  __shared__ float red[256];
  float acc = 0.f;
  for (int m = threadIdx.x; m < M; m += 256) acc += sdw[((size_t)m * (N + 1) + n) * ldx + 1];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) S[n] = red[0];
}

}  // namespace dbsde
