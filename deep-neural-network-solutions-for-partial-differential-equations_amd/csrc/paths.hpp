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

// --------------------------------------------------------------------------
// Cholesky-correlated device mode (with_corr...py:339-341: dW = L (sqrt(dt) z)):
// L^T staged in LDS once per workgroup, the uncorrelated increments of all
// paths of the workgroup staged per step, dW_d = sum_{k<=d} L[d][k] dwu_k as a
// VALU dot product per (path, d): one lane-distinct LDS read of L^T[k][d]
// (consecutive d -> conflict-free) and one broadcast 16-byte read of the
// four paths' dwu_k feed four FMAs.  Then the diagonal Euler step.
// Threads: G = 64 ceil(nb/64) per path group, 256/G groups, CP_PPT paths per
// thread.  nb <= 128.
// --------------------------------------------------------------------------
constexpr int CP_PPT = 4;
constexpr int CP_NBMAX = 128;

__global__ void __launch_bounds__(256) rollout_corr_kernel(RolloutArgs p) {
  extern __shared__ float smem[];
  const int nb = p.nb;
  const int G = (nb + 63) / 64 * 64, NG = 256 / G, PB = NG * CP_PPT;   // paths per block
  float* Lt = smem;                          // [nb][nb]
  float* zs = smem + ((nb * nb + 3) & ~3);    // [2][nb][PB], 16-byte aligned
  for (int i = threadIdx.x; i < nb * nb; i += 256) Lt[i] = p.Lt[i];
  const int tid = threadIdx.x, d = tid % G, grp = tid / G;
  const bool active_d = d < nb && grp < NG;
  const int wave_last = min(nb - 1, (tid / 64) * 64 % G + 63);   // largest d of this wave
  const int kmax = wave_last + 1;
  const int N1 = p.N + 1;
  const double dt64 = (double)p.T / (double)p.N;
  const float sqdt = sqrtf(p.T / (float)p.N);
  int mi[CP_PPT];
  bool ok[CP_PPT];
  float x[CP_PPT];
  FetchAcc fa[CP_PPT];
#pragma unroll
  for (int i = 0; i < CP_PPT; ++i) {
    mi[i] = blockIdx.x * PB + grp * CP_PPT + i;
    ok[i] = active_d && mi[i] < p.M;
    x[i] = ok[i] ? p.Xi[(p.xi_rows == 1 ? 0 : mi[i]) * p.D + d] : 0.f;
  }
  double tacc = 0.0;
  // time grid: the caller's t [M, N+1] when given (as step_block), else the
  // reference's fp32(fp64 cumsum of T/N)
  float t0[CP_PPT];
#pragma unroll
  for (int i = 0; i < CP_PPT; ++i) {
    t0[i] = (p.t && ok[i]) ? p.t[(size_t)mi[i] * N1] : 0.f;
    if (ok[i] && p.out != PATH_ROLLOUT) fa[i].put(p, mi[i], d, 0, t0[i], 0.f);
  }
  int buf = 0;
  for (int n0 = 0; n0 < p.N; n0 += 4) {
    float z[CP_PPT][4];
#pragma unroll
    for (int i = 0; i < CP_PPT; ++i) {
      if (ok[i]) philox_normal4(p.seed, p.offset, (uint32_t)(p.path0 + mi[i]), (uint32_t)(n0 >> 2), (uint32_t)d, z[i]);
      else z[i][0] = z[i][1] = z[i][2] = z[i][3] = 0.f;
    }
    for (int k4 = 0; k4 < 4 && n0 + k4 < p.N; ++k4) {
      const int n = n0 + k4;
      if (active_d) {
#pragma unroll
        for (int i = 0; i < CP_PPT; ++i) zs[(buf * nb + d) * PB + grp * CP_PPT + i] = sqdt * z[i][k4];
      }
      tacc += dt64;
      float t1[CP_PPT];
#pragma unroll
      for (int i = 0; i < CP_PPT; ++i) t1[i] = (p.t && ok[i]) ? p.t[(size_t)mi[i] * N1 + n + 1] : (float)tacc;
      __syncthreads();
      float acc[CP_PPT] = {};
      if (active_d) {
        const float* zb = zs + (size_t)buf * nb * PB + grp * CP_PPT;
        for (int k = 0; k < kmax; ++k) {
          const float l = Lt[k * nb + d];
          const float4 zz = *(const float4*)(zb + k * PB);
          acc[0] = fmaf(l, zz.x, acc[0]);
          acc[1] = fmaf(l, zz.y, acc[1]);
          acc[2] = fmaf(l, zz.z, acc[2]);
          acc[3] = fmaf(l, zz.w, acc[3]);
        }
      }
      buf ^= 1;
#pragma unroll
      for (int i = 0; i < CP_PPT; ++i) {
        if (!ok[i]) continue;
        if (p.out != PATH_ROLLOUT) {
          fa[i].put(p, mi[i], d, n + 1, t1[i], acc[i]);
          continue;
        }
        const size_t r = (size_t)mi[i] * N1 + n;
        float* xr = p.xin + r * p.ldx;
        xr[1 + d] = x[i];
        if (d == 0) {
          xr[0] = t0[i];
          xr[p.D + 1] = 1.0f;
        }
        const float dt = rn_sub(t1[i], t0[i]);
        const float sg = rn_add(rn_mul(p.sig_a, x[i]), p.sig_b);
        const float s = rn_mul(sg, acc[i]);
        p.sdw[r * p.ldx + 1 + d] = s;
        x[i] = rn_add(rn_add(x[i], rn_mul(rn_mul(p.mu_a, x[i]), dt)), s);
      }
#pragma unroll
      for (int i = 0; i < CP_PPT; ++i) t0[i] = t1[i];
    }
  }
  if (p.out != PATH_ROLLOUT) return;
#pragma unroll
  for (int i = 0; i < CP_PPT; ++i) {
    if (!ok[i]) continue;
    const size_t r = (size_t)mi[i] * N1 + p.N;
    float* xr = p.xin + r * p.ldx;
    xr[1 + d] = x[i];
    p.sdw[r * p.ldx + 1 + d] = 0.0f;
    if (d == 0) {
      xr[0] = t0[i];
      xr[p.D + 1] = 1.0f;
    }
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
