// evals.hip -- the references' exact / comparator solutions on the device:
// the closed forms the drivers compare the learned Y against
// (DeepBSDE.py:345-349, nd_BSPDE_case.py:587-658, with_corr...py:621-700) and
// the HJB Monte-Carlo value (hjb_implement.py:1088-1095).  Exported through
// include/dbsde.h (dbsde_exact, dbsde_hjb_mc); no context needed.
#include <hip/hip_runtime.h>

#include "../../include/dbsde.h"
#include "philox.hpp"

namespace dbsde {

__device__ __forceinline__ double ncdf(double x) { return 0.5 * erfc(-x * 0.70710678118654752440); }

// Black-Scholes call (q = 0) at time-to-maturity tau; the payoff and its
// 1 / 1/2 / 0 delta at tau <= 0 (nd_BSPDE_case.py:590-618)
__device__ __forceinline__ void bs_call(double S, double K, double tau, double r, double sig, double& price,
                                        double& delta) {
  if (tau > 0.0) {
    const double st = sig * sqrt(tau);
    const double d1 = (log(S / K) + (r + 0.5 * sig * sig) * tau) / st;
    const double d2 = d1 - st;
    price = S * ncdf(d1) - K * exp(-r * tau) * ncdf(d2);
    delta = ncdf(d1);
  } else {
    price = S - K > 0.0 ? S - K : 0.0;
    delta = S > K ? 1.0 : (S == K ? 0.5 : 0.0);
  }
}

struct ExactArgs {
  int kind, D;
  long long R;
  double T, p0, p1, p2;
  const float* t;
  const float* x;
  float* price;
  float* delta;
};

__global__ void __launch_bounds__(256) exact_kernel(ExactArgs a) {
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  const long long n = a.kind == DBSDE_EXACT_BS_CALL ? a.R * a.D : a.R;
  if (i >= n) return;
  const long long r = a.kind == DBSDE_EXACT_BS_CALL ? i / a.D : i;
  const double tau = a.T - (double)a.t[r];
  const float* xr = a.x + r * a.D;
  double price = 0.0, delta = 0.0;
  if (a.kind == DBSDE_EXACT_BSB) {            // exp((r + s^2)(T - t)) |x|^2
    double s2 = 0.0;
    for (int d = 0; d < a.D; ++d) s2 += (double)xr[d] * (double)xr[d];
    price = exp((a.p0 + a.p1 * a.p1) * tau) * s2;
  } else if (a.kind == DBSDE_EXACT_BS_CALL) {
    bs_call((double)a.x[i], a.p2, tau, a.p0, a.p1, price, delta);
  } else if (a.kind == DBSDE_EXACT_BASKET_AVG) {   // call on mean(x), sigma / sqrt(D)
    double sm = 0.0;
    for (int d = 0; d < a.D; ++d) sm += (double)xr[d];
    bs_call(sm / a.D, a.p2, tau, a.p0, a.p1 / sqrt((double)a.D), price, delta);
  } else {                                     // mean of the per-asset calls
    double ps = 0.0, ds = 0.0;
    for (int d = 0; d < a.D; ++d) {
      double pc, dc;
      bs_call((double)xr[d], a.p2, tau, a.p0, a.p1, pc, dc);
      ps += pc;
      ds += dc;
    }
    price = ps / a.D;
    delta = ds / a.D;
  }
  a.price[i] = (float)price;
  if (a.delta) a.delta[i] = (float)delta;
}

// HJB Monte-Carlo: block (p, c) sums exp(-g(x_p + s_p z_k)) = 1 / (1/2 + |y|^2/2)
// over its share of the samples k; normals z_k[4 q + j] = normal4 of counter
// (q, HJB_TAG, k, p) (oracle/philox.py hjb_value)
constexpr uint32_t HJB_TAG = 0x484A42u;
constexpr int HJB_CHUNKS = 64;
constexpr int HJB_DMAX = 4096;

__global__ void __launch_bounds__(256) hjb_mc_kernel(const float* t, const float* x, int D, float T, long long mc,
                                                     unsigned long long seed, double* part) {
  __shared__ float xs[HJB_DMAX];
  __shared__ double red[256];
  const int p = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += 256) xs[d] = x[(size_t)p * D + d];
  __syncthreads();
  const double s = sqrt(2.0 * fabs((double)T - (double)t[p]));
  const long long per = (mc + HJB_CHUNKS - 1) / HJB_CHUNKS;
  const long long k0 = (long long)blockIdx.y * per, k1 = k0 + per < mc ? k0 + per : mc;
  double acc = 0.0;
  for (long long k = k0 + threadIdx.x; k < k1; k += 256) {
    double ss = 0.0;
    for (int q = 0; q < (D + 3) / 4; ++q) {
      float z[4];
      philox_normal4(seed, (unsigned long long)p, (uint32_t)k, HJB_TAG, (uint32_t)q, z);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = 4 * q + j;
        if (d < D) {
          const double y = (double)xs[d] + s * (double)z[j];
          ss += y * y;
        }
      }
    }
    acc += 1.0 / (0.5 + 0.5 * ss);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)p * HJB_CHUNKS + blockIdx.y] = red[0];
}

__global__ void hjb_final_kernel(const double* part, int P, long long mc, float* u) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  double s = 0.0;
  for (int c = 0; c < HJB_CHUNKS; ++c) s += part[(size_t)p * HJB_CHUNKS + c];
  u[p] = (float)(-log(s / (double)mc));
}

}  // namespace dbsde

using namespace dbsde;

extern "C" {

int dbsde_exact(int kind, const float* t, const float* x, long long R, int D, float T, const double* params,
                float* price, float* delta, void* stream) {
  if (kind < DBSDE_EXACT_BSB || kind > DBSDE_EXACT_BASKET_MEAN || !t || !x || !params || !price || R < 1 || D < 1)
    return DBSDE_EINVAL;
  ExactArgs a{};
  a.kind = kind;
  a.D = D;
  a.R = R;
  a.T = T;
  a.p0 = params[0];
  a.p1 = params[1];
  a.p2 = kind == DBSDE_EXACT_BSB ? 0.0 : params[2];
  a.t = t;
  a.x = x;
  a.price = price;
  a.delta = delta;
  const long long n = kind == DBSDE_EXACT_BS_CALL ? R * D : R;
  exact_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a);
  return hipGetLastError() == hipSuccess ? DBSDE_OK : DBSDE_EHIP;
}

int dbsde_hjb_mc(const float* t, const float* x, int P, int D, float T, long long mc, unsigned long long seed,
                 float* u, void* stream) {
  if (!t || !x || !u || P < 1 || D < 1 || D > HJB_DMAX || mc < 1) return DBSDE_EINVAL;
  double* part = nullptr;
  if (hipMallocAsync((void**)&part, (size_t)P * HJB_CHUNKS * sizeof(double), (hipStream_t)stream) != hipSuccess)
    return DBSDE_ENOMEM;
  hjb_mc_kernel<<<dim3(P, HJB_CHUNKS), 256, 0, (hipStream_t)stream>>>(t, x, D, T, mc, seed, part);
  hjb_final_kernel<<<(P + 63) / 64, 64, 0, (hipStream_t)stream>>>(part, P, mc, u);
  const hipError_t e = hipGetLastError();
  (void)hipFreeAsync(part, (hipStream_t)stream);
  return e == hipSuccess ? DBSDE_OK : DBSDE_EHIP;
}

}  // extern "C"
