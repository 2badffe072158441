// vec.hpp -- flat-vector kernels of the L-BFGS optimizer (torch.optim.LBFGS as
// the reference builds it, nd_BSPDE_case.py:347-348: lr only, no clip; its
// closure re-runs loss_function + backward on the same batch, :357-361).
//
// The host drives torch's algorithm (fbsnn.py, LBFGS.step restated) and every
// vector operation runs here: fixed-order fp64 reductions (returned to the
// host, which branches on them as torch's Python code does), fp32 axpby, and
// the two-loop recursion as one single-workgroup launch (each of its 2 x num
// steps needs the previous step's global dot product, so one workgroup that
// owns every element avoids 2 x num grid-wide synchronisations).
#pragma once
#include <hip/hip_runtime.h>

namespace dbsde {

constexpr int VEC_RED_BLOCKS = 256;
constexpr int LBFGS_HMAX = 128;   // history entries per call (torch's default history_size is 100)

enum VecOp { VEC_DOT = 0, VEC_ASUM = 1, VEC_AMAX = 2 };

// per-block partials of sum a b / sum |a| / max |a| (fp64, fixed order)
__global__ void __launch_bounds__(256) vec_reduce_kernel(int op, const float* a, const float* b, long long n,
                                                         double* part) {
  __shared__ double red[256];
  double s = 0.0;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double x = a[i];
    if (op == VEC_DOT) s += x * (double)b[i];
    else if (op == VEC_ASUM) s += fabs(x);
    else s = fmax(s, fabs(x));
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] = op == VEC_AMAX ? fmax(red[threadIdx.x], red[threadIdx.x + k])
                                                           : red[threadIdx.x] + red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
__global__ void __launch_bounds__(256) vec_reduce_final_kernel(int op, const double* part, int nparts, double* out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) s = op == VEC_AMAX ? fmax(s, part[i]) : s + part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] = op == VEC_AMAX ? fmax(red[threadIdx.x], red[threadIdx.x + k])
                                                           : red[threadIdx.x] + red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

// z = alpha x + beta y (y may be null when beta == 0)
__global__ void __launch_bounds__(256) vec_axpby_kernel(float* z, const float* x, const float* y, long long n,
                                                        float alpha, float beta) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float v = alpha * x[i];
    z[i] = y ? v + beta * y[i] : v;
  }
}

struct LbfgsArgs {
  const float* g;
  const float* S;     // [slots][ld] steps s_i
  const float* Y;     // [slots][ld] gradient differences y_i
  long long ld, n;
  float* d;           // out: the direction; also q / r in place
  int num;            // history entries, oldest first
  float h_diag;
  int slot[LBFGS_HMAX];
  float ro[LBFGS_HMAX];
};

// one 1024-thread workgroup: fixed-order fp64 dot products (per-thread strided
// partials, then a tree), fp32 vector updates in torch's order:
//   q = -g;  for i = num-1..0: al_i = fp32(s_i . q) * ro_i;  q += -al_i y_i
//   r = q * H_diag;  for i = 0..num-1: be_i = fp32(y_i . r) * ro_i;  r += (al_i - be_i) s_i
__device__ inline double block_dot1024(const float* u, const float* v, long long n, double* red) {
  double s = 0.0;
  for (long long i = threadIdx.x; i < n; i += 1024) s += (double)u[i] * (double)v[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 512; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}
__global__ void __launch_bounds__(1024) lbfgs_direction_kernel(LbfgsArgs a) {
  __shared__ double red[1024];
  __shared__ float al[LBFGS_HMAX];
  float* q = a.d;
  for (long long i = threadIdx.x; i < a.n; i += 1024) q[i] = -a.g[i];
  __syncthreads();
  for (int h = a.num - 1; h >= 0; --h) {
    const float* s = a.S + (size_t)a.slot[h] * a.ld;
    const float* y = a.Y + (size_t)a.slot[h] * a.ld;
    const float alh = (float)block_dot1024(s, q, a.n, red) * a.ro[h];
    if (threadIdx.x == 0) al[h] = alh;
    for (long long i = threadIdx.x; i < a.n; i += 1024) q[i] = q[i] + (-alh) * y[i];
    __syncthreads();
  }
  for (long long i = threadIdx.x; i < a.n; i += 1024) q[i] = q[i] * a.h_diag;
  __syncthreads();
  for (int h = 0; h < a.num; ++h) {
    const float* s = a.S + (size_t)a.slot[h] * a.ld;
    const float* y = a.Y + (size_t)a.slot[h] * a.ld;
    const float be = (float)block_dot1024(y, q, a.n, red) * a.ro[h];
    const float c = al[h] - be;
    for (long long i = threadIdx.x; i < a.n; i += 1024) q[i] = q[i] + c * s[i];
    __syncthreads();
  }
}

}  // namespace dbsde
