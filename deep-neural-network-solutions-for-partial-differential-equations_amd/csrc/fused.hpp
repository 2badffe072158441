// fused.hpp -- shared pieces of the fused phase kernels (phase.hpp): their
// argument block, register tiles, compile-time activations, and the closed-form
// residual / cotangent of one row (DeepBSDE.py:223-240 restated).
#pragma once
#include <type_traits>

#include "kernels.hpp"

namespace dbsde {

// residual / cotangent inputs, shared by phase C (fused) and the forward-only
// loss kernel
struct CotanParams {
  int R, Rp, N1, D, Dp, gcols;
  const float* xin;         // [Rp, Dp]  [t, X, 1, 0..]
  const float* sdw;         // [Rp, Dp]  sigma dW (cols 1..D)
  const float* zfull;       // [Rp, Dp]  Z (cols 1..D)
  const float* u;           // [Rp]      Y
  const float* rowsum;      // [Rp, 8]   [s_zs, s_xz, s_zz, s_x, s_xx, z_1, u-mask, 0]
  const float* q3S;         // [N] or null
  float phi_r, phi_c, phi_zz, strike, g_alpha;
  int g_kind;
  // net_u VJP (dbsde_net_u_vjp): caller cotangents instead of the BSDE
  // residual ones -- ubar from ext_ub [Rp], zbar from the sdw rows
  int ext;
  const float* ext_ub;
};

struct FusedArgs {
  int R, N1, D, Dp, W, S;   // rows, N+1, D, padded D, padded level width, level stride
  int has_v, act;
  int tile0;                // first 64-row tile of this launch (path-chunked pipeline)
  int gcols;                // leading state columns entering g (row sums s_x, s_xx)
  int u_clamp;              // u = max(net, 0) (heston_dnnpde.py:568)
  float rho;
  const float* xin;         // [Rp, Dp]
  const float* beta[7];     // FC/Resnet level-j bias
  const float* wout;
  const float* bout;
  // phase A outputs
  float *Abuf, *H, *G, *Delta, *u, *zfull, *rowsum;  // rowsum [Rp, 8]
  const float* sdw;         // [Rp, Dp]
  // phase C: cotangents (computed in its prologue) and outputs
  CotanParams cp;
  float* zbar;              // [Rp, Dp] (written for the weight-gradient kernel)
  float* ubar;              // [Rp]
  float* u16;               // [Rp, 16] col 0 = ubar (split-K weight-gradient path) or null
  double* loss_part;        // [Rp / 64] per-workgroup loss sums
  float *Hdot, *Alpha;
  float* Adot;              // phase2 ADOT kernels: adot_j between the tangent and the reverse (tile order)
  // fragment images of the stage sequence of each pass (phase.hpp)
  // (fp32 images: two pieces per stage; split-bf16 images: one piece per
  // 32-wide input block, phase.hpp)
  const float* simgA[64];
  int snfA[64];
  int nA;
  const float* simgC[64];
  int snfC[64];
  int nC;
};

template <int TT>
struct Mat {
  floatx4 v[TT];
};

// activation with compile-time kind: value + first derivative, and first +
// second derivative (one sincos / tanh per element)
template <int ACT>
__device__ __forceinline__ void act_v1(float a, float& f, float& d1) {
  if constexpr (ACT == ACT_SINE) {
    fast_sincosf(a, f, d1);
  } else if constexpr (ACT == ACT_TANH) {
    f = tanhf(a);
    d1 = 1.f - f * f;
  } else {
    f = a > 0.f ? a : 0.f;
    d1 = a > 0.f ? 1.f : 0.f;
  }
}
template <int ACT>
__device__ __forceinline__ float act_1(float a) {
  if constexpr (ACT == ACT_SINE) {
    float sv, cv;
    fast_sincosf(a, sv, cv);
    return cv;
  } else if constexpr (ACT == ACT_TANH) {
    const float f = tanhf(a);
    return 1.f - f * f;
  } else {
    return a > 0.f ? 1.f : 0.f;
  }
}
template <int ACT>
__device__ __forceinline__ void act_12(float a, float& d1, float& d2) {
  if constexpr (ACT == ACT_SINE) {
    float sv;
    fast_sincosf(a, sv, d1);
    d2 = -sv;
  } else if constexpr (ACT == ACT_TANH) {
    const float f = tanhf(a);
    d1 = 1.f - f * f;
    d2 = -2.f * f * d1;
  } else {
    d1 = a > 0.f ? 1.f : 0.f;
    d2 = 0.f;
  }
}

// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E-1, so
// that per-level register arrays are indexed by constants (no scratch)
template <int B, int E>
struct SFor {
  template <class F>
  __device__ __forceinline__ static void run(F&& f) {
    if constexpr (B < E) {
      f(std::integral_constant<int, B>{});
      SFor<B + 1, E>::run(f);
    }
  }
};

template <int TT>
__device__ __forceinline__ void zero(Mat<TT>& m) {
#pragma unroll
  for (int t = 0; t < TT; ++t) m.v[t] = floatx4{0.f, 0.f, 0.f, 0.f};
}

// residual of a non-terminal row from its row sums rs, Y = y, Y_next = yn,
// dt and the Q3 sum: Y_{n+1} - Ytilde_{n+1} (DeepBSDE.py:223-228)
__device__ __forceinline__ float step_residual(const CotanParams& p, floatx4 rs0, floatx4 rs1, float y, float yn,
                                               float dt, float q3) {
  const float zs = p.q3S ? rs1[1] * q3 : rs0[0];
  const float phi = p.phi_r * (y - p.phi_c * rs0[1]) + p.phi_zz * rs0[2];
  return yn - (y + phi * dt + zs);
}

// cotangents of row r: ubar (d loss / d Y_r) and the per-row scalars the zbar
// entries need.  The loss of the row is res^2 + |Z - grad g|^2 (terminal).
// Every load is issued up front from clamped indices (one memory latency, not
// a chain of dependent ones).
struct RowCotan {
  bool valid, term;
  int n;
  float res, ub, coefY, dt, gsc, mask, q3s;
  float gA, gB;   // terminal: d g / d x_col = gA x_col + gB (terminal_dg as an affine map)
};
__device__ __forceinline__ RowCotan row_cotan(const CotanParams& p, int r) {
  RowCotan c{};
  c.valid = r < p.R;
  const int rr = c.valid ? r : 0;
  const int n = rr % p.N1;
  const bool term = n == p.N1 - 1;
  const int rn = term ? rr : rr + 1, rp = n >= 1 ? rr - 1 : rr;
  const floatx4 a0 = *(const floatx4*)(p.rowsum + (size_t)rr * 8), a1 = *(const floatx4*)(p.rowsum + (size_t)rr * 8 + 4);
  const floatx4 b0 = *(const floatx4*)(p.rowsum + (size_t)rp * 8), b1 = *(const floatx4*)(p.rowsum + (size_t)rp * 8 + 4);
  const float y = p.u[rr], yn = p.u[rn], yp = p.u[rp];
  const float t = p.xin[(size_t)rr * p.Dp], tn = p.xin[(size_t)rn * p.Dp], tp = p.xin[(size_t)rp * p.Dp];
  const float q = p.q3S ? p.q3S[term ? 0 : n] : 0.f, qp = p.q3S ? p.q3S[n >= 1 ? n - 1 : 0] : 0.f;
  c.n = n;
  c.term = term;
  c.mask = a1[2];
  if (term) {
    c.res = y - terminal_g(p.g_kind, a0[3], a1[0], p.gcols, p.strike, p.g_alpha, c.gsc);
    c.ub = 2.f * c.res;
    c.gA = p.g_kind == 0 ? 2.f : (p.g_kind == 3 ? c.gsc : 0.f);
    c.gB = (p.g_kind == 0 || p.g_kind == 3) ? 0.f : c.gsc;
  } else {
    c.dt = tn - t;
    c.res = step_residual(p, a0, a1, y, yn, c.dt, q);
    c.ub = -2.f * c.res * (1.f + p.phi_r * c.dt);
    c.q3s = q;
  }
  if (n >= 1) c.ub += 2.f * step_residual(p, b0, b1, yp, y, t - tp, qp);
  c.ub *= c.mask;
  c.coefY = -2.f * c.res;
  if (!c.valid) c.res = c.ub = c.coefY = 0.f;   // padding rows carry no cotangent
  return c;
}
// zbar of column col (1 <= col <= D) from x, z, (sigma dW) of that column;
// tz accumulates the terminal |Z - grad g|^2 over the g columns
// Branch-free (both row kinds evaluated, then selected): straight-line code
// per element, no divergence between terminal and interior rows of a wave.
__device__ __forceinline__ float col_zbar(const CotanParams& p, const RowCotan& c, int col, float xv, float zv,
                                          float sv, float& tz) {
  const float dphidz = -p.phi_r * p.phi_c * xv + 2.f * p.phi_zz * zv;
  const float sd = p.q3S ? c.q3s : sv;
  const float vn = c.mask * (c.coefY * (dphidz * c.dt + sd));
  const float e = zv - (c.gA * xv + c.gB);
  const bool ing = col <= p.gcols;
  tz += (c.term && ing) ? e * e : 0.f;
  const float vt = ing ? c.mask * (2.f * e) : 0.f;
  return c.term ? vt : vn;
}

// Forward-only loss (predict / loss_function without backward): per-block
// partial sums of the row losses; 16 threads per row, 16 rows per block.
#ifndef DBSDE_DEVICE_HELPERS_ONLY
__global__ void __launch_bounds__(256) cotan_kernel(CotanParams p, double* loss_part) {
  const int sub = threadIdx.x & 15;
  const int r = blockIdx.x * 16 + (threadIdx.x >> 4);
  double lv = 0.0;
  const RowCotan c = row_cotan(p, r);
  if (c.valid) {
    float tz = 0.f;
    if (c.term) {
      const float* xr = p.xin + (size_t)r * p.Dp;
      const float* zr = p.zfull + (size_t)r * p.Dp;
      const float* sr = p.sdw + (size_t)r * p.Dp;
      for (int col = 1 + sub; col <= p.D; col += 16) (void)col_zbar(p, c, col, xr[col], zr[col], sr[col], tz);
    }
    tz = red16(tz);
    if (sub == 0) lv = (double)(c.res * c.res + tz);
  }
  __shared__ double red[256];
  red[threadIdx.x] = lv;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss_part[blockIdx.x] = red[0];
}
#endif

}  // namespace dbsde
