// x3_acc.hip -- accuracy of the 3-way bf16 split product (x = hi + mid + lo,
// six v_mfma_f32_16x16x32_bf16 per 32-wide k block: lh, hl, mm, mh, hm, hh;
// dropped ml, lm, ll), with round-to-nearest parts (the kernels') and with
// truncating parts, against fp32-input MFMA
// (v_mfma_f32_16x16x4_f32) and an fp64 host reference, on one 16 x 16 output
// tile of out^T = W . act^T with K = 128, plus the permuted-k operand layout
// the phase kernels use (k slot (q, j) of block kb = feature 32 kb + 16 (j>>2)
// + 4 q + (j&3)).
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench/x3_acc tools/ubench/x3_acc.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned uintx4 __attribute__((ext_vector_type(4)));

constexpr int K = 128;

__device__ __forceinline__ float trunc16(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }
__device__ __forceinline__ unsigned hi2(float a, float b) {   // [bf16(a) | bf16(b) << 16], truncating
  return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}
// 8 values (v0: j = 0..3, v1: j = 4..7) -> hi / mid / lo bf16x8 operands
// RNE = 1: hi, mid rounded to nearest even (the kernels' split); 0: truncating
__device__ __forceinline__ float part(float x, int rne) { return rne ? (float)(__bf16)x : trunc16(x); }
__device__ __forceinline__ void split8(floatx4 v0, floatx4 v1, bf16x8& h, bf16x8& m, bf16x8& l, int rne) {
  float x[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  float r1[8], r2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    r1[j] = x[j] - part(x[j], rne);
    r2[j] = r1[j] - part(r1[j], rne);
    x[j] = part(x[j], rne);
    r1[j] = part(r1[j], rne);
  }
  uintx4 H, M, L;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    H[d] = hi2(x[2 * d], x[2 * d + 1]);
    M[d] = hi2(r1[2 * d], r1[2 * d + 1]);
    L[d] = hi2(r2[2 * d], r2[2 * d + 1]);
  }
  h = __builtin_bit_cast(bf16x8, H);
  m = __builtin_bit_cast(bf16x8, M);
  l = __builtin_bit_cast(bf16x8, L);
}

// W [16][K] row-major, X [16][K] row-major (X = act rows); out[16 feat][16 row]
__global__ void tile_kernel(const float* W, const float* X, float* out_f32, float* out_x3, int rne) {
  const int l = threadIdx.x, cl = l & 15, q = l >> 4;
  floatx4 acc = {0, 0, 0, 0};
  for (int s = 0; s < K / 4; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(W[cl * K + 4 * s + q], X[cl * K + 4 * s + q], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out_f32[(4 * q + r) * 16 + cl] = acc[r];
  floatx4 a3 = {0, 0, 0, 0};
  for (int kb = 0; kb < K / 32; ++kb) {
    floatx4 w0, w1, x0, x1;
    for (int j = 0; j < 4; ++j) {
      const int f0 = 32 * kb + 4 * q + j, f1 = f0 + 16;
      w0[j] = W[cl * K + f0];
      w1[j] = W[cl * K + f1];
      x0[j] = X[cl * K + f0];
      x1[j] = X[cl * K + f1];
    }
    bf16x8 wh, wm, wl, xh, xm, xl;
    split8(w0, w1, wh, wm, wl, rne);
    split8(x0, x1, xh, xm, xl, rne);
    a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xh, a3, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xl, a3, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, xm, a3, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, xh, a3, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xm, a3, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xh, a3, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) out_x3[(4 * q + r) * 16 + cl] = a3[r];
}

int main() {
  float *dW, *dX, *df, *dx;
  hipMalloc(&dW, 16 * K * 4);
  hipMalloc(&dX, 16 * K * 4);
  hipMalloc(&df, 256 * 4);
  hipMalloc(&dx, 256 * 4);
  int rc = 0;
  for (int rne = 1; rne >= 0; --rne) {
    std::mt19937 g(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    double worst_f32 = 0, worst_x3 = 0, sum_f32 = 0, sum_x3 = 0;
    int n = 0;
    for (int trial = 0; trial < 200; ++trial) {
      std::vector<float> W(16 * K), X(16 * K), of(256), ox(256);
      const float sc = std::pow(10.f, (float)(trial % 9) - 4.f);
      for (auto& v : W) v = nd(g) * 0.1f;
      for (auto& v : X) v = nd(g) * sc;
      hipMemcpy(dW, W.data(), W.size() * 4, hipMemcpyHostToDevice);
      hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice);
      tile_kernel<<<1, 64>>>(dW, dX, df, dx, rne);
      hipMemcpy(of.data(), df, 1024, hipMemcpyDeviceToHost);
      hipMemcpy(ox.data(), dx, 1024, hipMemcpyDeviceToHost);
      for (int f = 0; f < 16; ++f)
        for (int r = 0; r < 16; ++r) {
          double ref = 0, mag = 0;
          for (int k = 0; k < K; ++k) {
            ref += (double)W[f * K + k] * X[r * K + k];
            mag += std::fabs((double)W[f * K + k] * X[r * K + k]);
          }
          const double ef = std::fabs(of[f * 16 + r] - ref) / mag, ex = std::fabs(ox[f * 16 + r] - ref) / mag;
          worst_f32 = std::max(worst_f32, ef);
          worst_x3 = std::max(worst_x3, ex);
          sum_f32 += ef;
          sum_x3 += ex;
          ++n;
        }
    }
    printf("error / sum|w x| over %d outputs (K = %d): f32 MFMA mean %.3e max %.3e | x3 bf16 (%s parts) mean %.3e "
           "max %.3e\n",
           n, K, sum_f32 / n, worst_f32, rne ? "rounded" : "truncated", sum_x3 / n, worst_x3);
    if (rne && !(worst_x3 <= worst_f32 && sum_x3 <= sum_f32)) rc = 1;
  }
  return rc;
}
