// tnw.hip -- device code of the wave-owned weight-gradient contraction (see
// tnw.hpp).  Built as its own translation unit with
// -mllvm -amdgpu-mfma-vgpr-form=true: the 196 accumulators and the operand
// ring then live in arch VGPRs (253 registers, two waves per SIMD) instead of
// being split between AGPRs and VGPRs and copied on every loop trip.
#include "tnw.hpp"

namespace dbsde {

// one MFMA k-step (4 rows) of one product's operands: lane (i, kq) holds
// row 4g + kq, column 16m + i
template <int NB>
struct TnwStage {
  float a[NB], b[NB];
};

template <int NB>
__device__ __forceinline__ void tnw_load(const float* A, int lda, const float* B, int ldb, int row, int i,
                                         TnwStage<NB>& st) {
  const size_t r = (size_t)row;
#pragma unroll
  for (int m = 0; m < NB; ++m) {
    st.a[m] = A[r * lda + 16 * m + i];
    st.b[m] = B[r * ldb + 16 * m + i];
  }
}

template <int NB>
__device__ __forceinline__ void tnw_mma(floatx4 (&acc)[NB][NB], const TnwStage<NB>& st) {
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(st.a[m], st.b[n], acc[m][n], 0, 0, 0);
}

// acc += A[rows]^T B[rows] over k-steps [g0, g1), g1 - g0 a positive
// multiple of 4: three-stage register ring, steps g+1, g+2 in flight while
// step g is multiplied.  The loop body has no branches (prefetches past the
// slice are clamped to its last step and never used), so the accumulators
// stay in place and the waitcnts only cover the stage being consumed.
template <int NB>
__device__ __forceinline__ void tnw_product(floatx4 (&acc)[NB][NB], const float* A, int lda, const float* B, int ldb,
                                            int g0, int g1, int i, int kq) {
  TnwStage<NB> q0, q1, q2;
  const int gl = g1 - 1;
  // three-stage ring with a 3-step body (fixed rotation), then a 0-2 step tail
  tnw_load<NB>(A, lda, B, ldb, 4 * g0 + kq, i, q0);
  tnw_load<NB>(A, lda, B, ldb, 4 * (g0 + 1) + kq, i, q1);
  int g = g0;
  for (; g + 3 <= g1; g += 3) {
    tnw_load<NB>(A, lda, B, ldb, 4 * (g + 2) + kq, i, q2);
    __builtin_amdgcn_sched_barrier(0);
    tnw_mma<NB>(acc, q0);
    __builtin_amdgcn_sched_barrier(0);
    tnw_load<NB>(A, lda, B, ldb, 4 * min(g + 3, gl) + kq, i, q0);
    __builtin_amdgcn_sched_barrier(0);
    tnw_mma<NB>(acc, q1);
    __builtin_amdgcn_sched_barrier(0);
    tnw_load<NB>(A, lda, B, ldb, 4 * min(g + 4, gl) + kq, i, q1);
    __builtin_amdgcn_sched_barrier(0);
    tnw_mma<NB>(acc, q2);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (g < g1) tnw_mma<NB>(acc, q0);
  if (g + 1 < g1) tnw_mma<NB>(acc, q1);
}

// One workgroup = four waves = four problems of the same row slice: the four
// waves land on the four SIMDs of a CU, so the placement of the long-running
// waves is even.  XCD-aware mapping: the P/4 workgroups of a slice share
// blockIdx % 8.
template <int NB>
__global__ void __launch_bounds__(256, 1) tnw_kernel(TNWArgs a) {
  const int wg = blockIdx.x, wpg = a.P / 4;
  const int xcd = wg & 7, local = wg >> 3;
  const int s = a.s0 + (local / wpg) * 8 + xcd;
  const int p = a.order[(local - (local / wpg) * wpg) * 4 + (threadIdx.x >> 6)];
  const TNWProb& pr = a.prob[p];
  const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
  const int c0 = (int)((long long)s * a.nchunk / a.S), c1 = (int)((long long)(s + 1) * a.nchunk / a.S);

  floatx4 acc[NB][NB];
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int g0 = 4 * c0, g1 = 4 * c1;
  constexpr int T = 16 * NB;
  float* out = a.slab + ((size_t)s * a.P + p) * T * T;
  if (p == a.P - 1) {
    tnw_output<NB>(a, g0, g1, i, kq, out);
    return;
  }
  if (g1 > g0) {
    tnw_product<NB>(acc, pr.A1, pr.lda1, pr.B1, pr.ldb1, g0, g1, i, kq);
    tnw_product<NB>(acc, pr.A2, pr.lda2, pr.B2, pr.ldb2, g0, g1, i, kq);
  }
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v) out[(size_t)(16 * m + 4 * kq + v) * T + 16 * n + i] = acc[m][n][v];
}

template <int NB>
static void launch_nb(const TNWArgs& a, hipStream_t s) {
  tnw_kernel<NB><<<(unsigned)(a.sn * a.P / 4), 256, 0, s>>>(a);
}

// Launch errors are left for the caller's hipGetLastError.
int tnw_launch(int nb, const TNWArgs& a, hipStream_t s) {
  switch (nb) {
    case 1: launch_nb<1>(a, s); return 0;
    case 2: launch_nb<2>(a, s); return 0;
    case 3: launch_nb<3>(a, s); return 0;
    case 4: launch_nb<4>(a, s); return 0;
    case 5: launch_nb<5>(a, s); return 0;
    case 6: launch_nb<6>(a, s); return 0;
    case 7: launch_nb<7>(a, s); return 0;
    case 8: launch_nb<8>(a, s); return 0;
    default: return -1;
  }
}

}  // namespace dbsde
