// Weight-gradient contraction for the NAIS-Net layouts, one output tile per
// wave.
//
// loss.backward() (DeepBSDE.py:279) reduces every layer's parameter gradient
// over all R = M(N+1) network rows.  In the time-parallel formulation that is
// a sum of two transposed products per weight block,
//
//   x-stack block j (input layer j = 0, V_j for j >= 1):  alpha_j^T x + delta_j^T zbar
//   block matrix B_j (j = 1..K):                          alpha_j^T h_j' + delta_j^T hdot_j'
//
// with 16*NB x 16*NB outputs (NB = Wp/16 = Dp/16).  Each wave owns the whole
// tile of one problem over its own slice of rows, so every operand row is
// read exactly once per problem and no LDS or barrier is needed.  The 2K+1
// problems that share alpha_j/delta_j (and x/zbar) with a given row slice are
// dispatched to the same XCD (blockIdx round-robin over the 8 XCDs), so the
// shared operands are served from that XCD's L2.  The partial tile is written
// to a per-slice slab; slabsum_kernel (kernels.hpp) adds the slabs in a fixed
// order (fp64), so the result is deterministic.
//
// The output layer [w_out | b_out] gradient (sum_r ubar_r [h | 1] + hdot) is
// one more (one-block-row) problem on the same row slices.
#pragma once
#include <hip/hip_runtime.h>

namespace dbsde {

constexpr int TNW_PMAX = 2 * 6 + 1;  // K <= 6

struct TNWProb {
  const float* A1;
  const float* B1;
  const float* A2;
  const float* B2;
  int lda1, ldb1, lda2, ldb2;
};

struct TNWArgs {
  TNWProb prob[TNW_PMAX];
  int P;          // problems: 2K+1 weight blocks + the output layer (last)
  int order[TNW_PMAX + 3];   // problem of workgroup slot 4 g + wave (launch_tnw: operand-sharing groups)
  int S;          // row slices per problem (multiple of 8)
  int s0, sn;     // this launch: slices [s0, s0 + sn) (sn multiple of 8; sn = S for the whole reduction)
  int nchunk;     // Rp / 16
  float* slab;    // [S][P][16NB][16NB]
  // output layer operands
  const float* ubar;
  const float* Hk;
  const float* Hdk;
  int ldh;        // row stride of Hk/Hdk
  int R;          // valid rows
};

// Launch tnw_kernel<nb> over grid = S * P / 4 four-wave workgroups (tnw.hip,
// compiled on its own with VGPR-form MFMA so the 7x7 accumulator tile and a
// three-stage operand ring fit one register class).  Returns -1 for an
// unsupported nb; launch errors are left for hipGetLastError.
__attribute__((visibility("hidden"))) int tnw_launch(int nb, const TNWArgs& a, hipStream_t s);
// The same contraction in split-bf16 products (tnwx3.hip, 32-row k-steps; the
// row slices are whole 32-row steps).  nb = 7 only; -1 otherwise.
__attribute__((visibility("hidden"))) int tnw_x3_launch(int nb, const TNWArgs& a, hipStream_t s);

typedef float floatx4 __attribute__((ext_vector_type(4)));

// Output layer [w_out | b_out]: sum_r ubar_r h_r + hdot_r (and sum_r ubar_r)
// as a one-block-row product whose A operand [ubar | 1 | 0 ...] is formed in
// registers; row 0 of the tile is w_out, element (1, 0) is b_out.
template <int NB>
__device__ __forceinline__ void tnw_output(const TNWArgs& a, int g0, int g1, int i, int kq, float* out) {
  floatx4 acc[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) acc[n] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bs = 0.f;
#pragma unroll 4
  for (int g = g0; g < g1; ++g) {
    const int row = 4 * g + kq;
    const float ub = a.ubar[row];
    const float a1 = i == 0 ? ub : 0.f;
    const float a2 = (i == 0 && row < a.R) ? 1.f : 0.f;
    const float* h = a.Hk + (size_t)row * a.ldh + i;
    const float* hd = a.Hdk + (size_t)row * a.ldh + i;
    float b1[NB], b2[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      b1[n] = h[16 * n];
      b2[n] = hd[16 * n];
    }
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1[n], acc[n], 0, 0, 0);
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, b2[n], acc[n], 0, 0, 0);
    }
    bs += a1;
  }
  constexpr int T = 16 * NB;
#pragma unroll
  for (int n = 0; n < NB; ++n)
#pragma unroll
    for (int v = 0; v < 4; ++v) out[(size_t)(4 * kq + v) * T + 16 * n + i] = acc[n][v];
  // b_out partial: lanes 0, 16, 32, 48 hold the sums of their k rows
  const float b = (__shfl(bs, 0) + __shfl(bs, 16)) + (__shfl(bs, 32) + __shfl(bs, 48));
  if ((threadIdx.x & 63) == 0) out[T] = b;
}


}  // namespace dbsde
