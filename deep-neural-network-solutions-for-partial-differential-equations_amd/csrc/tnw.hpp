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
  int S;          // row slices per problem (multiple of 8)
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

}  // namespace dbsde
