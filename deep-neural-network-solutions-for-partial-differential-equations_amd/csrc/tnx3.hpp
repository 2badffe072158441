// tnx3.hpp -- the weight-gradient reduction GEMM of the per-layer (chain)
// layouts in split-bf16 products: the form of tn_gemm_kernel (kernels.hpp) for
// FC / Resnet networks whose widths have no fused phase kernels, e.g. config 4's
// FC-Sine [101, 256x4, 1] (hjb_implement.py:590-604).
//
//   slab[split][m][n] = sum over the split's rows r of  A0[r][m] B0[r][n]
//                                                      + A1[r][m] B1[r][n]
//   (loss.backward's weight gradients, DeepBSDE.py:279)
//
// One 4-wave workgroup per 128 x 128 output tile and row split, 64 x 64 (4 x 4
// MFMA blocks, 64 accumulators) per wave.  Per 32-row step the workgroup
// loads the A and B column strips once, splits every value into its exact
// hi + mid + lo bf16 parts once (phase.hpp split_two) and stores them in LDS
// as v_mfma_f32_16x16x32_bf16 fragment images; each wave then reads the
// fragments of its 4 A and 4 B blocks and issues the six products per block
// (phase.hpp: fp32-accurate).  Splitting cooperatively, each value once per
// workgroup, gives (a + b) / (a b) = 1/4 of a split per MFMA block against 2/7
// for the wave-owned 7 x 7 tile of tnwx3.hip.  The next step's global loads
// are in flight during the MFMAs.
//
// The slab layout is tn_gemm_kernel's ([split][mt 64][nt 64]), so the
// gradient finalize is shared.  The bias column of an FC / Resnet layer (the
// pair-0 "ones" column of tn_gemm_kernel) is the column sum of A0, accumulated
// in fp32 by the threads that load A0 and combined in a fixed order.
#pragma once
#include "phase.hpp"

namespace dbsde {

constexpr int TX_TILE = 128;

struct TnX3Step {
  float v[2][8];   // this thread's two 8-row column pieces
};

// column piece it (0..511) of a 128-wide strip: block it >> 6, lane (i, q) =
// rows 8 q .. 8 q + 7 of column 16 blk + i
__device__ __forceinline__ void tx3_load(TnX3Step& s, const float* X, int ld, int ncols, int col0, int r0) {
  const int t = threadIdx.x, lane = t & 63, i = lane & 15, q = lane >> 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int blk = (t >> 6) + 4 * h, col = col0 + 16 * blk + i;
    const float* p = X + (size_t)(r0 + 8 * q) * ld + col;
#pragma unroll
    for (int j = 0; j < 8; ++j) s.v[h][j] = col < ncols ? p[(size_t)j * ld] : 0.f;
  }
}
__device__ __forceinline__ void tx3_store(const TnX3Step& s, uintx4* img) {
  const int t = threadIdx.x, lane = t & 63;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int blk = (t >> 6) + 4 * h;
    uintx4 H, M, L;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const Dw3 r = split_two(s.v[h][2 * d], s.v[h][2 * d + 1]);
      H[d] = r.h;
      M[d] = r.m;
      L[d] = r.l;
    }
    img[(blk * 3 + 0) * 64 + lane] = H;
    img[(blk * 3 + 1) * 64 + lane] = M;
    img[(blk * 3 + 2) * 64 + lane] = L;
  }
}

// grid (tiles_m * tiles_n, splits, problems); rps = rows per split (multiple of 32)
// loads one (1) or two (2) steps ahead: measured equal on HJB and config 1
// (1.244 vs 1.238-1.247 ms, 0.492-0.499 vs 0.489-0.498 ms), 1 keeps the
// kernel at 184 registers
#ifndef DBSDE_TNX3_PD
#define DBSDE_TNX3_PD 1
#endif
#ifndef DBSDE_TNX3_XCD
#define DBSDE_TNX3_XCD 1
#endif
// XCD-aware order: workgroup i runs on XCD i % 8, so the grid is read as
// eight contiguous runs of (tile, split, problem), one per XCD -- the tiles of
// one split, which share their A / B column strips, run together on one XCD
// and read the strips once into its L2 instead of once per tile.
#ifndef DBSDE_TNX3_WAVES
#define DBSDE_TNX3_WAVES 3   // waves per SIMD the register budget targets (168 VGPRs; 2: 184, HJB 0.283 vs 0.267-0.271 ms)
#endif
__global__ void __launch_bounds__(256, DBSDE_TNX3_WAVES) tn_x3_kernel(TNArgs args, int rps) {
  const int nx = gridDim.x, ny = gridDim.y;
  int lin = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const int per = nx * ny * gridDim.z / 8;
  if (DBSDE_TNX3_XCD && lin < 8 * per) lin = (lin & 7) * per + (lin >> 3);
  const int tile = lin % nx, split = args.split0 + (lin / nx) % ny, prob = lin / (nx * ny);
  const TNProb& P = args.prob[prob];
  const int tiles_n = (P.nB[0] + TX_TILE - 1) / TX_TILE, tiles_m = (P.nA[0] + TX_TILE - 1) / TX_TILE;
  if (tile >= tiles_m * tiles_n) return;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int r_begin = split * rps, r_end = min(r_begin + rps, args.Rp);
  const int nstep = r_end > r_begin ? (r_end - r_begin) / 32 : 0;
  __shared__ uintx4 sa[8 * 3 * 64], sb[8 * 3 * 64];
  const int t = threadIdx.x, lane = t & 63, i = lane & 15, q = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6), wm = wave >> 1, wn = wave & 1;
  // the tile holding the bias column (or the last one, when it lies past the
  // B columns) also sums A0's columns
  const bool bias = P.ones_col >= 0 && tn == min(P.ones_col / TX_TILE, tiles_n - 1);
  floatx4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum[2] = {0.f, 0.f};
  const int total = nstep * P.npairs;
  // global loads DBSDE_TNX3_PD steps ahead: with two register sets a step's
  // strips have two steps of MFMA time to arrive from HBM (the loop is
  // unrolled by two so each set is named statically)
  TnX3Step ra0, rb0, ra1, rb1;
  auto load = [&](TnX3Step& a, TnX3Step& b, int it) __attribute__((always_inline)) {
    const int pr = it / nstep, st = it - pr * nstep;
    const int r0 = r_begin + 32 * st;
    tx3_load(a, P.A[pr], P.lda[pr], P.nA[pr], TX_TILE * tm, r0);
    tx3_load(b, P.B[pr], P.ldb[pr], P.nB[pr], TX_TILE * tn, r0);
  };
  constexpr int PD = DBSDE_TNX3_PD;
  auto step = [&](TnX3Step& ra, TnX3Step& rb, TnX3Step& na, TnX3Step& nb, int it) __attribute__((always_inline)) {
    if (bias && it < nstep) {   // pair 0: fixed row order within the thread
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[h] += ra.v[h][j];
    }
    tx3_store(ra, sa);
    tx3_store(rb, sb);
    __syncthreads();
    // PD 2: step it + 2 into this step's (now stored) registers; PD 1: it + 1
    // into the same set
    if (it + PD < total) load(PD == 2 ? ra : na, PD == 2 ? rb : nb, it + PD);
    uintx4 fb[4][3];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int p = 0; p < 3; ++p) fb[n][p] = sb[((4 * wn + n) * 3 + p) * 64 + lane];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      uintx4 fa[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) fa[p] = sa[((4 * wm + m) * 3 + p) * 64 + lane];
      const bf16x8 ah = __builtin_bit_cast(bf16x8, fa[0]), am = __builtin_bit_cast(bf16x8, fa[1]),
                   al = __builtin_bit_cast(bf16x8, fa[2]);
      // product-major over the four accumulators of the row: consecutive
      // MFMAs are independent (no dependent chain of six)
      const bf16x8 a6[6] = {al, ah, am, am, ah, ah};
      constexpr int bp[6] = {0, 2, 1, 0, 1, 0};   // b part: 0 hi, 1 mid, 2 lo
#pragma unroll
      for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a6[k], __builtin_bit_cast(bf16x8, fb[n][bp[k]]), acc[m][n], 0, 0, 0);
    }
    __syncthreads();
  };
  if (PD == 2) {
    if (total > 0) load(ra0, rb0, 0);
    if (total > 1) load(ra1, rb1, 1);
    for (int it = 0; it < total; it += 2) {
      step(ra0, rb0, ra0, rb0, it);
      if (it + 1 < total) step(ra1, rb1, ra1, rb1, it + 1);
    }
  } else {
    if (total > 0) load(ra0, rb0, 0);
    for (int it = 0; it < total; ++it) step(ra0, rb0, ra0, rb0, it);
  }
  const int ldo = P.nt * 64, nrows = P.mt * 64;
  float* out = P.slab + (size_t)split * nrows * ldo;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = TX_TILE * tm + 16 * (4 * wm + m) + 4 * q + v;
        const int col = TX_TILE * tn + 16 * (4 * wn + n) + i;
        if (row < nrows && col < ldo && !(bias && col == P.ones_col)) out[(size_t)row * ldo + col] = acc[m][n][v];
      }
  if (bias) {
    // lanes i, i + 16, i + 32, i + 48 hold the partial sums of column 16 blk + i
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float s = (__shfl(bsum[h], i) + __shfl(bsum[h], i + 16)) + (__shfl(bsum[h], i + 32) + __shfl(bsum[h], i + 48));
      const int row = TX_TILE * tm + 16 * ((t >> 6) + 4 * h) + i;
      if (q == 0 && row < nrows && P.ones_col < ldo) out[(size_t)row * ldo + P.ones_col] = s;
    }
  }
}

}  // namespace dbsde
