// tnwx3.hip -- the wave-owned weight-gradient contraction (tnw.hpp) in
// split-bf16 products.
//
// Each operand value is the exact sum of three bf16 parts (hi + mid + lo,
// see phase.hpp) and every 16x16 output block accumulates the six
// v_mfma_f32_16x16x32_bf16 products al.bh + ah.bl + am.bm + am.bh + ah.bm +
// ah.bh over a 32-row k-step; the dropped products stay within 2^-24 of each
// product, so the sums are as accurate as the fp32-input MFMA chain of
// tnw.hip (tools/ubench/x3_acc.hip) at 16/6 of its matrix rate.
//
// Operand layout of a 32-row step: lane (i, q) holds rows 8q .. 8q + 7 of
// column 16m + i of A (the A operand A^T[16m + i][row]) and of column 16n + i
// of B, eight dword loads per block.  One wave per SIMD (a 1024-wave grid):
// the 7x7 accumulator tile sits in AGPRs (this unit is built with the default
// MFMA register form), the split B operands of the step (84 VGPRs), the raw
// next step (112) and two split A blocks in VGPRs; the next step's loads are
// issued a whole step (294 MFMAs) ahead, and every A split runs between the
// MFMAs of the previous block (x3_products).
#include "tnw.hpp"

#ifndef DBSDE_TNW_INTERLEAVE
#define DBSDE_TNW_INTERLEAVE 1
#endif

namespace dbsde {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned uintx4 __attribute__((ext_vector_type(4)));

struct Split3 {
  bf16x8 h, m, l;
};

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned hi_pair(float a, float b) {
  return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}
// hi = bf16(x), mid = bf16(x - hi) (round to nearest even), lo = the exact
// remainder (phase.hpp split_two)
__device__ __forceinline__ Split3 split8(const float (&x)[8]) {
  uintx4 H, M, L;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const bf16x2 h = __builtin_convertvector(floatx2{x[2 * d], x[2 * d + 1]}, bf16x2);
    const float r0 = x[2 * d] - (float)h[0], r1 = x[2 * d + 1] - (float)h[1];
    const bf16x2 m = __builtin_convertvector(floatx2{r0, r1}, bf16x2);
    H[d] = __builtin_bit_cast(unsigned, h);
    M[d] = __builtin_bit_cast(unsigned, m);
    L[d] = hi_pair(r0 - (float)m[0], r1 - (float)m[1]);
  }
  return Split3{__builtin_bit_cast(bf16x8, H), __builtin_bit_cast(bf16x8, M), __builtin_bit_cast(bf16x8, L)};
}
__device__ __forceinline__ floatx4 mfma_bf(const bf16x8& a, const bf16x8& b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Operand loads through buffer descriptors: per lane one 32-bit byte offset
// (row, column i), the eight rows j of a lane's k group as SGPR offsets
// j * ld and the 16-column block m as the instruction's immediate offset, so
// a load costs no address arithmetic (the flat form spent a 64-bit add per
// load: 234 v_lshl_add_u64 per 294 MFMAs).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
}
template <int NB>
__device__ __forceinline__ void load_cols(float (&r)[NB][8], __amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned ld4) {
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int m = 0; m < NB; ++m) r[m][j] = bload1(rs, voff + 64u * m, (unsigned)j * ld4);
}

// acc += A1[rows]^T B1[rows] + A2[rows]^T B2[rows] over 32-row steps
// [g0, g1) of both products as one pipeline of 2 (g1 - g0) steps (the second
// product's first loads are in flight during the first product's last step).
// Per step: the B split (VALU) and the next step's B loads, then one
// scheduling region per A block m: its 42 MFMAs with the split of A block
// m + 1 interleaved one VALU per MFMA gap, and the next step's loads of A block
// m + 1.  The regions are pinned (sched_barrier): left alone, the scheduler
// sinks the next step's loads to the top of the next trip, right before their
// use.
template <int NB>
__device__ __forceinline__ void x3_products(floatx4 (&acc)[NB][NB], const TNWProb& pr, int g0, int g1, int i, int q) {
  const int n = g1 - g0, last = 2 * n - 1;
  const __amdgpu_buffer_rsrc_t rA1 = rsrc_of(pr.A1), rA2 = rsrc_of(pr.A2), rB1 = rsrc_of(pr.B1), rB2 = rsrc_of(pr.B2);
  const unsigned lda1 = 4u * pr.lda1, lda2 = 4u * pr.lda2, ldb1 = 4u * pr.ldb1, ldb2 = 4u * pr.ldb2;
  float ra[NB][8], rb[NB][8];
  load_cols<NB>(rb, rB1, ((32 * g0 + 8 * q) * ldb1) + 4u * i, ldb1);
  load_cols<NB>(ra, rA1, ((32 * g0 + 8 * q) * lda1) + 4u * i, lda1);
  Split3 sa = split8(ra[0]);   // A block 0 of the step (the last region splits the next step's)
  for (int k = 0; k <= last; ++k) {
    // the next step (clamped prefetch, unused past the end): product and row
    const int kn = min(k + 1, last), second = kn >= n;
    const __amdgpu_buffer_rsrc_t rA = second ? rA2 : rA1, rB = second ? rB2 : rB1;
    const unsigned lda = second ? lda2 : lda1, ldb = second ? ldb2 : ldb1;
    const unsigned nrow = 32 * (g0 + (second ? kn - n : kn)) + 8 * q;
    const unsigned voa = nrow * lda + 4u * i, vob = nrow * ldb + 4u * i;
    Split3 sb[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) sb[n] = split8(rb[n]);
    __builtin_amdgcn_sched_barrier(0);
    load_cols<NB>(rb, rB, vob, ldb);
#pragma unroll
    for (int j = 0; j < 8; ++j) ra[0][j] = bload1(rA, voa, (unsigned)j * lda);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < NB; ++m) {
      // region m splits A block m + 1 of this step, the last region block 0 of
      // the next step (loaded at this step's top)
      const Split3 san = split8(ra[m + 1 < NB ? m + 1 : 0]);
      if (m + 1 < NB) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ra[m + 1][j] = bload1(rA, voa + 64u * (m + 1), (unsigned)j * lda);
      }
#if DBSDE_TNW_INTERLEAVE
      // product-major: the NB accumulators of the row advance one product at
      // a time, so consecutive MFMAs are independent (a lone wave per SIMD
      // cannot hide the issue latency of a dependent chain of six)
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[m][n] = mfma_bf(sa.l, sb[n].h, acc[m][n]);
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[m][n] = mfma_bf(sa.h, sb[n].l, acc[m][n]);
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[m][n] = mfma_bf(sa.m, sb[n].m, acc[m][n]);
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[m][n] = mfma_bf(sa.m, sb[n].h, acc[m][n]);
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[m][n] = mfma_bf(sa.h, sb[n].m, acc[m][n]);
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[m][n] = mfma_bf(sa.h, sb[n].h, acc[m][n]);
#else
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        floatx4 c = acc[m][n];
        c = mfma_bf(sa.l, sb[n].h, c);
        c = mfma_bf(sa.h, sb[n].l, c);
        c = mfma_bf(sa.m, sb[n].m, c);
        c = mfma_bf(sa.m, sb[n].h, c);
        c = mfma_bf(sa.h, sb[n].m, c);
        acc[m][n] = mfma_bf(sa.h, sb[n].h, c);
      }
#endif
#pragma unroll
      for (int k = 0; k < 6 * NB; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);   // VALU
      }
      if (m + 1 < NB) __builtin_amdgcn_sched_group_barrier(0x020, 8, 0);   // VMEM read
      __builtin_amdgcn_sched_barrier(0);
      sa = san;
    }
  }
}

// the grid and problem / slice mapping of tnw_kernel (tnw.hip); slices are
// whole 32-row steps
template <int NB>
__global__ void __launch_bounds__(256, 1) tnw_x3_kernel(TNWArgs a) {
  const int wg = blockIdx.x, wpg = a.P / 4;
  const int xcd = wg & 7, local = wg >> 3;
  const int s = a.s0 + (local / wpg) * 8 + xcd;
  // wave-uniform problem index (its operand pointers go to SGPR buffer descriptors)
  const int p = __builtin_amdgcn_readfirstlane(a.order[(local - (local / wpg) * wpg) * 4 + (threadIdx.x >> 6)]);
  const TNWProb& pr = a.prob[p];
  const int lane = threadIdx.x & 63, i = lane & 15, q = lane >> 4;
  const int n32 = a.nchunk / 2;
  const int c0 = (int)((long long)s * n32 / a.S), c1 = (int)((long long)(s + 1) * n32 / a.S);
  constexpr int T = 16 * NB;
  float* out = a.slab + ((size_t)s * a.P + p) * T * T;
  if (p == a.P - 1) {
    tnw_output<NB>(a, 8 * c0, 8 * c1, i, q, out);
    return;
  }
  floatx4 acc[NB][NB];
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (c1 > c0) {
    x3_products<NB>(acc, pr, c0, c1, i, q);
  }
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v) out[(size_t)(16 * m + 4 * q + v) * T + 16 * n + i] = acc[m][n][v];
}

}  // namespace

int tnw_x3_launch(int nb, const TNWArgs& a, hipStream_t s) {
  if (nb != 7 || a.nchunk % 2 != 0) return -1;
  tnw_x3_kernel<7><<<(unsigned)(a.sn * a.P / 4), 256, 0, s>>>(a);
  return 0;
}

}  // namespace dbsde
