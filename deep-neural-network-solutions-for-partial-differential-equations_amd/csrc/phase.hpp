// phase.hpp -- register-resident fused phase kernels (gfx950).
//
// The two network passes of one deep-BSDE step, one wavefront per 16 rows
// (= 16 (path, time) pairs), 4 waves (64 rows, one wave per SIMD) per
// workgroup, two workgroups per CU (8-wave / 128-row workgroups sharing each
// staged weight piece measured slower: 0.305 -> 0.366 ms for the phases):
//   phaseA : forward (a_j, h_j, u) + input gradient (delta_j, g_j, Z) + the
//            per-row sums the residual needs (net_u, DeepBSDE.py:189-194)
//   phaseC : residuals and closed-form cotangents (ubar, zbar) of its rows,
//            forward tangent along zbar (adot_j, hdot_j) + reverse (p_j,
//            alpha_j) (loss.backward, DeepBSDE.py:279)
//
// Orientation.  Every layer is computed transposed, out^T = W . act^T: the
// weights are the MFMA A operand and the activations the B operand, so with
// v_mfma_f32_16x16x4_f32 lane l = cl + 16 q holds, for batch row cl, the
// output columns 16 o + 4 q + r (r = 0..3) of every 16-column block o.  That is
// exactly the B-operand layout the next layer needs, so activations never
// leave the registers between layers (no LDS re-layout, no per-layer barrier
// for activations, float4 global loads/stores of whole 16-byte column groups).
//
// Weights.  Each operand matrix is packed once per step (pack_tagged_kernel)
// into a t-major "fragment image": fragment (o, t) = 64 lanes x float4, lane l
// holding W[16 o + (l & 15)][16 t + 4 (l >> 4) .. + 3], at index t * TO + o.
// Every image is streamed through LDS in two pieces, input blocks [0, H) and
// [H, TI), H = ceil(TI / 2), double buffered with LDS-DMA
// (global_load_lds_dwordx4, one 1 KiB fragment per wave instruction): two
// workgroups fit in a CU (2 x 2 x 28 KB at TI = TO = 7).  Fragment reads are
// lane-linear ds_read_b128 (conflict-free).
//
// Stores.  An activation tile that the next layer also consumes (h, hdot,
// delta, g, alpha) is stored right after the next piece's barrier instead of
// just before it, so the vmcnt(0) that retires a piece's LDS-DMA does not
// wait on stores issued a few cycles earlier.
#pragma once
#include "fused.hpp"

namespace dbsde {

// Timing-only ablations of the 64-row phase kernels (profiles/r6_ab_phase.txt;
// results are wrong by construction, never built into the library): bit 0 no
// s_barrier per piece, bit 1 no weight-gradient operand stores (H, Delta, Hdot,
// Alpha, zbar), bit 2 no Abuf / G stores (phase C still loads them), bit 3 no
// wait for the piece DMA, bit 4 no operand splits (one perm instead of the
// hi / mid / lo split), bit 5 no LDS fragment reads (the piece's first
// fragment reused); the weight-gradient operand stores: bit 6 cached instead
// of non-temporal, bit 7 in tile order (1 KB contiguous per instruction),
// bit 8 column-major 16 x 16 blocks (4 dword stores per block), bits 9 / 10
// folded into the first 8192 / 512 rows (cache-resident footprints), bit 11
// into LDS instead, bit 12 the even blocks only.  The tiled layouts as real
// variants (phase kernels write, weight-gradient kernel reads) measured slower
// per step: profiles/r6_ab_phase.txt 5.
#ifndef DBSDE_AB_PHASE
#define DBSDE_AB_PHASE 0
#endif

constexpr int P3_WAVES = 4;
constexpr int P3_ROWS = 16 * P3_WAVES;
// split-bf16 weight ring depth: 3 pieces of 21 KiB (T = 7) per workgroup, two
// workgroups per CU (measured: 8-wave 128-row workgroups with a 6-deep ring,
// one per CU, 0.359 vs 0.310 ms for the phases, profiles/r3_ab_ring.txt)
constexpr int P3_NBUF_X3 = 3;

// B-operand-layout tile <-> row-major global matrix (float4 per 16-col block)
template <int TT>
__device__ __forceinline__ void bload(Mat<TT>& m, const float* base, int ld, int row0, int col0) {
  const int lane = threadIdx.x & 63;
  const float* p = base + (size_t)(row0 + (lane & 15)) * ld + col0 + 4 * (lane >> 4);
#pragma unroll
  for (int t = 0; t < TT; ++t) m.v[t] = *(const floatx4*)(p + 16 * t);
}
template <int TT>
__device__ __forceinline__ void bstore(const Mat<TT>& m, float* base, int ld, int row0, int col0) {
  const int lane = threadIdx.x & 63;
  float* p = base + (size_t)(row0 + (lane & 15)) * ld + col0 + 4 * (lane >> 4);
#pragma unroll
  for (int t = 0; t < TT; ++t) *(floatx4*)(p + 16 * t) = m.v[t];
}
// Abuf and G live only between phase A and phase C, so they use the register
// tile's own order: the 16 x 16 block at (row0, col0) is 256 contiguous floats
// (lane-major), one 1 KB contiguous access per instruction instead of 16
// 64-byte row pieces.  Needs row0, col0, ld multiples of 16.
template <int TT>
__device__ __forceinline__ void fstore(const Mat<TT>& m, float* base, int ld, int row0, int col0) {
  if constexpr (DBSDE_AB_PHASE & 4) return;
  const int lane = threadIdx.x & 63;
  float* p = base + (size_t)row0 * ld + col0 * 16 + 4 * lane;
#pragma unroll
  for (int t = 0; t < TT; ++t) *(floatx4*)(p + 256 * t) = m.v[t];
}
template <int TT>
__device__ __forceinline__ void fload(Mat<TT>& m, const float* base, int ld, int row0, int col0) {
  const int lane = threadIdx.x & 63;
  const float* p = base + (size_t)row0 * ld + col0 * 16 + 4 * lane;
#pragma unroll
  for (int t = 0; t < TT; ++t) m.v[t] = *(const floatx4*)(p + 256 * t);
}

// streaming store for the arrays only the weight-gradient kernel reads, after
// both phases (H, Delta, Hdot, Alpha, zbar): no L2 allocate, so Abuf / G / zfull,
// which phase C re-reads shortly after phase A wrote them, keep the cache
// (measured -13 us on the two phases, profiles/r2_ab_ntstore.txt)
template <int TT>
__device__ __forceinline__ void bstore_stream(const Mat<TT>& m, float* base, int ld, int row0, int col0) {
  if constexpr (DBSDE_AB_PHASE & 2) return;
  const int lane = threadIdx.x & 63;
  if constexpr (DBSDE_AB_PHASE & 128) {   // (ablation: tile order, 1 KB contiguous per instruction)
    float* p = base + (size_t)row0 * ld + col0 * 16 + 4 * lane;
#pragma unroll
    for (int t = 0; t < TT; ++t) __builtin_nontemporal_store(m.v[t], (floatx4*)(p + 256 * t));
    return;
  }
  if constexpr (DBSDE_AB_PHASE & 256) {   // (ablation: column-major 16x16 blocks, 4 dword stores)
    const int cl = lane & 15, q = lane >> 4;
    float* p = base + (size_t)row0 * ld + col0 * 16 + 64 * q + cl;
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) __builtin_nontemporal_store(m.v[t][r], p + 256 * t + 16 * r);
    return;
  }
  if constexpr (DBSDE_AB_PHASE & 2048) {   // (ablation: into LDS instead, over the ring's first KB)
#pragma unroll
    for (int t = 0; t < TT; ++t) asm volatile("ds_write_b128 %0, %1" ::"v"((unsigned)(16 * lane)), "v"(m.v[t]));
    return;
  }
  if constexpr (DBSDE_AB_PHASE & 512) row0 &= 8191;   // (ablation: a 60 MB footprint, MALL-resident)
  if constexpr (DBSDE_AB_PHASE & 1024) row0 &= 511;   // (ablation: a 4 MB footprint, L2-resident)
  float* p = base + (size_t)(row0 + (lane & 15)) * ld + col0 + 4 * (lane >> 4);
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    if constexpr (DBSDE_AB_PHASE & 4096)   // (ablation: the even blocks only)
      if (t & 1) continue;
    if constexpr (DBSDE_AB_PHASE & 64)     // (ablation: cached stores)
      *(floatx4*)(p + 16 * t) = m.v[t];
    else
      __builtin_nontemporal_store(m.v[t], (floatx4*)(p + 16 * t));
  }
}

// The LDS destination as a local-address-space pointer built from the low
// half of the generic address (the LDS offset; the aperture sits in the high
// half): the plain generic -> local cast carries a null check (s_cselect of
// src_shared_base per issue) that some register assignments cannot even encode.
__device__ __forceinline__ void glds16(const float* g, floatx4* l) {
  const unsigned off = (unsigned)(uintptr_t)l;
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)(uintptr_t)off, 16, 0, 0);
}
// s_waitcnt vmcnt(N) (expcnt / lgkmcnt untouched): vector-memory operations
// complete in issue order, so this waits for everything but the N youngest
// (N is clamped to the 6-bit field: waiting for more than asked is safe)
template <int N0>
__device__ __forceinline__ void vm_wait() {
  static_assert(N0 >= 0, "vmcnt count");
  constexpr int N = N0 < 63 ? N0 : 63;
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}
// workgroup barrier WITHOUT __syncthreads()'s release fence: that fence emits
// vmcnt(0), draining every store / load still in flight (the counted waits
// above would be lost).  lgkmcnt(0) first: this wave's LDS reads of the
// buffer the next DMA overwrites, and its LDS writes, are complete.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), vmcnt / expcnt untouched
  asm volatile("" ::: "memory");
  if constexpr (!(DBSDE_AB_PHASE & 1)) __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// acc[o] += sum_{t in [T0, T1)} W(o, t) . b(t); img = the piece holding
// fragment (o, t) at ((t - T0) * TO + o).
//   PF: the piece's fragments in that order, two per group (consecutive
//   fragments have different output blocks, so consecutive MFMAs never share
//   an accumulator), the next group's two ds_read_b128 issued before this
//   group's 8 MFMAs -- the LDS latency hides under 256 matrix-pipe cycles.
//   Otherwise output blocks in groups of 4 per input block, reads just ahead
//   of use (fewer live registers: phase C is at the 256-VGPR limit).
template <int TO, int TI, int T0, int T1, bool PF>
__device__ __forceinline__ void sgemm_piece(Mat<TO>& acc, const Mat<TI>& b, const floatx4* img, int lane) {
  if constexpr (PF) {
    constexpr int NF = (T1 - T0) * TO, NG = (NF + 1) / 2;
    floatx4 w[2][2];
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (k < NF) w[0][k] = img[k * 64 + lane];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g + 1 < NG) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int f = 2 * (g + 1) + k;
          if (f < NF) w[(g + 1) & 1][k] = img[f * 64 + lane];
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of this group's MFMAs
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int f = 2 * g + k;
          if (f < NF) {
            const int t = T0 + f / TO, o = f % TO;
            acc.v[o] = mfma4(w[g & 1][k][r], b.v[t][r], acc.v[o]);
          }
        }
    }
  } else {
    constexpr int OG = 4;
#pragma unroll
    for (int t = T0; t < T1; ++t) {
#pragma unroll
      for (int o0 = 0; o0 < TO; o0 += OG) {
        floatx4 w[OG];
#pragma unroll
        for (int o = 0; o < OG; ++o)
          if (o0 + o < TO) w[o] = img[((t - T0) * TO + o0 + o) * 64 + lane];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int o = 0; o < OG; ++o)
            if (o0 + o < TO) acc.v[o0 + o] = mfma4(w[o][r], b.v[t][r], acc.v[o0 + o]);
      }
    }
  }
}

// wave w copies fragments w, w + P3_WAVES, ... of an nf-fragment piece
__device__ __forceinline__ void piece_dma(const float* img, int nf, floatx4* buf, int wave, int lane) {
  for (int f = wave; f < nf; f += P3_WAVES) glds16(img + (size_t)f * 256 + lane * 4, buf + f * 64);
}
// the same with a compile-time fragment count (split-bf16 pieces: 3 TO), unrolled
template <int NF>
__device__ __forceinline__ void piece_dma_n(const float* img, floatx4* buf, int wave, int lane) {
#pragma unroll
  for (int k = 0; k < (NF + P3_WAVES - 1) / P3_WAVES; ++k) {
    const int f = wave + P3_WAVES * k;
    if (k < NF / P3_WAVES || f < NF) glds16(img + (size_t)f * 256 + lane * 4, buf + f * 64);
  }
}
// lane l of a VGPR pair holds piece l's image pointer (loaded once per kernel):
// a piece's pointer is two v_readlane_b32 instead of a scalar load from the
// kernel arguments after every barrier (the barrier's memory clobber forces
// the reload)
__device__ __forceinline__ const float* lane_ptr(unsigned long long v, int idx) {
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)v, idx), hi = __builtin_amdgcn_readlane((unsigned)(v >> 32), idx);
  return (const float*)(((unsigned long long)hi << 32) | lo);
}

// piece sequencer: wait for this piece, publish it, start the one NBUF - 1
// ahead (NBUF-buffer LDS ring; the fp32 kernels use 2, the split-bf16 kernels,
// whose pieces carry 1/4 of the MFMA work, P3_NBUF_X3).
// NYOUNG = vector-memory operations this wave is guaranteed to have issued
// after the piece's DMA (deferred stores, early loads): they may stay in flight
// across the barrier.  Under-counting is safe, over-counting is a race.  With
// NBUF > 2 the DMAs of the k = min(NBUF - 2, n - 1 - st) following pieces were
// also issued after this piece's: LC = a lower bound of this wave's chunks of
// each (waves copy 5 or 6 of 21), so k LC more may stay in flight.
//   NF > 0: every piece has NF fragments (the split-bf16 kernels) and the piece
//   pointers come from a per-lane table (lane_ptr, n <= 64).
//   NP > 0: the kernel's piece count at compile time (else the runtime n).
template <int NBUF, int LC, int NF = 0, int NP = 0>
struct PieceStagerT {
  static constexpr int nbuf = NBUF;
  static constexpr bool kRegs = false;   // (phasecs.hip's register-streamed feed: true)
  floatx4* wl;
  const float* const* img;
  const int* nf;
  int n, st, wave, lane, buf;
  unsigned long long ptab = 0;
  __device__ __forceinline__ void mark() {}
  __device__ __forceinline__ void dma(int k, floatx4* dst) {
    if constexpr (NF > 0)
      piece_dma_n<NF>(lane_ptr(ptab, k), dst, wave, lane);
    else
      piece_dma(img[k], nf[k], dst, wave, lane);
  }
  __device__ __forceinline__ int count() const { return NP > 0 ? NP : n; }
  __device__ __forceinline__ void start() {
    if constexpr (NF > 0) ptab = lane < count() ? (unsigned long long)img[lane] : 0ull;
#pragma unroll
    for (int k = 0; k < NBUF - 1; ++k)
      if (k < count()) dma(k, wl + k * buf);
  }
  // vm_wait<NYOUNG + LC k> for the runtime k (uniform) of younger pieces
  template <int NYOUNG, int K>
  __device__ __forceinline__ void wait_younger(int k) {
    if constexpr (K == 0) {
      vm_wait<NYOUNG>();
    } else {
      if (k >= K)
        vm_wait<NYOUNG + LC * K>();
      else
        wait_younger<NYOUNG, K - 1>(k);
    }
  }
  template <int NYOUNG>
  __device__ __forceinline__ const floatx4* next() {
    if constexpr (DBSDE_AB_PHASE & 8) {
    } else if constexpr (DBSDE_AB_PHASE & 6) {
      vm_wait<0>();   // the removed stores no longer pad the counts: drain (errs slow)
    } else if constexpr (NBUF > 2) {
      const int k = min(NBUF - 2, count() - 1 - st);
      wait_younger<NYOUNG, NBUF - 2>(k);
    } else {
      vm_wait<NYOUNG>();
    }
    lds_barrier();
    constexpr int DIST = NBUF - 1;
    if (st + DIST < count()) dma(st + DIST, wl + ((st + DIST) % NBUF) * buf);
    // nothing issued later may be hoisted above the DMA (the NYOUNG counts)
    __builtin_amdgcn_sched_barrier(0);
    const floatx4* cur = wl + (st % NBUF) * buf;
    ++st;
    return cur;
  }
};
// the kernels' stager: X3 pieces are 3 TO chunks, TO >= min(T, TD)
// NP: pieces of phase A (PH = 0: X0, {F_j, [X_j]}, {[Z_j], B_j}, Z0) or phase C
// (PH = 1: X0, [X_j], F_j, B_j), one per 32-wide input block in the X3 form
template <bool X3, int T, int TD, int K = 0, bool HV = false, int PH = 0>
using PieceStager = PieceStagerT<X3 ? P3_NBUF_X3 : 2, X3 ? (3 * (T < TD ? T : TD)) / P3_WAVES : 0, (X3 && T == TD) ? 3 * T : 0,
                                 (X3 && T == TD && K > 0)
                                     ? ((T + 1) / 2) * (PH == 0 ? 2 + 2 * K * (HV ? 2 : 1) : 1 + K * (HV ? 3 : 2))
                                     : 0>;


struct NoOp {
  __device__ __forceinline__ void operator()() const {}
};

// ---------------------------------------------------------------------------
// Split-bf16 products (X3 kernels).  An fp32 value is the exact sum of three
// bf16 parts, x = hi + mid + lo (hi and mid rounded to nearest even, lo the
// remainder: 8 + 8 + 8 significand bits), and W x is accumulated as the six
// v_mfma_f32_16x16x32_bf16 products Wl.xh + Wh.xl + Wm.xm + Wm.xh + Wh.xm +
// Wh.xh.  Every bf16 product is exact in the fp32 accumulator and the three
// dropped ones (Wm.xl, Wl.xm, Wl.xl) sum to at most 2^-24 of |W x| (the
// fp32 rounding bound of the product itself; unbiased, 3.5e-9 on average,
// tests/test_host_logic.py), so the result is as accurate as the fp32-input
// MFMA chain (tools/ubench/x3_acc.hip) at 16/6 of its rate on the matrix
// cores, which also leave the vector ALUs to the epilogues.
// Operand order: a 32-wide input block kb is the pair of 16-column register
// blocks (2 kb, 2 kb + 1) of the B-layout tile; lane (cl, q) element j holds
// column 32 kb + 16 (j >> 2) + 4 q + (j & 3) -- no data movement between
// layers, the weight image carries the same permutation (x3_off).
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef unsigned uintx4 __attribute__((ext_vector_type(4)));

struct Split3 {
  bf16x8 h, m, l;
};
// [upper half of a | upper half of b << 16]: two bf16 in one dword (exact
// when a and b are bf16 values)
__device__ __forceinline__ unsigned hi_pair(float a, float b) {
  return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}
// (x0, x1) -> dword d of the hi / mid / lo operands: hi = bf16(x) and mid =
// bf16(x - hi) rounded to nearest even (v_cvt_pk_bf16_f32), lo = the exact
// remainder (at most 8 significant bits, so a bf16 value)
struct Dw3 {
  unsigned h, m, l;
};
__device__ __forceinline__ Dw3 split_two(float x0, float x1) {
  if constexpr (DBSDE_AB_PHASE & 16) {
    const unsigned v = hi_pair(x0, x1);
    return Dw3{v, v, v};
  }
  const bf16x2 h = __builtin_convertvector(floatx2{x0, x1}, bf16x2);
  const float r0 = x0 - (float)h[0], r1 = x1 - (float)h[1];
  const bf16x2 m = __builtin_convertvector(floatx2{r0, r1}, bf16x2);
  return Dw3{__builtin_bit_cast(unsigned, h), __builtin_bit_cast(unsigned, m), hi_pair(r0 - (float)m[0], r1 - (float)m[1])};
}
template <int TI, int KB>
__device__ __forceinline__ Split3 split_block(const Mat<TI>& b) {
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int t = 2 * KB + (j >> 2);
    x[j] = t < TI ? b.v[t < TI ? t : 0][j & 3] : 0.f;
  }
  uintx4 H, M, L;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const Dw3 r = split_two(x[2 * d], x[2 * d + 1]);
    H[d] = r.h;
    M[d] = r.m;
    L[d] = r.l;
  }
  return Split3{__builtin_bit_cast(bf16x8, H), __builtin_bit_cast(bf16x8, M), __builtin_bit_cast(bf16x8, L)};
}
__device__ __forceinline__ floatx4 mfma_bf(uintx4 a, const bf16x8& b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), b, c, 0, 0, 0);
}
// split pair d (elements 2d, 2d + 1) of input block KB into dword d of the
// hi / mid / lo operands
template <int TI, int KB, int d>
__device__ __forceinline__ void split_pair(const Mat<TI>& b, uintx4& H, uintx4& M, uintx4& L) {
  float x[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int j = 2 * d + e, t = 2 * KB + (j >> 2);
    x[e] = t < TI ? b.v[t < TI ? t : 0][j & 3] : 0.f;
  }
  const Dw3 r = split_two(x[0], x[1]);
  H[d] = r.h;
  M[d] = r.m;
  L[d] = r.l;
}
// acc[o] += W(o, kb) . b(kb) over one piece = the TO fragments of input block
// kb, fragment o at chunks 3 o .. 3 o + 2 (hi, mid, lo).  Each fragment is one
// scheduling region: the next fragment's three ds_read_b128 first, then its six
// MFMAs with the split of the NEXT input block (KBN, one dword pair per
// fragment) interleaved two VALU per MFMA gap -- the LDS latency and the split
// hide under the matrix pipe.
//   PF = false (register-tight stages): a fragment's reads open its own region.
template <int TO, int TI, int KBN, bool PF>
__device__ __forceinline__ void sgemm_x3_piece(Mat<TO>& acc, const Split3& s, const floatx4* img, int lane,
                                               const Mat<TI>& b, uintx4 (&sn)[3]) {
  constexpr bool NEXT = KBN < (TI + 1) / 2;
  const uintx4* im = (const uintx4*)img;
  uintx4 w[PF ? 2 : 1][3];
  if constexpr (PF) {
#pragma unroll
    for (int p = 0; p < 3; ++p) w[0][p] = im[p * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);
  }
  SFor<0, TO>::run([&](auto oc) __attribute__((always_inline)) {
    constexpr int o = decltype(oc)::value;
    constexpr int OR = (DBSDE_AB_PHASE & 32) ? 0 : 1;   // (ablation: every fragment read is fragment 0's)
    if constexpr (PF && o + 1 < TO) {
#pragma unroll
      for (int p = 0; p < 3; ++p) w[(o + 1) & 1][p] = im[(3 * (o + 1) * OR + p) * 64 + lane];
    } else if constexpr (!PF) {
#pragma unroll
      for (int p = 0; p < 3; ++p) w[0][p] = im[(3 * o * OR + p) * 64 + lane];
    }
    if constexpr (NEXT && o < 4) split_pair<TI, NEXT ? KBN : 0, o>(b, sn[0], sn[1], sn[2]);
    // in the order the fragment parts arrive (hi, mid, lo: counted lgkmcnt
    // waits let the first MFMAs start before the later reads land)
    const uintx4* wc = w[PF ? (o & 1) : 0];
    floatx4 a = acc.v[o];
    a = mfma_bf(wc[0], s.l, a);
    a = mfma_bf(wc[0], s.m, a);
    a = mfma_bf(wc[1], s.m, a);
    a = mfma_bf(wc[1], s.h, a);
    a = mfma_bf(wc[2], s.h, a);
    acc.v[o] = mfma_bf(wc[0], s.h, a);
    if constexpr (!PF || o + 1 < TO) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);   // DS read
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // VALU
    }
    __builtin_amdgcn_sched_barrier(0);
  });
}
// The same piece with the MFMA chains of two fragments interleaved: one
// scheduling region per fragment pair (o0, o1), its twelve MFMAs alternating
// between the two accumulators, the next pair's six ds_read_b128 issued at
// the region's top (48 VGPRs of weight operands instead of 24).  A chain of
// six dependent v_mfma_f32_16x16x32_bf16 on one accumulator does not issue
// back to back; two interleaved chains do (tools/ubench/piece_x3.hip).
template <int TO, int TI, int KBN>
__device__ __forceinline__ void sgemm_x3_piece_pairs(Mat<TO>& acc, const Split3& s, const floatx4* img, int lane,
                                                     const Mat<TI>& b, uintx4 (&sn)[3]) {
  constexpr bool NEXT = KBN < (TI + 1) / 2;
  constexpr int NPR = (TO + 1) / 2;
  const uintx4* im = (const uintx4*)img;
  uintx4 w[2][2][3];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      if (k < TO) w[0][k][p] = im[(3 * k + p) * 64 + lane];
  __builtin_amdgcn_sched_barrier(0);
  SFor<0, NPR>::run([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    constexpr int o0 = 2 * g, o1 = 2 * g + 1;
    constexpr bool two = o1 < TO;
    constexpr int nrd = g + 1 < NPR ? 3 * ((2 * (g + 1) + 1 < TO) ? 2 : 1) : 0;   // next pair's reads
    if constexpr (g + 1 < NPR) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          if (2 * (g + 1) + k < TO) w[(g + 1) & 1][k][p] = im[(3 * (2 * (g + 1) + k) + p) * 64 + lane];
    }
    // the split of the next input block, one dword pair per region (4 pairs)
    if constexpr (NEXT && g < 4) split_pair<TI, NEXT ? KBN : 0, g>(b, sn[0], sn[1], sn[2]);
    if constexpr (NEXT && NPR < 4 && g == NPR - 1) {   // fewer regions than pairs: the rest here
      SFor<NPR, 4>::run([&](auto dc) __attribute__((always_inline)) {
        split_pair<TI, NEXT ? KBN : 0, decltype(dc)::value>(b, sn[0], sn[1], sn[2]);
      });
    }
    const uintx4* wa = w[g & 1][0];
    const uintx4* wb = w[g & 1][1];
    floatx4 a = acc.v[o0], c = acc.v[two ? o1 : o0];
    a = mfma_bf(wa[0], s.l, a);
    if constexpr (two) c = mfma_bf(wb[0], s.l, c);
    a = mfma_bf(wa[0], s.m, a);
    if constexpr (two) c = mfma_bf(wb[0], s.m, c);
    a = mfma_bf(wa[1], s.m, a);
    if constexpr (two) c = mfma_bf(wb[1], s.m, c);
    a = mfma_bf(wa[1], s.h, a);
    if constexpr (two) c = mfma_bf(wb[1], s.h, c);
    a = mfma_bf(wa[2], s.h, a);
    if constexpr (two) c = mfma_bf(wb[2], s.h, c);
    acc.v[o0] = mfma_bf(wa[0], s.h, a);
    if constexpr (two) acc.v[o1] = mfma_bf(wb[0], s.h, c);
    if constexpr (nrd > 0) __builtin_amdgcn_sched_group_barrier(0x100, nrd, 0);   // DS read
#pragma unroll
    for (int k = 0; k < (two ? 12 : 6); ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);   // VALU
    }
    __builtin_amdgcn_sched_barrier(0);
  });
}

// piece kind: 0 = sgemm_x3_piece (one chain at a time), 1 = fragment pairs
#ifndef DBSDE_PIECE_PAIRS
#define DBSDE_PIECE_PAIRS 0
#endif
// phase A: act'(a_j) recomputed from Abuf in the backward (1) or kept (0)
#ifndef DBSDE_A_RECOMP
#define DBSDE_A_RECOMP 0
#endif

// Vector-memory ops younger than piece KB's DMA (a lower bound for its
// vm_wait), DIST = ring depth - 1 the DMA lead: the previous stage's epilogue
// (NPRE ops, issued after the DMA of piece DIST - 1) for KB < DIST, and
// `after` (NAFTER ops, issued at piece 0 after the DMA of piece DIST) for
// 1 <= KB <= DIST.  A store is then waited for only once a DMA issued after
// it is needed.  DBSDE_VMCOUNT 0: the earlier tighter counts (KB 0 NPRE, KB 1
// NAFTER, none after), which made piece 1 wait for the epilogue's stores and
// piece 2 for `after`'s.
#ifndef DBSDE_VMCOUNT
#define DBSDE_VMCOUNT 1
#endif
template <int KB, int DIST, int NPRE, int NAFTER>
constexpr int piece_nyoung() {
  if constexpr (DBSDE_VMCOUNT == 0) return KB == 0 ? NPRE : (KB == 1 ? NAFTER : 0);
  return (KB < DIST ? NPRE : 0) + (KB >= 1 && KB <= DIST ? NAFTER : 0);
}
template <int TO, int TI, int NPRE, int NAFTER, int KB, bool PF, class SG, class F>
__device__ __forceinline__ void stage_x3_from(Mat<TO>& acc, const Mat<TI>& b, SG& sg, int lane, F&& after,
                                              const Split3& s) {
  constexpr int NKB = (TI + 1) / 2;
  if constexpr (KB < NKB) {
    const floatx4* w = sg.template next<piece_nyoung<KB, SG::nbuf - 1, NPRE, NAFTER>()>();
    if constexpr (KB == 0) {
      after();
      __builtin_amdgcn_sched_barrier(0);
    }
    uintx4 sn[3];
    if constexpr (DBSDE_PIECE_PAIRS && PF)
      sgemm_x3_piece_pairs<TO, TI, KB + 1>(acc, s, w, lane, b, sn);
    else
      sgemm_x3_piece<TO, TI, KB + 1, PF>(acc, s, w, lane, b, sn);
    sg.mark();
    if constexpr (KB + 1 < NKB)
      stage_x3_from<TO, TI, NPRE, NAFTER, KB + 1, PF>(
          acc, b, sg, lane, after,
          Split3{__builtin_bit_cast(bf16x8, sn[0]), __builtin_bit_cast(bf16x8, sn[1]), __builtin_bit_cast(bf16x8, sn[2])});
  }
}

// one stage = one operand image: two pieces (one when TI == 1), or in the X3
// kernels one piece per 32-wide input block; `after` runs right after the
// first piece's barrier (deferred stores, early loads).
// NPRE = vector-memory ops issued since the first piece's DMA (the previous
// stage's epilogue), NAFTER = the ops `after` issues (both lower bounds).
template <bool X3, int TO, int TI, int NPRE, int NAFTER, bool PF = false, class SG, class F>
__device__ __forceinline__ void stage_mm(Mat<TO>& acc, const Mat<TI>& b, SG& sg, int lane, F&& after) {
  if constexpr (X3) {
    stage_x3_from<TO, TI, NPRE, NAFTER, 0, PF>(acc, b, sg, lane, after, split_block<TI, 0>(b));
    return;
  }
  constexpr int H = (TI + 1) / 2;
  const floatx4* w = sg.template next<NPRE>();
  after();
  // keep the deferred stores / early loads here: left to itself the scheduler
  // sinks them to the end of the piece, right in front of the next vmcnt(0)
  __builtin_amdgcn_sched_barrier(0);
  sgemm_piece<TO, TI, 0, H, PF>(acc, b, w, lane);
  sg.mark();
  if constexpr (H < TI) {
    w = sg.template next<NAFTER>();
    sgemm_piece<TO, TI, H, TI, PF>(acc, b, w, lane);
    sg.mark();
  }
}

// ---------------------------------------------------------------------------
// phase A: forward + input gradient + Z (+ residual row sums)
// stage images (host order): X0, {F_j, [X_j]} j=1..K, {[Z_j], B_j} j=K..1, Z0
// ---------------------------------------------------------------------------
template <int T, int TD, int K, int ACT, bool HV, bool X3>
__global__ void __launch_bounds__(64 * P3_WAVES, 2 * P3_WAVES / 4) phaseA_kernel(FusedArgs p) {
  constexpr bool PFA = true;    // group-ahead fragment prefetch (sgemm_piece)
  constexpr int TB = T > TD ? T : TD, BUF = X3 ? 3 * TB * 64 : ((TB + 1) / 2) * TB * 64;
  __shared__ floatx4 wl[(X3 ? P3_NBUF_X3 : 2) * BUF];
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = blockIdx.x + p.tile0;   // 64-row tile (chunked launches offset it)
  const int row0 = tile * P3_ROWS + wave * 16;
  const int S = p.S, Wd = p.W;
  PieceStager<X3, T, TD, K, HV, 0> sg{wl, p.simgA, p.snfA, p.nA, 0, wave, lane, BUF};
  sg.start();
  Mat<TD> x;
  bload(x, p.xin, p.Dp, row0, 0);

  // act'(a_j) in registers, or (RECOMP, DBSDE_A_RECOMP) recomputed in the
  // backward from a_j reloaded out of Abuf (frees 3 T registers x 4 levels)
  constexpr bool RECOMP = DBSDE_A_RECOMP != 0;
  Mat<T> s1[RECOMP ? 1 : K + 1];
  Mat<T> h, acc;
  zero(acc);
  stage_mm<X3, T, TD, TD, 0, PFA>(acc, x, sg, lane, NoOp{});
  fstore(acc, p.Abuf, S, row0, 0);
#pragma unroll
  for (int o = 0; o < T; ++o)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float f, d;
      act_v1<ACT>(acc.v[o][r], f, d);
      h.v[o][r] = f;
      if constexpr (!RECOMP) s1[0].v[o][r] = d;
    }
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    zero(acc);
    stage_mm<X3, T, T, T, T, PFA>(acc, h, sg, lane, [&]() __attribute__((always_inline)) { bstore_stream(h, p.H, S, row0, (j - 1) * Wd); });
    if constexpr (HV) stage_mm<X3, T, TD, 0, 0, PFA>(acc, x, sg, lane, NoOp{});
#pragma unroll
    for (int o = 0; o < T; ++o) {
      if constexpr (!HV) {
        const floatx4 bb = *(const floatx4*)(p.beta[j - 1] + 16 * o + 4 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc.v[o][r] += bb[r];
      }
    }
    fstore(acc, p.Abuf, S, row0, j * Wd);
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float f, d;
        act_v1<ACT>(acc.v[o][r], f, d);
        if constexpr (!RECOMP) s1[j].v[o][r] = d;
        h.v[o][r] = f + p.rho * h.v[o][r];
      }
  });
  // u = h_{K+1} . w_out + b_out  (clamped at 0 for Heston, heston_dnnpde.py:568;
  // the clamp's gradient passes at u_raw >= 0, so Z = mask * grad u_raw)
  float umask = 1.f;
  {
    float us = 0.f;
#pragma unroll
    for (int o = 0; o < T; ++o) {
      const floatx4 wo = *(const floatx4*)(p.wout + 16 * o + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) us += h.v[o][r] * wo[r];
    }
    us += __shfl_xor(us, 16);
    us += __shfl_xor(us, 32);
    float uv = us + p.bout[0];
    if (p.u_clamp) {
      umask = uv >= 0.f ? 1.f : 0.f;
      uv = uv >= 0.f ? uv : 0.f;
    }
    if (q == 0) p.u[row0 + cl] = uv;
  }
  bstore_stream(h, p.H, S, row0, K * Wd);
  // input gradient: g_{K+1} = w_out, delta_K = w_out act'(a_K)
  Mat<T> g, dl;
#pragma unroll
  for (int o = 0; o < T; ++o) {
    const floatx4 wo = *(const floatx4*)(p.wout + 16 * o + 4 * q);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      g.v[o][r] = wo[r];
      // (acc still holds a_K)
      dl.v[o][r] = wo[r] * (RECOMP ? act_1<ACT>(acc.v[o][r]) : s1[RECOMP ? 0 : K].v[o][r]);
    }
  }
  Mat<TD> z;
  zero(z);
  Mat<T> av;   // RECOMP: a_{j-1}, reloaded
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    auto prev = [&]() __attribute__((always_inline)) {   // (g_j, delta_j) of the previous step
      if constexpr (j < K) fstore(g, p.G, S, row0, j * Wd);
      bstore_stream(dl, p.Delta, S, row0, j * Wd);
      if constexpr (RECOMP) fload(av, p.Abuf, S, row0, (j - 1) * Wd);
    };
    Mat<T> gn;
    zero(gn);
    constexpr int NPREV = (j < K ? 2 * T : T) + (RECOMP ? T : 0);
    if constexpr (HV) {
      stage_mm<X3, TD, T, 0, NPREV, PFA>(z, dl, sg, lane, prev);   // Z += delta_j V_j
      stage_mm<X3, T, T, 0, 0, PFA>(gn, dl, sg, lane, NoOp{});     // delta_j B_j
    } else {
      stage_mm<X3, T, T, 0, NPREV, PFA>(gn, dl, sg, lane, prev);
    }
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gv = gn.v[o][r] + p.rho * g.v[o][r];
        g.v[o][r] = gv;
        dl.v[o][r] = gv * (RECOMP ? act_1<ACT>(av.v[o][r]) : s1[RECOMP ? 0 : j - 1].v[o][r]);
      }
  });
  stage_mm<X3, TD, T, 0, 2 * T + TD, PFA>(z, dl, sg, lane, [&]() __attribute__((always_inline)) {   // Z += delta_0 W_in
    fstore(g, p.G, S, row0, 0);
    bstore_stream(dl, p.Delta, S, row0, 0);
    bload(x, p.xin, p.Dp, row0, 0);
  });
  if (p.u_clamp) {
#pragma unroll
    for (int o = 0; o < TD; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) z.v[o][r] *= umask;
  }
  bstore(z, p.zfull, p.Dp, row0, 0);
  // residual row sums of row cl: [s_zs, s_xz, s_zz, s_x, s_xx, z1]; s_x, s_xx
  // over the leading G state columns (the columns g reads)
  Mat<TD> sd;
  bload(sd, p.sdw, p.Dp, row0, 0);
  const int D = p.D, G = p.gcols;
  float s_zs = 0.f, s_xz = 0.f, s_zz = 0.f, s_x = 0.f, s_xx = 0.f, z1 = 0.f;
#pragma unroll
  for (int o = 0; o < TD; ++o)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 16 * o + 4 * q + r;
      const float zv = z.v[o][r], xv = x.v[o][r];
      if (c >= 1 && c <= D) {
        s_zs += zv * sd.v[o][r];
        s_xz += xv * zv;
        s_zz += zv * zv;
      }
      if (c >= 1 && c <= G) {
        s_x += xv;
        s_xx += xv * xv;
      }
      if (c == 1) z1 = zv;
    }
  float v6[6] = {s_zs, s_xz, s_zz, s_x, s_xx, z1};
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    v6[i] += __shfl_xor(v6[i], 16);
    v6[i] += __shfl_xor(v6[i], 32);
  }
  if (q == 0) {
    float* o = p.rowsum + (size_t)(row0 + cl) * 8;
    *(floatx4*)o = floatx4{v6[0], v6[1], v6[2], v6[3]};
    *(floatx4*)(o + 4) = floatx4{v6[4], v6[5], umask, 0.f};
  }
}

// ---------------------------------------------------------------------------
// phase C: cotangents + forward tangent along zbar + reverse over (primal, tangent)
// stage images (host order): X0, {F_j, [X_j]} j=1..K, B_j j=K..1
// ---------------------------------------------------------------------------
template <int T, int TD, int K, int ACT, bool HV, bool X3>
__global__ void __launch_bounds__(64 * P3_WAVES, 2 * P3_WAVES / 4) phaseC_kernel(FusedArgs p) {
  // prefetch in the tangent / reverse stages (the split-bf16 form is at the
  // register limit without it)
  constexpr bool PFC_T = !X3 || (HV && ACT != ACT_TANH), PFC_R = false;   // tanh: register-bound
  constexpr int TB = T > TD ? T : TD, BUF = X3 ? 3 * TB * 64 : ((TB + 1) / 2) * TB * 64;
  // ONE __shared__ array: with a second LDS object beside the LDS-DMA ring
  // hipcc waits vmcnt(0) before the first ds_read of every piece (the wave's
  // prefetched DMAs drained; cdna_hip_programming.md 5, trap 4(a))
  __shared__ floatx4 wl[(X3 ? P3_NBUF_X3 : 2) * BUF + P3_WAVES / 2];
  double* lsum = (double*)(wl + (X3 ? P3_NBUF_X3 : 2) * BUF);
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = blockIdx.x + p.tile0;   // 64-row tile (chunked launches offset it)
  const int row0 = tile * P3_ROWS + wave * 16;
  const int S = p.S, Wd = p.W;
  PieceStager<X3, T, TD, K, HV, 1> sg{wl, p.simgC, p.snfC, p.nC, 0, wave, lane, BUF};
  sg.start();

  // ---- residuals and closed-form cotangents of row cl (every lane of the row
  // computes them; the zbar columns 16 o + 4 q + r are this lane's)
  const CotanParams& cp = p.cp;
  const int r = row0 + cl;
  RowCotan rc = row_cotan(cp, r);
  if (cp.ext) {   // net_u VJP: the caller's (ubar, zbar), through the u-clamp mask
    rc.ub = rc.valid ? rc.mask * cp.ext_ub[r] : 0.f;
    rc.res = 0.f;
  }
  Mat<TD> zb;
  float tz = 0.f;
  {
    // all 3 TD row loads in flight at once (the branchy zbar formula would
    // otherwise split them into TD dependent memory round trips)
    const size_t off = (size_t)r * p.Dp + 4 * q;
    Mat<TD> xv, zv, sv;
#pragma unroll
    for (int o = 0; o < TD; ++o) {
      xv.v[o] = *(const floatx4*)(cp.xin + off + 16 * o);
      zv.v[o] = *(const floatx4*)(cp.zfull + off + 16 * o);
      sv.v[o] = *(const floatx4*)(cp.sdw + off + 16 * o);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int o = 0; o < TD; ++o)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int c = 16 * o + 4 * q + rr;
        zb.v[o][rr] = (rc.valid && c >= 1 && c <= p.D)
                          ? (cp.ext ? rc.mask * sv.v[o][rr] : col_zbar(cp, rc, c, xv.v[o][rr], zv.v[o][rr], sv.v[o][rr], tz))
                          : 0.f;
      }
  }
  bstore_stream(zb, p.zbar, p.Dp, row0, 0);
  tz += __shfl_xor(tz, 16);
  tz += __shfl_xor(tz, 32);
  {
    // loss of the workgroup's rows, fixed order: rows within the wave, then waves
    double lv = (rc.valid && q == 0) ? (double)(rc.res * rc.res + tz) : 0.0;
#pragma unroll
    for (int s = 1; s < 16; s <<= 1) lv += __shfl_xor(lv, s);
    if (lane == 0) lsum[wave] = lv;
    if (q == 0) {
      p.ubar[r] = rc.ub;
      if (p.u16) p.u16[(size_t)r * 16] = rc.ub;
    }
  }

  Mat<T> ad[K + 1];   // adot_j
  Mat<T> hd, av;
  // X-first (split-bf16 NAIS): the x-stack products zbar V_j^T of every
  // level come first, so zbar is dead before the block stages and the
  // tangent has the registers for the fragment prefetch.  Image order (host):
  // X0, X1..XK, F1..FK, B_K..B1 (else X0, {F_j, X_j}, B_K..B1).
  constexpr bool XFIRST = X3 && HV;
  zero(ad[0]);
  stage_mm<X3, T, TD, TD, T, PFC_T>(ad[0], zb, sg, lane, [&]() __attribute__((always_inline)) {
    fload(av, p.Abuf, S, row0, 0);
    if (threadIdx.x == 0) {   // fixed-order pairwise tree over the waves
      double l[P3_WAVES];
#pragma unroll
      for (int w = 0; w < P3_WAVES; ++w) l[w] = lsum[w];
#pragma unroll
      for (int h = 1; h < P3_WAVES; h <<= 1)
#pragma unroll
        for (int w = 0; w + h < P3_WAVES; w += 2 * h) l[w] += l[w + h];
      p.loss_part[tile] = l[0];
    }
  });
  if constexpr (XFIRST) {
    SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      zero(ad[j]);
      stage_mm<X3, T, TD, 0, 0, PFC_T>(ad[j], zb, sg, lane, NoOp{});
    });
  }
#pragma unroll
  for (int o = 0; o < T; ++o)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) hd.v[o][rr] = act_1<ACT>(av.v[o][rr]) * ad[0].v[o][rr];
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    if constexpr (!XFIRST) zero(ad[j]);
    stage_mm<X3, T, T, 0, 2 * T, PFC_T>(ad[j], hd, sg, lane, [&]() __attribute__((always_inline)) {
      bstore_stream(hd, p.Hdot, S, row0, (j - 1) * Wd);
      fload(av, p.Abuf, S, row0, j * Wd);
    });
    if constexpr (HV && !XFIRST) stage_mm<X3, T, TD, 0, 0, PFC_T>(ad[j], zb, sg, lane, NoOp{});
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) hd.v[o][rr] = act_1<ACT>(av.v[o][rr]) * ad[j].v[o][rr] + p.rho * hd.v[o][rr];
  });
  bstore_stream(hd, p.Hdot, S, row0, K * Wd);
  // reverse: p_{K+1} = ubar w_out ; alpha_K = w_out (ubar act'(a_K) + adot_K act''(a_K))
  Mat<T> pv, al;
  {
    const float ub = rc.ub;
#pragma unroll
    for (int o = 0; o < T; ++o) {
      const floatx4 wo = *(const floatx4*)(p.wout + 16 * o + 4 * q);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float d1, d2;
        act_12<ACT>(av.v[o][rr], d1, d2);
        pv.v[o][rr] = ub * wo[rr];
        al.v[o][rr] = wo[rr] * (ub * d1 + ad[K].v[o][rr] * d2);
      }
    }
  }
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    Mat<T> acc, gg;
    zero(acc);
    stage_mm<X3, T, T, 0, 3 * T, PFC_R>(acc, al, sg, lane, [&]() __attribute__((always_inline)) {   // alpha_j B_j
      bstore_stream(al, p.Alpha, S, row0, j * Wd);
      fload(av, p.Abuf, S, row0, (j - 1) * Wd);
      fload(gg, p.G, S, row0, (j - 1) * Wd);
    });
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float pp = acc.v[o][rr] + p.rho * pv.v[o][rr];
        pv.v[o][rr] = pp;
        float d1, d2;
        act_12<ACT>(av.v[o][rr], d1, d2);
        al.v[o][rr] = pp * d1 + gg.v[o][rr] * ad[j - 1].v[o][rr] * d2;
      }
  });
  bstore_stream(al, p.Alpha, S, row0, 0);
}

}  // namespace dbsde
