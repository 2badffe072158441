// phasecs.hip -- the column-split phase kernels (phasecs.hpp), built as their
// own translation unit.
#include <hip/hip_runtime.h>

// device helpers of kernels.hpp / fused.hpp only: their non-template kernels
// are defined once, in engine.hip
#define DBSDE_DEVICE_HELPERS_ONLY
#include "phasecs.hpp"

namespace dbsde {

namespace {

// this wave's output fragments of a layer: o0 = 2 wave, n = 2 (1 for the last
// wave at width 112).  The piece offset of fragment o0 and of the second one
// (clamped to the first when n = 1: that product is computed and dropped)
struct Own {
  int o0, n, off, f1;
};
template <int T>
__device__ __forceinline__ Own own_of(int wave) {
  const int o0 = 2 * wave, n = T - o0 >= 2 ? 2 : T - o0;
  return Own{o0, n, 3 * o0 * 64, n == 2 ? 3 : 0};
}

// element-wise select of two register values (a select of the references
// would become a dynamically indexed private array, i.e. scratch memory)
__device__ __forceinline__ floatx4 pick(bool c, floatx4 a, floatx4 b) {
  floatx4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = c ? a[i] : b[i];
  return r;
}
// the own fragments of a level, in the layouts of phase.hpp's fstore / fload
// (tile order) and bstore / bstore_stream (row-major); col0 = the level's
// first column + 16 o0.  Branch-free: with one own fragment (n = 1) the
// second access repeats the first (same address, same value), so the wave's
// vector-memory counts stay uniform and no control flow splits the stage.
__device__ __forceinline__ void fstore_n(const Mat<2>& m, float* base, int ld, int row0, int col0, int n) {
  const int lane = threadIdx.x & 63;
  float* p = base + (size_t)row0 * ld + col0 * 16 + 4 * lane;
  *(floatx4*)p = m.v[0];
  *(floatx4*)(p + (n > 1 ? 256 : 0)) = pick(n > 1, m.v[1], m.v[0]);
}
__device__ __forceinline__ void fload_n(Mat<2>& m, const float* base, int ld, int row0, int col0, int n) {
  const int lane = threadIdx.x & 63;
  const float* p = base + (size_t)row0 * ld + col0 * 16 + 4 * lane;
  m.v[0] = *(const floatx4*)p;
  m.v[1] = *(const floatx4*)(p + (n > 1 ? 256 : 0));
}
__device__ __forceinline__ void bstore_stream_n(const Mat<2>& m, float* base, int ld, int row0, int col0, int n) {
  const int lane = threadIdx.x & 63;
  float* p = base + (size_t)(row0 + (lane & 15)) * ld + col0 + 4 * (lane >> 4);
  __builtin_nontemporal_store(m.v[0], (floatx4*)p);
  __builtin_nontemporal_store(pick(n > 1, m.v[1], m.v[0]), (floatx4*)(p + (n > 1 ? 16 : 0)));
}
__device__ __forceinline__ void bstore_n(const Mat<2>& m, float* base, int ld, int row0, int col0, int n) {
  const int lane = threadIdx.x & 63;
  float* p = base + (size_t)(row0 + (lane & 15)) * ld + col0 + 4 * (lane >> 4);
  *(floatx4*)p = m.v[0];
  *(floatx4*)(p + (n > 1 ? 16 : 0)) = pick(n > 1, m.v[1], m.v[0]);
}
__device__ __forceinline__ void bload_n(Mat<2>& m, const float* base, int ld, int row0, int col0, int n) {
  const int lane = threadIdx.x & 63;
  const float* p = base + (size_t)(row0 + (lane & 15)) * ld + col0 + 4 * (lane >> 4);
  m.v[0] = *(const floatx4*)p;
  m.v[1] = *(const floatx4*)(p + (n > 1 ? 16 : 0));
}
// a 16-column vector (w_out, a bias) at the own fragments; zero past n
__device__ __forceinline__ floatx4 vec_at(const float* v, int o, int q, bool ok) {
  const floatx4 x = *(const floatx4*)(v + 16 * (ok ? o : 0) + 4 * q);
  return pick(ok, x, floatx4{0.f, 0.f, 0.f, 0.f});
}

// the layer-input exchange: own fragments in, the whole B-operand tile out.
// DBL (register-streamed weights, no per-piece barrier): two tiles used in
// turn, so a wave that runs a stage ahead never overwrites the tile a slower
// wave has still to read (the next write to a tile is a stage barrier later)
template <int T, bool DBL>
struct XEx {
  floatx4* base;
  int wr;
  const floatx4* rd;
};
template <int T, bool DBL>
__device__ __forceinline__ void xput(const Mat<2>& m, XEx<T, DBL>& x, const Own& w, int lane) {
  floatx4* t = x.base + x.wr * (T * 64);
  t[w.o0 * 64 + lane] = m.v[0];
  t[(w.o0 + (w.n > 1 ? 1 : 0)) * 64 + lane] = pick(w.n > 1, m.v[1], m.v[0]);
  x.rd = t;
  if constexpr (DBL) x.wr ^= 1;
}

// register-streamed weights: each wave loads only its own two fragments of
// each piece straight into registers, two pieces ahead (global_load_dwordx4,
// 1 KiB per fragment chunk, coalesced); no LDS ring, no per-piece barrier --
// the waves meet only at the stage barriers of the activation exchange.
struct WFrag {
  uintx4 w0[3], w1[3];
};
#ifndef DBSDE_CS_DEPTH
#define DBSDE_CS_DEPTH 2
#endif
template <int NP>
struct WStream {
  static constexpr bool kRegs = true;
  static constexpr int DEPTH = DBSDE_CS_DEPTH;   // pieces in flight (2 or 3)
  unsigned long long ptab;   // lane l: piece l's image (lane_ptr)
  int st, off, f1, lane;
  WFrag a, b, c2;
  __device__ __forceinline__ void fetch(WFrag& f, int k) {
    const int kk = k < NP ? k : NP - 1;   // past the end: the last piece again (unused)
    const uintx4* im = (const uintx4*)(lane_ptr(ptab, kk) + off);
#pragma unroll
    for (int p = 0; p < 3; ++p) f.w0[p] = im[p * 64 + lane];
#pragma unroll
    for (int p = 0; p < 3; ++p) f.w1[p] = im[(f1 + p) * 64 + lane];
  }
  __device__ __forceinline__ void init(const float* const* img, const Own& w, int ln) {
    lane = ln;
    st = 0;
    off = 3 * w.o0 * 256;
    f1 = w.f1;
    ptab = lane < NP ? (unsigned long long)img[lane] : 0ull;
    fetch(a, 0);
    fetch(b, 1);
    if constexpr (DEPTH == 3) fetch(c2, 2);
  }
  __device__ __forceinline__ WFrag next() {
    const WFrag c = a;
    a = b;
    if constexpr (DEPTH == 3) {
      b = c2;
      fetch(c2, st + 3);
    } else {
      fetch(b, st + 2);
    }
    ++st;
    return c;
  }
};
// the piece count of a phase (phase.hpp PieceStager's NP)
template <int T, int K, bool HV, int PH>
constexpr int cs_pieces() {
  return ((T + 1) / 2) * (PH == 0 ? 2 + 2 * K * (HV ? 2 : 1) : 1 + K * (HV ? 3 : 2));
}
template <int TT>
__device__ __forceinline__ void xget(Mat<TT>& m, const floatx4* xb, int lane) {
#pragma unroll
  for (int o = 0; o < TT; ++o) m.v[o] = xb[o * 64 + lane];
}

// acc[0..1] += W(own fragments, kb) . b(kb) over one piece: the six
// ds_read_b128 of the two fragments first, then their twelve MFMAs as two
// interleaved chains (each fragment's products in phase.hpp's order, so its
// accumulation is the same), the split of the next input block (all four
// dword pairs) between them
template <int TI, int KBN>
__device__ __forceinline__ void sgemm_cs_piece(Mat<2>& acc, const Split3& s, const floatx4* img, int f1, int lane,
                                               const Mat<TI>& b, uintx4 (&sn)[3]) {
  constexpr bool NEXT = KBN < (TI + 1) / 2;
  const uintx4* im = (const uintx4*)img;
  uintx4 w0[3], w1[3];
#pragma unroll
  for (int p = 0; p < 3; ++p) w0[p] = im[p * 64 + lane];
#pragma unroll
  for (int p = 0; p < 3; ++p) w1[p] = im[(f1 + p) * 64 + lane];
  if constexpr (NEXT) {
    split_pair<TI, NEXT ? KBN : 0, 0>(b, sn[0], sn[1], sn[2]);
    split_pair<TI, NEXT ? KBN : 0, 1>(b, sn[0], sn[1], sn[2]);
    split_pair<TI, NEXT ? KBN : 0, 2>(b, sn[0], sn[1], sn[2]);
    split_pair<TI, NEXT ? KBN : 0, 3>(b, sn[0], sn[1], sn[2]);
  }
  floatx4 a = acc.v[0], c = acc.v[1];
  a = mfma_bf(w0[0], s.l, a);
  c = mfma_bf(w1[0], s.l, c);
  a = mfma_bf(w0[0], s.m, a);
  c = mfma_bf(w1[0], s.m, c);
  a = mfma_bf(w0[1], s.m, a);
  c = mfma_bf(w1[1], s.m, c);
  a = mfma_bf(w0[1], s.h, a);
  c = mfma_bf(w1[1], s.h, c);
  a = mfma_bf(w0[2], s.h, a);
  c = mfma_bf(w1[2], s.h, c);
  acc.v[0] = mfma_bf(w0[0], s.h, a);
  acc.v[1] = mfma_bf(w1[0], s.h, c);
  __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);   // DS read
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // VALU
  }
  __builtin_amdgcn_sched_barrier(0);
}

// the register-streamed piece: as sgemm_cs_piece, operands already in registers
template <int TI, int KBN>
__device__ __forceinline__ void sgemm_cs_regs(Mat<2>& acc, const Split3& s, const WFrag& f, const Mat<TI>& b,
                                              uintx4 (&sn)[3]) {
  constexpr bool NEXT = KBN < (TI + 1) / 2;
  if constexpr (NEXT) {
    split_pair<TI, NEXT ? KBN : 0, 0>(b, sn[0], sn[1], sn[2]);
    split_pair<TI, NEXT ? KBN : 0, 1>(b, sn[0], sn[1], sn[2]);
    split_pair<TI, NEXT ? KBN : 0, 2>(b, sn[0], sn[1], sn[2]);
    split_pair<TI, NEXT ? KBN : 0, 3>(b, sn[0], sn[1], sn[2]);
  }
  floatx4 a = acc.v[0], c = acc.v[1];
  a = mfma_bf(f.w0[0], s.l, a);
  c = mfma_bf(f.w1[0], s.l, c);
  a = mfma_bf(f.w0[0], s.m, a);
  c = mfma_bf(f.w1[0], s.m, c);
  a = mfma_bf(f.w0[1], s.m, a);
  c = mfma_bf(f.w1[1], s.m, c);
  a = mfma_bf(f.w0[1], s.h, a);
  c = mfma_bf(f.w1[1], s.h, c);
  a = mfma_bf(f.w0[2], s.h, a);
  c = mfma_bf(f.w1[2], s.h, c);
  acc.v[0] = mfma_bf(f.w0[0], s.h, a);
  acc.v[1] = mfma_bf(f.w1[0], s.h, c);
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // VALU
  }
  __builtin_amdgcn_sched_barrier(0);
}
template <int TI, int KB, class SG>
__device__ __forceinline__ void stage_csr_from(Mat<2>& acc, const Mat<TI>& b, SG& sg, const Split3& s) {
  constexpr int NKB = (TI + 1) / 2;
  if constexpr (KB < NKB) {
    const WFrag f = sg.next();
    __builtin_amdgcn_sched_barrier(0);   // the next pieces' loads issue before this piece's MFMAs
    uintx4 sn[3];
    sgemm_cs_regs<TI, KB + 1>(acc, s, f, b, sn);
    if constexpr (KB + 1 < NKB)
      stage_csr_from<TI, KB + 1>(
          acc, b, sg,
          Split3{__builtin_bit_cast(bf16x8, sn[0]), __builtin_bit_cast(bf16x8, sn[1]), __builtin_bit_cast(bf16x8, sn[2])});
  }
}

template <int TI, int NPRE, int NAFTER, int KB, class SG>
__device__ __forceinline__ void stage_cs_from(Mat<2>& acc, const Mat<TI>& b, SG& sg, int lane, const Own& w,
                                              const Split3& s) {
  constexpr int NKB = (TI + 1) / 2;
  if constexpr (KB < NKB) {
    const floatx4* wp = sg.template next<piece_nyoung<KB, SG::nbuf - 1, NPRE, NAFTER>()>();
    uintx4 sn[3];
    sgemm_cs_piece<TI, KB + 1>(acc, s, wp + w.off, w.f1, lane, b, sn);
    if constexpr (KB + 1 < NKB)
      stage_cs_from<TI, NPRE, NAFTER, KB + 1>(
          acc, b, sg, lane, w,
          Split3{__builtin_bit_cast(bf16x8, sn[0]), __builtin_bit_cast(bf16x8, sn[1]), __builtin_bit_cast(bf16x8, sn[2])});
  }
}
// one stage: the own output fragments += the stage's image . b, one piece per
// 32-wide input block.  XIN: b is the previous level's exchanged tile, read
// from LDS after the first piece's barrier (which publishes it); `after` runs
// right after that barrier (deferred stores, early loads).  NPRE / NAFTER as
// phase.hpp stage_mm (lower bounds over the four waves).
template <int TI, int NPRE, int NAFTER, bool XIN, class SG, class X, class F>
__device__ __forceinline__ void stage_cs(Mat<2>& acc, Mat<TI>& b, SG& sg, int lane, const Own& w, const X& xb,
                                         F&& after) {
  constexpr int NKB = (TI + 1) / 2;
  if constexpr (SG::kRegs) {
    if constexpr (XIN) {
      lds_barrier();   // publishes the exchange tile (and keeps every vector-memory op in flight)
      xget(b, xb.rd, lane);
    }
    after();
    __builtin_amdgcn_sched_barrier(0);
    stage_csr_from<TI, 0>(acc, b, sg, split_block<TI, 0>(b));
  } else {
    const floatx4* wp = sg.template next<piece_nyoung<0, SG::nbuf - 1, NPRE, NAFTER>()>();
    if constexpr (XIN) xget(b, xb.rd, lane);
    after();
    __builtin_amdgcn_sched_barrier(0);
    const Split3 s = split_block<TI, 0>(b);
    uintx4 sn[3];
    sgemm_cs_piece<TI, 1>(acc, s, wp + w.off, w.f1, lane, b, sn);
    if constexpr (NKB > 1)
      stage_cs_from<TI, NPRE, NAFTER, 1>(
          acc, b, sg, lane, w,
          Split3{__builtin_bit_cast(bf16x8, sn[0]), __builtin_bit_cast(bf16x8, sn[1]), __builtin_bit_cast(bf16x8, sn[2])});
  }
}

#ifndef DBSDE_CS_REG
#define DBSDE_CS_REG 1
#endif
// the weight feed of a phase: register-streamed (DBSDE_CS_REG=1) or the
// 64-row kernels' LDS-DMA ring shared by the four waves
template <bool REG, int T, int TD, int K, bool HV, int PH>
struct FeedOf {
  using type = PieceStager<true, T, TD, K, HV, PH>;
};
template <int T, int TD, int K, bool HV, int PH>
struct FeedOf<true, T, TD, K, HV, PH> {
  using type = WStream<cs_pieces<T, K, HV, PH>()>;
};

}  // namespace

// ---------------------------------------------------------------------------
// phase A, column split: forward + input gradient + Z + residual row sums of
// one 16-row tile (phase.hpp phaseA_kernel, same images and outputs)
// ---------------------------------------------------------------------------
template <int T, int TD, int K, int ACT, bool HV>
__global__ void __launch_bounds__(64 * P3_WAVES, 2) phaseAcs_kernel(FusedArgs p) {
  static_assert(T == TD && T == 7, "column-split kernels: width-112 levels");
  constexpr bool REG = DBSDE_CS_REG != 0;
  constexpr int BUF = 3 * T * 64, RING = REG ? 0 : P3_NBUF_X3 * BUF, NX = REG ? 2 : 1;
  // ONE __shared__ array (phase.hpp phaseC_kernel): the weight ring (LDS
  // feed), the exchange tile(s), the cross-wave sums [4 waves][16 rows][8]
  __shared__ floatx4 wl[RING + NX * T * 64 + P3_WAVES * 16 * 8 / 4];
  XEx<T, REG> xb{wl + RING, 0, wl + RING};
  float* red = (float*)(wl + RING + NX * T * 64);
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Own w = own_of<T>(wave);
  const int tile = blockIdx.x + p.tile0;
  const int row0 = tile * CS_ROWS;
  const int S = p.S, Wd = p.W, c0 = 16 * w.o0;
  typename FeedOf<REG, T, TD, K, HV, 0>::type sg;
  if constexpr (REG) {
    sg.init(p.simgA, w, lane);
  } else {
    sg = {wl, p.simgA, p.snfA, p.nA, 0, wave, lane, BUF};
    sg.start();
  }
  Mat<TD> x;
  bload(x, p.xin, p.Dp, row0, 0);

  Mat<2> s1[K + 1];   // act'(a_j), own fragments
  Mat<2> acc, ho;     // a_j / h_j, own fragments
  Mat<T> hf;          // h_j, the whole tile (exchange)
  zero(acc);
  stage_cs<TD, TD, 0, false>(acc, x, sg, lane, w, xb, NoOp{});
  fstore_n(acc, p.Abuf, S, row0, c0, w.n);
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float f, d;
      act_v1<ACT>(acc.v[o][r], f, d);
      ho.v[o][r] = f;
      s1[0].v[o][r] = d;
    }
  xput(ho, xb, w, lane);
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    zero(acc);
    stage_cs<T, 1, 1, true>(acc, hf, sg, lane, w, xb, [&]() __attribute__((always_inline)) {
      bstore_stream_n(ho, p.H, S, row0, (j - 1) * Wd + c0, w.n);
    });
    if constexpr (HV) stage_cs<TD, 0, 0, false>(acc, x, sg, lane, w, xb, NoOp{});
    if constexpr (!HV) {
#pragma unroll
      for (int o = 0; o < 2; ++o) {
        const floatx4 bb = vec_at(p.beta[j - 1], w.o0 + o, q, o < w.n);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc.v[o][r] += bb[r];
      }
    }
    fstore_n(acc, p.Abuf, S, row0, j * Wd + c0, w.n);
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float f, d;
        act_v1<ACT>(acc.v[o][r], f, d);
        s1[j].v[o][r] = d;
        ho.v[o][r] = f + p.rho * ho.v[o][r];
      }
    if constexpr (j < K) xput(ho, xb, w, lane);
  });
  // u = h_{K+1} . w_out + b_out: the waves' partial dots, summed in wave order
  float umask = 1.f;
  {
    float us = 0.f;
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      const floatx4 wo = vec_at(p.wout, w.o0 + o, q, o < w.n);
#pragma unroll
      for (int r = 0; r < 4; ++r) us += ho.v[o][r] * wo[r];
    }
    us += __shfl_xor(us, 16);
    us += __shfl_xor(us, 32);
    if (q == 0) red[wave * 16 + cl] = us;
    lds_barrier();
    float uv = ((red[cl] + red[16 + cl]) + (red[32 + cl] + red[48 + cl])) + p.bout[0];
    if (p.u_clamp) {
      umask = uv >= 0.f ? 1.f : 0.f;
      uv = uv >= 0.f ? uv : 0.f;
    }
    if (wave == 0 && q == 0) p.u[row0 + cl] = uv;
  }
  bstore_stream_n(ho, p.H, S, row0, K * Wd + c0, w.n);
  // input gradient: g_{K+1} = w_out, delta_K = w_out act'(a_K)
  Mat<2> g, dl;
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const floatx4 wo = vec_at(p.wout, w.o0 + o, q, o < w.n);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      g.v[o][r] = wo[r];
      dl.v[o][r] = wo[r] * s1[K].v[o][r];
    }
  }
  xput(dl, xb, w, lane);
  Mat<2> z;
  zero(z);
  Mat<T> df;   // delta_j, the whole tile
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    auto prev = [&]() __attribute__((always_inline)) {   // (g_j, delta_j) of the previous step
      if constexpr (j < K) fstore_n(g, p.G, S, row0, j * Wd + c0, w.n);
      bstore_stream_n(dl, p.Delta, S, row0, j * Wd + c0, w.n);
    };
    Mat<2> gn;
    zero(gn);
    constexpr int NPREV = j < K ? 2 : 1;
    if constexpr (HV) {
      stage_cs<T, 0, NPREV, true>(z, df, sg, lane, w, xb, prev);       // Z += delta_j V_j
      stage_cs<T, 0, 0, false>(gn, df, sg, lane, w, xb, NoOp{});       // delta_j B_j
    } else {
      stage_cs<T, 0, NPREV, true>(gn, df, sg, lane, w, xb, prev);
    }
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gv = gn.v[o][r] + p.rho * g.v[o][r];
        g.v[o][r] = gv;
        dl.v[o][r] = gv * s1[j - 1].v[o][r];
      }
    xput(dl, xb, w, lane);
  });
  stage_cs<T, 0, 2, true>(z, df, sg, lane, w, xb, [&]() __attribute__((always_inline)) {   // Z += delta_0 W_in
    fstore_n(g, p.G, S, row0, c0, w.n);
    bstore_stream_n(dl, p.Delta, S, row0, c0, w.n);
  });
  if (p.u_clamp) {
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) z.v[o][r] *= umask;
  }
  bstore_n(z, p.zfull, p.Dp, row0, c0, w.n);
  // residual row sums of row cl over the own columns, then over the waves in
  // order: [s_zs, s_xz, s_zz, s_x, s_xx, z1]
  Mat<2> xo, sd;
  bload_n(xo, p.xin, p.Dp, row0, c0, w.n);
  bload_n(sd, p.sdw, p.Dp, row0, c0, w.n);
  const int D = p.D, G = p.gcols;
  float v6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = c0 + 16 * o + 4 * q + r;
      const bool in = o < w.n;
      const float zv = z.v[o][r], xv = xo.v[o][r];
      if (in && c >= 1 && c <= D) {
        v6[0] += zv * sd.v[o][r];
        v6[1] += xv * zv;
        v6[2] += zv * zv;
      }
      if (in && c >= 1 && c <= G) {
        v6[3] += xv;
        v6[4] += xv * xv;
      }
      if (c == 1) v6[5] = zv;
    }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    v6[i] += __shfl_xor(v6[i], 16);
    v6[i] += __shfl_xor(v6[i], 32);
  }
  float* rw = red + P3_WAVES * 16;   // past the u partials (read before the Z stages' barriers)
  if (q == 0) {
#pragma unroll
    for (int i = 0; i < 6; ++i) rw[(wave * 16 + cl) * 6 + i] = v6[i];
  }
  lds_barrier();
  if (wave == 0 && q == 0) {
    float t[6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
      t[i] = (rw[cl * 6 + i] + rw[(16 + cl) * 6 + i]) + (rw[(32 + cl) * 6 + i] + rw[(48 + cl) * 6 + i]);
    float* o = p.rowsum + (size_t)(row0 + cl) * 8;
    *(floatx4*)o = floatx4{t[0], t[1], t[2], t[3]};
    *(floatx4*)(o + 4) = floatx4{t[4], t[5], umask, 0.f};
  }
}

// ---------------------------------------------------------------------------
// phase C, column split: cotangents + forward tangent along zbar + reverse of
// one 16-row tile (phase.hpp phaseC_kernel, same images and outputs)
// ---------------------------------------------------------------------------
template <int T, int TD, int K, int ACT, bool HV>
__global__ void __launch_bounds__(64 * P3_WAVES, 2) phaseCcs_kernel(FusedArgs p) {
  static_assert(T == TD && T == 7, "column-split kernels: width-112 levels");
  constexpr bool REG = DBSDE_CS_REG != 0;
  constexpr int BUF = 3 * T * 64, RING = REG ? 0 : P3_NBUF_X3 * BUF, NX = REG ? 2 : 1;
  __shared__ floatx4 wl[RING + NX * T * 64];
  XEx<T, REG> xb{wl + RING, 0, wl + RING};
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Own w = own_of<T>(wave);
  const int tile = blockIdx.x + p.tile0;
  const int row0 = tile * CS_ROWS;
  const int S = p.S, Wd = p.W, c0 = 16 * w.o0;
  typename FeedOf<REG, T, TD, K, HV, 1>::type sg;
  if constexpr (REG) {
    sg.init(p.simgC, w, lane);
  } else {
    sg = {wl, p.simgC, p.snfC, p.nC, 0, wave, lane, BUF};
    sg.start();
  }

  // residuals and cotangents of row cl (every wave: the whole zbar tile is
  // the x-stack stages' input)
  const CotanParams& cp = p.cp;
  const int r = row0 + cl;
  RowCotan rc = row_cotan(cp, r);
  if (cp.ext) {
    rc.ub = rc.valid ? rc.mask * cp.ext_ub[r] : 0.f;
    rc.res = 0.f;
  }
  Mat<TD> zb;
  float tz = 0.f;
  {
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
  tz += __shfl_xor(tz, 16);
  tz += __shfl_xor(tz, 32);
  if (wave == 0) {
    bstore_stream(zb, p.zbar, p.Dp, row0, 0);
    double lv = (rc.valid && q == 0) ? (double)(rc.res * rc.res + tz) : 0.0;
#pragma unroll
    for (int s = 1; s < 16; s <<= 1) lv += __shfl_xor(lv, s);
    if (lane == 0) p.loss_part[tile] = lv;
    if (q == 0) {
      p.ubar[r] = rc.ub;
      if (p.u16) p.u16[(size_t)r * 16] = rc.ub;
    }
  }

  Mat<2> ad[K + 1];   // adot_j, own fragments
  Mat<2> hdo, avo;    // hdot_j, a_j (own)
  Mat<T> hf;          // hdot_j, the whole tile
  constexpr bool XFIRST = HV;   // image order X0, X1..XK, F1..FK, B_K..B1 (phase.hpp)
  zero(ad[0]);
  stage_cs<TD, 0, 1, false>(ad[0], zb, sg, lane, w, xb, [&]() __attribute__((always_inline)) {
    fload_n(avo, p.Abuf, S, row0, c0, w.n);
  });
  if constexpr (XFIRST) {
    SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      zero(ad[j]);
      stage_cs<TD, 0, 0, false>(ad[j], zb, sg, lane, w, xb, NoOp{});
    });
  }
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) hdo.v[o][rr] = act_1<ACT>(avo.v[o][rr]) * ad[0].v[o][rr];
  xput(hdo, xb, w, lane);
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    if constexpr (!XFIRST) zero(ad[j]);
    stage_cs<T, 0, 2, true>(ad[j], hf, sg, lane, w, xb, [&]() __attribute__((always_inline)) {
      bstore_stream_n(hdo, p.Hdot, S, row0, (j - 1) * Wd + c0, w.n);
      fload_n(avo, p.Abuf, S, row0, j * Wd + c0, w.n);
    });
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) hdo.v[o][rr] = act_1<ACT>(avo.v[o][rr]) * ad[j].v[o][rr] + p.rho * hdo.v[o][rr];
    if constexpr (j < K) xput(hdo, xb, w, lane);
  });
  bstore_stream_n(hdo, p.Hdot, S, row0, K * Wd + c0, w.n);
  // reverse: p_{K+1} = ubar w_out ; alpha_K = w_out (ubar act'(a_K) + adot_K act''(a_K))
  Mat<2> pv, al;
  {
    const float ub = rc.ub;
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      const floatx4 wo = vec_at(p.wout, w.o0 + o, q, o < w.n);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float d1, d2;
        act_12<ACT>(avo.v[o][rr], d1, d2);
        pv.v[o][rr] = ub * wo[rr];
        al.v[o][rr] = wo[rr] * (ub * d1 + ad[K].v[o][rr] * d2);
      }
    }
  }
  xput(al, xb, w, lane);
  Mat<T> af;   // alpha_j, the whole tile
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    Mat<2> acc, gg;
    zero(acc);
    stage_cs<T, 0, 3, true>(acc, af, sg, lane, w, xb, [&]() __attribute__((always_inline)) {   // alpha_j B_j
      bstore_stream_n(al, p.Alpha, S, row0, j * Wd + c0, w.n);
      fload_n(avo, p.Abuf, S, row0, (j - 1) * Wd + c0, w.n);
      fload_n(gg, p.G, S, row0, (j - 1) * Wd + c0, w.n);
    });
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float pp = acc.v[o][rr] + p.rho * pv.v[o][rr];
        pv.v[o][rr] = pp;
        float d1, d2;
        act_12<ACT>(avo.v[o][rr], d1, d2);
        al.v[o][rr] = pp * d1 + gg.v[o][rr] * ad[j - 1].v[o][rr] * d2;
      }
    if constexpr (j > 1) xput(al, xb, w, lane);
  });
  bstore_stream_n(al, p.Alpha, S, row0, c0, w.n);
}

#define DBSDE_PHASECS_DEFINE(T, TD, K, ACT, HV)                           \
  template __global__ void phaseAcs_kernel<T, TD, K, ACT, HV>(FusedArgs); \
  template __global__ void phaseCcs_kernel<T, TD, K, ACT, HV>(FusedArgs);
DBSDE_PHASECS_INSTANCES(DBSDE_PHASECS_DEFINE)
#undef DBSDE_PHASECS_DEFINE

}  // namespace dbsde
