// phase2.hip -- the two-tile fused phase kernels (phase2.hpp), built as their
// own translation unit.
#include <hip/hip_runtime.h>

// device helpers of kernels.hpp / fused.hpp only: their non-template kernels
// are defined once, in engine.hip
#define DBSDE_DEVICE_HELPERS_ONLY
#include "phase2.hpp"

// fragment pairs in the one-tile kernels: bit 0 phase A, bit 1 phase C
#ifndef DBSDE_P2_PAIRS
#define DBSDE_P2_PAIRS 3
#endif

namespace dbsde {

// stager: split-bf16 pieces; T == TD: every piece 3 T fragments (compile-time
// piece count and a per-lane pointer table), else the runtime piece tables
template <int T, int TD, int K, bool HV, int PH, int NBUF>
using PieceStager2 = PieceStagerT<NBUF, (3 * (T < TD ? T : TD)) / P3_WAVES, T == TD ? 3 * T : 0,
                                  T == TD ? ((T + 1) / 2) * (PH == 0 ? 2 + 2 * K * (HV ? 2 : 1) : 1 + K * (HV ? 3 : 2))
                                          : 0>;

// acc[t][o] += W(o, kb) . b[t](kb) over one piece for the NT tiles: per
// fragment o the next fragment's three ds_read_b128 first, then the 6 NT
// MFMAs, with the split of the next input block of every tile (KBN; one dword
// pair per tile per fragment, o < 4) interleaved two VALU per MFMA gap.
template <int TO, int TI, int KBN, int NT>
__device__ __forceinline__ void sgemm_x3_piece_nt(Mat<TO> (&acc)[NT], const Split3 (&s)[NT], const floatx4* img,
                                                  int lane, const Mat<TI> (&b)[NT], uintx4 (&sn)[NT][3]) {
  constexpr bool NEXT = KBN < (TI + 1) / 2;
  const uintx4* im = (const uintx4*)img;
  uintx4 w[2][3];
#pragma unroll
  for (int p = 0; p < 3; ++p) w[0][p] = im[p * 64 + lane];
  __builtin_amdgcn_sched_barrier(0);
  SFor<0, TO>::run([&](auto oc) __attribute__((always_inline)) {
    constexpr int o = decltype(oc)::value;
    if constexpr (o + 1 < TO) {
#pragma unroll
      for (int p = 0; p < 3; ++p) w[(o + 1) & 1][p] = im[(3 * (o + 1) + p) * 64 + lane];
    }
    if constexpr (NEXT && o < 4) {
#pragma unroll
      for (int t = 0; t < NT; ++t) split_pair<TI, NEXT ? KBN : 0, o>(b[t], sn[t][0], sn[t][1], sn[t][2]);
    }
    const uintx4* wc = w[o & 1];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      floatx4 a = acc[t].v[o];
      a = mfma_bf(wc[0], s[t].l, a);
      a = mfma_bf(wc[0], s[t].m, a);
      a = mfma_bf(wc[1], s[t].m, a);
      a = mfma_bf(wc[1], s[t].h, a);
      a = mfma_bf(wc[2], s[t].h, a);
      acc[t].v[o] = mfma_bf(wc[0], s[t].h, a);
    }
    if constexpr (o + 1 < TO) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);   // DS read
#pragma unroll
    for (int k = 0; k < 6 * NT; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // VALU
    }
    __builtin_amdgcn_sched_barrier(0);
  });
}

template <int TO, int TI, int NPRE, int NAFTER, int KB, int NT, bool PR, class SG, class F>
__device__ __forceinline__ void stage_nt_from(Mat<TO> (&acc)[NT], const Mat<TI> (&b)[NT], SG& sg, int lane, F&& after,
                                              const Split3 (&s)[NT]) {
  constexpr int NKB = (TI + 1) / 2;
  if constexpr (KB < NKB) {
    const floatx4* w = sg.template next<piece_nyoung<KB, SG::nbuf - 1, NPRE, NAFTER>()>();
    if constexpr (KB == 0) {
      after();
      __builtin_amdgcn_sched_barrier(0);
    }
    uintx4 sn[NT][3];
    if constexpr (PR && NT == 1)
      sgemm_x3_piece_pairs<TO, TI, KB + 1>(acc[0], s[0], w, lane, b[0], sn[0]);
    else
      sgemm_x3_piece_nt<TO, TI, KB + 1, NT>(acc, s, w, lane, b, sn);
    if constexpr (KB + 1 < NKB) {
      Split3 s2[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        s2[t] = Split3{__builtin_bit_cast(bf16x8, sn[t][0]), __builtin_bit_cast(bf16x8, sn[t][1]),
                       __builtin_bit_cast(bf16x8, sn[t][2])};
      stage_nt_from<TO, TI, NPRE, NAFTER, KB + 1, NT, PR>(acc, b, sg, lane, after, s2);
    }
  }
}
// one stage = one operand image, one piece per 32-wide input block; `after`
// runs right after the first piece's barrier.  NPRE / NAFTER as stage_mm.
//   PR: one tile per wave (one wave per SIMD) -- the fragments in pairs, two
//   interleaved MFMA chains (sgemm_x3_piece_pairs): a lone wave cannot hide
//   the dependent issue of one chain (tools/ubench/piece_x3.hip: 59 -> 76 %)
template <int TO, int TI, int NPRE, int NAFTER, int NT, bool PR = false, class SG, class F>
__device__ __forceinline__ void stage_nt(Mat<TO> (&acc)[NT], const Mat<TI> (&b)[NT], SG& sg, int lane, F&& after) {
  Split3 s[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) s[t] = split_block<TI, 0>(b[t]);
  stage_nt_from<TO, TI, NPRE, NAFTER, 0, NT, PR>(acc, b, sg, lane, after, s);
}

template <int NT, int TT>
__device__ __forceinline__ void zero_nt(Mat<TT> (&m)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) zero(m[t]);
}

// ---------------------------------------------------------------------------
// phase A, two tiles per wave: forward + input gradient + Z (+ residual row
// sums).  Stage images as phaseA_kernel.
// ---------------------------------------------------------------------------
template <int T, int TD, int K, int ACT, bool HV, int NT, int NBUF, bool ADOT>
__global__ void __launch_bounds__(64 * P3_WAVES, 1) phaseA2_kernel(FusedArgs p) {
  constexpr int TB = T > TD ? T : TD, BUF = 3 * TB * 64, ROWS = 16 * NT * P3_WAVES;
  constexpr bool PRA = NT == 1 && (DBSDE_P2_PAIRS & 1);
  __shared__ floatx4 wl[NBUF * BUF];
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = blockIdx.x + p.tile0;   // ROWS-row tile (chunked launches offset it)
  const int row0 = tile * ROWS + wave * 16 * NT;   // register tile t: rows row0 + 16 t ..
  const int S = p.S, Wd = p.W;
  PieceStager2<T, TD, K, HV, 0, NBUF> sg{wl, p.simgA, p.snfA, p.nA, 0, wave, lane, BUF};
  sg.start();
  Mat<TD> x[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bload(x[t], p.xin, p.Dp, row0 + 16 * t, 0);

  Mat<T> h[NT], acc[NT];
  zero_nt(acc);
  stage_nt<T, TD, NT * TD, 0, NT, PRA>(acc, x, sg, lane, NoOp{});
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    fstore(acc[t], p.Abuf, S, row0 + 16 * t, 0);
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float f, d;
        act_v1<ACT>(acc[t].v[o][r], f, d);
        h[t].v[o][r] = f;
      }
  }
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    zero_nt(acc);
    stage_nt<T, T, NT * T, NT * T, NT, PRA>(acc, h, sg, lane, [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int t = 0; t < NT; ++t) bstore_stream(h[t], p.H, S, row0 + 16 * t, (j - 1) * Wd);
    });
    if constexpr (HV) stage_nt<T, TD, 0, 0, NT, PRA>(acc, x, sg, lane, NoOp{});
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr (!HV) {
#pragma unroll
        for (int o = 0; o < T; ++o) {
          const floatx4 bb = *(const floatx4*)(p.beta[j - 1] + 16 * o + 4 * q);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[t].v[o][r] += bb[r];
        }
      }
      fstore(acc[t], p.Abuf, S, row0 + 16 * t, j * Wd);
#pragma unroll
      for (int o = 0; o < T; ++o)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float f, d;
          act_v1<ACT>(acc[t].v[o][r], f, d);
          h[t].v[o][r] = f + p.rho * h[t].v[o][r];
        }
    }
  });
  // u = h_{K+1} . w_out + b_out (clamped at 0 for Heston, heston_dnnpde.py:568)
  float umask[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float us = 0.f;
#pragma unroll
    for (int o = 0; o < T; ++o) {
      const floatx4 wo = *(const floatx4*)(p.wout + 16 * o + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) us += h[t].v[o][r] * wo[r];
    }
    us += __shfl_xor(us, 16);
    us += __shfl_xor(us, 32);
    float uv = us + p.bout[0];
    umask[t] = 1.f;
    if (p.u_clamp) {
      umask[t] = uv >= 0.f ? 1.f : 0.f;
      uv = uv >= 0.f ? uv : 0.f;
    }
    if (q == 0) p.u[row0 + 16 * t + cl] = uv;
    bstore_stream(h[t], p.H, S, row0 + 16 * t, K * Wd);
  }
  // input gradient: g_{K+1} = w_out, delta_K = w_out act'(a_K) (acc still holds a_K)
  Mat<T> g[NT], dl[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int o = 0; o < T; ++o) {
      const floatx4 wo = *(const floatx4*)(p.wout + 16 * o + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        g[t].v[o][r] = wo[r];
        dl[t].v[o][r] = wo[r] * act_1<ACT>(acc[t].v[o][r]);
      }
    }
  Mat<TD> z[NT];
  zero_nt(z);
  Mat<T> av[NT];   // a_{j-1}, reloaded from Abuf for act'(a_{j-1})
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    auto prev = [&]() __attribute__((always_inline)) {   // (g_j, delta_j) of the previous step; a_{j-1}
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if constexpr (j < K) fstore(g[t], p.G, S, row0 + 16 * t, j * Wd);
        bstore_stream(dl[t], p.Delta, S, row0 + 16 * t, j * Wd);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) fload(av[t], p.Abuf, S, row0 + 16 * t, (j - 1) * Wd);
    };
    Mat<T> gn[NT];
    zero_nt(gn);
    constexpr int NPREV = NT * ((j < K ? 2 * T : T) + T);
    if constexpr (HV) {
      stage_nt<TD, T, 0, NPREV, NT, PRA>(z, dl, sg, lane, prev);   // Z += delta_j V_j
      stage_nt<T, T, 0, 0, NT, PRA>(gn, dl, sg, lane, NoOp{});     // delta_j B_j
    } else {
      stage_nt<T, T, 0, NPREV, NT, PRA>(gn, dl, sg, lane, prev);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int o = 0; o < T; ++o)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gv = gn[t].v[o][r] + p.rho * g[t].v[o][r];
          g[t].v[o][r] = gv;
          dl[t].v[o][r] = gv * act_1<ACT>(av[t].v[o][r]);
        }
  });
  stage_nt<TD, T, 0, NT * (2 * T + TD), NT, PRA>(z, dl, sg, lane, [&]() __attribute__((always_inline)) {   // Z += delta_0 W_in
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      fstore(g[t], p.G, S, row0 + 16 * t, 0);
      bstore_stream(dl[t], p.Delta, S, row0 + 16 * t, 0);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) bload(x[t], p.xin, p.Dp, row0 + 16 * t, 0);
  });
  const int D = p.D, G = p.gcols;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (p.u_clamp) {
#pragma unroll
      for (int o = 0; o < TD; ++o)
#pragma unroll
        for (int r = 0; r < 4; ++r) z[t].v[o][r] *= umask[t];
    }
    const int rt = row0 + 16 * t;
    bstore(z[t], p.zfull, p.Dp, rt, 0);
    // residual row sums of row cl: [s_zs, s_xz, s_zz, s_x, s_xx, z1]; s_x, s_xx
    // over the leading G state columns (the columns g reads)
    Mat<TD> sd;
    bload(sd, p.sdw, p.Dp, rt, 0);
    float s_zs = 0.f, s_xz = 0.f, s_zz = 0.f, s_x = 0.f, s_xx = 0.f, z1 = 0.f;
#pragma unroll
    for (int o = 0; o < TD; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * o + 4 * q + r;
        const float zv = z[t].v[o][r], xv = x[t].v[o][r];
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
      float* o = p.rowsum + (size_t)(rt + cl) * 8;
      *(floatx4*)o = floatx4{v6[0], v6[1], v6[2], v6[3]};
      *(floatx4*)(o + 4) = floatx4{v6[4], v6[5], umask[t], 0.f};
    }
  }
}

// ---------------------------------------------------------------------------
// phase C, two tiles per wave: cotangents + forward tangent along zbar +
// reverse over (primal, tangent).  Stage images as phaseC_kernel (X-first
// order for the x-stack networks).
// ---------------------------------------------------------------------------
template <int T, int TD, int K, int ACT, bool HV, int NT, int NBUF, bool ADOT>
__global__ void __launch_bounds__(64 * P3_WAVES, 1) phaseC2_kernel(FusedArgs p) {
  constexpr int TB = T > TD ? T : TD, BUF = 3 * TB * 64, ROWS = 16 * NT * P3_WAVES;
  constexpr bool PRC = NT == 1 && (DBSDE_P2_PAIRS & 2) && ACT != ACT_TANH;   // tanh: spills with pairs
  // one __shared__ array (the loss slots after the ring): see phaseC_kernel
  __shared__ floatx4 wl[NBUF * BUF + P3_WAVES / 2];
  double* lsum = (double*)(wl + NBUF * BUF);
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = blockIdx.x + p.tile0;
  const int row0 = tile * ROWS + wave * 16 * NT;
  const int S = p.S, Wd = p.W;
  PieceStager2<T, TD, K, HV, 1, NBUF> sg{wl, p.simgC, p.snfC, p.nC, 0, wave, lane, BUF};
  sg.start();

  // ---- residuals and closed-form cotangents of rows (row0 + 16 t + cl)
  const CotanParams& cp = p.cp;
  RowCotan rc[NT];
  Mat<TD> zb[NT];
  double lv = 0.0;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int r = row0 + 16 * t + cl;
    rc[t] = row_cotan(cp, r);
    if (cp.ext) {   // net_u VJP: the caller's (ubar, zbar), through the u-clamp mask
      rc[t].ub = rc[t].valid ? rc[t].mask * cp.ext_ub[r] : 0.f;
      rc[t].res = 0.f;
    }
    float tz = 0.f;
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
        zb[t].v[o][rr] = (rc[t].valid && c >= 1 && c <= p.D)
                             ? (cp.ext ? rc[t].mask * sv.v[o][rr]
                                       : col_zbar(cp, rc[t], c, xv.v[o][rr], zv.v[o][rr], sv.v[o][rr], tz))
                             : 0.f;
      }
    bstore_stream(zb[t], p.zbar, p.Dp, row0 + 16 * t, 0);
    tz += __shfl_xor(tz, 16);
    tz += __shfl_xor(tz, 32);
    // loss of the rows, fixed order: rows within a tile, tiles, then waves
    double lt = (rc[t].valid && q == 0) ? (double)(rc[t].res * rc[t].res + tz) : 0.0;
#pragma unroll
    for (int s = 1; s < 16; s <<= 1) lt += __shfl_xor(lt, s);
    lv += lt;
    if (q == 0) {
      p.ubar[r] = rc[t].ub;
      if (p.u16) p.u16[(size_t)r * 16] = rc[t].ub;
    }
  }
  if (lane == 0) lsum[wave] = lv;

  // adot_j: all levels in registers, or (ADOT) the current level only, with
  // every level stored to Adot for the reverse
  constexpr int NAD = ADOT ? 1 : K + 1;
  Mat<T> ad[NAD][NT];
  Mat<T> hd[NT], av[NT];
  constexpr bool XFIRST = HV && !ADOT;
  zero_nt(ad[0]);
  stage_nt<T, TD, NT * TD, NT * T, NT, PRC>(ad[0], zb, sg, lane, [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < NT; ++t) fload(av[t], p.Abuf, S, row0 + 16 * t, 0);
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
      zero_nt(ad[j]);
      stage_nt<T, TD, 0, 0, NT, PRC>(ad[j], zb, sg, lane, NoOp{});
    });
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) hd[t].v[o][rr] = act_1<ACT>(av[t].v[o][rr]) * ad[0][t].v[o][rr];
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    constexpr int ja = ADOT ? 0 : j;
    if constexpr (ADOT) {
      // this level's accumulators reuse the registers of the previous one
#pragma unroll
      for (int t = 0; t < NT; ++t) fstore(ad[0][t], p.Adot, S, row0 + 16 * t, (j - 1) * Wd);
    }
    if constexpr (!XFIRST) zero_nt(ad[ja]);
    constexpr int NAF = 2 * NT * T;   // (ADOT: the Adot stores are older, not counted)
    stage_nt<T, T, 0, NAF, NT, PRC>(ad[ja], hd, sg, lane, [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int t = 0; t < NT; ++t) bstore_stream(hd[t], p.Hdot, S, row0 + 16 * t, (j - 1) * Wd);
#pragma unroll
      for (int t = 0; t < NT; ++t) fload(av[t], p.Abuf, S, row0 + 16 * t, j * Wd);
    });
    if constexpr (HV && !XFIRST) stage_nt<T, TD, 0, 0, NT, PRC>(ad[ja], zb, sg, lane, NoOp{});
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int o = 0; o < T; ++o)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          hd[t].v[o][rr] = act_1<ACT>(av[t].v[o][rr]) * ad[ja][t].v[o][rr] + p.rho * hd[t].v[o][rr];
  });
  constexpr int jK = ADOT ? 0 : K;   // ad[jK] = adot_K
  // reverse: p_{K+1} = ubar w_out ; alpha_K = w_out (ubar act'(a_K) + adot_K act''(a_K))
  Mat<T> pv[NT], al[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bstore_stream(hd[t], p.Hdot, S, row0 + 16 * t, K * Wd);
    const float ub = rc[t].ub;
#pragma unroll
    for (int o = 0; o < T; ++o) {
      const floatx4 wo = *(const floatx4*)(p.wout + 16 * o + 4 * q);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float d1, d2;
        act_12<ACT>(av[t].v[o][rr], d1, d2);
        pv[t].v[o][rr] = ub * wo[rr];
        al[t].v[o][rr] = wo[rr] * (ub * d1 + ad[jK][t].v[o][rr] * d2);
      }
    }
  }
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    Mat<T> gg[NT];
    Mat<T> adr[ADOT ? NT : 1];   // ADOT: adot_{j-1} reloaded
    // p_j = rho p_{j+1} + alpha_j B_j, accumulated in place (rho is 0 or 1)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int o = 0; o < T; ++o)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) pv[t].v[o][rr] *= p.rho;
    constexpr int NAF = (ADOT ? 4 : 3) * NT * T;
    stage_nt<T, T, 0, NAF, NT, PRC>(pv, al, sg, lane, [&]() __attribute__((always_inline)) {   // alpha_j B_j
#pragma unroll
      for (int t = 0; t < NT; ++t) bstore_stream(al[t], p.Alpha, S, row0 + 16 * t, j * Wd);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        fload(av[t], p.Abuf, S, row0 + 16 * t, (j - 1) * Wd);
        fload(gg[t], p.G, S, row0 + 16 * t, (j - 1) * Wd);
        if constexpr (ADOT) fload(adr[t], p.Adot, S, row0 + 16 * t, (j - 1) * Wd);
      }
    });
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int o = 0; o < T; ++o)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          float d1, d2;
          act_12<ACT>(av[t].v[o][rr], d1, d2);
          const float a1 = ADOT ? adr[ADOT ? t : 0].v[o][rr] : ad[ADOT ? 0 : j - 1][t].v[o][rr];
          al[t].v[o][rr] = pv[t].v[o][rr] * d1 + gg[t].v[o][rr] * a1 * d2;
        }
  });
#pragma unroll
  for (int t = 0; t < NT; ++t) bstore_stream(al[t], p.Alpha, S, row0 + 16 * t, 0);
}

#define DBSDE_PHASE2_DEFINE(T, TD, K, ACT, HV, NT, NBUF, ADOT)                           \
  template __global__ void phaseA2_kernel<T, TD, K, ACT, HV, NT, NBUF, ADOT>(FusedArgs); \
  template __global__ void phaseC2_kernel<T, TD, K, ACT, HV, NT, NBUF, ADOT>(FusedArgs);
DBSDE_PHASE2_INSTANCES(DBSDE_PHASE2_DEFINE)
#undef DBSDE_PHASE2_DEFINE

}  // namespace dbsde
