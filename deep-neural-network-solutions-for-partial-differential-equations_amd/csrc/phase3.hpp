// phase3.hpp -- register-resident phase kernels, 4-wave workgroups (gfx950).
//
// Same arithmetic, orientation and operand images as phase.hpp (weights are
// the MFMA A operand from LDS fragment images, activations the B operand in
// registers), with the workgroup cut to 4 waves = 64 rows, one wave per SIMD.
// Two such workgroups share a CU and run independently, so while one wave of
// a SIMD is in its activation epilogue (sincos) or waiting on memory, the
// other can keep the matrix pipe busy; the 8-wave phase.hpp kernels hold both
// waves of a SIMD in lock step at every stage barrier.
//
// LDS.  Every stage image is streamed in two pieces, input blocks [0, H) and
// [H, TI) with H = ceil(TI / 2), so two double-buffered workgroups fit in a
// CU (2 x 2 x 28 KB at TI = TO = 7).  The images are t-major for this: the
// fragment of (output block o, input block t) sits at index t * TO + o, so a
// piece is one contiguous run of fragments (pack_tagged_kernel, ftout > 0).
//
// Stores.  An activation tile that the next layer also consumes (h, hdot,
// delta, g, alpha) is stored right after the next piece's barrier instead of
// just before it, so the vmcnt(0) that retires a piece's LDS-DMA does not
// wait on stores issued a few cycles earlier.
#pragma once
#include "phase.hpp"

namespace dbsde {

constexpr int P3_WAVES = 4;
constexpr int P3_ROWS = 16 * P3_WAVES;

// acc[o] += sum_{t in [T0, T1)} W(o, t) . b(t); img = the piece holding
// fragment (o, t) at ((t - T0) * TO + o)
template <int TO, int TI, int T0, int T1, int OG = 4>
__device__ __forceinline__ void sgemm_piece(Mat<TO>& acc, const Mat<TI>& b, const floatx4* img, int lane) {
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

// wave w copies fragments w, w + 4, ... of an nf-fragment piece
__device__ __forceinline__ void piece_dma(const float* img, int nf, floatx4* buf, int wave, int lane) {
  for (int f = wave; f < nf; f += P3_WAVES) glds16(img + (size_t)f * 256 + lane * 4, buf + f * 64);
}

// piece sequencer: wait for this piece, publish it, start the next one
struct PieceStager {
  floatx4* wl;
  const float* const* img;
  const int* nf;
  int n, st, wave, lane, buf;
  __device__ __forceinline__ const floatx4* next() {
#ifdef DBSDE_EXP_NOSTAGE
    if (st++ > 0) return wl;   // timing experiment only: every piece reuses piece 0, no DMA, no barrier
    vm_wait0();
    __syncthreads();
    return wl;
#endif
    vm_wait0();
    __syncthreads();
    if (st + 1 < n) piece_dma(img[st + 1], nf[st + 1], wl + ((st + 1) & 1) * buf, wave, lane);
    const floatx4* cur = wl + (st & 1) * buf;
    ++st;
    return cur;
  }
};

struct NoOp {
  __device__ __forceinline__ void operator()() const {}
};

// one stage = one operand image: two pieces (one when TI == 1); `after` runs
// right after the first piece's barrier (deferred stores, early loads)
template <int TO, int TI, class F>
__device__ __forceinline__ void stage_mm(Mat<TO>& acc, const Mat<TI>& b, PieceStager& sg, int lane, F&& after) {
  constexpr int H = (TI + 1) / 2;
  const floatx4* w = sg.next();
  after();
  sgemm_piece<TO, TI, 0, H>(acc, b, w, lane);
  if constexpr (H < TI) {
    w = sg.next();
    sgemm_piece<TO, TI, H, TI>(acc, b, w, lane);
  }
}

// ---------------------------------------------------------------------------
// phase A: forward + input gradient + Z (+ residual row sums)
// stage images (host order): X0, {F_j, [X_j]} j=1..K, {[Z_j], B_j} j=K..1, Z0
// ---------------------------------------------------------------------------
template <int T, int TD, int K, int ACT>
__global__ void __launch_bounds__(256, 2) phaseA3_kernel(FusedArgs p) {
  constexpr int TB = T > TD ? T : TD, BUF = ((TB + 1) / 2) * TB * 64;
  __shared__ floatx4 wl[2 * BUF];
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = blockIdx.x * P3_ROWS + wave * 16;
  const int S = p.S, Wd = p.W;
  PieceStager sg{wl, p.simgA, p.snfA, p.nA, 0, wave, lane, BUF};
  piece_dma(p.simgA[0], p.snfA[0], wl, wave, lane);
  Mat<TD> x;
  bload(x, p.xin, p.Dp, row0, 0);

  Mat<T> s1[K + 1];   // act'(a_j)
  Mat<T> h, acc;
  zero(acc);
  stage_mm<T, TD>(acc, x, sg, lane, NoOp{});
  bstore(acc, p.Abuf, S, row0, 0);
#pragma unroll
  for (int o = 0; o < T; ++o)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float f, d;
      act_v1<ACT>(acc.v[o][r], f, d);
      h.v[o][r] = f;
      s1[0].v[o][r] = d;
    }
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    zero(acc);
    stage_mm<T, T>(acc, h, sg, lane, [&]() __attribute__((always_inline)) { bstore(h, p.H, S, row0, (j - 1) * Wd); });
    if (p.has_v) stage_mm<T, TD>(acc, x, sg, lane, NoOp{});
#pragma unroll
    for (int o = 0; o < T; ++o) {
      const floatx4 bb = p.has_v ? floatx4{0.f, 0.f, 0.f, 0.f} : *(const floatx4*)(p.beta[j - 1] + 16 * o + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc.v[o][r] += bb[r];
    }
    bstore(acc, p.Abuf, S, row0, j * Wd);
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float f, d;
        act_v1<ACT>(acc.v[o][r], f, d);
        s1[j].v[o][r] = d;
        h.v[o][r] = f + p.rho * h.v[o][r];
      }
  });
  // u = h_{K+1} . w_out + b_out
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
    if (q == 0) p.u[row0 + cl] = us + p.bout[0];
  }
  bstore(h, p.H, S, row0, K * Wd);
  // input gradient: g_{K+1} = w_out, delta_K = w_out act'(a_K)
  Mat<T> g, dl;
#pragma unroll
  for (int o = 0; o < T; ++o) {
    const floatx4 wo = *(const floatx4*)(p.wout + 16 * o + 4 * q);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      g.v[o][r] = wo[r];
      dl.v[o][r] = wo[r] * s1[K].v[o][r];
    }
  }
  Mat<TD> z;
  zero(z);
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    auto prev = [&]() __attribute__((always_inline)) {   // (g_j, delta_j) of the previous step
      if constexpr (j < K) bstore(g, p.G, S, row0, j * Wd);
      bstore(dl, p.Delta, S, row0, j * Wd);
    };
    Mat<T> gn;
    zero(gn);
    if (p.has_v) {
      stage_mm<TD, T>(z, dl, sg, lane, prev);      // Z += delta_j V_j
      stage_mm<T, T>(gn, dl, sg, lane, NoOp{});    // delta_j B_j
    } else {
      stage_mm<T, T>(gn, dl, sg, lane, prev);
    }
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gv = gn.v[o][r] + p.rho * g.v[o][r];
        g.v[o][r] = gv;
        dl.v[o][r] = gv * s1[j - 1].v[o][r];
      }
  });
  stage_mm<TD, T>(z, dl, sg, lane, [&]() __attribute__((always_inline)) {   // Z += delta_0 W_in
    bstore(g, p.G, S, row0, 0);
    bstore(dl, p.Delta, S, row0, 0);
    bload(x, p.xin, p.Dp, row0, 0);
  });
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
#pragma unroll
    for (int i = 0; i < 6; ++i) o[i] = v6[i];
  }
}

// ---------------------------------------------------------------------------
// phase C: forward tangent along zbar + reverse over (primal, tangent)
// stage images (host order): X0, {F_j, [X_j]} j=1..K, B_j j=K..1
// ---------------------------------------------------------------------------
template <int T, int TD, int K, int ACT>
__global__ void __launch_bounds__(256, 2) phaseC3_kernel(FusedArgs p) {
  constexpr int TB = T > TD ? T : TD, BUF = ((TB + 1) / 2) * TB * 64;
  __shared__ floatx4 wl[2 * BUF];
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = blockIdx.x * P3_ROWS + wave * 16;
  const int S = p.S, Wd = p.W;
  PieceStager sg{wl, p.simgC, p.snfC, p.nC, 0, wave, lane, BUF};
  piece_dma(p.simgC[0], p.snfC[0], wl, wave, lane);
  Mat<TD> zb;
  bload(zb, p.zbar, p.Dp, row0, 0);

  Mat<T> ad[K + 1];   // adot_j
  Mat<T> hd, av;
  zero(ad[0]);
  stage_mm<T, TD>(ad[0], zb, sg, lane, [&]() __attribute__((always_inline)) { bload(av, p.Abuf, S, row0, 0); });
#pragma unroll
  for (int o = 0; o < T; ++o)
#pragma unroll
    for (int r = 0; r < 4; ++r) hd.v[o][r] = act_1<ACT>(av.v[o][r]) * ad[0].v[o][r];
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    zero(ad[j]);
    stage_mm<T, T>(ad[j], hd, sg, lane, [&]() __attribute__((always_inline)) {
      bstore(hd, p.Hdot, S, row0, (j - 1) * Wd);
      bload(av, p.Abuf, S, row0, j * Wd);
    });
    if (p.has_v) stage_mm<T, TD>(ad[j], zb, sg, lane, NoOp{});
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) hd.v[o][r] = act_1<ACT>(av.v[o][r]) * ad[j].v[o][r] + p.rho * hd.v[o][r];
  });
  bstore(hd, p.Hdot, S, row0, K * Wd);
  // reverse: p_{K+1} = ubar w_out ; alpha_K = w_out (ubar act'(a_K) + adot_K act''(a_K))
  Mat<T> pv, al;
  {
    const float ub = p.ubar[row0 + cl];
#pragma unroll
    for (int o = 0; o < T; ++o) {
      const floatx4 wo = *(const floatx4*)(p.wout + 16 * o + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float d1, d2;
        act_12<ACT>(av.v[o][r], d1, d2);
        pv.v[o][r] = ub * wo[r];
        al.v[o][r] = wo[r] * (ub * d1 + ad[K].v[o][r] * d2);
      }
    }
  }
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    Mat<T> acc, gg;
    zero(acc);
    stage_mm<T, T>(acc, al, sg, lane, [&]() __attribute__((always_inline)) {   // alpha_j B_j
      bstore(al, p.Alpha, S, row0, j * Wd);
      bload(av, p.Abuf, S, row0, (j - 1) * Wd);
      bload(gg, p.G, S, row0, (j - 1) * Wd);
    });
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pp = acc.v[o][r] + p.rho * pv.v[o][r];
        pv.v[o][r] = pp;
        float d1, d2;
        act_12<ACT>(av.v[o][r], d1, d2);
        al.v[o][r] = pp * d1 + gg.v[o][r] * ad[j - 1].v[o][r] * d2;
      }
  });
  bstore(al, p.Alpha, S, row0, 0);
}

}  // namespace dbsde
