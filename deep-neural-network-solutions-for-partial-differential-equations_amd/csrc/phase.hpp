// phase.hpp -- register-resident phase kernels (gfx950).
//
// The two network passes of the step, one wavefront per 16 rows:
//   phaseA2 : forward (a_j, h_j, u) + input gradient (delta_j, g_j, Z) + the
//             per-row sums the residual needs
//   phaseC2 : forward tangent along zbar (adot_j, hdot_j) + reverse (p_j, alpha_j)
//
// Orientation.  Every layer is computed transposed, out^T = W . act^T: the
// weights are the MFMA A operand and the activations the B operand, so with
// v_mfma_f32_16x16x4_f32 lane l = cl + 16 q holds, for batch row cl, the
// output columns 16 o + 4 q + r (r = 0..3) of every 16-column block o.  That is
// exactly the B-operand layout the next layer needs (k-step (t, r) pairs
// logical k = q with column 16 t + 4 q + r), so activations never leave the
// registers between layers: no LDS re-layout, no per-layer barrier for
// activations, float4 global loads/stores of whole 16-byte column groups.
//
// Weights.  Each operand matrix is packed once per step (pack_tagged_kernel)
// into a "fragment image": fragment (o, t) is 64 lanes x float4 with lane l
// holding W[16 o + (l & 15)][16 t + 4 (l >> 4) .. + 3].  A workgroup of 8 waves
// (128 rows, two waves per SIMD) streams the images of its stage sequence
// through two LDS buffers with LDS-DMA (global_load_lds_dwordx4, one 1 KiB
// fragment per wave-instruction, no VGPRs): while stage s computes out of one
// buffer the image of stage s+1 lands in the other, and one barrier per stage
// (not per K chunk) publishes it.  Fragment reads are lane-linear ds_read_b128
// (conflict-free).
#pragma once
#include "fused.hpp"

namespace dbsde {

constexpr int PH_WAVES = 8;
constexpr int PH_ROWS = 16 * PH_WAVES;  // rows per workgroup; Rp is padded to this

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
#ifdef DBSDE_EXP_NOSTORE
  if (base != nullptr) return;   // timing experiment only: activation stores dropped
#endif
  const int lane = threadIdx.x & 63;
  float* p = base + (size_t)(row0 + (lane & 15)) * ld + col0 + 4 * (lane >> 4);
#pragma unroll
  for (int t = 0; t < TT; ++t) *(floatx4*)(p + 16 * t) = m.v[t];
}

__device__ __forceinline__ void glds16(const float* g, floatx4* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
// wave w copies fragments w, w + 8, ... of an nf-fragment image
__device__ __forceinline__ void stage_dma(const float* img, int nf, floatx4* buf, int wave, int lane) {
  for (int f = wave; f < nf; f += PH_WAVES) glds16(img + (size_t)f * 256 + lane * 4, buf + f * 64);
}
__device__ __forceinline__ void vm_wait0() { __builtin_amdgcn_s_waitcnt(0x0F70); }   // vmcnt(0)

// acc[o] += W(o, :) . b  over TI input blocks; W from a fragment image in LDS
// Output blocks are taken in groups of at most OG (fragment registers 4 OG;
// OG >= 2 keeps consecutive MFMAs on independent accumulators).
template <int TO, int TI, int OG = 4>
__device__ __forceinline__ void sgemm(Mat<TO>& acc, const Mat<TI>& b, const floatx4* img, int lane) {
#pragma unroll
  for (int t = 0; t < TI; ++t) {
#pragma unroll
    for (int o0 = 0; o0 < TO; o0 += OG) {
      constexpr int dummy = 0;
      (void)dummy;
      floatx4 w[OG];
#pragma unroll
      for (int o = 0; o < OG; ++o)
        if (o0 + o < TO) w[o] = img[((o0 + o) * TI + t) * 64 + lane];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int o = 0; o < OG; ++o)
          if (o0 + o < TO) acc.v[o0 + o] = mfma4(w[o][r], b.v[t][r], acc.v[o0 + o]);
    }
  }
}

// stage sequencer: wait for this stage's image, publish it, start the next one
struct Stager {
  floatx4* wl;
  const float* const* img;
  const int* nf;
  int n, st, wave, lane, buf;
  __device__ __forceinline__ const floatx4* next() {
    vm_wait0();
    __syncthreads();
    if (st + 1 < n) stage_dma(img[st + 1], nf[st + 1], wl + ((st + 1) & 1) * buf, wave, lane);
    const floatx4* cur = wl + (st & 1) * buf;
    ++st;
    return cur;
  }
};

// ---------------------------------------------------------------------------
// phase A: forward + input gradient + Z (+ residual row sums)
// stage images (host order): X0, {F_j, [X_j]} j=1..K, {[Z_j], B_j} j=K..1, Z0
// ---------------------------------------------------------------------------
template <int T, int TD, int K, int ACT>
__global__ void __launch_bounds__(512, 2) phaseA2_kernel(FusedArgs p) {
  constexpr int TB = T > TD ? T : TD, BUF = TB * TB * 64;
  __shared__ floatx4 wl[2 * BUF];
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = blockIdx.x * PH_ROWS + wave * 16;
  const int S = p.S, Wd = p.W;
  Stager sg{wl, p.simgA, p.snfA, p.nA, 0, wave, lane, BUF};
  stage_dma(p.simgA[0], p.snfA[0], wl, wave, lane);
  Mat<TD> x;
  bload(x, p.xin, p.Dp, row0, 0);

  Mat<T> s1[K + 1];   // act'(a_j)
  Mat<T> h, acc;
  {  // level 0
    const floatx4* w = sg.next();
    zero(acc);
    sgemm<T, TD>(acc, x, w, lane);
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float f, d;
        act_v1<ACT>(acc.v[o][r], f, d);
        h.v[o][r] = f;
        s1[0].v[o][r] = d;
      }
    bstore(acc, p.Abuf, S, row0, 0);
    bstore(h, p.H, S, row0, 0);
  }
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const floatx4* w = sg.next();
    zero(acc);
    sgemm<T, T>(acc, h, w, lane);
    if (p.has_v) {
      w = sg.next();
      sgemm<T, TD>(acc, x, w, lane);
    }
#pragma unroll
    for (int o = 0; o < T; ++o) {
      const floatx4 bb = p.has_v ? floatx4{0.f, 0.f, 0.f, 0.f} : *(const floatx4*)(p.beta[j - 1] + 16 * o + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = acc.v[o][r] + bb[r];
        acc.v[o][r] = a;
        float f, d;
        act_v1<ACT>(a, f, d);
        s1[j].v[o][r] = d;
        h.v[o][r] = f + p.rho * h.v[o][r];
      }
    }
    bstore(acc, p.Abuf, S, row0, j * Wd);
    bstore(h, p.H, S, row0, j * Wd);
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
  bstore(dl, p.Delta, S, row0, K * Wd);
  Mat<TD> z;
  zero(z);
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    const floatx4* w;
    if (p.has_v) {
      w = sg.next();
      sgemm<TD, T>(z, dl, w, lane);   // Z += delta_j V_j
    }
    w = sg.next();
    Mat<T> gn;
    zero(gn);
    sgemm<T, T>(gn, dl, w, lane);    // delta_j B_j
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gv = gn.v[o][r] + p.rho * g.v[o][r];
        g.v[o][r] = gv;
        dl.v[o][r] = gv * s1[j - 1].v[o][r];
      }
    bstore(g, p.G, S, row0, (j - 1) * Wd);
    bstore(dl, p.Delta, S, row0, (j - 1) * Wd);
  });
  {
    const floatx4* w = sg.next();
    bload(x, p.xin, p.Dp, row0, 0);
    sgemm<TD, T>(z, dl, w, lane);    // Z += delta_0 W_in
  }
  bstore(z, p.zfull, p.Dp, row0, 0);
  // residual row sums of row cl: [s_zs, s_xz, s_zz, s_x, s_xx, z1]
  Mat<TD> sd;
  bload(sd, p.sdw, p.Dp, row0, 0);
  const int D = p.D;
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
__global__ void __launch_bounds__(512, 2) phaseC2_kernel(FusedArgs p) {
  constexpr int TB = T > TD ? T : TD, BUF = TB * TB * 64;
  __shared__ floatx4 wl[2 * BUF];
  const int lane = threadIdx.x & 63, q = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = blockIdx.x * PH_ROWS + wave * 16;
  const int S = p.S, Wd = p.W;
  Stager sg{wl, p.simgC, p.snfC, p.nC, 0, wave, lane, BUF};
  stage_dma(p.simgC[0], p.snfC[0], wl, wave, lane);
  Mat<TD> zb;
  bload(zb, p.zbar, p.Dp, row0, 0);

  Mat<T> ad[K + 1];   // adot_j
  Mat<T> hd, av;
  {  // tangent level 0
    const floatx4* w = sg.next();
    bload(av, p.Abuf, S, row0, 0);
    zero(ad[0]);
    sgemm<T, TD>(ad[0], zb, w, lane);
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) hd.v[o][r] = act_1<ACT>(av.v[o][r]) * ad[0].v[o][r];
    bstore(hd, p.Hdot, S, row0, 0);
  }
  SFor<1, K + 1>::run([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const floatx4* w = sg.next();
    bload(av, p.Abuf, S, row0, j * Wd);
    zero(ad[j]);
    sgemm<T, T>(ad[j], hd, w, lane);
    if (p.has_v) {
      w = sg.next();
      sgemm<T, TD>(ad[j], zb, w, lane);
    }
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 4; ++r) hd.v[o][r] = act_1<ACT>(av.v[o][r]) * ad[j].v[o][r] + p.rho * hd.v[o][r];
    bstore(hd, p.Hdot, S, row0, j * Wd);
  });
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
    bstore(al, p.Alpha, S, row0, K * Wd);
  }
  SFor<0, K>::run([&](auto ic) __attribute__((always_inline)) {
    constexpr int j = K - decltype(ic)::value;
    const floatx4* w = sg.next();
    bload(av, p.Abuf, S, row0, (j - 1) * Wd);
    Mat<T> acc;
    zero(acc);
    sgemm<T, T>(acc, al, w, lane);   // alpha_j B_j
    Mat<T> gg;
    bload(gg, p.G, S, row0, (j - 1) * Wd);
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
    bstore(al, p.Alpha, S, row0, (j - 1) * Wd);
  });
}

}  // namespace dbsde
