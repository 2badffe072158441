// Microbenchmark: the split-bf16 piece loop of the phase kernels (phase.hpp
// sgemm_x3_piece) in isolation -- one 21 KiB weight piece resident in LDS,
// no barriers, no LDS-DMA, no global memory -- to measure what the inner loop
// itself sustains on the matrix cores.  Per piece and wave: 7 fragments x 3
// ds_read_b128, 7 x 6 dependent v_mfma_f32_16x16x32_bf16 chains, and the
// split of the next 32-wide input block (4 dword pairs).
//   mode 0: phase.hpp's sgemm_x3_piece (PF, split interleaved)
//   mode 1: the same without the split work (last piece of a stage)
//   mode 2: weights held in registers (no fragment reads), with the split
//   mode 3: two fragments' MFMA chains interleaved (independent accumulators
//           back to back), with the split
//   mode 4: all 21 fragment parts read first, product-major MFMA order
//   mode 5: pairs of fragments interleaved, the next pair read ahead
// An empty asm memory clobber per iteration keeps the LDS reads in the loop.
// Each at 1 and 2 waves per SIMD (1 or 2 four-wave workgroups per CU).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I<csrc> piece_x3.hip -o piece_x3
#include <hip/hip_runtime.h>

#include <cstdio>

#include "phase.hpp"

using namespace dbsde;

template <int KBN>
__device__ __forceinline__ void piece_interleaved(Mat<7>& acc, const Split3& s, const floatx4* img, int lane,
                                                  const Mat<7>& b, uintx4 (&sn)[3]) {
  const uintx4* im = (const uintx4*)img;
  SFor<0, 4>::run([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    constexpr int o0 = 2 * g, o1 = 2 * g + 1;
    uintx4 w0[3], w1[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) w0[p] = im[(3 * o0 + p) * 64 + lane];
    if constexpr (o1 < 7) {
#pragma unroll
      for (int p = 0; p < 3; ++p) w1[p] = im[(3 * o1 + p) * 64 + lane];
    }
    split_pair<7, KBN, g>(b, sn[0], sn[1], sn[2]);
    floatx4 a = acc.v[o0], c = o1 < 7 ? acc.v[o1 < 7 ? o1 : 0] : floatx4{0, 0, 0, 0};
    a = mfma_bf(w0[0], s.l, a);
    if constexpr (o1 < 7) c = mfma_bf(w1[0], s.l, c);
    a = mfma_bf(w0[0], s.m, a);
    if constexpr (o1 < 7) c = mfma_bf(w1[0], s.m, c);
    a = mfma_bf(w0[1], s.m, a);
    if constexpr (o1 < 7) c = mfma_bf(w1[1], s.m, c);
    a = mfma_bf(w0[1], s.h, a);
    if constexpr (o1 < 7) c = mfma_bf(w1[1], s.h, c);
    a = mfma_bf(w0[2], s.h, a);
    if constexpr (o1 < 7) c = mfma_bf(w1[2], s.h, c);
    acc.v[o0] = mfma_bf(w0[0], s.h, a);
    if constexpr (o1 < 7) acc.v[o1] = mfma_bf(w1[0], s.h, c);
  });
}

// mode 4: every fragment's three parts read first (84 VGPRs), then the six
// products in product-major order (7 independent chains back to back)
__device__ __forceinline__ void piece_productmajor(Mat<7>& acc, const Split3& s, const floatx4* img, int lane) {
  const uintx4* im = (const uintx4*)img;
  uintx4 w[7][3];
#pragma unroll
  for (int o = 0; o < 7; ++o)
#pragma unroll
    for (int p = 0; p < 3; ++p) w[o][p] = im[(3 * o + p) * 64 + lane];
#pragma unroll
  for (int o = 0; o < 7; ++o) acc.v[o] = mfma_bf(w[o][0], s.l, acc.v[o]);
#pragma unroll
  for (int o = 0; o < 7; ++o) acc.v[o] = mfma_bf(w[o][0], s.m, acc.v[o]);
#pragma unroll
  for (int o = 0; o < 7; ++o) acc.v[o] = mfma_bf(w[o][1], s.m, acc.v[o]);
#pragma unroll
  for (int o = 0; o < 7; ++o) acc.v[o] = mfma_bf(w[o][1], s.h, acc.v[o]);
#pragma unroll
  for (int o = 0; o < 7; ++o) acc.v[o] = mfma_bf(w[o][2], s.h, acc.v[o]);
#pragma unroll
  for (int o = 0; o < 7; ++o) acc.v[o] = mfma_bf(w[o][0], s.h, acc.v[o]);
}
// mode 5: pairs of fragments, each pair's two chains interleaved, the next
// pair's six reads issued ahead (48 VGPRs of weights)
__device__ __forceinline__ void piece_pairs(Mat<7>& acc, const Split3& s, const floatx4* img, int lane) {
  const uintx4* im = (const uintx4*)img;
  uintx4 w[2][2][3];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int p = 0; p < 3; ++p) w[0][k][p] = im[(3 * k + p) * 64 + lane];
  SFor<0, 4>::run([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    constexpr int o0 = 2 * g, o1 = 2 * g + 1;
    if constexpr (g + 1 < 4) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          if (2 * (g + 1) + k < 7) w[(g + 1) & 1][k][p] = im[(3 * (2 * (g + 1) + k) + p) * 64 + lane];
    }
    const auto& wa = w[g & 1][0];
    const auto& wb = w[g & 1][1];
    floatx4 a = acc.v[o0], c = acc.v[o1 < 7 ? o1 : 0];
    a = mfma_bf(wa[0], s.l, a);
    if constexpr (o1 < 7) c = mfma_bf(wb[0], s.l, c);
    a = mfma_bf(wa[0], s.m, a);
    if constexpr (o1 < 7) c = mfma_bf(wb[0], s.m, c);
    a = mfma_bf(wa[1], s.m, a);
    if constexpr (o1 < 7) c = mfma_bf(wb[1], s.m, c);
    a = mfma_bf(wa[1], s.h, a);
    if constexpr (o1 < 7) c = mfma_bf(wb[1], s.h, c);
    a = mfma_bf(wa[2], s.h, a);
    if constexpr (o1 < 7) c = mfma_bf(wb[2], s.h, c);
    acc.v[o0] = mfma_bf(wa[0], s.h, a);
    if constexpr (o1 < 7) acc.v[o1] = mfma_bf(wb[0], s.h, c);
    __builtin_amdgcn_sched_barrier(0);
  });
}

template <int MODE>
__device__ __forceinline__ void one_piece(Mat<7>& acc, const Split3& s, const floatx4* w, int lane, const Mat<7>& b,
                                          uintx4 (&sn)[3], const uintx4 (&wr)[21]) {
  if constexpr (MODE == 0) {
    sgemm_x3_piece<7, 7, 1, true>(acc, s, w, lane, b, sn);
  } else if constexpr (MODE == 1) {
    sgemm_x3_piece<7, 7, 4, true>(acc, s, w, lane, b, sn);
  } else if constexpr (MODE == 2) {
#pragma unroll
    for (int o = 0; o < 7; ++o) {
      if (o < 4) split_pair<7, 1, 0>(b, sn[0], sn[1], sn[2]);
      floatx4 a = acc.v[o];
      a = mfma_bf(wr[3 * o], s.l, a);
      a = mfma_bf(wr[3 * o], s.m, a);
      a = mfma_bf(wr[3 * o + 1], s.m, a);
      a = mfma_bf(wr[3 * o + 1], s.h, a);
      a = mfma_bf(wr[3 * o + 2], s.h, a);
      acc.v[o] = mfma_bf(wr[3 * o], s.h, a);
    }
  } else if constexpr (MODE == 3) {
    piece_interleaved<1>(acc, s, w, lane, b, sn);
  } else if constexpr (MODE == 4) {
    piece_productmajor(acc, s, w, lane);
  } else {
    piece_pairs(acc, s, w, lane);
  }
  if constexpr (MODE >= 4) {   // no split work: the same operand again
    sn[0] = __builtin_bit_cast(uintx4, s.h);
    sn[1] = __builtin_bit_cast(uintx4, s.m);
    sn[2] = __builtin_bit_cast(uintx4, s.l);
  }
}

// mode 6/7: the phase kernels' piece pipeline -- PieceStager (3-buffer LDS
// ring, LDS-DMA of each piece two ahead from a 56-piece image in global memory
// (L2 resident), counted vmcnt wait + barrier per piece) around
// sgemm_x3_piece (6) or the pairs piece (7)
// mode 8: mode 6 plus the phase kernels' activation stores: after every 4th
// piece (one level) the wave stores its 16 x 112 accumulator tile twice (as
// fstore + bstore_stream do: 2 x 7 KiB per level and wave) into a large
// streaming buffer -- the HBM write stream of phase A (~185 MB per dispatch)
template <int MODE, int WPS>
__global__ void __launch_bounds__(256, WPS) kern_staged(float* out, const float* const* pieces, int iters,
                                                       float* sink, long long sink_floats) {
  constexpr int BUF = 3 * 7 * 64;
  __shared__ floatx4 wl[P3_NBUF_X3 * BUF];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  Mat<7> b, acc;
#pragma unroll
  for (int t = 0; t < 7; ++t) {
    b.v[t] = floatx4{1.f, 0.5f, 0.25f, 0.125f} * (float)(lane + t + 1) * 1.0001f;
    acc.v[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  Split3 s = split_block<7, 0>(b);
  long long so = ((long long)blockIdx.x * 4 + wave) * 16 * 112 * 14;
  for (int it = 0; it < iters; ++it) {
    PieceStagerT<P3_NBUF_X3, 5, 21, 56> sg{wl, pieces, nullptr, 56, 0, wave, lane, BUF};
    sg.start();
    SFor<0, 56>::run([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      const floatx4* w = sg.template next<0>();
      if constexpr (MODE == 8 && k % 4 == 0 && k > 0) {
        float* base = sink + (so % (sink_floats - 2 * 16 * 112)) ;
        fstore(acc, base, 112, 0, 0);
        bstore_stream(acc, base + 16 * 112, 112, 0, 0);
        so += (long long)gridDim.x * 4 * 16 * 112 * 2;
      }
      if constexpr (MODE == 9 && k >= 4) {   // the same bytes, 3 or 4 of the 14 stores after each piece's barrier
        float* base = sink + (so % (sink_floats - 2 * 16 * 112));
        constexpr int i0 = (k % 4) * 4, i1 = i0 + 4 < 14 ? i0 + 4 : 14;
        const int l = threadIdx.x & 63;
#pragma unroll
        for (int i = i0; i < i1; ++i) {
          if (i < 7)
            *(floatx4*)(base + 256 * i + 4 * l) = acc.v[i < 7 ? i : 0];
          else
            __builtin_nontemporal_store(acc.v[i - 7 < 7 ? i - 7 : 0],
                                        (floatx4*)(base + 16 * 112 + (l & 15) * 112 + 4 * (l >> 4) + 16 * (i - 7)));
        }
        if (k % 4 == 3) so += (long long)gridDim.x * 4 * 16 * 112 * 2;
      }
      uintx4 sn[3];
      if constexpr (MODE == 6 || MODE == 8 || MODE == 9)
        sgemm_x3_piece<7, 7, 1, true>(acc, s, w, lane, b, sn);
      else
        sgemm_x3_piece_pairs<7, 7, 1>(acc, s, w, lane, b, sn);
      s = Split3{__builtin_bit_cast(bf16x8, sn[0]), __builtin_bit_cast(bf16x8, sn[1]), __builtin_bit_cast(bf16x8, sn[2])};
    });
  }
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 7; ++t) sum += acc.v[t][0] + acc.v[t][1] + acc.v[t][2] + acc.v[t][3];
  out[blockIdx.x * 256 + threadIdx.x] = sum;
}

template <int MODE, int WPS>
__global__ void __launch_bounds__(256, WPS) kern(float* out, int iters) {
  __shared__ floatx4 wl[3 * 7 * 64];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 3 * 7 * 64; i += 256) {
    const unsigned u = 0x3f803f80u ^ (unsigned)(i * 2654435761u & 0x007f007fu);
    wl[i] = __builtin_bit_cast(floatx4, uintx4{u, u ^ 0x10001u, u ^ 0x20002u, u ^ 0x30003u});
  }
  __syncthreads();
  Mat<7> b, acc;
#pragma unroll
  for (int t = 0; t < 7; ++t) {
    b.v[t] = floatx4{1.f, 0.5f, 0.25f, 0.125f} * (float)(lane + t + 1) * 1.0001f;
    acc.v[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  uintx4 wr[21];
#pragma unroll
  for (int k = 0; k < 21; ++k) wr[k] = ((const uintx4*)wl)[k * 64 + lane];
  Split3 s = split_block<7, 0>(b);
  for (int it = 0; it < iters; ++it) {
    asm volatile("" ::: "memory");   // the weight reads stay in the loop (no hoisting)
    uintx4 sn[3];
    one_piece<MODE>(acc, s, wl, lane, b, sn, wr);
    s = Split3{__builtin_bit_cast(bf16x8, sn[0]), __builtin_bit_cast(bf16x8, sn[1]), __builtin_bit_cast(bf16x8, sn[2])};
  }
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 7; ++t) sum += acc.v[t][0] + acc.v[t][1] + acc.v[t][2] + acc.v[t][3];
  out[blockIdx.x * 256 + threadIdx.x] = sum;
}

template <int MODE, int WPS>
void run(const char* name) {
  const int blocks = 256 * WPS, iters = 4000;
  float* out;
  (void)hipMalloc(&out, blocks * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  kern<MODE, WPS><<<blocks, 256>>>(out, iters);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(e0);
    kern<MODE, WPS><<<blocks, 256>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  // 42 MFMAs per piece and wave, 16 x 16 x 32 x 2 flops each
  const double mfmas = 42.0 * iters * blocks * 4, flops = mfmas * 16 * 16 * 32 * 2;
  printf("%-34s waves/SIMD=%d  %.3f ms  %.0f bf16 TF/s  %.1f%% of 2500  ns/piece/wave %.1f\n", name, WPS, best,
         flops / best / 1e9, flops / best / 1e9 / 25.0, best * 1e6 / iters);
  (void)hipFree(out);
}

template <int MODE, int WPS>
void run_staged(const char* name, int blocks_per_cu_x) {
  const int blocks = 256 * WPS * blocks_per_cu_x / 2, iters = 40;
  float* out;
  (void)hipMalloc(&out, blocks * 256 * 4);
  float* img;
  (void)hipMalloc(&img, 56 * 21 * 1024);
  (void)hipMemset(img, 0x3f, 56 * 21 * 1024);
  const float* h[64];
  for (int k = 0; k < 64; ++k) h[k] = img + (size_t)(k % 56) * 21 * 256;
  const float** dp;
  (void)hipMalloc(&dp, sizeof(h));
  (void)hipMemcpy(dp, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const long long sink_floats = 256LL << 20;   // 1 GiB streaming target
  float* sink;
  (void)hipMalloc(&sink, sink_floats * 4);
  kern_staged<MODE, WPS><<<blocks, 256>>>(out, dp, iters, sink, sink_floats);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(e0);
    kern_staged<MODE, WPS><<<blocks, 256>>>(out, dp, iters, sink, sink_floats);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  const double mfmas = 42.0 * 56 * iters * blocks * 4, flops = mfmas * 16 * 16 * 32 * 2;
  // per-wave time of one piece: a SIMD runs WPS * blocks_per_cu_x / 2 waves
  printf("%-34s waves/SIMD=%d  %.3f ms  %.0f bf16 TF/s  %.1f%% of 2500  ns/piece/wave-slot %.1f\n", name,
         WPS * blocks_per_cu_x / 2, best, flops / best / 1e9, flops / best / 1e9 / 25.0, best * 1e6 / (iters * 56));
  (void)hipFree(out);
  (void)hipFree(img);
  (void)hipFree(dp);
  (void)hipFree(sink);
}

int main() {
  run_staged<6, 1>("staged sgemm_x3_piece", 2);
  run_staged<6, 2>("staged sgemm_x3_piece", 2);
  run_staged<8, 1>("staged + level stores", 2);
  run_staged<8, 2>("staged + level stores", 2);
  run_staged<9, 1>("staged + spread stores", 2);
  run_staged<9, 2>("staged + spread stores", 2);
  return 0;
  run<0, 1>("sgemm_x3_piece (split)");
  run<0, 2>("sgemm_x3_piece (split)");
  run<1, 1>("sgemm_x3_piece (no split)");
  run<1, 2>("sgemm_x3_piece (no split)");
  run<2, 1>("weights in registers (split)");
  run<2, 2>("weights in registers (split)");
  run<3, 1>("two chains interleaved (split)");
  run<3, 2>("two chains interleaved (split)");
  run<4, 1>("product-major, 21 reads first");
  run<4, 2>("product-major, 21 reads first");
  run<5, 1>("fragment pairs, next pair ahead");
  run<5, 2>("fragment pairs, next pair ahead");
  return 0;
}
