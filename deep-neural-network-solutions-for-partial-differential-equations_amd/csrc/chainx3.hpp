// chainx3.hpp -- the per-layer chain GEMM (kernels.hpp chain_gemm_kernel) in
// split-bf16 products, for the layouts the fused phase kernels do not cover
// (FC / Resnet at widths other than 16 and 110/112, e.g. config 4's
// FC-Sine [101, 256x4, 1], hjb_implement.py:590-604).
//
//   C[Rp, NP] = A[Rp, K] . W^T,  W [NP, K] held as a split-bf16 fragment image
//   (phase.hpp / x3_off: the weight packer's image of this layer), with the
//   chain epilogues unchanged (same accumulator layout as the fp32 form).
//
// The activations are the MFMA A operand: lane (r, q) of a wave holds row
// r of its 16 rows and the 8 k values 32 kb + 16 (j >> 2) + 4 q + (j & 3) of
// input block kb -- two float4 loads -- split into hi / mid / lo bf16 in
// registers; the weight fragment of output block o and input block kb is the
// B operand as stored in the image (lane (c, q) holds W[16 o + c][same k]).
// Six v_mfma_f32_16x16x32_bf16 per product block (phase.hpp: fp32-accurate).
// The NT weight fragments of a 32-wide input block (NT x 3 KiB, contiguous in
// the image) go to LDS by LDS-DMA, double buffered, one block ahead; the A
// rows of the next block are loaded a block ahead into registers.
#pragma once
#include "phase.hpp"

namespace dbsde {

template <int NT>
__device__ __forceinline__ void chain_x3_mainloop(const ChainArgs& p, int row0, int col0, floatx4 (&acc)[NT]) {
  __shared__ floatx4 Bs[2][NT * 3 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int TI = p.x3_ti, nkb = (TI + 1) / 2;
  // fragment (o, kb) of the image is at bf16 offset (kb * tout + o) * 1536
  const unsigned short* img = p.x3_img + (size_t)(col0 >> 4) * 1536;
  const size_t kb_stride = (size_t)p.x3_tout * 1536;
  const float* Ar = p.A + (size_t)(row0 + wave * 16 + (lane & 15)) * p.lda + 4 * q;
  auto dma = [&](int kb, int buf) {
    const unsigned short* src = img + kb * kb_stride;
    for (int ch = wave; ch < NT * 3; ch += 4) glds16((const float*)(src + ch * 512 + lane * 8), &Bs[buf][ch * 64]);
  };
  auto aload = [&](int kb, floatx4& a0, floatx4& a1) {
    const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
    a0 = 2 * kb < TI ? *(const floatx4*)(Ar + 32 * kb) : z;
    a1 = 2 * kb + 1 < TI ? *(const floatx4*)(Ar + 32 * kb + 16) : z;
  };
  floatx4 a0, a1, n0, n1;
  dma(0, 0);
  aload(0, a0, a1);
  for (int kb = 0; kb < nkb; ++kb) {
    const int buf = kb & 1;
    vm_wait<0>();   // this wave's DMA chunks and A rows of block kb
    __syncthreads();   // every wave's chunks landed; buffer buf ^ 1 no longer read
    if (kb + 1 < nkb) {
      dma(kb + 1, buf ^ 1);
      aload(kb + 1, n0, n1);
    }
    uintx4 H, M, L;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const float x0 = d < 2 ? a0[2 * d] : a1[2 * d - 4], x1 = d < 2 ? a0[2 * d + 1] : a1[2 * d - 3];
      const Dw3 r = split_two(x0, x1);
      H[d] = r.h;
      M[d] = r.m;
      L[d] = r.l;
    }
    const bf16x8 sh = __builtin_bit_cast(bf16x8, H), sm = __builtin_bit_cast(bf16x8, M),
                 sl = __builtin_bit_cast(bf16x8, L);
    const uintx4* bw = (const uintx4*)&Bs[buf][0];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16x8 wh = __builtin_bit_cast(bf16x8, bw[(3 * t + 0) * 64 + lane]);
      const bf16x8 wm = __builtin_bit_cast(bf16x8, bw[(3 * t + 1) * 64 + lane]);
      const bf16x8 wl = __builtin_bit_cast(bf16x8, bw[(3 * t + 2) * 64 + lane]);
      floatx4 c = acc[t];
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sl, wh, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sh, wl, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sm, wm, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sm, wh, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sh, wm, c, 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sh, wh, c, 0, 0, 0);
    }
    a0 = n0;
    a1 = n1;
  }
}

}  // namespace dbsde
