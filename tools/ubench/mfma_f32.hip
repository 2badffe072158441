// Microbenchmark: v_mfma_f32_16x16x4_f32 throughput in the fused kernels'
// shape (7 output tiles per wave).  mode 0: operands in registers; mode 1:
// A (1 b128) + B (7 b128) re-read from LDS every 16-deep chunk.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ void __launch_bounds__(256) kern(float* out, int iters) {
  __shared__ float L[2][7 * 16 * 24 + 16 * 120];
  const int lane = threadIdx.x & 63, cl = lane & 15, q = lane >> 4;
  for (int i = threadIdx.x; i < 2 * (7 * 16 * 24 + 16 * 120); i += 256) (&L[0][0])[i] = 0.001f * (i & 7);
  __syncthreads();
  floatx4 acc[7];
  for (int t = 0; t < 7; ++t) acc[t] = floatx4{0, 0, 0, 0};
  floatx4 a = floatx4{1.f, 0.5f, 0.25f, 0.125f} * (float)(lane + 1);
  floatx4 b[7];
  for (int t = 0; t < 7; ++t) b[t] = a * (float)(t + 1);
  for (int it = 0; it < iters; ++it) {
    if (MODE == 1) {
      const float* Bs = L[it & 1];
      a = *(const floatx4*)(Bs + 7 * 16 * 24 + cl * 120 + 4 * q + 16 * (it % 7));
#pragma unroll
      for (int t = 0; t < 7; ++t) b[t] = *(const floatx4*)(Bs + (16 * t + cl) * 24 + 4 * q);
    }
#pragma unroll
    for (int t = 0; t < 7; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[t].x, acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 7; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[t].y, acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 7; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[t].z, acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 7; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[t].w, acc[t], 0, 0, 0);
  }
  float s = 0;
  for (int t = 0; t < 7; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int MODE>
void run(int blocks_per_cu, const char* name) {
  const int cus = 256, blocks = cus * blocks_per_cu, iters = 2000;
  float* out;
  (void)hipMalloc(&out, blocks * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  kern<MODE><<<blocks, 256>>>(out, iters);
  (void)hipEventRecord(e0);
  kern<MODE><<<blocks, 256>>>(out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 16 * 16 * 4 * 28.0 * iters * blocks * 4;
  printf("%-22s waves/SIMD=%d  %.3f ms  %.1f TFLOP/s\n", name, blocks_per_cu, ms, flops / ms / 1e9);
  (void)hipFree(out);
}
int main() {
  for (int w = 1; w <= 4; ++w) run<0>(w, "registers");
  for (int w = 1; w <= 4; ++w) run<1>(w, "lds operands");
  return 0;
}
