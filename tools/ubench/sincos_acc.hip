// Accuracy of the product dbsde::fast_sincosf (v_sin_f32 / v_cos_f32 after a
// Cody-Waite 2*pi reduction) and, for comparison, of the plain fract(a/2pi)
// form, against fp64 libm on the host, over |a| <= A for several A.
// Build: hipcc -O3 --offload-arch=gfx950 -o sincos_acc sincos_acc.hip
#include <hip/hip_runtime.h>
#include "../../deep-neural-network-solutions-for-partial-differential-equations_amd/csrc/kernels.hpp"
#include <cmath>
#include <cstdio>
#include <vector>

template <int PLAIN>
__global__ void kern(const float* a, float* s, float* c, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (!PLAIN) {
    dbsde::fast_sincosf(a[i], s[i], c[i]);
    return;
  }
  const float rev = __builtin_amdgcn_fractf(a[i] * 0.15915494309189535f);
  s[i] = __builtin_amdgcn_sinf(rev);
  c[i] = __builtin_amdgcn_cosf(rev);
}

int main() {
  const int n = 1 << 22;
  std::vector<float> a(n), s(n), c(n);
  float *da, *ds, *dc;
  if (hipMalloc(&da, n * 4) || hipMalloc(&ds, n * 4) || hipMalloc(&dc, n * 4)) return 1;
  for (int plain = 0; plain < 2; ++plain)
  for (float A : {1.f, 4.f, 16.f, 64.f, 1024.f, 16384.f}) {
    for (int i = 0; i < n; ++i) a[i] = A * (2.f * (i + 0.5f) / n - 1.f);
    (void)hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
    if (plain) kern<1><<<(n + 255) / 256, 256>>>(da, ds, dc, n);
    else kern<0><<<(n + 255) / 256, 256>>>(da, ds, dc, n);
    (void)hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
    double es = 0, ec = 0;
    for (int i = 0; i < n; ++i) {
      es = fmax(es, fabs(s[i] - sin((double)a[i])));
      ec = fmax(ec, fabs(c[i] - cos((double)a[i])));
    }
    printf("%s |a|<=%g  max abs err sin %.3e cos %.3e  (2^-23 = %.3e)\n", plain ? "fract   " : "product ", A, es, ec, ldexp(1.0, -23));
  }
  return 0;
}
