// philox.hpp -- Philox4x32-10 counter-based generator and Box-Muller normals
// (device side of the Brownian increments; restated in oracle/philox.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dbsde {

// --------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11; Random123 constants) + Box-Muller
// --------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// Four standard normals from one Philox block: both Box-Muller outputs of the
// uniform pairs (c0, c1) and (c2, c3).  Counter (d, n/4, m, offset), key
// (seed ^ offset_hi, seed_hi); z[k] is the draw of step 4 (n/4) + k.
__device__ __forceinline__ void philox_normal4(unsigned long long seed, unsigned long long offset, uint32_t m,
                                               uint32_t nq, uint32_t d, float z[4]) {
  uint32_t c[4] = {d, nq, m, (uint32_t)offset};
  philox4x32_10(c, (uint32_t)seed ^ (uint32_t)(offset >> 32), (uint32_t)(seed >> 32));
  const float u1 = ((float)(c[0] >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
  const float u2 = (float)(c[1] >> 8) * (1.0f / 16777216.0f);            // [0, 1)
  const float u3 = ((float)(c[2] >> 8) + 1.0f) * (1.0f / 16777216.0f);
  const float u4 = (float)(c[3] >> 8) * (1.0f / 16777216.0f);
  // Box-Muller on the transcendental unit: -2 ln u = -2 ln2 log2 u (v_log_f32),
  // v_sqrt_f32, and sin / cos of 2 pi u straight from v_sin_f32 / v_cos_f32,
  // whose argument is in revolutions (u in [0, 1): no range reduction).  Each
  // is accurate to ~1 ulp; the normals stay within 2e-6 of the fp64 oracle
  // (tests/test_gpu_device_rng.py) at a fraction of the libm cost.
  const float r1 = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  const float r2 = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u3));
  z[0] = r1 * __builtin_amdgcn_cosf(u2);
  z[1] = r1 * __builtin_amdgcn_sinf(u2);
  z[2] = r2 * __builtin_amdgcn_cosf(u4);
  z[3] = r2 * __builtin_amdgcn_sinf(u4);
}

}  // namespace dbsde
