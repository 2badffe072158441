// phase2.hpp -- the fused phase kernels with two 16-row tiles per wave (gfx950).
//
// Same algorithm, image order and operand layout as phase.hpp (read that
// header first); what changes is the work per staged weight piece.  A wave
// owns 32 rows (two 16-row register tiles), a 4-wave workgroup 128 rows, one
// workgroup per CU with the whole 512-entry register file per wave (one wave
// per SIMD).  Every fragment read from LDS feeds 12 MFMAs (two tiles x six
// split-bf16 products) instead of 6, so per MFMA the kernel issues half the
// LDS-DMA, half the fragment reads and half the barriers of the 16-row form,
// and each weight byte streamed from L2 serves 128 rows instead of 64.  The
// ring is 4 pieces deep (3 in flight, 84 KiB).
//
// Phase A keeps no act'(a_j) registers (they would need 224 per wave): the
// backward reloads a_j from Abuf, which it wrote a few stages earlier, and
// recomputes act'(a_j) -- the same reload phase C makes.
#pragma once
#include "phase.hpp"

namespace dbsde {

constexpr int Q_NT = 2;                            // 16-row tiles per wave
constexpr int Q_ROWS = 16 * Q_NT * P3_WAVES;       // rows per workgroup
constexpr int Q_NBUF = 4;                          // split-bf16 weight ring depth

template <int T, int K, int ACT, bool HV>
__global__ void __launch_bounds__(64 * P3_WAVES, 1) phaseA2_kernel(FusedArgs p);
template <int T, int K, int ACT, bool HV>
__global__ void __launch_bounds__(64 * P3_WAVES, 1) phaseC2_kernel(FusedArgs p);

// the instantiations phase2.hip builds (its own translation unit, compiled in
// parallel with engine.hip)
#define DBSDE_PHASE2_INSTANCES(X) \
  X(7, 3, 0, true) X(7, 3, 0, false) X(7, 3, 1, true) X(7, 3, 1, false) X(7, 3, 2, true) X(7, 3, 2, false)
#define DBSDE_PHASE2_EXTERN(T, K, ACT, HV)                                  \
  extern template __global__ void phaseA2_kernel<T, K, ACT, HV>(FusedArgs); \
  extern template __global__ void phaseC2_kernel<T, K, ACT, HV>(FusedArgs);
DBSDE_PHASE2_INSTANCES(DBSDE_PHASE2_EXTERN)
#undef DBSDE_PHASE2_EXTERN

}  // namespace dbsde
