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
// The same kernels with one tile per wave and 48 KiB pieces serve the FC
// width-256 network of config 4 (hjb_implement.py:590-604), where one 16-row
// tile already fills the register file (a level is 64 VGPRs per lane).
//
// Phase A keeps no act'(a_j) registers (they would need 224 per wave): the
// backward reloads a_j from Abuf, which it wrote a few stages earlier, and
// recomputes act'(a_j) -- the same reload phase C makes.
#pragma once
#include "phase.hpp"

namespace dbsde {

// Template parameters of the phase2 kernels:
//   T, TD   level / state width in 16-column blocks (T != TD: runtime piece
//           tables, pieces of 3 TO fragments for the stage's TO)
//   K, ACT, HV  as phase.hpp
//   NT      16-row register tiles per wave (rows per workgroup 64 NT)
//   NBUF    LDS ring depth in pieces of 3 max(T, TD) KiB
//   ADOT    phase C keeps adot_j in memory (Adot, tile order) between the
//           tangent and the reverse instead of registers (wide levels), and
//           runs the x-stack products level by level (no X-first order)
template <int T, int TD, int K, int ACT, bool HV, int NT, int NBUF, bool ADOT>
__global__ void __launch_bounds__(64 * P3_WAVES, 1) phaseA2_kernel(FusedArgs p);
template <int T, int TD, int K, int ACT, bool HV, int NT, int NBUF, bool ADOT>
__global__ void __launch_bounds__(64 * P3_WAVES, 1) phaseC2_kernel(FusedArgs p);

// the instantiations phase2.hip builds (its own translation unit, compiled in
// parallel with engine.hip): config 4's FC [101,256x4,1] and config 1's FC
// [2,256x4,1] (call_option_1d.py), one tile per wave, 48 KiB pieces, adot
// through memory.  (The width-112 networks with two tiles
// per wave, X(7, 7, 3, ACT, HV, 2, 4, ADOT), measured slower than phase.hpp's
// two 4-wave workgroups per CU: 0.386 / 0.406 ms against 0.293 ms for the
// phase section at the north star)
#define DBSDE_PHASE2_INSTANCES(X)                                                                   \
  X(16, 7, 3, 0, false, 1, 3, true) X(16, 7, 3, 1, false, 1, 3, true) X(16, 7, 3, 2, false, 1, 3, true) \
  X(16, 1, 3, 0, false, 1, 3, true) X(16, 1, 3, 1, false, 1, 3, true) X(16, 1, 3, 2, false, 1, 3, true)
#define DBSDE_PHASE2_EXTERN(T, TD, K, ACT, HV, NT, NBUF, ADOT)                                   \
  extern template __global__ void phaseA2_kernel<T, TD, K, ACT, HV, NT, NBUF, ADOT>(FusedArgs); \
  extern template __global__ void phaseC2_kernel<T, TD, K, ACT, HV, NT, NBUF, ADOT>(FusedArgs);
DBSDE_PHASE2_INSTANCES(DBSDE_PHASE2_EXTERN)
#undef DBSDE_PHASE2_EXTERN

}  // namespace dbsde
