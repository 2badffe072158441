// phasecs.hpp -- column-split phase kernels for small path counts (gfx950).
//
// The kernels of phase.hpp give each wave its own 16 rows, so a 4-wave
// workgroup covers 64 rows and a step of M paths has M (N + 1) / 64
// workgroups.  At the per-rank shapes of strong scaling (M = 128 / 256 paths
// per GPU: 102 / 204 workgroups on 256 CUs) the chip is mostly idle and the
// step time is one workgroup's serial chain of 56 weight pieces.
//
// Here the four waves of a workgroup share the SAME 16 rows and split each
// layer's output blocks: wave w computes output fragments 2w, 2w + 1 (the
// last wave one, at width 112), i.e. 12 of a piece's 42 split-bf16 MFMAs.
// The staged weight pieces, their order and the LDS-DMA ring are those of
// phase.hpp (the same host images); a wave just reads its two fragments of
// each piece.  A layer's full input (h_j, delta_j, hdot_j, alpha_j) is
// assembled through a 7 KiB LDS exchange: each wave writes its output
// fragments in the B-operand register layout, the next piece's barrier
// publishes them, and every wave reads all seven back.  4x the workgroups,
// 2/7 of the MFMA chain per wave, so the step's critical path shrinks ~3.5x
// when the 64-row kernels cannot fill the chip.
//
// Cross-wave sums (u = h_{K+1} . w_out, the residual row sums over the Z
// columns) go through a small LDS area in a fixed order.
#pragma once
#include "phase.hpp"

namespace dbsde {

constexpr int CS_ROWS = 16;   // rows per workgroup

template <int T, int TD, int K, int ACT, bool HV>
__global__ void __launch_bounds__(64 * P3_WAVES, 2) phaseAcs_kernel(FusedArgs p);
template <int T, int TD, int K, int ACT, bool HV>
__global__ void __launch_bounds__(64 * P3_WAVES, 2) phaseCcs_kernel(FusedArgs p);

// the instantiations phasecs.hip builds: the width-112 split-bf16 networks
// (NAIS-Net / Naisnet with the x-stack, FC / Resnet without) x 3 activations
#define DBSDE_PHASECS_INSTANCES(X) \
  X(7, 7, 3, 0, true) X(7, 7, 3, 1, true) X(7, 7, 3, 2, true) X(7, 7, 3, 0, false) X(7, 7, 3, 1, false) X(7, 7, 3, 2, false)
#define DBSDE_PHASECS_EXTERN(T, TD, K, ACT, HV)                                   \
  extern template __global__ void phaseAcs_kernel<T, TD, K, ACT, HV>(FusedArgs); \
  extern template __global__ void phaseCcs_kernel<T, TD, K, ACT, HV>(FusedArgs);
DBSDE_PHASECS_INSTANCES(DBSDE_PHASECS_EXTERN)
#undef DBSDE_PHASECS_EXTERN

}  // namespace dbsde
