// clockstamp.hip -- diagnostic only (tools/clock_probe.py): the shader clock
// at one moment of a stream, measured in a kernel.  One wave reads
// s_memrealtime (100 MHz) and s_memtime (shader cycles), spins until 2 us of
// real time have passed (bounded: at most 1e6 trips), reads both again and
// stores the two deltas with a vector store: clock MHz = 100 * dcycles /
// dreal.  Launched between the steps of the bench loop, it reads the clock
// the chip holds at that point of the run (MI355X_MICROARCH.md, DVFS item 6).
#include <hip/hip_runtime.h>

__global__ void __launch_bounds__(64) clockstamp_kernel(unsigned long long* out, int slot) {
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = r0, c1 = c0;
  for (int it = 0; it < 1000000 && r1 - r0 < 200; ++it) {
    r1 = __builtin_amdgcn_s_memrealtime();
    c1 = __builtin_amdgcn_s_memtime();
  }
  if (threadIdx.x == 0) {
    out[2 * slot] = c1 - c0;
    out[2 * slot + 1] = r1 - r0;
  }
}

extern "C" int clockstamp_launch(void* out, int slot, void* stream) {
  clockstamp_kernel<<<1, 64, 0, (hipStream_t)stream>>>((unsigned long long*)out, slot);
  return (int)hipGetLastError();
}
