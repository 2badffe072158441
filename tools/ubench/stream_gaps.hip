// stream_gaps.hip -- queue cost of the step's stream structure, eager vs
// captured graph.  Spin kernels of fixed duration stand in for the step's
// launches (durations from the round-5 kernel trace, us):
//   main : rtr(7) pack(6) [record fork] [wait roll] A0(110) C0(120) tnw0(140) [wait join] fin(15) projb(13)
//   pipe2: [wait fork] A1(110) C1(120) tnw1(140) [record join]
//   pf   : [wait fork] roll(37) [record roll]   (the next step's paths)
// Variants: eager (as the engine issues it), graph (one iteration captured and
// replayed), and eager without the roll wait (one event wait fewer on main).
//   hipcc -O3 --offload-arch=gfx950 -o stream_gaps stream_gaps.hip && ./stream_gaps
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// every workgroup spins `ticks` of the 100 MHz constant clock, then writes
// one word (vector store) so the kernel has an observable effect
__global__ void spin(unsigned long long ticks, int* out) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

struct Ctx {
  hipStream_t s, p2, pf;
  hipEvent_t fork, join, roll;
  int* buf;
  unsigned* flag;     // stream memory-op variant: [0] fork, [1] join
  unsigned epoch = 0;
  bool memops = false;
};

static void k(hipStream_t s, int grid, double us, int* buf) {
  hipLaunchKernelGGL(spin, dim3(grid), dim3(256), 0, s, (unsigned long long)(us * 100.0), buf);
}

// one step; roll_wait: main waits for the previous step's roll before A0
static void step(Ctx& c, bool roll_wait, bool first) {
  k(c.s, 64, 7, c.buf);     // rtr
  k(c.s, 64, 6, c.buf);     // pack
  ++c.epoch;
  if (c.memops) {
    CK(hipStreamWriteValue32(c.s, c.flag, c.epoch, 0));
    CK(hipStreamWaitValue32(c.p2, c.flag, c.epoch, hipStreamWaitValueGte, 0xFFFFFFFFu));
    CK(hipStreamWaitValue32(c.pf, c.flag, c.epoch, hipStreamWaitValueGte, 0xFFFFFFFFu));
  } else {
    CK(hipEventRecord(c.fork, c.s));
    CK(hipStreamWaitEvent(c.p2, c.fork, 0));
    CK(hipStreamWaitEvent(c.pf, c.fork, 0));
  }
  if (roll_wait && !first) CK(hipStreamWaitEvent(c.s, c.roll, 0));
  k(c.pf, 100, 37, c.buf);  // roll (next step)
  CK(hipEventRecord(c.roll, c.pf));
  k(c.s, 256, 110, c.buf);  // A0
  k(c.p2, 256, 110, c.buf); // A1
  k(c.s, 256, 120, c.buf);  // C0
  k(c.p2, 256, 120, c.buf); // C1
  k(c.s, 256, 140, c.buf);  // tnw0
  k(c.p2, 256, 140, c.buf); // tnw1
  if (c.memops) {
    CK(hipStreamWriteValue32(c.p2, c.flag + 1, c.epoch, 0));
    CK(hipStreamWaitValue32(c.s, c.flag + 1, c.epoch, hipStreamWaitValueGte, 0xFFFFFFFFu));
  } else {
    CK(hipEventRecord(c.join, c.p2));
    CK(hipStreamWaitEvent(c.s, c.join, 0));
  }
  k(c.s, 441, 15, c.buf);   // fin
  k(c.s, 64, 13, c.buf);    // projb
}

// argv[1]: 0 = events (DisableTiming), 1 = + DisableSystemFence, 2 = stream memory ops
int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  Ctx c;
  c.memops = mode == 2;
  const unsigned evf = hipEventDisableTiming | (mode == 1 ? hipEventDisableSystemFence : 0);
  printf("mode %d\n", mode);
  CK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c.p2, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c.pf, hipStreamNonBlocking));
  CK(hipEventCreateWithFlags(&c.fork, evf));
  CK(hipEventCreateWithFlags(&c.join, evf));
  CK(hipEventCreateWithFlags(&c.roll, evf));
  CK(hipMalloc(&c.buf, 4096 * sizeof(int)));
  CK(hipMalloc(&c.flag, 64));
  CK(hipMemset(c.flag, 0, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 200;
  const double ideal = 7 + 6 + 110 + 120 + 140 + 15 + 13;
  for (int rep = 0; rep < 1; ++rep) {
    for (int v = 0; v < 2; ++v) {   // eager with / without the roll wait
      for (int i = 0; i < 20; ++i) step(c, v == 0, i == 0);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, c.s));
      for (int i = 0; i < iters; ++i) step(c, v == 0, false);
      CK(hipEventRecord(e1, c.s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("eager%s  %.1f us/step (ideal %.0f)\n", v == 0 ? "         " : " no-rollw", 1e3 * ms / iters, ideal);
    }
    // graph: capture one step (fork/join through the events), replay
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipDeviceSynchronize());
    CK(hipStreamBeginCapture(c.s, hipStreamCaptureModeGlobal));
    step(c, false, true);   // within one capture the roll is produced, then joined at the end
    CK(hipStreamWaitEvent(c.s, c.roll, 0));
    CK(hipStreamEndCapture(c.s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, c.s));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, c.s));
    for (int i = 0; i < iters; ++i) CK(hipGraphLaunch(ge, c.s));
    CK(hipEventRecord(e1, c.s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("graph (%zu nodes) %.1f us/step (ideal %.0f)\n", nn, 1e3 * ms / iters, ideal);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    // single stream, no events at all (the serial lower bound of the same launches: A0 A1 C0 C1 ...)
    for (int pass = 0; pass < 2; ++pass) {
      CK(hipDeviceSynchronize());
      if (pass) CK(hipEventRecord(e0, c.s));
      for (int i = 0; i < (pass ? iters : 20); ++i) {
        k(c.s, 64, 7, c.buf);
        k(c.s, 64, 6, c.buf);
        k(c.s, 512, 110, c.buf);
        k(c.s, 512, 120, c.buf);
        k(c.s, 512, 140, c.buf);
        k(c.s, 441, 15, c.buf);
        k(c.s, 64, 13, c.buf);
      }
      if (pass) {
        CK(hipEventRecord(e1, c.s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("one stream, merged chunks %.1f us/step (ideal %.0f)\n", 1e3 * ms / iters, ideal);
      }
    }
  }
  return 0;
}
