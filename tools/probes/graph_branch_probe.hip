// Probe: do independent branches of a captured hipGraph (fork/join via events on a second
// stream) run concurrently on gfx950?  Two single-workgroup kernels that each spin ~50 us.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__global__ void spin(long long cycles, int* out) {
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

int main() {
  int* d; CHK(hipMalloc(&d, 4096));
  hipStream_t s1, s2; CHK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CHK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, join, e0, e1; CHK(hipEventCreateWithFlags(&fork, hipEventDisableTiming)); CHK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const long long cyc = 100000;  // clock64 ~ 100 MHz constant clock? measured below
  // single kernel time
  for (int mode = 0; mode < 3; ++mode) {
    hipGraph_t g; hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    if (mode == 0) {
      spin<<<1, 64, 0, s1>>>(cyc, d);
    } else if (mode == 1) {  // serial pair
      spin<<<1, 64, 0, s1>>>(cyc, d);
      spin<<<1, 64, 0, s1>>>(cyc, d + 1);
    } else {                 // forked pair
      CHK(hipEventRecord(fork, s1));
      CHK(hipStreamWaitEvent(s2, fork, 0));
      spin<<<1, 64, 0, s1>>>(cyc, d);
      spin<<<1, 64, 0, s2>>>(cyc, d + 1);
      CHK(hipEventRecord(join, s2));
      CHK(hipStreamWaitEvent(s1, join, 0));
    }
    CHK(hipStreamEndCapture(s1, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(ge, s1)); CHK(hipStreamSynchronize(s1));
    CHK(hipEventRecord(e0, s1));
    for (int i = 0; i < 20; ++i) CHK(hipGraphLaunch(ge, s1));
    CHK(hipEventRecord(e1, s1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("mode %d (%s): %.1f us per graph\n", mode, mode == 0 ? "one kernel" : mode == 1 ? "serial pair" : "forked pair", ms * 1000 / 20);
  }
  // eager two-stream concurrency
  CHK(hipEventRecord(e0, s1));
  for (int i = 0; i < 20; ++i) {
    CHK(hipEventRecord(fork, s1)); CHK(hipStreamWaitEvent(s2, fork, 0));
    spin<<<1, 64, 0, s1>>>(cyc, d); spin<<<1, 64, 0, s2>>>(cyc, d + 1);
    CHK(hipEventRecord(join, s2)); CHK(hipStreamWaitEvent(s1, join, 0));
  }
  CHK(hipEventRecord(e1, s1)); CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  printf("eager forked pair: %.1f us per iteration\n", ms * 1000 / 20);
  return 0;
}
