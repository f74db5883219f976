// gap_probe.hip -- per-kernel cost of back-to-back dependent kernels (stream launches and one
// captured graph), as a function of the bytes each kernel writes: tells a fixed launch gap from
// a kernel-boundary cost that grows with dirty L2 lines.
//   hipcc --offload-arch=gfx950 -O3 gap_probe.hip -o gap_probe && ./gap_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void write_kernel(double* __restrict__ p, size_t n, double v) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = v + (double)i;
}

int main() {
  const int NK = 20, REPS = 50;
  const size_t sizes[] = {0, 64 << 10, 512 << 10, 4 << 20, 32 << 20};
  double* buf;
  CK(hipMalloc(&buf, (size_t)64 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (size_t bytes : sizes) {
    const size_t n = bytes / 8;
    const int grid = n == 0 ? 1 : (int)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024);
    auto enqueue = [&]() {
      for (int k = 0; k < NK; ++k)
        hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(256), 0, s, buf + (k & 1) * ((size_t)4 << 20), n, (double)k);
    };
    // stream launches
    enqueue();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < REPS; ++r) enqueue();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms_stream;
    CK(hipEventElapsedTime(&ms_stream, e0, e1));
    // one graph of NK kernels
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    enqueue();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < REPS; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms_graph;
    CK(hipEventElapsedTime(&ms_graph, e0, e1));
    printf("bytes/kernel %9zu grid %5d: stream %.2f us/kernel, graph %.2f us/kernel\n", bytes, grid,
           1e3 * ms_stream / (REPS * NK), 1e3 * ms_graph / (REPS * NK));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipFree(buf));
  return 0;
}
