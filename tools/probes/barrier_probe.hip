// Probe: cost of a dependent kernel boundary (graph of empty kernels) vs a device-wide barrier
// inside one persistent kernel (256 WGs, agent-scope fences, cross-XCD data hand-off checked).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__global__ void empty_kernel(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

__global__ void tiny_work(double* buf, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) buf[i] = buf[i] * 1.0000001 + 1.0;
}

struct Bar {
  unsigned int count;
  unsigned int gen;
};

__device__ __forceinline__ void grid_barrier(Bar* b, unsigned int nblocks, unsigned int& my_gen) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();  // release this WG's writes (agent scope: L2 writeback across XCDs)
    const unsigned int g = my_gen;
    const unsigned int old = atomicAdd(&b->count, 1u);
    if (old == nblocks - 1) {
      b->count = 0;
      __threadfence();
      atomicAdd(&b->gen, 1u);
    } else {
      while (__hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __threadfence();  // acquire
  }
  my_gen++;
  __syncthreads();
}

// each phase: WG b writes its 512-double slot; after the barrier it reads slot (b+37)%nb and
// checks the value written in this phase
__global__ void persistent(Bar* bar, double* data, int phases, int* errors) {
  const unsigned int nb = gridDim.x;
  unsigned int my_gen = 0;
  if (threadIdx.x == 0) my_gen = __hip_atomic_load(&bar->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  __shared__ unsigned int sg;
  if (threadIdx.x == 0) sg = my_gen;
  __syncthreads();
  my_gen = sg;
  for (int ph = 0; ph < phases; ++ph) {
    double* mine = data + (size_t)blockIdx.x * 512;
    for (int i = threadIdx.x; i < 512; i += blockDim.x) mine[i] = ph * 1000.0 + blockIdx.x + i * 1e-3;
    grid_barrier(bar, nb, my_gen);
    const int other = (blockIdx.x + 37) % nb;
    const double* o = data + (size_t)other * 512;
    int bad = 0;
    for (int i = threadIdx.x; i < 512; i += blockDim.x) bad += (o[i] != ph * 1000.0 + other + i * 1e-3);
    if (bad) atomicAdd(errors, bad);
    grid_barrier(bar, nb, my_gen);
  }
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  printf("%s CUs %d\n", prop.name, prop.multiProcessorCount);
  int* p;
  CHK(hipMalloc(&p, 64));
  CHK(hipMemset(p, 0, 64));
  hipStream_t s;
  CHK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int NK = 200;
  const int grid = prop.multiProcessorCount;
  for (int variant = 0; variant < 2; ++variant) {
    hipGraph_t g;
    hipGraphExec_t ge;
    double* buf;
    CHK(hipMalloc(&buf, sizeof(double) * 65536));
    CHK(hipMemset(buf, 0, sizeof(double) * 65536));
    CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < NK; ++k) {
      if (variant == 0)
        hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, s, p);
      else
        hipLaunchKernelGGL(tiny_work, dim3(256), dim3(256), 0, s, buf, 65536);
    }
    CHK(hipStreamEndCapture(s, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(ge, s));
    CHK(hipStreamSynchronize(s));
    CHK(hipEventRecord(e0, s));
    for (int r = 0; r < 5; ++r) CHK(hipGraphLaunch(ge, s));
    CHK(hipEventRecord(e1, s));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("graph of %d %s kernels (%d WGs): %.3f us per kernel\n", NK, variant ? "tiny-work" : "empty",
           grid, ms * 1000.0 / (5 * NK));
  }
  Bar* bar;
  CHK(hipMalloc(&bar, sizeof(Bar)));
  CHK(hipMemset(bar, 0, sizeof(Bar)));
  double* data;
  CHK(hipMalloc(&data, sizeof(double) * 512 * grid));
  int* err;
  CHK(hipMalloc(&err, sizeof(int)));
  CHK(hipMemset(err, 0, sizeof(int)));
  int nbper = 0;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nbper, persistent, 256, 0));
  printf("persistent occupancy %d blocks/CU\n", nbper);
  const int PH = 500;
  void* args[] = {&bar, &data, (void*)&PH, &err};
  int phases = PH;
  args[2] = &phases;
  CHK(hipLaunchCooperativeKernel((void*)persistent, dim3(grid), dim3(256), args, 0, s));
  CHK(hipStreamSynchronize(s));
  CHK(hipEventRecord(e0, s));
  CHK(hipLaunchCooperativeKernel((void*)persistent, dim3(grid), dim3(256), args, 0, s));
  CHK(hipEventRecord(e1, s));
  CHK(hipEventSynchronize(e1));
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  int herr = -1;
  CHK(hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost));
  printf("persistent: %d barriers in %.3f us -> %.3f us per barrier (incl. 4 KB write/read per WG), errors %d\n",
         2 * PH, ms * 1000.0, ms * 1000.0 / (2 * PH), herr);
  return 0;
}
