// Probe: verify the lane layout of v_mfma_f64_16x16x4_f64 on gfx950 and
// measure fp64 MFMA / VALU / transcendental throughput on one CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef double double4_t __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(const double* A, const double* B, double* D) {
  // A: 16x4 row-major, B: 4x16 row-major, D: 16x16 row-major
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  double4_t c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    // hypothesis: col = l&15, row = (l>>4) + 4*r  ... store raw for host check
    D[(l * 4) + r] = c[r];
  }
}

__global__ void mfma_rate(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double4_t c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

__global__ void fma_rate(double* out, int iters) {
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
  double x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  const double m = 0.999999, a = 1e-7;
  for (int i = 0; i < iters; ++i) {
    x0 = fma(x0, m, a); x1 = fma(x1, m, a); x2 = fma(x2, m, a); x3 = fma(x3, m, a);
    x4 = fma(x4, m, a); x5 = fma(x5, m, a); x6 = fma(x6, m, a); x7 = fma(x7, m, a);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

__global__ void trans_rate(double* out, int iters) {
  double x = threadIdx.x * 1e-3 + blockIdx.x * 1e-6, acc = 0;
  for (int i = 0; i < iters; ++i) {
    double s, c;
    sincos(x, &s, &c);
    acc += exp(-x) * c + s;
    x += 1e-3;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  double hA[64], hB[64], hD[256];
  for (int i = 0; i < 64; ++i) { hA[i] = (i * 7 % 13) - 6; hB[i] = (i * 5 % 11) - 5 + 0.5 * (i % 3); }
  double *dA, *dB, *dD;
  hipMalloc(&dA, 64 * 8); hipMalloc(&dB, 64 * 8); hipMalloc(&dD, 256 * 8);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  layout_kernel<<<1, 64>>>(dA, dB, dD);
  hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
  double ref[256];
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
    double s = 0; for (int k = 0; k < 4; ++k) s += hA[i * 4 + k] * hB[k * 16 + j];
    ref[i * 16 + j] = s;
  }
  // test hypotheses
  int bad1 = 0, bad2 = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    double v = hD[l * 4 + r];
    int col = l & 15;
    int row1 = (l >> 4) + 4 * r;      // guide
    int row2 = (l >> 4) * 4 + r;      // f32-style
    if (v != ref[row1 * 16 + col]) bad1++;
    if (v != ref[row2 * 16 + col]) bad2++;
  }
  printf("layout: guide(row=(l>>4)+4r) mismatches=%d ; f32-style(row=4(l>>4)+r) mismatches=%d\n", bad1, bad2);

  double* dout; hipMalloc(&dout, 1 << 24);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int cus = 256;
  for (int rep = 0; rep < 2; ++rep) {
    int iters = 4096;
    hipEventRecord(e0);
    mfma_rate<<<cus * 4, 256>>>(dout, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = (double)cus * 4 * 4 * iters * 4 * 2048.0;
    printf("mfma f64 16x16x4: %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
    hipEventRecord(e0);
    fma_rate<<<cus * 4, 256>>>(dout, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    flops = (double)cus * 4 * 256 * iters * 8 * 2.0;
    printf("v_fma_f64: %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
    int titers = 256;
    hipEventRecord(e0);
    trans_rate<<<cus * 4, 256>>>(dout, titers);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double evals = (double)cus * 4 * 256 * titers;
    printf("exp+sincos f64: %.3f ms  %.3f G(exp+sincos)/s\n", ms, evals / ms / 1e6);
  }
  // launch latency: empty kernel chain
  hipEventRecord(e0);
  for (int i = 0; i < 1000; ++i) fma_rate<<<256, 64>>>(dout, 1);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("1000 tiny dependent launches: %.3f us each\n", ms);
  return 0;
}
