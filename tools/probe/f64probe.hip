#include <hip/hip_runtime.h>
#include <cstdio>
template <int OP>
__global__ void k(double* out, int iters, double a, double b) {
  double x[8];
  unsigned u[8];
  for (int i = 0; i < 8; ++i) { x[i] = threadIdx.x + i; u[i] = threadIdx.x * 7 + i; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) x[i] = x[i] * a;
      if constexpr (OP == 1) x[i] = x[i] + a;
      if constexpr (OP == 2) x[i] = __builtin_fma(x[i], a, b);
      if constexpr (OP == 3) { x[i] += (double)u[i]; u[i] += 3; }
      if constexpr (OP == 4) { float f = (float)x[i]; x[i] = (double)(f * (float)a); }
    }
  }
  double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  double* d; hipMalloc(&d, 8 << 20);
  const int blocks = 256 * 8, thr = 256, iters = 4096;
  const char* names[] = {"mul_f64", "add_f64", "fma_f64", "cvt_f64_u32+add", "f32 mul + 2 cvt"};
  for (int op = 0; op < 5; ++op) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      switch (op) {
        case 0: k<0><<<blocks, thr>>>(d, iters, 1.0000001, 0.5); break;
        case 1: k<1><<<blocks, thr>>>(d, iters, 1.0000001, 0.5); break;
        case 2: k<2><<<blocks, thr>>>(d, iters, 1.0000001, 0.5); break;
        case 3: k<3><<<blocks, thr>>>(d, iters, 1.0000001, 0.5); break;
        case 4: k<4><<<blocks, thr>>>(d, iters, 1.0000001, 0.5); break;
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double winst = (double)blocks * thr / 64 * iters * 8;  // wave-instructions of the op
    printf("%-18s %.3f ms  %.2f G wave-inst/s  cycles/wave-inst/SIMD @2.4GHz = %.2f\n", names[op], ms,
           winst / ms / 1e6, 1024.0 * 2.4e9 / (winst / ms * 1e3));
  }
  return 0;
}
