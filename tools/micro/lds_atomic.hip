// Micro-benchmark: LDS atomic add throughput on gfx950 for several address patterns.
// hipcc --offload-arch=gfx950 -O3 lds_atomic.hip -o lds_atomic && ./lds_atomic
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE, bool RET>
__global__ __launch_bounds__(1024) void k(unsigned int* out, int iters, unsigned int seed) {
  __shared__ unsigned int tab[32768];
  for (int i = threadIdx.x; i < 32768; i += 1024) tab[i] = 0;
  __syncthreads();
  unsigned int x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  unsigned int acc = 0;
  const int lane = threadIdx.x & 63;
  for (int it = 0; it < iters; ++it) {
    unsigned int a;
    x = x * 1664525u + 1013904223u;
    if (MODE == 0) a = (threadIdx.x + it * 1024) & 32767;            // lane-linear, no conflict
    else if (MODE == 1) a = (x >> 8) & 32767;                         // random
    else if (MODE == 2) a = (threadIdx.x >> 6) * 64 + (it & 7);       // whole wave one address
    else a = ((x >> 8) & 3) * 64 + lane;                              // 4 lanes per bank... (lane-distinct)
    if (RET) acc += atomicAdd(&tab[a], 1u);
    else atomicAdd(&tab[a], 1u);
  }
  __syncthreads();
  if (RET) out[blockIdx.x * 1024 + threadIdx.x] = acc;
  else out[blockIdx.x * 1024 + threadIdx.x] = tab[threadIdx.x];
}

template <int MODE, bool RET>
void run(unsigned int* d, const char* name) {
  const int iters = 4096, blocks = 256 * 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((k<MODE, RET>), dim3(blocks), dim3(1024), 0, 0, d, iters, 1u);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<MODE, RET>), dim3(blocks), dim3(1024), 0, 0, d, iters, 2u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  // wave-instructions per CU: blocks/256 CUs * 16 waves * iters
  const double winstr = (double)blocks / 256 * 16 * iters;
  const double cyc = ms * 1e-3 * 2.4e9;
  printf("%-28s %s: %.2f ms, %.2f CU-cycles per wave-atomic\n", name, RET ? "rtn " : "nort", ms, cyc / winstr);
}

int main() {
  unsigned int* d;
  hipMalloc(&d, 256 * 4 * 1024 * 4);
  run<0, true>(d, "lane-linear");
  run<0, false>(d, "lane-linear");
  run<1, true>(d, "random 32K words");
  run<1, false>(d, "random 32K words");
  run<2, true>(d, "same address per wave");
  run<2, false>(d, "same address per wave");
  run<3, true>(d, "4-way bank (distinct addr)");
  run<3, false>(d, "4-way bank (distinct addr)");
  hipFree(d);
  return 0;
}
