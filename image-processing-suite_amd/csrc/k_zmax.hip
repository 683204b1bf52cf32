// a5: z max-projection (MaxProjection.py:45, np.maximum.reduce(images) on uint16 planes).
// Pure streaming: Z x 2 B read + 2 B written per pixel; 16 B (8 px) per lane per load.
#include "cpx_internal.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ unsigned int max_u16x2(unsigned int a, unsigned int b) {
  unsigned int lo = max(a & 0xffffu, b & 0xffffu);
  unsigned int hi = max(a >> 16, b >> 16);
  return lo | (hi << 16);
}

__global__ __launch_bounds__(kThreads) void k_zmax_vec(const uint4* __restrict__ src, int Z,
                                                        long long n8, uint4* __restrict__ out,
                                                        int G) {
  const long long total = n8 * G;
  for (long long t = (long long)blockIdx.x * kThreads + threadIdx.x; t < total;
       t += (long long)gridDim.x * kThreads) {
    const long long g = t / n8, v = t - g * n8;
    const uint4* s = src + g * Z * n8 + v;
    uint4 m = s[0];
    for (int z = 1; z < Z; ++z) {
      uint4 x = s[(long long)z * n8];
      m.x = max_u16x2(m.x, x.x);
      m.y = max_u16x2(m.y, x.y);
      m.z = max_u16x2(m.z, x.z);
      m.w = max_u16x2(m.w, x.w);
    }
    out[g * n8 + v] = m;
  }
}

__global__ __launch_bounds__(kThreads) void k_zmax_scalar(const unsigned short* __restrict__ src,
                                                           int Z, long long N,
                                                           unsigned short* __restrict__ out, int G) {
  const long long total = N * G;
  for (long long t = (long long)blockIdx.x * kThreads + threadIdx.x; t < total;
       t += (long long)gridDim.x * kThreads) {
    const long long g = t / N, i = t - g * N;
    const unsigned short* s = src + g * Z * N + i;
    unsigned short m = s[0];
    for (int z = 1; z < Z; ++z) m = max(m, s[(long long)z * N]);
    out[g * N + i] = m;
  }
}

}  // namespace

extern "C" int cpx_zmax_u16(cpx_ctx* ctx, const uint16_t* src_dev, int G, int Z, int64_t N,
                            uint16_t* out_dev) {
  CPX_REQUIRE(ctx && src_dev && out_dev, CPX_ERR_ARG, "cpx_zmax_u16: null argument");
  CPX_REQUIRE(G > 0 && Z > 0 && N > 0, CPX_ERR_ARG, "cpx_zmax_u16: bad sizes G=%d Z=%d N=%lld", G,
              Z, (long long)N);
  const bool vec = (N % 8 == 0) && ((uintptr_t)src_dev % 16 == 0) && ((uintptr_t)out_dev % 16 == 0);
  const long long work = vec ? (N / 8) * G : N * G;
  int grid = (int)std::min<long long>((work + kThreads - 1) / kThreads, (long long)ctx->n_cu * 8);
  if (grid < 1) grid = 1;
  if (vec)
    hipLaunchKernelGGL(k_zmax_vec, dim3(grid), dim3(kThreads), 0, ctx->stream,
                       (const uint4*)src_dev, Z, (long long)(N / 8), (uint4*)out_dev, G);
  else
    hipLaunchKernelGGL(k_zmax_scalar, dim3(grid), dim3(kThreads), 0, ctx->stream,
                       (const unsigned short*)src_dev, Z, (long long)N, (unsigned short*)out_dev, G);
  CPX_CHECK_LAUNCH("k_zmax");
  return CPX_OK;
}
