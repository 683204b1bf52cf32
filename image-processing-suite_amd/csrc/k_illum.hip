// a1 + a4: flat-field illumination correction fused with the PercentMaximal statistics.
//
// Reference arithmetic restated:
//   Illumination_QC_mult.py:145   img = tifffile.imread(path).astype(float)     (uint16 -> f64)
//   Illumination_QC_mult.py:148-150  img = img / illum_cache[i]   (f64 / illum dtype -> f64)
//   Illumination_QC_mult.py:73-95 calculate_saturation_cp_exact: 100*count(px == max)/n
//   Cellpose_GPU_s3fs.py:72       tifffile.imread(path) / channel_correction[n]
//                                 (numpy promotion: uint16 / float32 -> float32)
// One pass over HBM: read raw u16 (2 B/px) + illum (4 B/px, L2/MALL-resident across FOVs),
// write the fp32 corrected plane (4 B/px), and reduce {max, count(max), min, sum, nan, inf} of
// the fp64 quotient per plane.  Reductions are fixed-order (per-block partials -> one
// finishing block per plane), so results are bit-reproducible run to run.
#include "cpx_internal.h"
#include <math.h>

namespace {

constexpr int kThreads = 256;
constexpr int kBlocksPerPlane = 64;

struct Partial {
  double max_q, min_q, sum_q;
  long long count_max;
  int has_nan, has_inf;
};

struct Acc {
  double m;      // running max
  long long c;   // count of m
  double mn;     // running min
  double s;      // sum
  int nan, inf;
  __device__ void init() {
    m = -INFINITY;
    c = 0;
    mn = INFINITY;
    s = 0.0;
    nan = 0;
    inf = 0;
  }
  __device__ __forceinline__ void add(double v) {
    if (v != v) {  // NaN: np.max -> NaN, and no pixel compares equal to NaN
      nan = 1;
      return;
    }
    if (isinf(v)) inf = 1;
    if (v > m) {
      m = v;
      c = 1;
    } else if (v == m) {
      c += 1;
    }
    mn = v < mn ? v : mn;
    s += v;
  }
  __device__ __forceinline__ void merge(double om, long long oc, double omn, double os, int onan,
                                        int oinf) {
    if (om > m) {
      m = om;
      c = oc;
    } else if (om == m) {
      c += oc;
    }
    mn = omn < mn ? omn : mn;
    s += os;
    nan |= onan;
    inf |= oinf;
  }
};

__device__ __forceinline__ void wave_merge(Acc& a) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double om = __shfl_xor(a.m, off, 64);
    long long oc = __shfl_xor(a.c, off, 64);
    double omn = __shfl_xor(a.mn, off, 64);
    double os = __shfl_xor(a.s, off, 64);
    int onan = __shfl_xor(a.nan, off, 64);
    int oinf = __shfl_xor(a.inf, off, 64);
    a.merge(om, oc, omn, os, onan, oinf);
  }
}

// Quotient for one pixel.  ILLUM: 0 none, 1 f32, 2 f64, 3 = `illum` is the float64 image itself.
template <int ILLUM>
__device__ __forceinline__ void quot(unsigned short r, const void* illum, long long idx, double& q,
                                     float& f) {
  if (ILLUM == 1) {
    float il = static_cast<const float*>(illum)[idx];
    q = (double)r / (double)il;     // QC path: f64 / f32 -> f64 (exact operands)
    f = (float)r / il;              // producer path: u16 / f32 -> f32, correctly rounded
  } else if (ILLUM == 2) {
    double il = static_cast<const double*>(illum)[idx];
    q = (double)r / il;
    f = (float)q;                   // producer path would be f64; stored as fp32
  } else if (ILLUM == 3) {
    q = static_cast<const double*>(illum)[idx];
    f = (float)q;
  } else {
    q = (double)r;
    f = (float)r;
  }
}

template <int ILLUM, bool VEC>
__global__ __launch_bounds__(kThreads) void k_illum_correct(const unsigned short* __restrict__ raw,
                                                             const void* __restrict__ illum, int C,
                                                             long long N, float* __restrict__ corr,
                                                             Partial* __restrict__ partials) {
  const int plane = blockIdx.y;
  const int ch = plane % C;
  const unsigned short* rp = raw + (long long)plane * N;
  float* cp = corr ? corr + (long long)plane * N : nullptr;
  const long long ibase = (long long)ch * N;
  Acc a;
  a.init();
  if (VEC) {
    // 8 pixels per thread-iteration: 16 B of raw, 32 B of illum (f32), 32 B of output.
    const long long n8 = N >> 3;
    const long long per_block = (n8 + gridDim.x - 1) / gridDim.x;
    const long long beg = per_block * blockIdx.x;
    const long long end = min(n8, beg + per_block);
    for (long long v = beg + threadIdx.x; v < end; v += kThreads) {
      uint4 rv = reinterpret_cast<const uint4*>(rp)[v];
      unsigned short r8[8];
      r8[0] = rv.x & 0xffff; r8[1] = rv.x >> 16; r8[2] = rv.y & 0xffff; r8[3] = rv.y >> 16;
      r8[4] = rv.z & 0xffff; r8[5] = rv.z >> 16; r8[6] = rv.w & 0xffff; r8[7] = rv.w >> 16;
      float f8[8];
      if (ILLUM == 1) {
        const float4* ip = reinterpret_cast<const float4*>(static_cast<const float*>(illum) + ibase);
        float4 i0 = ip[2 * v], i1 = ip[2 * v + 1];
        float il[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          double q = (double)r8[k] / (double)il[k];
          f8[k] = (float)r8[k] / il[k];
          a.add(q);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          double q;
          quot<ILLUM>(r8[k], illum, ibase + v * 8 + k, q, f8[k]);
          a.add(q);
        }
      }
      if (cp) {
        float4* op = reinterpret_cast<float4*>(cp);
        op[2 * v] = make_float4(f8[0], f8[1], f8[2], f8[3]);
        op[2 * v + 1] = make_float4(f8[4], f8[5], f8[6], f8[7]);
      }
    }
  } else {
    const long long per_block = (N + gridDim.x - 1) / gridDim.x;
    const long long beg = per_block * blockIdx.x;
    const long long end = min(N, beg + per_block);
    for (long long i = beg + threadIdx.x; i < end; i += kThreads) {
      double q;
      float f;
      quot<ILLUM>(rp[i], illum, ibase + i, q, f);
      a.add(q);
      if (cp) cp[i] = f;
    }
  }
  // block reduction: wave -> LDS -> wave 0 (fixed order)
  wave_merge(a);
  __shared__ Partial sp[kThreads / 64];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) sp[wid] = Partial{a.m, a.mn, a.s, a.c, a.nan, a.inf};
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc b;
    b.init();
    for (int w = 0; w < kThreads / 64; ++w)
      b.merge(sp[w].max_q, sp[w].count_max, sp[w].min_q, sp[w].sum_q, sp[w].has_nan, sp[w].has_inf);
    partials[(long long)plane * gridDim.x + blockIdx.x] = Partial{b.m, b.mn, b.s, b.c, b.nan, b.inf};
  }
}

__global__ void k_illum_finish(const Partial* __restrict__ partials, int nb, long long N,
                               cpx_plane_stats* __restrict__ stats) {
  const int plane = blockIdx.x;
  if (threadIdx.x != 0) return;
  Acc b;
  b.init();
  for (int i = 0; i < nb; ++i) {
    const Partial& p = partials[(long long)plane * nb + i];
    b.merge(p.max_q, p.count_max, p.min_q, p.sum_q, p.has_nan, p.has_inf);
  }
  cpx_plane_stats s;
  s.n = N;
  s.has_nan = b.nan;
  s.has_inf = b.inf;
  s.sum_q = b.nan ? NAN : b.s;
  s.max_q = b.nan ? NAN : b.m;
  s.min_q = b.nan ? NAN : b.mn;
  s.count_max = b.nan ? 0 : b.c;
  // calculate_saturation_cp_exact: 100.0 * float(count) / float(n); 0.0 for an empty plane
  s.pct_max = (N == 0) ? 0.0 : (100.0 * (double)s.count_max) / (double)N;
  s._pad = 0;
  stats[plane] = s;
}

}  // namespace

extern "C" int cpx_illum_correct(cpx_ctx* ctx, const uint16_t* raw_dev, const void* illum_dev,
                                 int illum_dtype, int C, int n_planes, int H, int W,
                                 float* corr_dev, cpx_plane_stats* stats_dev) {
  CPX_REQUIRE(ctx && raw_dev && stats_dev, CPX_ERR_ARG, "cpx_illum_correct: null argument");
  CPX_REQUIRE(C > 0 && n_planes > 0 && H > 0 && W > 0, CPX_ERR_ARG,
              "cpx_illum_correct: bad sizes C=%d n_planes=%d H=%d W=%d", C, n_planes, H, W);
  CPX_REQUIRE(illum_dtype == CPX_DTYPE_NONE || illum_dev != nullptr, CPX_ERR_ARG,
              "cpx_illum_correct: illum dtype %d without data", illum_dtype);
  CPX_REQUIRE(illum_dtype >= 0 && illum_dtype <= 3, CPX_ERR_ARG, "bad illum dtype %d", illum_dtype);
  CPX_REQUIRE(n_planes <= 65535, CPX_ERR_ARG, "cpx_illum_correct: too many planes");
  const long long N = (long long)H * W;
  const int nb = kBlocksPerPlane;
  Partial* partials = (Partial*)cpx_ws(ctx, WS_PARTIALS, sizeof(Partial) * (size_t)nb * n_planes);
  if (!partials) return CPX_ERR_OOM;
  dim3 grid(nb, n_planes);
  const bool vec = (N % 8 == 0) && ((uintptr_t)raw_dev % 16 == 0) &&
                   (corr_dev == nullptr || (uintptr_t)corr_dev % 16 == 0) &&
                   (illum_dtype != CPX_DTYPE_F32 || (uintptr_t)illum_dev % 16 == 0);
  const void* il = illum_dtype == CPX_DTYPE_NONE ? nullptr : illum_dev;
#define LAUNCH(IL, V) \
  hipLaunchKernelGGL((k_illum_correct<IL, V>), grid, dim3(kThreads), 0, ctx->stream, raw_dev, il, C, N, corr_dev, partials)
  if (vec) {
    if (illum_dtype == CPX_DTYPE_F32) LAUNCH(1, true);
    else if (illum_dtype == CPX_DTYPE_F64) LAUNCH(2, true);
    else if (illum_dtype == CPX_DTYPE_IMAGE_F64) LAUNCH(3, true);
    else LAUNCH(0, true);
  } else {
    if (illum_dtype == CPX_DTYPE_F32) LAUNCH(1, false);
    else if (illum_dtype == CPX_DTYPE_F64) LAUNCH(2, false);
    else if (illum_dtype == CPX_DTYPE_IMAGE_F64) LAUNCH(3, false);
    else LAUNCH(0, false);
  }
#undef LAUNCH
  CPX_CHECK_LAUNCH("k_illum_correct");
  hipLaunchKernelGGL(k_illum_finish, dim3(n_planes), dim3(64), 0, ctx->stream, partials, nb, N,
                     stats_dev);
  CPX_CHECK_LAUNCH("k_illum_finish");
  return CPX_OK;
}
