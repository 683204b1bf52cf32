// f3: the embedding consumer's preprocessing, Cellpose_GPU_s3fs.py:177-187 —
// every kept crop channel, already scale_to_8bit'ed by cpx_crops (crops8), goes through
// PIL L -> RGB -> transformers' TimmWrapperImageProcessor for timm/tf_efficientnetv2_l.in21k:
// Image.resize(D, BICUBIC) (Pillow's 8-bit fixed-point resampler, libImaging/Resample.c),
// CenterCrop(D) (identity for square crops), ToTensor (/255, fp32), Normalize((x-m)/s, fp32),
// and the model's fp16 autocast rounds the result to fp16.  R = G = B, so one plane is resampled
// and written three times.  Arithmetic restated in oracle/embed_oracle.py (pinned to Pillow).
//
// Two passes as Pillow: k_embed_h resamples the rows of every image (S x S -> S x D, 8-bit with
// clamp), k_embed_v the columns (S x D -> D x D) and writes the normalised fp16 planes.  Integer
// coefficients per output position (int32, 2^22 fixed point, <= 5 taps for bicubic upsampling)
// are computed on the host in fp64 exactly as Pillow does and cached per (S, D).
#include "cpx_internal.h"
#include <hip/hip_fp16.h>
#include <math.h>
#include <vector>

namespace {

constexpr int kPrec = 32 - 8 - 2;  // Pillow PRECISION_BITS
constexpr int kMaxTaps = 8;
constexpr int kRowsH = 8;          // source rows per k_embed_h block
constexpr int kRowsV = 4;          // output rows per k_embed_v block

struct Coeffs {
  const int* xmin;   // [D]
  const int* count;  // [D]
  const int* k;      // [D][kMaxTaps]
};

__device__ __forceinline__ int clip8(int ss) {
  const int v = ss >> kPrec;  // arithmetic shift: Pillow's lookup of ss >> PRECISION_BITS
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

__global__ __launch_bounds__(1024) void k_embed_h(const unsigned char* __restrict__ src,
                                                  const long long* __restrict__ idx, int S, int D,
                                                  Coeffs c, unsigned char* __restrict__ tmp) {
  extern __shared__ unsigned char rows[];  // kRowsH x S
  const int n = blockIdx.x;
  const int r0 = blockIdx.y * kRowsH;
  const int nr = min(kRowsH, S - r0);
  const unsigned char* img = src + idx[n] * (long long)S * S;
  for (int i = threadIdx.x; i < nr * S; i += blockDim.x) rows[i] = img[(long long)r0 * S + i];
  __syncthreads();
  for (int x = threadIdx.x; x < D; x += blockDim.x) {
    const int xm = c.xmin[x], cnt = c.count[x];
    const int* k = c.k + x * kMaxTaps;
    for (int r = 0; r < nr; ++r) {
      int ss = 1 << (kPrec - 1);
      for (int t = 0; t < cnt; ++t) ss += (int)rows[r * S + xm + t] * k[t];
      tmp[((long long)n * S + r0 + r) * D + x] = (unsigned char)clip8(ss);
    }
  }
}

__global__ __launch_bounds__(1024) void k_embed_v(const unsigned char* __restrict__ tmp, int S, int D,
                                                  Coeffs c, float mean, float stdv,
                                                  __half* __restrict__ out) {
  const int n = blockIdx.x;
  const int y0 = blockIdx.y * kRowsV;
  const long long plane = (long long)D * D;
  for (int x = threadIdx.x; x < D; x += blockDim.x) {
    for (int y = y0; y < min(D, y0 + kRowsV); ++y) {
      const int ym = c.xmin[y], cnt = c.count[y];
      const int* k = c.k + y * kMaxTaps;
      int ss = 1 << (kPrec - 1);
      for (int t = 0; t < cnt; ++t) ss += (int)tmp[((long long)n * S + ym + t) * D + x] * k[t];
      const float v = ((float)clip8(ss) / 255.0f - mean) / stdv;  // ToTensor, Normalize (fp32)
      const __half h = __float2half_rn(v);                         // autocast fp16
      __half* o = out + (long long)n * 3 * plane + (long long)y * D + x;
      o[0] = h;
      o[plane] = h;
      o[2 * plane] = h;
    }
  }
}

double bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// libImaging/Resample.c precompute_coeffs + normalize_coeffs_8bpc for one axis
bool coeffs_8bpc(int in, int out, int* xmin, int* count, int* k) {
  const double scale = (double)in / out;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  if ((int)ceil(support) * 2 + 1 > kMaxTaps) return false;
  const double ss = 1.0 / filterscale;
  for (int xx = 0; xx < out; ++xx) {
    const double center = (xx + 0.5) * scale;
    int x0 = (int)(center - support + 0.5);
    if (x0 < 0) x0 = 0;
    int x1 = (int)(center + support + 0.5);
    if (x1 > in) x1 = in;
    x1 -= x0;
    double w[kMaxTaps];
    double ww = 0.0;
    for (int x = 0; x < x1; ++x) {
      w[x] = bicubic((x + x0 - center + 0.5) * ss);
      ww += w[x];
    }
    for (int x = 0; x < kMaxTaps; ++x) {
      int v = 0;
      if (x < x1) {
        const double n = ww != 0.0 ? w[x] / ww : w[x];
        v = n < 0 ? (int)(-0.5 + n * (1 << kPrec)) : (int)(0.5 + n * (1 << kPrec));
      }
      k[xx * kMaxTaps + x] = v;
    }
    xmin[xx] = x0;
    count[xx] = x1;
  }
  return true;
}

}  // namespace

extern "C" int cpx_embed_preprocess(cpx_ctx* ctx, const uint8_t* crops8_dev, const int64_t* index_dev,
                                    int N, int S, int D, float mean, float stdv, void* out_dev) {
  CPX_REQUIRE(ctx && crops8_dev && index_dev && out_dev, CPX_ERR_ARG, "cpx_embed_preprocess: null argument");
  CPX_REQUIRE(N > 0 && N <= 65535 && S > 0 && S <= 4096 && D > 0 && D <= 4096 && stdv != 0.0f,
              CPX_ERR_ARG, "cpx_embed_preprocess: bad sizes");
  // coefficient table (both axes are S -> D), cached by (S, D)
  const size_t words = (size_t)D * (2 + kMaxTaps);
  int* tab = (int*)cpx_ws(ctx, WS_EMBED, words * sizeof(int) + (size_t)N * S * D + 256);
  if (!tab) return CPX_ERR_OOM;
  unsigned char* tmp = (unsigned char*)(tab + words) + (256 - (words * sizeof(int)) % 256) % 256;
  if (ctx->embed_key[0] != S || ctx->embed_key[1] != D || ctx->embed_gen != ctx->ws_gen[WS_EMBED]) {
    std::vector<int> h(words);
    CPX_REQUIRE(coeffs_8bpc(S, D, &h[0], &h[D], &h[2 * D]), CPX_ERR_ARG,
                "cpx_embed_preprocess: downscale factor too large");
    CPX_CHECK_HIP(hipMemcpyAsync(tab, h.data(), words * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
    CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    ctx->embed_key[0] = S;
    ctx->embed_key[1] = D;
    ctx->embed_gen = ctx->ws_gen[WS_EMBED];
  }
  Coeffs c{tab, tab + D, tab + 2 * D};
  const int th = std::min(1024, (D + 63) / 64 * 64);
  hipLaunchKernelGGL(k_embed_h, dim3(N, cpx_div_up(S, kRowsH)), dim3(th), kRowsH * S, ctx->stream,
                     (const unsigned char*)crops8_dev, (const long long*)index_dev, S, D, c, tmp);
  hipLaunchKernelGGL(k_embed_v, dim3(N, cpx_div_up(D, kRowsV)), dim3(th), 0, ctx->stream,
                     (const unsigned char*)tmp, S, D, c, mean, stdv, (__half*)out_dev);
  CPX_CHECK_LAUNCH("cpx_embed_preprocess");
  return CPX_OK;
}
