// f3 per-cell embeddings: the EfficientNetV2-L forward of the reference's consumer
// (Cellpose_GPU_s3fs.py:109-110,184-194: timm tf_efficientnetv2_l under fp16 autocast,
// `pooler_output`) on the fp16 matrix cores.  Activations are NHWC fp16, every product is an fp16
// x fp16 MFMA with fp32 accumulation, BatchNorm is folded to a per-channel scale/shift applied to
// the fp32 accumulator, followed by SiLU and the residual add, and each stored activation is
// rounded to fp16 once (autocast rounds after every op; the checkpoint is a remote download, so
// the embedding values are parity-unpinned either way — tests compare with the fp32 module).
//
//   k_eff_stem  conv3x3/2 3 -> 32 + BN + SiLU on the preprocessed NCHW images (VALU; 27 taps)
//   k_eff_conv  implicit-GEMM convolution (1x1 or 3x3, stride 1 or 2, TF 'same' padding) on
//               v_mfma_f32_32x32x16_f16: a 256-thread block computes 64 output channels x 64
//               pixels of one image, K in chunks of 32 (one tap, 32 input channels) staged in
//               LDS (16-byte chunks XOR-swizzled, conflict-free fragment reads) from registers,
//               double-buffered; an optional per-(image, input channel) gate (squeeze-excite)
//               multiplies the weight tile as it is staged; epilogue scale/shift, SiLU, residual
//   k_eff_dw    depthwise 3x3 (stride 1 or 2) + BN + SiLU, fp32 taps; per-block channel sums of
//               the output (the SE mean) in fixed order
//   k_eff_se    per image: channel means -> reduce 1x1 + SiLU -> expand 1x1 + sigmoid = gate
//   k_eff_pool  global average pool of the head -> fp32 pooler_output [N][1280]
#include "cpx_internal.h"
#include <math.h>

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kET = 256;  // k_eff_conv block: 4 waves, 2 x 2 wave tiles of 32 x 32
constexpr int kEB = 64;   // output channels / pixels per block
constexpr int kEK = 32;   // K chunk

__device__ __forceinline__ float silu(float v) { return v / (1.0f + expf(-v)); }

// TF 'same' padding (timm Conv2dSame): output ceil(i / s), pad_lo = total / 2
__host__ __device__ inline int same_out(int i, int s) { return (i + s - 1) / s; }
__host__ __device__ inline int same_pad_lo(int i, int k, int s) {
  const int tot = (same_out(i, s) - 1) * s + k - i;
  return tot > 0 ? tot / 2 : 0;
}

__device__ __forceinline__ int eswz(int row) { return (row >> 2) & 3; }

// 8 halves scaled by 8 fp32 gates (one rounding)
__device__ __forceinline__ uint4 gate8(uint4 w, const float* g) {
  f16x8 h = __builtin_bit_cast(f16x8, w);
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = (_Float16)((float)h[k] * g[k]);
  return __builtin_bit_cast(uint4, h);
}

__global__ __launch_bounds__(kET) void k_eff_conv(const _Float16* __restrict__ in, int Hi, int Wi, int Cin,
                                                  const _Float16* __restrict__ w, int Cout, int ks, int stride,
                                                  int Ho, int Wo, int pad_y, int pad_x, int tiles_per_img,
                                                  const float* __restrict__ scale, const float* __restrict__ shift,
                                                  int act, const _Float16* __restrict__ res,
                                                  const float* __restrict__ gate, _Float16* __restrict__ out) {
  __shared__ uint4 sA[2][kEB * 4];
  __shared__ uint4 sB[2][kEB * 4];
  const int n = blockIdx.x / tiles_per_img;
  const int p0 = (blockIdx.x - n * tiles_per_img) * kEB;
  const int co0 = blockIdx.y * kEB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mw = wid & 1, pw = wid >> 1;
  const int l32 = lane & 31, h = lane >> 5;
  const int K = ks * ks * Cin;
  const int nk = K / kEK;
  const int HWo = Ho * Wo;
  // this thread's staging slot: row (channel / pixel) and 16-byte chunk of the 64-byte K chunk
  const int srow = tid >> 2, sc = tid & 3;
  const int sslot = srow * 4 + (sc ^ eswz(srow));
  const int co = co0 + srow;
  const int px = p0 + srow;
  const bool pvalid = px < HWo;
  const int oy = pvalid ? px / Wo : 0, ox = pvalid ? px - (px / Wo) * Wo : 0;
  const _Float16* inb = in + (long long)n * Hi * Wi * Cin;
  const float* gb = gate ? gate + (long long)n * Cin : nullptr;
  auto load = [&](int kc, uint4& a, uint4& b) {
    const int k0 = kc * kEK;
    const int tap = k0 / Cin, ci = k0 - tap * Cin + 8 * sc;
    a = make_uint4(0u, 0u, 0u, 0u);
    if (co < Cout) {
      a = *reinterpret_cast<const uint4*>(w + (long long)co * K + k0 + 8 * sc);
      if (gb) a = gate8(a, gb + ci);
    }
    b = make_uint4(0u, 0u, 0u, 0u);
    const int ky = tap / ks, kx = tap - (tap / ks) * ks;
    const int iy = oy * stride + ky - pad_y, ix = ox * stride + kx - pad_x;
    if (pvalid && (unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi)
      b = *reinterpret_cast<const uint4*>(inb + ((long long)iy * Wi + ix) * Cin + ci);
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  uint4 ra, rb;
  load(0, ra, rb);
  sA[0][sslot] = ra;
  sB[0][sslot] = rb;
  __syncthreads();
  const int ar = mw * 32 + l32, br = pw * 32 + l32;
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = kc & 1;
    if (kc + 1 < nk) load(kc + 1, ra, rb);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int c = 2 * st + h;
      const f16x8 fa = __builtin_bit_cast(f16x8, sA[buf][ar * 4 + (c ^ eswz(ar))]);
      const f16x8 fb = __builtin_bit_cast(f16x8, sB[buf][br * 4 + (c ^ eswz(br))]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa, fb, acc, 0, 0, 0);
    }
    if (kc + 1 < nk) {
      sA[buf ^ 1][sslot] = ra;
      sB[buf ^ 1][sslot] = rb;
    }
    __syncthreads();
  }
  // epilogue: lane (l32, h) holds pixel p0 + pw*32 + l32, channels 8 g + 4 h + {0..3}
  const int opx = p0 + pw * 32 + l32;
  if (opx >= HWo) return;
  const long long obase = ((long long)n * HWo + opx) * Cout;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int c = co0 + mw * 32 + 8 * g + 4 * h;
    if (c >= Cout) continue;
    f16x4 o;
    float rv[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (res) {
      const f16x4 r4 = *reinterpret_cast<const f16x4*>(res + obase + c);
#pragma unroll
      for (int k = 0; k < 4; ++k) rv[k] = (float)r4[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v = acc[4 * g + k] * scale[c + k] + shift[c + k];
      if (act) v = silu(v);
      o[k] = (_Float16)(v + rv[k]);
    }
    *reinterpret_cast<f16x4*>(out + obase + c) = o;
  }
}

// stem: conv3x3/2 3 -> 32 on NCHW fp16 [N][3][H][W] -> NHWC fp16 [N][Ho][Wo][32], BN + SiLU
__global__ __launch_bounds__(256) void k_eff_stem(const _Float16* __restrict__ x, int H, int W, int Ho, int Wo,
                                                  int pad_y, int pad_x, const float* __restrict__ w,
                                                  const float* __restrict__ scale,
                                                  const float* __restrict__ shift, _Float16* __restrict__ out) {
  __shared__ float sw[32 * 27];
  for (int i = threadIdx.x; i < 32 * 27; i += 256) sw[i] = w[i];
  __syncthreads();
  const int n = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= Ho * Wo) return;
  const int oy = p / Wo, ox = p - (p / Wo) * Wo;
  float xv[27];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iy = oy * 2 + ky - pad_y, ix = ox * 2 + kx - pad_x;
        xv[c * 9 + ky * 3 + kx] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                                      ? (float)x[(((long long)n * 3 + c) * H + iy) * W + ix] : 0.0f;
      }
  _Float16* o = out + ((long long)n * Ho * Wo + p) * 32;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f16x8 v8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int co = 8 * q + k;
      float s = 0.0f;
#pragma unroll
      for (int t = 0; t < 27; ++t) s += sw[co * 27 + t] * xv[t];
      v8[k] = (_Float16)silu(s * scale[co] + shift[co]);
    }
    *reinterpret_cast<f16x8*>(o + 8 * q) = v8;
  }
}

// depthwise 3x3: block = 64 pixels of one image x 64 channels (8 channel groups of 8 x 32 pixel
// lanes, two pixels each); partial[n][pblk][c] = sum of the block's outputs (fp32, as stored)
constexpr int kDwP = 64;
__global__ __launch_bounds__(256) void k_eff_dw(const _Float16* __restrict__ in, int Hi, int Wi, int C, int stride,
                                                int Ho, int Wo, int pad_y, int pad_x, int pblks,
                                                const float* __restrict__ w, const float* __restrict__ scale,
                                                const float* __restrict__ shift, _Float16* __restrict__ out,
                                                float* __restrict__ partial) {
  __shared__ float sred[32][65];
  const int n = blockIdx.x / pblks, pb = blockIdx.x - n * pblks;
  const int c0 = blockIdx.y * 64 + 8 * (threadIdx.x & 7);
  const int pl = threadIdx.x >> 3;  // 0..31
  float wt[8][9], sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[k][t] = w[(c0 + k) * 9 + t];
    sc[k] = scale[c0 + k];
    sh[k] = shift[c0 + k];
  }
  float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const _Float16* inb = in + (long long)n * Hi * Wi * C;
#pragma unroll
  for (int u = 0; u < kDwP / 32; ++u) {
    const int p = pb * kDwP + pl + 32 * u;
    if (p >= Ho * Wo) continue;
    const int oy = p / Wo, ox = p - (p / Wo) * Wo;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iy = oy * stride + ky - pad_y, ix = ox * stride + kx - pad_x;
        if ((unsigned)iy >= (unsigned)Hi || (unsigned)ix >= (unsigned)Wi) continue;
        const f16x8 v = *reinterpret_cast<const f16x8*>(inb + ((long long)iy * Wi + ix) * C + c0);
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] += wt[k][ky * 3 + kx] * (float)v[k];
      }
    f16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[k] = (_Float16)silu(a[k] * sc[k] + sh[k]);
      sum[k] += (float)o[k];
    }
    *reinterpret_cast<f16x8*>(out + ((long long)n * Ho * Wo + p) * C + c0) = o;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) sred[pl][8 * (threadIdx.x & 7) + k] = sum[k];
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0.0f;
    for (int q = 0; q < 32; ++q) s += sred[q][threadIdx.x];
    partial[((long long)n * pblks + pb) * C + blockIdx.y * 64 + threadIdx.x] = s;
  }
}

// squeeze-excite gate per image: mean over pixels (fixed-order sum of the block partials),
// r = silu(br + Wr mean) (rd outputs), gate = sigmoid(be + We r) (C outputs)
__global__ __launch_bounds__(256) void k_eff_se(const float* __restrict__ partial, int pblks, int HW, int C, int rd,
                                                const float* __restrict__ wr, const float* __restrict__ br,
                                                const float* __restrict__ we, const float* __restrict__ be,
                                                float* __restrict__ gate) {
  extern __shared__ float sm[];  // mean [C], r [rd]
  float* mean = sm;
  float* r = sm + C;
  const int n = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.0f;
    for (int b = 0; b < pblks; ++b) s += partial[((long long)n * pblks + b) * C + c];
    mean[c] = s / (float)HW;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < rd; j += 256) {
    float s = br[j];
    const float* wj = wr + (long long)j * C;
    for (int c = 0; c < C; ++c) s += wj[c] * mean[c];
    r[j] = silu(s);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = be[c];
    const float* wc = we + (long long)c * rd;
    for (int j = 0; j < rd; ++j) s += wc[j] * r[j];
    gate[(long long)n * C + c] = 1.0f / (1.0f + expf(-s));
  }
}

// global average pool: NHWC fp16 [N][HW][C] -> fp32 [N][C]
__global__ __launch_bounds__(256) void k_eff_pool(const _Float16* __restrict__ in, int HW, int C,
                                                  float* __restrict__ out) {
  const int n = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.0f;
  for (int p = 0; p < HW; ++p) s += (float)in[((long long)n * HW + p) * C + c];
  out[(long long)n * C + c] = s / (float)HW;
}

}  // namespace

extern "C" int cpx_effnet_stem(cpx_ctx* ctx, const void* x, int N, int H, int W, const float* w,
                               const float* scale, const float* shift, void* out) {
  CPX_REQUIRE(ctx && x && w && scale && shift && out, CPX_ERR_ARG, "cpx_effnet_stem: null argument");
  CPX_REQUIRE(N > 0 && N <= 65535 && H > 2 && W > 2, CPX_ERR_ARG, "cpx_effnet_stem: bad sizes");
  const int Ho = same_out(H, 2), Wo = same_out(W, 2);
  hipLaunchKernelGGL(k_eff_stem, dim3(cpx_div_up(Ho * Wo, 256), N), dim3(256), 0, ctx->stream,
                     (const _Float16*)x, H, W, Ho, Wo, same_pad_lo(H, 3, 2), same_pad_lo(W, 3, 2), w, scale,
                     shift, (_Float16*)out);
  CPX_CHECK_LAUNCH("k_eff_stem");
  return CPX_OK;
}

extern "C" int cpx_effnet_conv(cpx_ctx* ctx, const void* in, int N, int H, int W, int cin, int cout, int ks,
                               int stride, const void* w, const float* scale, const float* shift, int act,
                               const void* res, const float* gate, void* out) {
  CPX_REQUIRE(ctx && in && w && scale && shift && out, CPX_ERR_ARG, "cpx_effnet_conv: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0 && (ks == 1 || ks == 3) && (stride == 1 || stride == 2) &&
                  cin % kEK == 0 && cout % 4 == 0 && cout > 0,
              CPX_ERR_ARG, "cpx_effnet_conv: unsupported shape (ks %d stride %d cin %d cout %d)", ks, stride,
              cin, cout);
  CPX_REQUIRE(((uintptr_t)in | (uintptr_t)w | (uintptr_t)out | (uintptr_t)res) % 16 == 0, CPX_ERR_ARG,
              "cpx_effnet_conv: misaligned buffers");
  CPX_REQUIRE(!res || stride == 1, CPX_ERR_ARG, "cpx_effnet_conv: residual needs stride 1");
  const int Ho = same_out(H, stride), Wo = same_out(W, stride);
  const int tpi = cpx_div_up(Ho * Wo, kEB);
  const long long gx = (long long)N * tpi;
  CPX_REQUIRE(gx < (1LL << 31), CPX_ERR_ARG, "cpx_effnet_conv: too many tiles");
  hipLaunchKernelGGL(k_eff_conv, dim3((unsigned)gx, cpx_div_up(cout, kEB)), dim3(kET), 0, ctx->stream,
                     (const _Float16*)in, H, W, cin, (const _Float16*)w, cout, ks, stride, Ho, Wo,
                     same_pad_lo(H, ks, stride), same_pad_lo(W, ks, stride), tpi, scale, shift, act,
                     (const _Float16*)res, gate, (_Float16*)out);
  CPX_CHECK_LAUNCH("k_eff_conv");
  return CPX_OK;
}

extern "C" int cpx_effnet_dw(cpx_ctx* ctx, const void* in, int N, int H, int W, int C, int stride,
                             const float* w, const float* scale, const float* shift, void* out,
                             float* partial) {
  CPX_REQUIRE(ctx && in && w && scale && shift && out && partial, CPX_ERR_ARG, "cpx_effnet_dw: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0 && C % 64 == 0 && (stride == 1 || stride == 2), CPX_ERR_ARG,
              "cpx_effnet_dw: unsupported shape (C %d stride %d)", C, stride);
  const int Ho = same_out(H, stride), Wo = same_out(W, stride);
  const int pblks = cpx_div_up(Ho * Wo, kDwP);
  hipLaunchKernelGGL(k_eff_dw, dim3(N * pblks, C / 64), dim3(256), 0, ctx->stream, (const _Float16*)in, H, W, C,
                     stride, Ho, Wo, same_pad_lo(H, 3, stride), same_pad_lo(W, 3, stride), pblks, w, scale, shift,
                     (_Float16*)out, partial);
  CPX_CHECK_LAUNCH("k_eff_dw");
  return CPX_OK;
}

extern "C" int cpx_effnet_dw_blocks(int H, int W, int stride) {
  return cpx_div_up(same_out(H, stride) * same_out(W, stride), kDwP);
}

extern "C" int cpx_effnet_se(cpx_ctx* ctx, const float* partial, int N, int pblks, int HW, int C, int rd,
                             const float* wr, const float* br, const float* we, const float* be, float* gate) {
  CPX_REQUIRE(ctx && partial && wr && br && we && be && gate, CPX_ERR_ARG, "cpx_effnet_se: null argument");
  CPX_REQUIRE(N > 0 && pblks > 0 && HW > 0 && C > 0 && rd > 0 && (C + rd) * 4 <= 64 * 1024, CPX_ERR_ARG,
              "cpx_effnet_se: bad sizes");
  hipLaunchKernelGGL(k_eff_se, dim3(N), dim3(256), sizeof(float) * (C + rd), ctx->stream, partial, pblks, HW, C,
                     rd, wr, br, we, be, gate);
  CPX_CHECK_LAUNCH("k_eff_se");
  return CPX_OK;
}

extern "C" int cpx_effnet_pool(cpx_ctx* ctx, const void* in, int N, int HW, int C, float* out) {
  CPX_REQUIRE(ctx && in && out && N > 0 && HW > 0 && C > 0, CPX_ERR_ARG, "cpx_effnet_pool: bad argument");
  hipLaunchKernelGGL(k_eff_pool, dim3(cpx_div_up(C, 256), N), dim3(256), 0, ctx->stream, (const _Float16*)in, HW,
                     C, out);
  CPX_CHECK_LAUNCH("k_eff_pool");
  return CPX_OK;
}
