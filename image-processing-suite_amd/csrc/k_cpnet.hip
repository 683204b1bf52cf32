// a4 CPnet glue: fused conv epilogues and pre-activations on bf16 NHWC activations.
//
// Cellpose's CPnet (resnet_torch.py: batchconv = BatchNorm -> ReLU -> Conv2d, residual sums,
// style bias added before BatchNorm in the up path) runs eagerly as ~9 full-tensor passes per
// convolution (conv, bias, residual add, style add, BatchNorm, ReLU).  Here each MIOpen
// convolution (no bias) is followed by ONE pass that applies everything up to the next
// convolution's input (cpx/cpnet_fused.py builds the schedule):
//   t = conv + bias[c] (+ res, optionally read from the 2x-downsampled residual = nearest
//       upsampling fused into the read)          -> y_out (the residual stream, if wanted)
//   u = t (+ style[n, c])
//   z = scale[c] * u + shift[c] (eval BatchNorm), ReLU -> z_out (the next conv's input,
//       optionally written 2x nearest-upsampled)
// and the down path's 2x2 max-pool is fused with the following BatchNorm+ReLU.  Arithmetic in
// fp32, one bf16 rounding (RNE) per stored tensor.  All passes are HBM-bound elementwise:
// 16-byte vectors (8 channels) per thread, grid sized to the chip.
#include "cpx_internal.h"

namespace {

constexpr int kET = 256;

__device__ __forceinline__ float bf2f(unsigned short h) {
  return __uint_as_float((unsigned int)h << 16);
}

__device__ __forceinline__ unsigned short f2bf(float f) {  // round to nearest even
  unsigned int u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (unsigned short)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const unsigned int w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(w[k] << 16);
    f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// two fp32 -> packed bf16 pair, round to nearest even (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned int pk2(float lo, float hi) {
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned int, v);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pk2(f[0], f[1]);
  v.y = pk2(f[2], f[3]);
  v.z = pk2(f[4], f[5]);
  v.w = pk2(f[6], f[7]);
  return v;
}

struct EpiArgs {
  const unsigned short* conv;
  const float* bias;
  const unsigned short* res;
  const float* style;
  const float* scale;
  const float* shift;
  unsigned short* y;
  unsigned short* z;
  int N, Hh, Ww, Cn, res_up, relu, z_up;
};

// vector path: Cn % 8 == 0, one uint4 (8 channels of one pixel) per thread iteration
__global__ __launch_bounds__(kET) void k_cpnet_epi8(EpiArgs a) {
  const long long P = (long long)a.Hh * a.Ww;
  const long long n8 = (long long)a.N * P * a.Cn / 8;
  const int cv = a.Cn / 8;
  for (long long v = (long long)blockIdx.x * kET + threadIdx.x; v < n8;
       v += (long long)gridDim.x * kET) {
    const long long pix = v / cv;
    const int c0 = (int)(v - pix * cv) * 8;
    float t[8];
    if (a.conv) {
      unpack8(reinterpret_cast<const uint4*>(a.conv)[v], t);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] = 0.0f;
    }
    if (a.bias) {
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] += a.bias[c0 + k];
    }
    const long long n = pix / P;
    if (a.res) {
      long long rv = v;
      if (a.res_up) {
        const long long rem = pix - n * P;
        const int h = (int)(rem / a.Ww), w = (int)(rem - (long long)h * a.Ww);
        const long long rp = (n * (a.Hh >> 1) + (h >> 1)) * (a.Ww >> 1) + (w >> 1);
        rv = rp * cv + c0 / 8;
      }
      float r[8];
      unpack8(reinterpret_cast<const uint4*>(a.res)[rv], r);
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] += r[k];
    }
    if (a.y) reinterpret_cast<uint4*>(a.y)[v] = pack8(t);
    if (!a.z) continue;
    if (a.style) {
      const float* s = a.style + n * a.Cn + c0;
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] += s[k];
    }
    if (a.scale) {
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] = a.scale[c0 + k] * t[k] + a.shift[c0 + k];
    }
    if (a.relu) {
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] = fmaxf(t[k], 0.0f);
    }
    const uint4 zv = pack8(t);
    if (!a.z_up) {
      reinterpret_cast<uint4*>(a.z)[v] = zv;
    } else {
      const long long rem = pix - n * P;
      const int h = (int)(rem / a.Ww), w = (int)(rem - (long long)h * a.Ww);
      const long long W2 = 2LL * a.Ww;
      const long long base = (n * 2LL * a.Hh + 2LL * h) * W2 + 2LL * w;
      uint4* z4 = reinterpret_cast<uint4*>(a.z);
      z4[base * cv + c0 / 8] = zv;
      z4[(base + 1) * cv + c0 / 8] = zv;
      z4[(base + W2) * cv + c0 / 8] = zv;
      z4[(base + W2 + 1) * cv + c0 / 8] = zv;
    }
  }
}

// scalar path (few channels: the 2-channel network input, the 3-channel head)
__global__ __launch_bounds__(kET) void k_cpnet_epi1(EpiArgs a) {
  const long long P = (long long)a.Hh * a.Ww;
  const long long ne = (long long)a.N * P * a.Cn;
  for (long long e = (long long)blockIdx.x * kET + threadIdx.x; e < ne;
       e += (long long)gridDim.x * kET) {
    const long long pix = e / a.Cn;
    const int c = (int)(e - pix * a.Cn);
    const long long n = pix / P;
    const long long rem = pix - n * P;
    const int h = (int)(rem / a.Ww), w = (int)(rem - (long long)h * a.Ww);
    float t = a.conv ? bf2f(a.conv[e]) : 0.0f;
    if (a.bias) t += a.bias[c];
    if (a.res) {
      long long re = e;
      if (a.res_up) re = ((n * (a.Hh >> 1) + (h >> 1)) * (a.Ww >> 1) + (w >> 1)) * a.Cn + c;
      t += bf2f(a.res[re]);
    }
    if (a.y) a.y[e] = f2bf(t);
    if (!a.z) continue;
    if (a.style) t += a.style[n * a.Cn + c];
    if (a.scale) t = a.scale[c] * t + a.shift[c];
    if (a.relu) t = fmaxf(t, 0.0f);
    const unsigned short zb = f2bf(t);
    if (!a.z_up) {
      a.z[e] = zb;
    } else {
      const long long W2 = 2LL * a.Ww;
      const long long base = (n * 2LL * a.Hh + 2LL * h) * W2 + 2LL * w;
      a.z[base * a.Cn + c] = zb;
      a.z[(base + 1) * a.Cn + c] = zb;
      a.z[(base + W2) * a.Cn + c] = zb;
      a.z[(base + W2 + 1) * a.Cn + c] = zb;
    }
  }
}

// 2x2 max-pool (stride 2) of [N, 2Hh, 2Ww, Cn] -> x_out [N, Hh, Ww, Cn], and
// z_out = ReLU(scale * x + shift) of the pooled tensor (both optional)
__global__ __launch_bounds__(kET) void k_cpnet_pool8(const unsigned short* __restrict__ in,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift, int relu,
                                                     int N, int Hh, int Ww, int Cn,
                                                     unsigned short* __restrict__ xo,
                                                     unsigned short* __restrict__ zo) {
  const long long P = (long long)Hh * Ww;
  const int cv = Cn / 8;
  const long long n8 = (long long)N * P * cv;
  const long long W2 = 2LL * Ww;
  const uint4* in4 = reinterpret_cast<const uint4*>(in);
  for (long long v = (long long)blockIdx.x * kET + threadIdx.x; v < n8;
       v += (long long)gridDim.x * kET) {
    const long long pix = v / cv;
    const int c8 = (int)(v - pix * cv);
    const long long n = pix / P;
    const long long rem = pix - n * P;
    const int h = (int)(rem / Ww), w = (int)(rem - (long long)h * Ww);
    const long long base = (n * 2LL * Hh + 2LL * h) * W2 + 2LL * w;
    float m[8], q[8];
    unpack8(in4[base * cv + c8], m);
    unpack8(in4[(base + 1) * cv + c8], q);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = fmaxf(m[k], q[k]);
    unpack8(in4[(base + W2) * cv + c8], q);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = fmaxf(m[k], q[k]);
    unpack8(in4[(base + W2 + 1) * cv + c8], q);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = fmaxf(m[k], q[k]);
    if (xo) reinterpret_cast<uint4*>(xo)[v] = pack8(m);  // max of bf16 values is exact
    if (zo) {
      const int c0 = c8 * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float t = scale ? scale[c0 + k] * m[k] + shift[c0 + k] : m[k];
        m[k] = relu ? fmaxf(t, 0.0f) : t;
      }
      reinterpret_cast<uint4*>(zo)[v] = pack8(m);
    }
  }
}

int grid_for(cpx_ctx* ctx, long long work) {
  const long long g = (work + kET - 1) / kET;
  const long long cap = 8LL * ctx->n_cu * 4;  // ~8 waves per SIMD in flight, grid-stride beyond
  return (int)std::max(1LL, std::min(g, cap));
}

}  // namespace

extern "C" int cpx_cpnet_epilogue(cpx_ctx* ctx, const void* conv, const float* bias,
                                  const void* res, int res_up, const float* style,
                                  const float* scale, const float* shift, int relu, int N, int Hh,
                                  int Ww, int Cn, void* y_out, void* z_out, int z_up) {
  CPX_REQUIRE(ctx && (y_out || z_out), CPX_ERR_ARG, "cpx_cpnet_epilogue: null argument");
  CPX_REQUIRE(N > 0 && Hh > 0 && Ww > 0 && Cn > 0, CPX_ERR_ARG, "cpx_cpnet_epilogue: bad sizes");
  CPX_REQUIRE(!(scale == nullptr) == !(shift == nullptr), CPX_ERR_ARG,
              "cpx_cpnet_epilogue: scale and shift go together");
  CPX_REQUIRE(!res_up || ((Hh % 2) == 0 && (Ww % 2) == 0), CPX_ERR_ARG,
              "cpx_cpnet_epilogue: res_up needs even sizes");
  EpiArgs a{(const unsigned short*)conv, bias, (const unsigned short*)res, style, scale, shift,
            (unsigned short*)y_out, (unsigned short*)z_out, N, Hh, Ww, Cn, res_up, relu, z_up};
  const long long ne = (long long)N * Hh * Ww * Cn;
  const bool vec = (Cn % 8) == 0 &&
                   ((uintptr_t)conv | (uintptr_t)res | (uintptr_t)y_out | (uintptr_t)z_out) % 16 == 0;
  if (vec) {
    hipLaunchKernelGGL(k_cpnet_epi8, dim3(grid_for(ctx, ne / 8)), dim3(kET), 0, ctx->stream, a);
    CPX_CHECK_LAUNCH("k_cpnet_epi8");
  } else {
    hipLaunchKernelGGL(k_cpnet_epi1, dim3(grid_for(ctx, ne)), dim3(kET), 0, ctx->stream, a);
    CPX_CHECK_LAUNCH("k_cpnet_epi1");
  }
  return CPX_OK;
}

extern "C" int cpx_cpnet_pool(cpx_ctx* ctx, const void* in, const float* scale,
                              const float* shift, int relu, int N, int Hh, int Ww, int Cn,
                              void* x_out, void* z_out) {
  CPX_REQUIRE(ctx && in && (x_out || z_out), CPX_ERR_ARG, "cpx_cpnet_pool: null argument");
  CPX_REQUIRE(N > 0 && Hh > 0 && Ww > 0 && Cn > 0 && Cn % 8 == 0, CPX_ERR_ARG,
              "cpx_cpnet_pool: bad sizes (channels must be a multiple of 8)");
  CPX_REQUIRE(!(scale == nullptr) == !(shift == nullptr), CPX_ERR_ARG,
              "cpx_cpnet_pool: scale and shift go together");
  CPX_REQUIRE(((uintptr_t)in | (uintptr_t)x_out | (uintptr_t)z_out) % 16 == 0, CPX_ERR_ARG,
              "cpx_cpnet_pool: buffers must be 16-byte aligned");
  const long long n8 = (long long)N * Hh * Ww * Cn / 8;
  hipLaunchKernelGGL(k_cpnet_pool8, dim3(grid_for(ctx, n8)), dim3(kET), 0, ctx->stream,
                     (const unsigned short*)in, scale, shift, relu, N, Hh, Ww, Cn,
                     (unsigned short*)x_out, (unsigned short*)z_out);
  CPX_CHECK_LAUNCH("k_cpnet_pool8");
  return CPX_OK;
}

// ---------------------------------------------------------------------------------------------
// CPnet stem: the first down block's entry on the 2-channel network input x, one pass instead
// of four (input BatchNorm+ReLU pass, MIOpen 3x3 2->32 conv + its epilogue pass, MIOpen 1x1
// projection):  z0 = bf16(relu(scale0 * x + shift0)) is formed while the 18 x 18 halo tile is
// staged in LDS, then per pixel 32 outputs of the 3x3 conv (K = 18, fp32 FMAs; the weights are
// block-uniform scalar loads) with bias0 -> BatchNorm1 -> ReLU -> z_out, and the 1x1
// projection of the raw x -> p_out.  Memory-bound: 4 B read, 128 B written per pixel.
namespace {

constexpr int kSTY = 16, kSTX = 16;

__global__ __launch_bounds__(kSTY * kSTX) void k_cpnet_stem(
    const unsigned short* __restrict__ x, int N, int H, int W, const float* __restrict__ scale0,
    const float* __restrict__ shift0, const float* __restrict__ w0, const float* __restrict__ bias0,
    const float* __restrict__ scale1, const float* __restrict__ shift1,
    const float* __restrict__ wp, unsigned short* __restrict__ p_out,
    unsigned short* __restrict__ z_out, int tiles_x, int tiles_y) {
  __shared__ float sz[2][kSTY + 2][kSTX + 2];
  const int tiles = tiles_x * tiles_y;
  const int n = blockIdx.x / tiles, t = blockIdx.x - n * tiles;
  const int ty0 = (t / tiles_x) * kSTY, tx0 = (t % tiles_x) * kSTX;
  const float s00 = scale0[0], s01 = scale0[1], h00 = shift0[0], h01 = shift0[1];
  for (int i = threadIdx.x; i < (kSTY + 2) * (kSTX + 2); i += kSTY * kSTX) {
    const int hy = i / (kSTX + 2), hx = i - hy * (kSTX + 2);
    const int gy = ty0 + hy - 1, gx = tx0 + hx - 1;
    float a = 0.0f, b = 0.0f;  // zero padding of z0 (the conv input)
    if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
      const unsigned int v = *reinterpret_cast<const unsigned int*>(x + (((long long)n * H + gy) * W + gx) * 2);
      a = (float)(__bf16)fmaxf(s00 * __uint_as_float(v << 16) + h00, 0.0f);
      b = (float)(__bf16)fmaxf(s01 * __uint_as_float(v & 0xffff0000u) + h01, 0.0f);
    }
    sz[0][hy][hx] = a;
    sz[1][hy][hx] = b;
  }
  __syncthreads();
  const int ly = threadIdx.x / kSTX, lx = threadIdx.x - ly * kSTX;
  const int gy = ty0 + ly, gx = tx0 + lx;
  if (gy >= H || gx >= W) return;
  const long long pix = ((long long)n * H + gy) * W + gx;
  float in[18];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < 9; ++k) in[c * 9 + k] = sz[c][ly + k / 3][lx + k % 3];
  const unsigned int xv = *reinterpret_cast<const unsigned int*>(x + pix * 2);
  const float x0 = __uint_as_float(xv << 16), x1 = __uint_as_float(xv & 0xffff0000u);
  uint4* zo = reinterpret_cast<uint4*>(z_out + pix * 32);
  uint4* po = reinterpret_cast<uint4*>(p_out + pix * 32);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float zf[8], pf[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int co = q * 8 + e;
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < 18; ++k) acc = __builtin_fmaf(w0[co * 18 + k], in[k], acc);
      zf[e] = fmaxf(__builtin_fmaf(scale1[co], acc + bias0[co], shift1[co]), 0.0f);
      pf[e] = __builtin_fmaf(wp[co * 2], x0, wp[co * 2 + 1] * x1);
    }
    zo[q] = pack8(zf);
    po[q] = pack8(pf);
  }
}

}  // namespace

extern "C" int cpx_cpnet_stem(cpx_ctx* ctx, const void* x, int N, int H, int W,
                              const float* scale0, const float* shift0, const float* w0,
                              const float* bias0, const float* scale1, const float* shift1,
                              const float* wp, void* p_out, void* z_out) {
  CPX_REQUIRE(ctx && x && scale0 && shift0 && w0 && bias0 && scale1 && shift1 && wp && p_out && z_out,
              CPX_ERR_ARG, "cpx_cpnet_stem: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0, CPX_ERR_ARG, "cpx_cpnet_stem: bad sizes");
  CPX_REQUIRE(((uintptr_t)x % 4) == 0 && ((uintptr_t)p_out | (uintptr_t)z_out) % 16 == 0,
              CPX_ERR_ARG, "cpx_cpnet_stem: misaligned buffers");
  const int tx = cpx_div_up(W, kSTX), ty = cpx_div_up(H, kSTY);
  const long long blocks = (long long)N * tx * ty;
  CPX_REQUIRE(blocks < (1LL << 31), CPX_ERR_ARG, "cpx_cpnet_stem: too many tiles");
  hipLaunchKernelGGL(k_cpnet_stem, dim3((unsigned)blocks), dim3(kSTY * kSTX), 0, ctx->stream,
                     (const unsigned short*)x, N, H, W, scale0, shift0, w0, bias0, scale1, shift1,
                     wp, (unsigned short*)p_out, (unsigned short*)z_out, tx, ty);
  CPX_CHECK_LAUNCH("k_cpnet_stem");
  return CPX_OK;
}
