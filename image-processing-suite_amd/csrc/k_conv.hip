// a4 CPnet 3x3 convolution (pad 1, stride 1) on bf16 NHWC activations, implicit GEMM on the
// gfx950 matrix cores (v_mfma_f32_32x32x16_bf16) with the CPnet epilogue fused in.
//
// GEMM view per block: D[cout][pixel] = sum over (tap, cin) W[cout][cin][tap] * X[pixel+tap][cin]
// for a TY x TX spatial tile of one image and BN output channels:
//   * the input halo (TY+2) x (TX+2) x CK (one cin slab) and the weights [tap][BN][CK] of the
//     slab are staged in LDS as 16-byte chunks, XOR-swizzled so the ds_read_b128 fragment reads
//     (16 lanes = 16 different pixels / output channels at one 16-byte column) hit distinct
//     bank slots;
//   * 4 waves split the tile's 32-pixel subtiles; each wave owns all BN output channels
//     (BN/32 x subtiles accumulators of 16 fp32), A = weights (row = cout), B = pixels;
//   * epilogue straight from the accumulators (fp32): bias, residual (optionally read
//     nearest-upsampled), residual-stream store, style bias, eval BatchNorm, ReLU, and the next
//     convolution's input store (optionally 2x nearest-upsampled) — the semantics of
//     cpx_cpnet_epilogue (k_cpnet.hip) without the bf16 round trip of the raw convolution.
// Accumulator layout (32x32x16): lane l holds pixel (l & 31) and output channels
// (r & 3) + 8 (r >> 2) + 4 (l >> 5) of its 16 registers r: four runs of 4 consecutive channels,
// stored as 8-byte NHWC pieces.
#include "cpx_internal.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct ConvEpi {
  const float* bias;
  const unsigned short* res;
  const float* style;
  const float* scale;
  const float* shift;
  unsigned short* y;
  unsigned short* z;
  int res_up, relu, z_up;
};

__device__ __forceinline__ unsigned short f2bf(float f) {  // round to nearest even
  unsigned int u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (unsigned short)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

// 16-byte chunk swizzle: chunk q of LDS row `row` (a pixel or an output channel) lives at
// slot q ^ swz(row); with Q chunks per row this makes (row mod 16) -> distinct bank slots.
template <int Q>
__device__ __forceinline__ int swz(int row) {
  if constexpr (Q >= 16) return row & 15;
  else if constexpr (Q == 8) return (row >> 1) & 7;
  else if constexpr (Q == 4) return (row >> 2) & 3;
  else if constexpr (Q == 2) return (row >> 3) & 1;
  else return 0;
}

template <int CIN, int COUT, int BN, int TY, int TX, int CK>
__global__ __launch_bounds__(256) void k_conv3x3(const unsigned short* __restrict__ in,
                                                 const unsigned short* __restrict__ wpk,
                                                 ConvEpi ep, int N, int H, int W, int tiles_x,
                                                 int tiles_y) {
  constexpr int HY = TY + 2, HX = TX + 2, NPIX = HY * HX;
  constexpr int Q = CK / 8;
  constexpr int NCH = CIN / CK;
  constexpr int P = TY * TX;
  constexpr int NPT = P / 32;
  constexpr int WPT = NPT / 4;
  constexpr int NMT = BN / 32;
  static_assert(CIN % CK == 0 && CK % 16 == 0 && COUT % BN == 0 && BN % 32 == 0, "shape");
  static_assert(P % 128 == 0, "4 waves x 32-pixel subtiles");
  __shared__ uint4 sIn[NPIX * Q];
  __shared__ uint4 sW[9 * BN * Q];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int tiles = tiles_x * tiles_y;
  const int n = blockIdx.x / tiles;
  const int t = blockIdx.x - n * tiles;
  const int ty0 = (t / tiles_x) * TY, tx0 = (t % tiles_x) * TX;
  const int nb = blockIdx.y;

  f32x16 acc[NMT][WPT];
#pragma unroll
  for (int m = 0; m < NMT; ++m)
#pragma unroll
    for (int p = 0; p < WPT; ++p)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][p][r] = 0.0f;

  // per-lane LDS pixel rows of this wave's subtiles (tap 0,0)
  int lin0[WPT];
#pragma unroll
  for (int p = 0; p < WPT; ++p) {
    const int px = (wid * WPT + p) * 32 + l32;
    lin0[p] = (px / TX) * HX + (px % TX);
  }

  const uint4* w4 = reinterpret_cast<const uint4*>(wpk);
  for (int ch = 0; ch < NCH; ++ch) {
    // stage the input halo slab
    for (int i = threadIdx.x; i < NPIX * Q; i += 256) {
      const int lin = i / Q, q = i - lin * Q;
      const int hy = lin / HX, hx = lin - hy * HX;
      const int gy = ty0 + hy - 1, gx = tx0 + hx - 1;
      uint4 v = {0u, 0u, 0u, 0u};
      if (gy >= 0 && gy < H && gx >= 0 && gx < W)
        v = *reinterpret_cast<const uint4*>(in + (((long long)n * H + gy) * W + gx) * CIN + ch * CK + q * 8);
      sIn[lin * Q + (q ^ swz<Q>(lin))] = v;
    }
    // stage the weight slab [tap][BN][CK]
    const long long wb = ((long long)(nb * NCH + ch) * 9 * BN) * Q;
    for (int i = threadIdx.x; i < 9 * BN * Q; i += 256) {
      const int row = i / Q, q = i - row * Q;
      sW[row * Q + (q ^ swz<Q>(row))] = w4[wb + i];
    }
    __syncthreads();
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
      for (int kk = 0; kk < CK / 16; ++kk) {
        const int qa = kk * 2 + h;
        bf16x8 a[NMT], b[WPT];
#pragma unroll
        for (int m = 0; m < NMT; ++m) {
          const int row = tap * BN + m * 32 + l32;
          const uint4 v = sW[row * Q + (qa ^ swz<Q>(row))];
          a[m] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int p = 0; p < WPT; ++p) {
          const int lin = lin0[p] + ky * HX + kx;
          const uint4 v = sIn[lin * Q + (qa ^ swz<Q>(lin))];
          b[p] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int m = 0; m < NMT; ++m)
#pragma unroll
          for (int p = 0; p < WPT; ++p)
            acc[m][p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m], b[p], acc[m][p], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // fused epilogue
#pragma unroll
  for (int p = 0; p < WPT; ++p) {
    const int px = (wid * WPT + p) * 32 + l32;
    const int gy = ty0 + px / TX, gx = tx0 + px % TX;
    if (gy >= H || gx >= W) continue;
    const long long pix = ((long long)n * H + gy) * W + gx;
    long long rpix = pix;
    if (ep.res_up) rpix = ((long long)n * (H >> 1) + (gy >> 1)) * (W >> 1) + (gx >> 1);
#pragma unroll
    for (int m = 0; m < NMT; ++m) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = nb * BN + m * 32 + 8 * g + 4 * h;
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = acc[m][p][4 * g + k];
        if (ep.bias) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] += ep.bias[c0 + k];
        }
        if (ep.res) {
          const uint2 r = *reinterpret_cast<const uint2*>(ep.res + rpix * COUT + c0);
          v[0] += __uint_as_float(r.x << 16);
          v[1] += __uint_as_float(r.x & 0xffff0000u);
          v[2] += __uint_as_float(r.y << 16);
          v[3] += __uint_as_float(r.y & 0xffff0000u);
        }
        if (ep.y) {
          uint2 o;
          o.x = (unsigned int)f2bf(v[0]) | ((unsigned int)f2bf(v[1]) << 16);
          o.y = (unsigned int)f2bf(v[2]) | ((unsigned int)f2bf(v[3]) << 16);
          *reinterpret_cast<uint2*>(ep.y + pix * COUT + c0) = o;
        }
        if (!ep.z) continue;
        if (ep.style) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] += ep.style[(long long)n * COUT + c0 + k];
        }
        if (ep.scale) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = ep.scale[c0 + k] * v[k] + ep.shift[c0 + k];
        }
        if (ep.relu) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = fmaxf(v[k], 0.0f);
        }
        uint2 o;
        o.x = (unsigned int)f2bf(v[0]) | ((unsigned int)f2bf(v[1]) << 16);
        o.y = (unsigned int)f2bf(v[2]) | ((unsigned int)f2bf(v[3]) << 16);
        if (!ep.z_up) {
          *reinterpret_cast<uint2*>(ep.z + pix * COUT + c0) = o;
        } else {
          const long long W2 = 2LL * W;
          const long long b2 = ((long long)n * 2 * H + 2LL * gy) * W2 + 2LL * gx;
          *reinterpret_cast<uint2*>(ep.z + b2 * COUT + c0) = o;
          *reinterpret_cast<uint2*>(ep.z + (b2 + 1) * COUT + c0) = o;
          *reinterpret_cast<uint2*>(ep.z + (b2 + W2) * COUT + c0) = o;
          *reinterpret_cast<uint2*>(ep.z + (b2 + W2 + 1) * COUT + c0) = o;
        }
      }
    }
  }
}

struct ConvCfg {
  int bn, ck, ty, tx;
};

// tile configuration per (Cin, Cout); must match the instantiations in launch()
bool conv_cfg(int cin, int cout, ConvCfg* c) {
  c->ck = 32;
  c->tx = 16;
  if (cout == 32) {
    c->bn = 32;
    c->ty = 16;
  } else if (cout == 64) {
    c->bn = 64;
    c->ty = 16;
  } else if (cout == 128 || cout == 256) {
    c->bn = 64;
    c->ty = 8;
  } else {
    return false;
  }
  return (cin == 32 || cin == 64 || cin == 128 || cin == 256);
}

template <int CIN, int COUT, int BN, int TY, int TX, int CK>
int launch(cpx_ctx* ctx, const void* in, const void* wpk, const ConvEpi& ep, int N, int H, int W) {
  const int tx = cpx_div_up(W, TX), ty = cpx_div_up(H, TY);
  const long long blocks = (long long)N * tx * ty;
  CPX_REQUIRE(blocks < (1LL << 31), CPX_ERR_ARG, "cpx_cpnet_conv3x3: too many tiles");
  hipLaunchKernelGGL((k_conv3x3<CIN, COUT, BN, TY, TX, CK>), dim3((unsigned)blocks, COUT / BN),
                     dim3(256), 0, ctx->stream, (const unsigned short*)in,
                     (const unsigned short*)wpk, ep, N, H, W, tx, ty);
  CPX_CHECK_LAUNCH("k_conv3x3");
  return CPX_OK;
}

}  // namespace

extern "C" int cpx_cpnet_conv_cfg(int cin, int cout, int* bn, int* ck) {
  ConvCfg c;
  if (!conv_cfg(cin, cout, &c)) return CPX_ERR_SHAPE;
  if (bn) *bn = c.bn;
  if (ck) *ck = c.ck;
  return CPX_OK;
}

extern "C" int cpx_cpnet_conv3x3(cpx_ctx* ctx, const void* in, int N, int H, int W, int cin,
                                 int cout, const void* wpk, const float* bias, const void* res,
                                 int res_up, const float* style, const float* scale,
                                 const float* shift, int relu, void* y_out, void* z_out,
                                 int z_up) {
  CPX_REQUIRE(ctx && in && wpk && (y_out || z_out), CPX_ERR_ARG,
              "cpx_cpnet_conv3x3: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0, CPX_ERR_ARG, "cpx_cpnet_conv3x3: bad sizes");
  CPX_REQUIRE(!(scale == nullptr) == !(shift == nullptr), CPX_ERR_ARG,
              "cpx_cpnet_conv3x3: scale and shift go together");
  CPX_REQUIRE(!res_up || ((H % 2) == 0 && (W % 2) == 0), CPX_ERR_ARG,
              "cpx_cpnet_conv3x3: res_up needs even sizes");
  CPX_REQUIRE(((uintptr_t)in | (uintptr_t)wpk) % 16 == 0 &&
                  ((uintptr_t)res | (uintptr_t)y_out | (uintptr_t)z_out) % 8 == 0,
              CPX_ERR_ARG, "cpx_cpnet_conv3x3: misaligned buffers");
  ConvEpi ep{bias, (const unsigned short*)res, style, scale, shift, (unsigned short*)y_out,
             (unsigned short*)z_out, res_up, relu, z_up};
#define CPX_CONV(CI, CO, BN_, TY_)                                   \
  if (cin == CI && cout == CO)                                       \
    return launch<CI, CO, BN_, TY_, 16, 32>(ctx, in, wpk, ep, N, H, W);
  CPX_CONV(32, 32, 32, 16)
  CPX_CONV(64, 32, 32, 16)
  CPX_CONV(32, 64, 64, 16)
  CPX_CONV(64, 64, 64, 16)
  CPX_CONV(128, 64, 64, 16)
  CPX_CONV(64, 128, 64, 8)
  CPX_CONV(128, 128, 64, 8)
  CPX_CONV(256, 128, 64, 8)
  CPX_CONV(128, 256, 64, 8)
  CPX_CONV(256, 256, 64, 8)
#undef CPX_CONV
  cpx_set_error("cpx_cpnet_conv3x3: unsupported channels %d -> %d", cin, cout);
  return CPX_ERR_SHAPE;
}
