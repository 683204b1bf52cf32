// a6 CPnet 3x3 convolution (pad 1, stride 1) on bf16 NHWC activations, implicit GEMM on the
// gfx950 matrix cores (v_mfma_f32_32x32x16_bf16) with the CPnet epilogue fused in.
//
// GEMM view per block: D[cout][pixel] = sum over (tap, cin) W[cout][cin][tap] * X[pixel+tap][cin]
// for a TY x TX spatial tile of one image and BM output channels (k_conv3x3w):
//   * 512 threads = 8 waves = (BM/32 channel slices) x (8/(BM/32) pixel groups); a wave owns one
//     32-channel slice of a group of 32-pixel subtiles (A = weights, row = cout; B = pixels);
//   * input channels go in slabs of 16: the slab's input halo (TY+2) x (TX+2) x 16 and its
//     weights [tap][BM][16] are double-buffered in LDS and filled by LDS-DMA
//     (global_load_lds_dwordx4, no staging registers), so slab c+1 streams in while slab c's
//     MFMAs run; the halo is staged once and reused by all 9 taps;
//   * tiles are sized per level so that the 9-tap weight slab is reused over 392-512 pixels and
//     the widths of the CPnet levels (224, 112, 56, 28) split into whole tiles;
//   * epilogue from the fp32 accumulators: bias, residual (optionally read nearest-upsampled),
//     residual-stream store, style bias, eval BatchNorm, ReLU, and the next convolution's input
//     store (optionally 2x nearest-upsampled) — the semantics of cpx_cpnet_epilogue
//     (k_cpnet.hip) without the bf16 round trip of the raw convolution.  The accumulator layout
//     scatters 8-byte pieces over 32 pixels per store instruction, so the residual tile and each
//     output tile go through the (by then idle) staging LDS: HBM sees whole-line 16-byte
//     loads/stores only.
// Accumulator layout (32x32x16): lane l holds pixel (l & 31) and output channels
// (r & 3) + 8 (r >> 2) + 4 (l >> 5) of its 16 registers r: four runs of 4 consecutive channels.
#include "cpx_internal.h"
#include <type_traits>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

struct ConvEpi {
  const float* bias;
  const unsigned short* res;
  const float* style;
  const float* scale;
  const float* shift;
  unsigned short* y;
  unsigned short* z;
  int res_up, relu, z_up;
  // optional CPnet output head on z (cout 32 only): head[pixel][j] = head_b[j] +
  // sum_c head_w[j][c] * bf16(z[c]), j < n_head <= 4; z itself is then not stored
  const float* head_w;
  const float* head_b;
  unsigned short* head;
  int n_head;
};

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

// two fp32 -> packed bf16 pair, round to nearest even (v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned int pk_bf16(float lo, float hi) {
  bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned int, v);
}

// LDS-DMA writes are lane-linear (wave base + lane x 16 B), so the weight chunks' XOR swizzle is
// applied on the source address, and the input halo is stored unswizzled (32-byte pixel rows:
// a 2-way bank conflict on the fragment reads, hidden under the MFMAs).  Outside-image halo
// pixels are DMA'd from a 16-byte zero block.
__device__ uint4 g_conv_zero16 = {0u, 0u, 0u, 0u};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

template <int CIN, int COUT, int BM, int TY, int TX>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
void k_conv3x3w(const unsigned short* __restrict__ in, const unsigned short* __restrict__ wpk,
                ConvEpi ep, int N, int H, int W, int tiles_x, int tiles_y) {
  constexpr int NT = 512, NWV = NT / 64;
  constexpr int CK = 16, Q = 2;
  constexpr int MW = BM / 32, PW = NWV / MW;  // waves: MW channel slices x PW pixel groups
  constexpr int HY = TY + 2, HX = TX + 2, NPIX = HY * HX;
  constexpr int NCH = CIN / CK;
  constexpr int P = TY * TX;
  constexpr int NS = (P + 31) / 32;    // 32-pixel subtiles of the tile
  constexpr int NSH = (NS + PW - 1) / PW;   // subtiles per pixel group (the last may have fewer)
  constexpr int NSL = NS - (PW - 1) * NSH;
  constexpr int QB = BM / 8;
  constexpr int SW = 9 * BM * Q, SI = (NPIX * Q + 63) / 64 * 64, SB = SW + SI;  // 16-byte slots
  constexpr int NWW = SW / 64, NWIN = SI / 64;                  // DMA wave-instructions per slab
  constexpr int JW = (NWW + NWV - 1) / NWV, JI = (NWIN + NWV - 1) / NWV;
  constexpr int OUT_R = (P * QB + NT - 1) / NT;
  static_assert(CIN % CK == 0 && COUT % BM == 0 && BM % 32 == 0 && NWV % MW == 0, "shape");
  static_assert(NSL > 0, "every pixel group needs a subtile");
  static_assert(SW % 64 == 0 && SI % 64 == 0, "DMA instructions must not straddle regions");
  static_assert(P * QB <= 2 * SB, "output tile must fit the staging LDS");
  __shared__ uint4 smem[2 * SB];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int mt = wid % MW, ph = wid / MW;  // 32-channel slice, pixel group
  const int h = lane >> 5, l32 = lane & 31;
  const int tiles = tiles_x * tiles_y;
  const int n = blockIdx.x / tiles;
  const int t = blockIdx.x - n * tiles;
  const int ty0 = (t / tiles_x) * TY, tx0 = (t % tiles_x) * TX;
  const int nb = blockIdx.y;
  const unsigned short* inb = in + (long long)n * H * W * CIN;
  const uint4* w4 = reinterpret_cast<const uint4*>(wpk);

  // slab ch -> LDS buffer buf by DMA.  Wave w issues weight instructions w, w+8, .. (slots
  // [64 j, 64 j + 64): 2 chunks per row, chunk swizzle (row >> 3) & 1 = (lane >> 4) & 1 applied on
  // the source) and input-halo instructions w, w+8, ... of the halo region; the halo source
  // offsets (-1 = outside the image -> zero chunk) do not depend on the slab: computed once.
  const int fW = (lane & ~1) | ((lane & 1) ^ ((lane >> 4) & 1));
  int inOff[JI];
#pragma unroll
  for (int jj = 0; jj < JI; ++jj) {
    const int si = (wid + NWV * jj) * 64 + lane;
    const int lin = min(si >> 1, NPIX - 1), q = si & 1;
    const int hy = lin / HX, hx = lin - hy * HX;
    const int gy = ty0 + hy - 1, gx = tx0 + hx - 1;
    inOff[jj] = ((unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W) ? (gy * W + gx) * CIN + q * 8 : -1;
  }
  auto issue = [&](int ch, int buf) {
    const uint4* wsl = w4 + (long long)(nb * NCH + ch) * SW;
    uint4* dst = smem + buf * SB;
#pragma unroll
    for (int jj = 0; jj < JW; ++jj) {
      const int j = wid + NWV * jj;
      if (j < NWW)
        __builtin_amdgcn_global_load_lds((glb_void_t*)(wsl + j * 64 + fW), (lds_void_t*)(dst + j * 64), 16, 0, 0);
    }
#pragma unroll
    for (int jj = 0; jj < JI; ++jj) {
      const int j = wid + NWV * jj;
      if (j < NWIN) {
        const uint4* src = inOff[jj] >= 0 ? reinterpret_cast<const uint4*>(inb + inOff[jj] + ch * CK) : &g_conv_zero16;
        __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(dst + SW + j * 64), 16, 0, 0);
      }
    }
  };

  f32x16 acc[NSH];
#pragma unroll
  for (int p = 0; p < NSH; ++p)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[p][r] = 0.0f;

  // this wave's subtiles ph*NSH + p (p < nsub); padding lanes read a valid row, never stored
  const int nsub = min(NSH, NS - ph * NSH);
  int bIn[NSH];
#pragma unroll
  for (int p = 0; p < NSH; ++p) {
    const int px = min((ph * NSH + p) * 32 + l32, P - 1);
    bIn[p] = SW + ((px / TX) * HX + (px % TX)) * Q + h;
  }
  const int bW = (mt * 32 + l32) * Q + (h ^ ((l32 >> 3) & 1));

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int ch = 0; ch < NCH; ++ch) {
    if (ch + 1 < NCH) issue(ch + 1, (ch + 1) & 1);
    const uint4* sb = smem + (ch & 1) * SB;
    // wave-uniform subtile count, resolved to one of two unrolled bodies (no per-MFMA branch)
    auto mma = [&](auto cnt) {
      constexpr int C = decltype(cnt)::value;
#pragma unroll 1
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - 3 * (tap / 3);
        const bf16x8 a = __builtin_bit_cast(bf16x8, sb[bW + tap * BM * Q]);
#pragma unroll
        for (int p = 0; p < C; ++p) {
          const bf16x8 b = __builtin_bit_cast(bf16x8, sb[bIn[p] + (ky * HX + kx) * Q]);
          acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[p], 0, 0, 0);
        }
      }
    };
    if (nsub == NSH) mma(std::integral_constant<int, NSH>{});
    else mma(std::integral_constant<int, NSL>{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue (same semantics as k_conv3x3), output tile [P][QB] staged in LDS ----
  const int cb = nb * BM + mt * 32 + 4 * h;  // + 8 g: this lane's channel runs
  auto gpix = [&](int px) -> long long {
    const int gy = ty0 + px / TX, gx = tx0 + px % TX;
    if (px >= P || gy >= H || gx >= W) return -1;
    return ((long long)n * H + gy) * W + gx;
  };
  auto piece = [&](int px, int g) -> uint2* {
    const int k = mt * 4 + g;
    return reinterpret_cast<uint2*>(smem + px * QB + (k ^ swz<QB>(px))) + h;
  };
  auto cvec = [&](const float* v, int g) -> float4 {
    return *reinterpret_cast<const float4*>(v + cb + 8 * g);
  };
  if (ep.bias) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bv = cvec(ep.bias, g);
#pragma unroll
      for (int p = 0; p < NSH; ++p) {
        acc[p][4 * g + 0] += bv.x;
        acc[p][4 * g + 1] += bv.y;
        acc[p][4 * g + 2] += bv.z;
        acc[p][4 * g + 3] += bv.w;
      }
    }
  }
  if (ep.res) {
#pragma unroll
    for (int r = 0; r < OUT_R; ++r) {
      const int i = threadIdx.x + r * NT;
      if (i < P * QB) {
        const int px = i / QB, k = i - px * QB;
        const int gy = ty0 + px / TX, gx = tx0 + px % TX;
        uint4 v = {0u, 0u, 0u, 0u};
        if (gy < H && gx < W) {
          const long long rp = ep.res_up ? ((long long)n * (H >> 1) + (gy >> 1)) * (W >> 1) + (gx >> 1)
                                         : ((long long)n * H + gy) * W + gx;
          v = *reinterpret_cast<const uint4*>(ep.res + rp * COUT + nb * BM + k * 8);
        }
        smem[px * QB + (k ^ swz<QB>(px))] = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < NSH; ++p) {
      const int px = min((ph * NSH + p) * 32 + l32, P - 1);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint2 r = *piece(px, g);
        acc[p][4 * g + 0] += __uint_as_float(r.x << 16);
        acc[p][4 * g + 1] += __uint_as_float(r.x & 0xffff0000u);
        acc[p][4 * g + 2] += __uint_as_float(r.y << 16);
        acc[p][4 * g + 3] += __uint_as_float(r.y & 0xffff0000u);
      }
    }
    __syncthreads();
  }
  auto stage = [&]() {
#pragma unroll
    for (int p = 0; p < NSH; ++p) {
      const int px = (ph * NSH + p) * 32 + l32;
      if (px < P) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint2 o;
          o.x = pk_bf16(acc[p][4 * g + 0], acc[p][4 * g + 1]);
          o.y = pk_bf16(acc[p][4 * g + 2], acc[p][4 * g + 3]);
          *piece(px, g) = o;
        }
      }
    }
  };
  auto drain = [&](unsigned short* dst) {
#pragma unroll
    for (int r = 0; r < OUT_R; ++r) {
      const int i = threadIdx.x + r * NT;
      const int px = i / QB, k = i - px * QB;
      const long long gp = gpix(px);
      if (i < P * QB && gp >= 0)
        *reinterpret_cast<uint4*>(dst + gp * COUT + nb * BM + k * 8) = smem[px * QB + (k ^ swz<QB>(px))];
    }
  };
  if (ep.y) {
    stage();
    __syncthreads();
    drain(ep.y);
    __syncthreads();
  }
  if (!ep.z && !ep.head) return;
  if (ep.style) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 sv = cvec(ep.style + (long long)n * COUT, g);
#pragma unroll
      for (int p = 0; p < NSH; ++p) {
        acc[p][4 * g + 0] += sv.x;
        acc[p][4 * g + 1] += sv.y;
        acc[p][4 * g + 2] += sv.z;
        acc[p][4 * g + 3] += sv.w;
      }
    }
  }
  if (ep.scale) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 sc = cvec(ep.scale, g), sh = cvec(ep.shift, g);
#pragma unroll
      for (int p = 0; p < NSH; ++p) {
        acc[p][4 * g + 0] = sc.x * acc[p][4 * g + 0] + sh.x;
        acc[p][4 * g + 1] = sc.y * acc[p][4 * g + 1] + sh.y;
        acc[p][4 * g + 2] = sc.z * acc[p][4 * g + 2] + sh.z;
        acc[p][4 * g + 3] = sc.w * acc[p][4 * g + 3] + sh.w;
      }
    }
  }
  if (ep.relu) {
#pragma unroll
    for (int p = 0; p < NSH; ++p)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[p][r] = fmaxf(acc[p][r], 0.0f);
  }
  if constexpr (BM == 32) {
    if (ep.head) {
      // each lane holds 16 of its pixel's 32 channels (8 g + 4 h + k); the lane pair
      // (l, l ^ 32) completes the dot products
#pragma unroll
      for (int p = 0; p < NSH; ++p) {
        float o[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int c = 8 * g + 4 * h + k;
            const float zb = (float)(__bf16)acc[p][4 * g + k];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (j < ep.n_head) o[j] += ep.head_w[j * 32 + c] * zb;
          }
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += __shfl_xor(o[j], 32, 64);
        const int px = (ph * NSH + p) * 32 + l32;
        const long long gp = gpix(px);
        if (h == 0 && p < nsub && gp >= 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < ep.n_head) {
              const __bf16 v = (__bf16)(o[j] + ep.head_b[j]);
              ep.head[gp * ep.n_head + j] = __builtin_bit_cast(unsigned short, v);
            }
        }
      }
      return;
    }
  }
  stage();
  __syncthreads();
  if (!ep.z_up) {
    drain(ep.z);
  } else {
    const long long W2 = 2LL * W;
#pragma unroll
    for (int r = 0; r < 4 * OUT_R; ++r) {
      const int i = threadIdx.x + r * NT;
      if (i >= 4 * P * QB) continue;
      const int k = i % QB;
      const int d = i / QB;
      const int dy = d / (2 * TX), dx = d - dy * (2 * TX);
      const int px = (dy >> 1) * TX + (dx >> 1);
      const int gy = ty0 + (dy >> 1), gx = tx0 + (dx >> 1);
      if (gy >= H || gx >= W) continue;
      const long long dp = ((long long)n * 2 * H + 2LL * ty0 + dy) * W2 + 2LL * tx0 + dx;
      *reinterpret_cast<uint4*>(ep.z + dp * COUT + nb * BM + k * 8) = smem[px * QB + (k ^ swz<QB>(px))];
    }
  }
}

struct ConvCfg {
  int bn, ck, ty, tx;
};

// tile configuration per (Cin, Cout); must match the instantiations in launch()
bool conv_cfg(int cin, int cout, ConvCfg* c) {
  c->ck = 16;  // k_conv3x3w: 16-channel slabs, BM output channels per block
  if (cout == 32) {
    c->bn = 32;
    c->ty = 16;
    c->tx = 32;
  } else if (cout == 64) {
    c->bn = 64;
    c->ty = 16;
    c->tx = 28;
  } else if (cout == 128 || cout == 256) {
    c->bn = 128;
    c->ty = 14;
    c->tx = 28;
  } else {
    return false;
  }
  return (cin == 32 || cin == 64 || cin == 128 || cin == 256);
}

template <int CIN, int COUT, int BM, int TY, int TX>
int launch_wide(cpx_ctx* ctx, const void* in, const void* wpk, const ConvEpi& ep, int N, int H, int W) {
  const int tx = cpx_div_up(W, TX), ty = cpx_div_up(H, TY);
  const long long blocks = (long long)N * tx * ty;
  CPX_REQUIRE(blocks < (1LL << 31), CPX_ERR_ARG, "cpx_cpnet_conv3x3: too many tiles");
  hipLaunchKernelGGL((k_conv3x3w<CIN, COUT, BM, TY, TX>), dim3((unsigned)blocks, COUT / BM),
                     dim3(512), 0, ctx->stream, (const unsigned short*)in,
                     (const unsigned short*)wpk, ep, N, H, W, tx, ty);
  CPX_CHECK_LAUNCH("k_conv3x3w");
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

static int conv3x3_impl(cpx_ctx* ctx, const void* in, int N, int H, int W, int cin, int cout,
                        const void* wpk, const float* bias, const void* res, int res_up,
                        const float* style, const float* scale, const float* shift, int relu,
                        void* y_out, void* z_out, int z_up, const float* head_w,
                        const float* head_b, int n_head, void* head_out) {
  CPX_REQUIRE(ctx && in && wpk && (y_out || z_out || head_out), CPX_ERR_ARG,
              "cpx_cpnet_conv3x3: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0, CPX_ERR_ARG, "cpx_cpnet_conv3x3: bad sizes");
  CPX_REQUIRE(!(scale == nullptr) == !(shift == nullptr), CPX_ERR_ARG,
              "cpx_cpnet_conv3x3: scale and shift go together");
  CPX_REQUIRE(!res_up || ((H % 2) == 0 && (W % 2) == 0), CPX_ERR_ARG,
              "cpx_cpnet_conv3x3: res_up needs even sizes");
  CPX_REQUIRE(((uintptr_t)in | (uintptr_t)wpk) % 16 == 0 &&
                  ((uintptr_t)res | (uintptr_t)y_out | (uintptr_t)z_out) % 16 == 0,
              CPX_ERR_ARG, "cpx_cpnet_conv3x3: misaligned buffers");
  CPX_REQUIRE(!head_out || (cout == 32 && !z_out && head_w && head_b && n_head >= 1 && n_head <= 4),
              CPX_ERR_ARG, "cpx_cpnet_conv3x3_head: head needs cout 32, no z_out, 1..4 outputs");
  ConvEpi ep{bias, (const unsigned short*)res, style, scale, shift, (unsigned short*)y_out,
             (unsigned short*)z_out, res_up, relu, z_up, head_w, head_b,
             (unsigned short*)head_out, n_head};

#define CPX_CONVW(CI, CO, BM_, TY_, TX_)                             \
  if (cin == CI && cout == CO)                                       \
    return launch_wide<CI, CO, BM_, TY_, TX_>(ctx, in, wpk, ep, N, H, W);
  CPX_CONVW(32, 32, 32, 16, 32)
  CPX_CONVW(64, 32, 32, 16, 32)
  CPX_CONVW(32, 64, 64, 16, 28)
  CPX_CONVW(64, 64, 64, 16, 28)
  CPX_CONVW(128, 64, 64, 16, 28)
  CPX_CONVW(64, 128, 128, 14, 28)
  CPX_CONVW(128, 128, 128, 14, 28)
  CPX_CONVW(256, 128, 128, 14, 28)
  CPX_CONVW(128, 256, 128, 14, 28)
  CPX_CONVW(256, 256, 128, 14, 28)
#undef CPX_CONVW
  cpx_set_error("cpx_cpnet_conv3x3: unsupported channels %d -> %d", cin, cout);
  return CPX_ERR_SHAPE;
}

extern "C" int cpx_cpnet_conv3x3(cpx_ctx* ctx, const void* in, int N, int H, int W, int cin,
                                 int cout, const void* wpk, const float* bias, const void* res,
                                 int res_up, const float* style, const float* scale,
                                 const float* shift, int relu, void* y_out, void* z_out,
                                 int z_up) {
  return conv3x3_impl(ctx, in, N, H, W, cin, cout, wpk, bias, res, res_up, style, scale, shift,
                      relu, y_out, z_out, z_up, nullptr, nullptr, 0, nullptr);
}

extern "C" int cpx_cpnet_conv3x3_head(cpx_ctx* ctx, const void* in, int N, int H, int W, int cin,
                                      int cout, const void* wpk, const float* bias,
                                      const void* res, int res_up, const float* style,
                                      const float* scale, const float* shift, int relu,
                                      void* y_out, const float* head_w, const float* head_b,
                                      int n_head, void* head_out) {
  CPX_REQUIRE(head_out != nullptr, CPX_ERR_ARG, "cpx_cpnet_conv3x3_head: null head output");
  return conv3x3_impl(ctx, in, N, H, W, cin, cout, wpk, bias, res, res_up, style, scale, shift,
                      relu, y_out, nullptr, 0, head_w, head_b, n_head, head_out);
}
