// a6 CPnet at the reference's precision: 3x3 / 1x1 convolutions on split-fp16 activations
// (f16x3), the stem, the max-pool and the style vector — the fp32 U-Net of
// Cellpose_GPU_s3fs.py:108,143 (CellposeModel(gpu, model_type='nuclei'), no half precision)
// on the gfx950 fp16 matrix cores.
//
// Split format.  A value a (fp32) is stored as two fp16 halves, hi = f16(a) (round to nearest)
// and lo = f16((a - hi) * 2^11); a is read back as hi + lo * 2^-11 (one rounding), within
// 2^-22 |a| (below f16's normal range: 2^-35 absolute).  Activation tensors are NHWC with the
// channels in slabs of 16: per pixel and slab, 16 hi halves then 16 lo halves (64 bytes), i.e.
// 4 bytes per channel like fp32.  |a| >= 65504 does not fit: producers raise ovf[n] for the
// image n (network tile) whose activation it was, so the host can re-run only those FOVs.
// Products.  With weights split the same way (host, once), a product w x = wh xh + wh xl' 2^-11
// + wl' xh 2^-11 + O(2^-22 w x): per 16 input channels three v_mfma_f32_32x32x16_f16,
//   acc0 += Wh Xh,   acc1 += Wh Xl' + Wl' Xh,   result = acc0 + acc1 * 2^-11,
// fp32 accumulation as the fp32 network (products of two fp16 are exact in fp32).  Measured
// against the fp32 CPU network this reproduces its masks and object IDs, which
// the bf16 kernels of k_conv.hip do not.
//
// k_conv_x3<KS, CIN, COUT, BM, TY, TX, WM, WN>: implicit GEMM D[cout][pixel] = sum over (tap,
// cin) W[cout][cin][tap] X[pixel + tap][cin] for a TY x TX tile of one image and BM output
// channels; 512 threads = 8 waves = (BM / 32 / WM channel groups) x (pixel groups of WN 32-pixel
// subtiles); a wave owns WM 32-channel slices x WN subtiles (2 accumulator sets).  Input
// channels go in slabs of 16: the slab's halo tile (64 B per pixel) and its [tap][BM][hi|lo][16]
// weights are double-buffered in LDS and filled by LDS-DMA (global_load_lds_dwordx4), the
// 16-byte chunks XOR-swizzled on the source address (chunk c of row r at slot c ^ ((r >> 2) & 3))
// so the fragment reads are bank-conflict free.  Epilogue (same semantics as k_conv.hip): bias,
// residual (split, optionally read nearest-upsampled), residual-stream store, style bias, eval
// BatchNorm, ReLU, next-input store (optionally 2x nearest-upsampled) or the CPnet output head
// (fp32), all on the fp32 values; output tiles go through LDS as whole 16-byte chunks.
#include "cpx_internal.h"
#include <type_traits>
#include <stdlib.h>

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr float kLoScale = 2048.0f;
constexpr float kLoInv = 1.0f / 2048.0f;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

__device__ uint4 g_x3_zero16 = {0u, 0u, 0u, 0u};

__device__ __forceinline__ int swz4(int row) { return (row >> 2) & 3; }

// output-tile chunk swizzle (Q chunks per pixel row)
template <int Q>
__device__ __forceinline__ int swzq(int row) {
  if constexpr (Q >= 16) return row & 15;
  else if constexpr (Q == 8) return (row >> 1) & 7;
  else if constexpr (Q == 4) return (row >> 2) & 3;
  else return 0;
}

// 4 fp32 -> (hi, lo) 8-byte pieces; bad |= not representable.  A value outside the fp16 range
// is stored saturated (+-65504, NaN -> -65504): the image is flagged and re-run in fp32 by the
// host, and no inf / NaN reaches the kernels after the network (flows stay finite)
__device__ __forceinline__ void split4(float a, float b, float c, float d, uint2& hi, uint2& lo, bool& bad) {
  const float v[4] = {a, b, c, d};
  f16x4 h, l;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    bad |= !(fabsf(v[k]) < 65504.0f);
    const float vc = fminf(fmaxf(v[k], -65504.0f), 65504.0f);
    const _Float16 t = (_Float16)vc;
    h[k] = t;
    l[k] = (_Float16)((vc - (float)t) * kLoScale);
  }
  hi = __builtin_bit_cast(uint2, h);
  lo = __builtin_bit_cast(uint2, l);
}

__device__ __forceinline__ void join4(const uint2& hi, const uint2& lo, float* out) {
  const f16x4 h = __builtin_bit_cast(f16x4, hi), l = __builtin_bit_cast(f16x4, lo);
#pragma unroll
  for (int k = 0; k < 4; ++k) out[k] = (float)h[k] + (float)l[k] * kLoInv;
}

// 8 channels: hi chunk + lo chunk -> fp32
__device__ __forceinline__ void join8(const uint4& hi, const uint4& lo, float* out) {
  join4(make_uint2(hi.x, hi.y), make_uint2(lo.x, lo.y), out);
  join4(make_uint2(hi.z, hi.w), make_uint2(lo.z, lo.w), out + 4);
}

__device__ __forceinline__ void split8(const float* v, uint4& hi, uint4& lo, bool& bad) {
  uint2 h0, l0, h1, l1;
  split4(v[0], v[1], v[2], v[3], h0, l0, bad);
  split4(v[4], v[5], v[6], v[7], h1, l1, bad);
  hi = make_uint4(h0.x, h0.y, h1.x, h1.y);
  lo = make_uint4(l0.x, l0.y, l1.x, l1.y);
}

// The epilogue's y / z tile stores are non-temporal (streamed past L2: the next reader is another
// launch, and the halo lines the tile loop prefetches stay cached; p32 2.22 -> 2.17 ms per call,
// the deep levels unchanged, `gpurun_out/r05j`)

struct X3Epi {
  const float* bias;
  const uint4* res;    // split [N][h][w][COUT] (res_up: [N][h/2][w/2][COUT])
  const float* style;  // [N][style_stride] (+ channel)
  const float* scale;
  const float* shift;
  uint4* y;            // residual stream (split)
  uint4* z;            // next convolution's input (split; z_up: 2x nearest-upsampled)
  int res_up, relu, z_up, style_stride;
  const float* head_w;  // [n_head][32]
  const float* head_b;
  float* head;          // fp32 [N][h][w][n_head]
  int n_head;
  int* ovf;
  int in_up;  // the input is the (H/2) x (W/2) tensor read 2x nearest-upsampled
  // block projection folded into the convolution (k_conv_x3 with CIN2 > 0): after the 3x3 slabs
  // of `in`, CIN2 / 16 one-tap slabs of in2 [N][H][W][CIN2] (split) with weights wpk2
  // [COUT/BM][CIN2/16][BM][hi|lo][16] accumulate conv1x1(in2, wp) into the same sums
  const uint4* in2;
  const uint4* wpk2;
  // 2x2/2 max-pool of the y tile (k_cpnet_pool_x3's arithmetic, fused into the epilogue of a down
  // block's last convolution): pool_x [N][H/2][W/2][COUT] = the maximum's own hi/lo pair and
  // pool_z = split(relu(pool_scale x + pool_shift)), the next block's input and its BatchNorm+ReLU
  uint4* pool_x;
  uint4* pool_z;
  const float* pool_scale;
  const float* pool_shift;
};

// Epilogue of a 3x3 / 1x1 convolution tile on its fp32 values (acc0 = the joined sums): bias,
// residual, residual-stream store, style, eval BatchNorm, ReLU, next-input store or output head.
// Every thread of the block takes part (the output tile is staged through smem); waves without a
// subtile (j >= nsub) only move data.
// res_lds (optional): the residual tile already in LDS in the staging layout (k_conv_x3 DMAs it
// into its free slab buffer during the last slab); y is then staged in `smem` and z in the
// residual's buffer (y-less calls: z in `smem`), which needs two block barriers instead of six and
// no global-load wait.
template <int COUT, int BM, int TY, int TX, int WM, int WN>
__device__ __forceinline__ void x3_epilogue(f32x16 (&acc0)[WM][WN], const X3Epi& ep, uint4* smem, int n,
                                            int nb, int ty0, int tx0, int H, int W, int mw, int pg, int nsub,
                                            int tid = -1, uint4* res_lds = nullptr) {
  // tid: threadIdx.x, or a per-tile opaque copy of it from a persistent caller (the staging
  // offsets derived from it are then recomputed per tile instead of hoisted and spilled)
  if (tid < 0) tid = threadIdx.x;
  uint4* const ybuf = smem;
  uint4* const zbuf = (res_lds && ep.y) ? res_lds : smem;
  constexpr int NT = 512;
  constexpr int P = TY * TX;
  constexpr int QB = BM / 4;
  constexpr int QC = COUT / 4;
  constexpr int OUT_R = (P * QB + NT - 1) / NT;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5, l32 = lane & 31;
  bool bad = false;
  auto gpix = [&](int px) -> long long {
    const int gy = ty0 + px / TX, gx = tx0 + px % TX;
    if (px >= P || gy >= H || gx >= W) return -1;
    return ((long long)n * H + gy) * W + gx;
  };
  // lane's channel group (m, g): channels cb(m) + 8 g + {0..3} of the block, slab (m', g >> 1)
  auto slice = [&](int m) { return mw * WM + m; };
  auto piece = [&](const uint4* buf, int px, int m, int g, int lo) -> uint2* {
    const int q = (slice(m) * 2 + (g >> 1)) * 4 + 2 * lo + (g & 1);
    return reinterpret_cast<uint2*>(const_cast<uint4*>(buf) + px * QB + (q ^ swzq<QB>(px))) + h;
  };
  auto chan = [&](int m, int g) { return nb * BM + slice(m) * 32 + 8 * g + 4 * h; };
  if (ep.bias) {
#pragma unroll
    for (int m = 0; m < WM; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bv = *reinterpret_cast<const float4*>(ep.bias + chan(m, g));
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          acc0[m][j][4 * g + 0] += bv.x;
          acc0[m][j][4 * g + 1] += bv.y;
          acc0[m][j][4 * g + 2] += bv.z;
          acc0[m][j][4 * g + 3] += bv.w;
        }
      }
  }
  if (ep.res) {
    const uint4* rbuf = res_lds ? res_lds : smem;
    if (!res_lds) {
#pragma unroll
      for (int r = 0; r < OUT_R; ++r) {
        const int i = tid + r * NT;
        if (i < P * QB) {
          const int px = i / QB, k = i - px * QB;
          const int gy = ty0 + px / TX, gx = tx0 + px % TX;
          uint4 v = {0u, 0u, 0u, 0u};
          if (gy < H && gx < W) {
            const long long rp = ep.res_up ? ((long long)n * (H >> 1) + (gy >> 1)) * (W >> 1) + (gx >> 1)
                                           : ((long long)n * H + gy) * W + gx;
            v = ep.res[rp * QC + nb * QB + k];
          }
          smem[px * QB + (k ^ swzq<QB>(px))] = v;
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int px = min((pg * WN + j) * 32 + l32, P - 1);
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float rv[4];
          join4(*piece(rbuf, px, m, g, 0), *piece(rbuf, px, m, g, 1), rv);
#pragma unroll
          for (int k = 0; k < 4; ++k) acc0[m][j][4 * g + k] += rv[k];
        }
    }
    if (!res_lds) __syncthreads();  // (res_lds: y is staged in the other buffer, z after y's barrier)
  }
  auto stage = [&](uint4* buf) {
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int px = (pg * WN + j) * 32 + l32;
      if (j < nsub && px < P) {
#pragma unroll
        for (int m = 0; m < WM; ++m)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            uint2 hi, lo;
            split4(acc0[m][j][4 * g], acc0[m][j][4 * g + 1], acc0[m][j][4 * g + 2], acc0[m][j][4 * g + 3],
                   hi, lo, bad);
            *piece(buf, px, m, g, 0) = hi;
            *piece(buf, px, m, g, 1) = lo;
          }
      }
    }
  };
  auto drain = [&](const uint4* buf, uint4* dst) {
#pragma unroll
    for (int r = 0; r < OUT_R; ++r) {
      const int i = tid + r * NT;
      const int px = i / QB, k = i - px * QB;
      const long long gp = gpix(px);
      if (i < P * QB && gp >= 0) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, buf[px * QB + (k ^ swzq<QB>(px))]),
                                    reinterpret_cast<u32x4*>(dst + gp * QC + nb * QB + k));
      }
    }
  };
  auto flag = [&]() {
    if (ep.ovf && __ballot(bad)) {
      if (lane == 0) atomicOr(ep.ovf + n, 1);
    }
  };
  if (ep.y) {
    stage(ybuf);
    __syncthreads();
    drain(ybuf, ep.y);
    if (ep.pool_x) {
      // pooled pixel (py, px) of the tile from staged pixels (2py + a, 2px + b), first maximum in
      // the order (0,0) (0,1) (1,0) (1,1) as k_cpnet_pool_x3; one item per (pooled pixel, group of 8)
      static_assert(TY % 2 == 0 && TX % 2 == 0, "pooled tiles");
      constexpr int PH = TY / 2, PW2 = TX / 2, G8 = BM / 8;
      for (int it = tid; it < PH * PW2 * G8; it += NT) {
        const int gi = it % G8, pp = it / G8;
        const int py = pp / PW2, px = pp - py * PW2;
        const int gy = ty0 / 2 + py, gx = tx0 / 2 + px;
        if (2 * gy >= H || 2 * gx >= W) continue;
        const int q = (gi >> 1) * 4 + (gi & 1);  // hi chunk of the group in the block; lo = q + 2
        float best[8];
        f16x8 mh, ml;
#pragma unroll
        for (int sidx = 0; sidx < 4; ++sidx) {
          const int spx = (2 * py + (sidx >> 1)) * TX + 2 * px + (sidx & 1);
          const uint4 ch = ybuf[spx * QB + (q ^ swzq<QB>(spx))];
          const uint4 cl = ybuf[spx * QB + ((q + 2) ^ swzq<QB>(spx))];
          float f[8];
          join8(ch, cl, f);
          const f16x8 fh = __builtin_bit_cast(f16x8, ch), fl = __builtin_bit_cast(f16x8, cl);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (sidx == 0 || f[k] > best[k]) {  // max_pool2d: first maximum
              best[k] = f[k];
              mh[k] = fh[k];
              ml[k] = fl[k];
            }
        }
        const long long op = ((long long)n * (H / 2) + gy) * (W / 2) + gx;
        ep.pool_x[op * QC + nb * QB + q] = __builtin_bit_cast(uint4, mh);
        ep.pool_x[op * QC + nb * QB + q + 2] = __builtin_bit_cast(uint4, ml);
        const int c0 = nb * BM + gi * 8;
        float zz[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) zz[k] = fmaxf(ep.pool_scale[c0 + k] * best[k] + ep.pool_shift[c0 + k], 0.0f);
        uint4 zh, zl;
        split8(zz, zh, zl, bad);
        ep.pool_z[op * QC + nb * QB + q] = zh;
        ep.pool_z[op * QC + nb * QB + q + 2] = zl;
      }
    }
    if (zbuf == ybuf) __syncthreads();  // z is staged over y's tile
  }
  if (!ep.z && !ep.head) {
    flag();
    return;
  }
  if (ep.style) {
#pragma unroll
    for (int m = 0; m < WM; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 sv = *reinterpret_cast<const float4*>(ep.style + (long long)n * ep.style_stride + chan(m, g));
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          acc0[m][j][4 * g + 0] += sv.x;
          acc0[m][j][4 * g + 1] += sv.y;
          acc0[m][j][4 * g + 2] += sv.z;
          acc0[m][j][4 * g + 3] += sv.w;
        }
      }
  }
  if (ep.scale) {
#pragma unroll
    for (int m = 0; m < WM; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 sc = *reinterpret_cast<const float4*>(ep.scale + chan(m, g));
        const float4 sh = *reinterpret_cast<const float4*>(ep.shift + chan(m, g));
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          acc0[m][j][4 * g + 0] = sc.x * acc0[m][j][4 * g + 0] + sh.x;
          acc0[m][j][4 * g + 1] = sc.y * acc0[m][j][4 * g + 1] + sh.y;
          acc0[m][j][4 * g + 2] = sc.z * acc0[m][j][4 * g + 2] + sh.z;
          acc0[m][j][4 * g + 3] = sc.w * acc0[m][j][4 * g + 3] + sh.w;
        }
      }
  }
  if (ep.relu) {
#pragma unroll
    for (int m = 0; m < WM; ++m)
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc0[m][j][r] = fmaxf(acc0[m][j][r], 0.0f);
  }
  if constexpr (COUT == 32 && BM == 32 && WM == 1) {
    if (ep.head) {
      // fp32 output 1x1 convolution: lane l and l ^ 32 hold the two halves of a pixel's channels
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        float o[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int c = 8 * g + 4 * h + k;
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (q < ep.n_head) o[q] = __builtin_fmaf(ep.head_w[q * 32 + c], acc0[0][j][4 * g + k], o[q]);
          }
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] += __shfl_xor(o[q], 32, 64);
        const int px = (pg * WN + j) * 32 + l32;
        const long long gp = gpix(px);
        if (h == 0 && j < nsub && gp >= 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (q < ep.n_head) ep.head[gp * ep.n_head + q] = o[q] + ep.head_b[q];
        }
      }
      flag();
      return;
    }
  }
  stage(zbuf);
  __syncthreads();
  if (!ep.z_up) {
    drain(zbuf, ep.z);
  } else {
    const long long W2 = 2LL * W;
#pragma unroll
    for (int r = 0; r < 4 * OUT_R; ++r) {
      const int i = tid + r * NT;
      if (i >= 4 * P * QB) continue;
      const int k = i % QB;
      const int d = i / QB;
      const int dy = d / (2 * TX), dx = d - dy * (2 * TX);
      const int px = (dy >> 1) * TX + (dx >> 1);
      const int gy = ty0 + (dy >> 1), gx = tx0 + (dx >> 1);
      if (gy >= H || gx >= W) continue;
      const long long dp = ((long long)n * 2 * H + 2LL * ty0 + dy) * W2 + 2LL * tx0 + dx;
      ep.z[dp * QC + nb * QB + k] = zbuf[px * QB + (k ^ swzq<QB>(px))];
    }
  }
  flag();
}

// Instruction-scheduling hint after an unrolled tap loop: iglp_opt(0), the compiler's MFMA /
// DS-read interleave — the 32-channel-block kernels 2.5-3 % faster, bit-identical outputs
// (`gpurun_out/r05y`; sched_group_barrier groups that issue tap t + 1's fragment reads before tap
// t's MFMAs measured ~1 %).  The 224^2 persistent kernel takes the same hint after each slab's
// taps (-2.3 %, `gpurun_out/r05z`); the multi-fragment loop with one tap per iteration does not
// (+-1 % and more spills).
__device__ __forceinline__ void x3_sched() { __builtin_amdgcn_iglp_opt(0); }

template <int KS, int CIN, int COUT, int BM, int TY, int TX, int WM, int WN, int WPE, int CIN2 = 0, int NBUF = 2>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_conv_x3(const uint4* __restrict__ in, const uint4* __restrict__ wpk, X3Epi ep, int N, int H,
               int W, int tiles_x, int tiles_y) {
  constexpr int NT = 512, NWV = NT / 64;
  constexpr int T = KS * KS, HALO = KS / 2;
  constexpr int MWV = BM / (32 * WM), PW = NWV / MWV;
  constexpr int HY = TY + KS - 1, HX = TX + KS - 1, NPIX = HY * HX;
  constexpr int NCH = CIN / 16;
  constexpr int NCH2 = CIN2 / 16, QI2 = CIN2 / 4;     // folded projection slabs (one tap each)
  constexpr int NW2 = BM * 4 / 64;                    // their weight DMA rows
  static_assert(CIN2 == 0 || (KS == 3 && CIN2 % 16 == 0), "projection slabs fold into a 3x3 conv");
  constexpr int P = TY * TX, NS = (P + 31) / 32;
  constexpr int SW = T * BM * 4;                      // 16-byte slots [tap][BM][4 chunks]
  constexpr int SI = (NPIX * 4 + 63) / 64 * 64;       // [halo pixel][4 chunks]
  constexpr int SB = SW + SI;
  constexpr int NWW = SW / 64, NWIN = SI / 64;
  constexpr int JW = (NWW + NWV - 1) / NWV, JI = (NWIN + NWV - 1) / NWV;
  constexpr int QB = BM / 4;                          // output chunks per pixel (hi + lo)
  constexpr int QC = COUT / 4;                        // chunks per pixel of a COUT tensor
  constexpr int QI = CIN / 4;
  constexpr int OUT_R = (P * QB + NT - 1) / NT;
  static_assert(CIN % 16 == 0 && COUT % BM == 0 && BM % (32 * WM) == 0 && NWV % MWV == 0, "shape");
  static_assert(PW * WN >= NS, "every subtile needs a wave");
  static_assert(SW % 64 == 0, "weight DMA rows");
  // NBUF 2: slab c + 1 streams into the second buffer under slab c's MFMAs; NBUF 1: one slab
  // buffer (half the LDS per block, so more blocks per CU cover each other's DMA waits)
  static_assert(NBUF == 1 || NBUF == 2, "slab buffers");
  constexpr int SMEM = NBUF == 2 ? 2 * SB : (P * QB > SB ? P * QB : SB);
  static_assert(P * QB <= SMEM, "output tile must fit the staging LDS");
  // projection slabs packed PK per slab buffer: a projection slab reads only the tile's centre
  // pixels (P * 4 slots, no halo) and one tap of weights (BM * 4 slots), so two fit where a 3x3
  // slab's nine weight taps and halo go — half the DMA waits and barriers of the projection
  constexpr int NPR = (P * 4 + 63) / 64;              // centre-pixel DMA rows of one projection slab
  constexpr int PK = (CIN2 > 0 && 2 * BM * 4 + 2 * NPR * 64 <= SB) ? 2 : 1;
  constexpr int NCHP = (NCH2 + PK - 1) / PK;          // projection slab buffers
  static_assert(SMEM * 16 <= 163840, "LDS");
  __shared__ uint4 smem[SMEM];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int mw = wid % MWV, pg = wid / MWV;
  const int h = lane >> 5, l32 = lane & 31;
  const int tiles = tiles_x * tiles_y;
  // XCD-aware order: the hardware deals consecutive block ids round-robin over the 8 XCDs, so
  // block b runs on XCD b % 8; give each XCD a contiguous run of items instead.  An item is
  // (tile, output-channel block nb) with nb fastest, so the COUT / BM blocks of one tile run
  // together on one XCD and read its input halo once from HBM (the rest from that XCD's L2), and
  // vertically adjacent tiles (which share halo rows) meet in the same L2
  constexpr int NB = COUT / BM;
  const int G = gridDim.x, xq = G >> 3, xr = G & 7, xb = blockIdx.x & 7;
  const int bid = xb * xq + min(xb, xr) + (blockIdx.x >> 3);
  const int tile = bid / NB, nb = bid - tile * NB;
  const int n = tile / tiles;
  const int t = tile - n * tiles;
  const int ty0 = (t / tiles_x) * TY, tx0 = (t % tiles_x) * TX;
  // in_up: the source pixel of (gy, gx) is (gy / 2, gx / 2) of the half-size input (nearest 2x
  // upsampling folded into the halo DMA; the L2 serves each source line to four output pixels)
  const int iu = ep.in_up, Wi = W >> iu;
  const uint4* inb = in + (long long)n * (H >> iu) * Wi * QI;

  // DMA sources: weights (lane-constant swizzle), halo pixel + chunk (slab-independent)
  const int fW = (lane & ~3) | ((lane & 3) ^ ((lane >> 4) & 3));
  int inPC[JI];  // source pixel * 4 + swizzled chunk, -1 outside the image
#pragma unroll
  for (int jj = 0; jj < JI; ++jj) {
    const int si = (wid + NWV * jj) * 64 + lane;
    const int hp = si >> 2, cq = si & 3;
    const int hy = hp / HX, hx = hp - (hp / HX) * HX;
    const int gy = ty0 + hy - HALO, gx = tx0 + hx - HALO;
    inPC[jj] = (hp < NPIX && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W)
                   ? ((gy >> iu) * Wi + (gx >> iu)) * 4 + (cq ^ swz4(hp)) : -1;
  }
  const uint4* inb2 = CIN2 ? ep.in2 + (long long)n * H * W * QI2 : nullptr;
  // the residual tile, DMA'd during the last slab into the slab buffer that slab does not use, in
  // the epilogue's staging layout (chunk k of pixel px at px * QB + (k ^ swzq(px)))
  constexpr int NCHT_ = NCH + NCHP;
  constexpr bool kResPre = NBUF == 2 && P * QB <= SB;
  uint4* const bufO = smem + (NBUF == 2 ? ((NCHT_ - 1) & 1) * SB : 0);  // the last slab's buffer
  uint4* const bufR = smem + (NBUF == 2 ? (NCHT_ & 1) * SB : 0);        // free during the last slab
  auto issue_res = [&]() {
    constexpr int NRR = (P * QB + 63) / 64, JR = (NRR + NWV - 1) / NWV;
#pragma unroll
    for (int jj = 0; jj < JR; ++jj) {
      const int j = wid + NWV * jj;
      if (j < NRR) {
        const int sl = j * 64 + lane;
        const int px = sl / QB, kk = (sl - (sl / QB) * QB) ^ swzq<QB>(px);
        const int gy = ty0 + px / TX, gx = tx0 + px % TX;
        const uint4* src = &g_x3_zero16;
        if (sl < P * QB && gy < H && gx < W) {
          const long long rp = ep.res_up ? ((long long)n * (H >> 1) + (gy >> 1)) * (W >> 1) + (gx >> 1)
                                         : ((long long)n * H + gy) * W + gx;
          src = ep.res + rp * QC + nb * QB + kk;
        }
        __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(bufR + j * 64), 16, 0, 0);
      }
    }
  };
  // slab ch < NCH: the 3x3 weights and the halo of `in`; ch >= NCH: a projection slab (one tap
  // of weights, the halo of in2 — only its centre is read)
  auto issue = [&](int ch, int buf) {
    uint4* dst = smem + buf * SB;
    if (CIN2 == 0 || ch < NCH) {
      const uint4* wsl = wpk + (long long)(nb * NCH + ch) * SW;
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
          const uint4* src = inPC[jj] >= 0 ? inb + (long long)(inPC[jj] >> 2) * QI + (inPC[jj] & 3) + ch * 4
                                           : &g_x3_zero16;
          __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(dst + SW + j * 64), 16, 0, 0);
        }
      }
    } else if constexpr (PK == 1) {
      const int c2 = ch - NCH;
      const uint4* wsl = ep.wpk2 + (long long)(nb * NCH2 + c2) * (BM * 4);
      if (wid < NW2)
        __builtin_amdgcn_global_load_lds((glb_void_t*)(wsl + wid * 64 + fW), (lds_void_t*)(dst + wid * 64), 16, 0, 0);
#pragma unroll
      for (int jj = 0; jj < JI; ++jj) {
        const int j = wid + NWV * jj;
        if (j < NWIN) {
          const uint4* src = inPC[jj] >= 0 ? inb2 + (long long)(inPC[jj] >> 2) * QI2 + (inPC[jj] & 3) + c2 * 4
                                           : &g_x3_zero16;
          __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(dst + SW + j * 64), 16, 0, 0);
        }
      }
    } else {
      // packed: weights of slab u at [u BM 4, ...), its centre pixels at [PK BM 4 + u NPR 64, ...)
      // (pixel p, chunk k at slot p * 4 + (k ^ swz4(p)), as the halo layout without the halo)
#pragma unroll
      for (int u = 0; u < PK; ++u) {
        const int c2 = (ch - NCH) * PK + u;
        if (c2 < NCH2) {
          const uint4* wsl = ep.wpk2 + (long long)(nb * NCH2 + c2) * (BM * 4);
          if (wid < NW2)
            __builtin_amdgcn_global_load_lds((glb_void_t*)(wsl + wid * 64 + fW),
                                             (lds_void_t*)(dst + u * BM * 4 + wid * 64), 16, 0, 0);
#pragma unroll
          for (int jj = 0; jj < (NPR + NWV - 1) / NWV; ++jj) {
            const int j = wid + NWV * jj;
            if (j < NPR) {
              const int si = j * 64 + lane, pp = si >> 2, cq = si & 3;
              const int gy = ty0 + pp / TX, gx = tx0 + pp % TX;
              const uint4* src = (pp < P && gy < H && gx < W)
                                     ? inb2 + ((long long)gy * W + gx) * QI2 + (cq ^ swz4(pp)) + c2 * 4
                                     : &g_x3_zero16;
              __builtin_amdgcn_global_load_lds((glb_void_t*)src,
                                               (lds_void_t*)(dst + PK * BM * 4 + u * NPR * 64 + j * 64), 16, 0, 0);
            }
          }
        }
      }
    }
  };

  f32x16 acc0[WM][WN], acc1[WM][WN];
#pragma unroll
  for (int m = 0; m < WM; ++m)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc0[m][j][r] = 0.0f;
        acc1[m][j][r] = 0.0f;
      }

  const int nsub = max(0, min(WN, NS - pg * WN));
  int aS[WM];
#pragma unroll
  for (int m = 0; m < WM; ++m) {
    const int r = (mw * WM + m) * 32 + l32;
    aS[m] = r * 4 + (h ^ swz4(r));
  }
  int hp0[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int px = min((pg * WN + j) * 32 + l32, P - 1);
    hp0[j] = (px / TX) * HX + (px % TX);
  }

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr int NCHT = NCH + NCHP;
  // weights of tap `tw` against the halo at (ky, kx) of slab buffer sb, over C subtiles
  auto tapbody = [&](auto cnt, const uint4* sb, int tw, int ky, int kx) {
    constexpr int C = decltype(cnt)::value;
    f16x8 ah[WM], al[WM];
#pragma unroll
    for (int m = 0; m < WM; ++m) {
      ah[m] = __builtin_bit_cast(f16x8, sb[aS[m] + tw * BM * 4]);
      al[m] = __builtin_bit_cast(f16x8, sb[(aS[m] ^ 2) + tw * BM * 4]);
    }
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const int hp = hp0[j] + ky * HX + kx;
      const int bs = SW + hp * 4 + (h ^ swz4(hp));
      const f16x8 bh = __builtin_bit_cast(f16x8, sb[bs]);
      const f16x8 bl = __builtin_bit_cast(f16x8, sb[bs ^ 2]);
#pragma unroll
      for (int m = 0; m < WM; ++m) {
        acc0[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[m], bh, acc0[m][j], 0, 0, 0);
        acc1[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[m], bl, acc1[m][j], 0, 0, 0);
        acc1[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[m], bh, acc1[m][j], 0, 0, 0);
      }
    }
  };
  // the wave's subtile count as a compile-time constant
  auto per_nsub = [&](auto body) {
    if constexpr (WN == 1) {
      if (nsub == 1) body(std::integral_constant<int, 1>{});
    } else if constexpr (WN == 2) {
      if (nsub == 2) body(std::integral_constant<int, 2>{});
      else if (nsub == 1) body(std::integral_constant<int, 1>{});
    } else {
      static_assert(WN <= 2, "WN");
    }
  };
  for (int ch = 0; ch < NCH; ++ch) {
    if (NBUF == 2 && ch + 1 < NCHT) issue(ch + 1, (ch + 1) & 1);
    if (kResPre && ch + 1 == NCHT && ep.res) issue_res();
    const uint4* sb = smem + (NBUF == 2 ? (ch & 1) * SB : 0);
    per_nsub([&](auto cnt) {
      if constexpr (WM * WN == 1) {
        // single-fragment waves: all taps unrolled, the next tap's reads scheduled under this
        // tap's MFMAs; larger wave tiles keep one tap per iteration (register budget)
#pragma unroll
        for (int tap = 0; tap < T; ++tap) tapbody(cnt, sb, tap, tap / KS, tap % KS);
        x3_sched();
      } else {
        // multi-fragment waves: the two-slice BM 64 tile (WM 2, WN 1) unrolls all nine taps with
        // the interleave hint, like the single-fragment loop, where the registers allow it (no
        // folded projection, CIN >= 64): -6 to -7.5 % on those kernels, bit-identical
        // (`gpurun_out/r05ab`); CIN 32, the projection-folded forms and the WN 2 tiles spill
        // unrolled and keep one tap per iteration
        if constexpr (WM == 2 && WN == 1 && CIN2 == 0 && CIN >= 64) {
#pragma unroll
          for (int tap = 0; tap < T; ++tap) tapbody(cnt, sb, tap, tap / KS, tap % KS);
          x3_sched();
        } else {
#pragma unroll 1
          for (int tap = 0; tap < T; ++tap) tapbody(cnt, sb, tap, tap / KS, tap % KS);
        }
      }
    });
    if (NBUF == 1) {  // every wave is done with the buffer before the next slab lands in it
      __syncthreads();
      if (ch + 1 < NCHT) issue(ch + 1, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // folded projection: one centre tap per slab of in2 (weight slot 0)
#pragma unroll 1
  for (int ch = NCH; ch < NCHT; ++ch) {
    if (NBUF == 2 && ch + 1 < NCHT) issue(ch + 1, (ch + 1) & 1);
    if (kResPre && ch + 1 == NCHT && ep.res) issue_res();
    const uint4* sb = smem + (NBUF == 2 ? (ch & 1) * SB : 0);
    if constexpr (PK == 1) {
      per_nsub([&](auto cnt) { tapbody(cnt, sb, 0, HALO, HALO); });
    } else {
      // the packed slabs in channel order, each the centre tap's MFMAs of tapbody
      per_nsub([&](auto cnt) {
        constexpr int C = decltype(cnt)::value;
#pragma unroll
        for (int u = 0; u < PK; ++u) {
          if ((ch - NCH) * PK + u < NCH2) {
            f16x8 ah[WM], al[WM];
#pragma unroll
            for (int m = 0; m < WM; ++m) {
              ah[m] = __builtin_bit_cast(f16x8, sb[aS[m] + u * BM * 4]);
              al[m] = __builtin_bit_cast(f16x8, sb[(aS[m] ^ 2) + u * BM * 4]);
            }
#pragma unroll
            for (int j = 0; j < C; ++j) {
              const int pp = min((pg * WN + j) * 32 + l32, P - 1);
              const int bs = PK * BM * 4 + u * NPR * 64 + pp * 4 + (h ^ swz4(pp));
              const f16x8 bh = __builtin_bit_cast(f16x8, sb[bs]);
              const f16x8 bl = __builtin_bit_cast(f16x8, sb[bs ^ 2]);
#pragma unroll
              for (int m = 0; m < WM; ++m) {
                acc0[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[m], bh, acc0[m][j], 0, 0, 0);
                acc1[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[m], bl, acc1[m][j], 0, 0, 0);
                acc1[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[m], bh, acc1[m][j], 0, 0, 0);
              }
            }
          }
        }
      });
    }
    if (NBUF == 1) {
      __syncthreads();
      if (ch + 1 < NCHT) issue(ch + 1, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue on the fp32 values ----
#pragma unroll
  for (int m = 0; m < WM; ++m)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc0[m][j][r] += acc1[m][j][r] * kLoInv;  // exact product, one rounding

  if constexpr (kResPre)
    x3_epilogue<COUT, BM, TY, TX, WM, WN>(acc0, ep, bufO, n, nb, ty0, tx0, H, W, mw, pg, nsub, -1,
                                          ep.res ? bufR : nullptr);
  else
    x3_epilogue<COUT, BM, TY, TX, WM, WN>(acc0, ep, smem, n, nb, ty0, tx0, H, W, mw, pg, nsub);
}

// The 224^2 level's 32 -> 32 convolutions as a persistent grid: both slabs of the weights
// (36 KiB) are loaded into LDS once per block, and each block walks a run of 8 x 32 tiles loading
// only the tile's halo (both slabs, 43.5 KiB: one wait per tile instead of a weight + halo DMA per
// slab); the halo buffer then stages the tile's epilogue.  80 KiB per block, two per CU.  The
// tiles of one XCD form a contiguous range that its blocks walk in step, so vertically adjacent
// tiles (which share halo rows) are in flight together in that XCD's L2.  Per output pixel the
// sums are formed in k_conv_x3's slab / tap / MFMA order: bit-identical results.
template <int kP32Touch>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
void k_conv_x3_p32(const uint4* __restrict__ in, const uint4* __restrict__ wpk, X3Epi ep, int N, int H,
                   int W, int tiles_x, int tiles_y) {
  constexpr int NWV = 8, BM = 32, T = 9, TY = 8, TX = 32, HX = TX + 2, NPIX = (TY + 2) * HX;
  constexpr int NCH = 2, QI = 8;
  constexpr int SW = T * BM * 4;                   // one slab's weights, 16-byte slots
  constexpr int SI = (NPIX * 4 + 63) / 64 * 64;    // one slab of the halo
  constexpr int NWW = NCH * SW / 64, NWIN = SI / 64;
  constexpr int JW = (NWW + NWV - 1) / NWV, JI = (NWIN + NWV - 1) / NWV;
  static_assert(TY * TX * (BM / 4) <= NCH * SI, "the epilogue stages in the halo buffer");
  static_assert((NCH * SW + NCH * SI) * 16 <= 81920, "two blocks per CU");
  __shared__ uint4 smem[NCH * SW + NCH * SI];
  uint4* sx = smem + NCH * SW;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int tiles = tiles_x * tiles_y, total = N * tiles;
  const int G = gridDim.x, xb = blockIdx.x & 7, ng = G < 8 ? G : 8;
  const int lo = (int)((long long)total * xb / ng), hi = (int)((long long)total * (xb + 1) / ng);
  const int nbx = (G - xb + 7) >> 3;  // blocks on this XCD
  const int fW = (lane & ~3) | ((lane & 3) ^ ((lane >> 4) & 3));
#pragma unroll
  for (int jj = 0; jj < JW; ++jj) {
    const int j = wid + NWV * jj;
    if (j < NWW)
      __builtin_amdgcn_global_load_lds((glb_void_t*)(wpk + j * 64 + fW), (lds_void_t*)(smem + j * 64), 16, 0, 0);
  }
  unsigned touch = 0;
  const int aS = l32 * 4 + (h ^ swz4(l32));
  const int px = wid * 32 + l32;
  const int hp0 = (px / TX) * HX + (px % TX);
  for (int t = lo + (blockIdx.x >> 3); t < hi; t += nbx) {
    const int n = t / tiles, tt = t - n * tiles;
    const int ty0 = (tt / tiles_x) * TY, tx0 = (tt % tiles_x) * TX;
    const uint4* inb = in + (long long)n * H * W * QI;
#pragma unroll
    for (int jj = 0; jj < JI; ++jj) {
      const int j = wid + NWV * jj;
      if (j < NWIN) {
        const int si = j * 64 + lane;
        const int hp = si >> 2, cq = si & 3;
        const int hy = hp / HX, hx = hp - (hp / HX) * HX;
        const int gy = ty0 + hy - 1, gx = tx0 + hx - 1;
        const int off = (hp < NPIX && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W)
                            ? (gy * W + gx) * QI + (cq ^ swz4(hp)) : -1;
#pragma unroll
        for (int s = 0; s < NCH; ++s) {
          const uint4* src = off >= 0 ? inb + off + s * 4 : &g_x3_zero16;
          __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(sx + s * SI + j * 64), 16, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned tv0 = 0, tv1 = 0;
    if (kP32Touch) {
      // L2 prefetch while the MFMAs run: one 128-byte line per thread of this tile's residual
      // (read by the epilogue) and, in mode 1, of the block's next halo (DMA'd at the next tile's
      // top); the loaded words are first used at the tile's end (no wait before the MFMAs) and
      // only feed `touch`, consumed after the loop
      const int i = threadIdx.x;
      if (ep.res && i < TY * TX) {
        const int gy = ty0 + i / TX, gx = tx0 + i % TX;
        if (gy < H && gx < W) {
          const long long rp = ep.res_up ? ((long long)n * (H >> 1) + (gy >> 1)) * (W >> 1) + (gx >> 1)
                                         : ((long long)n * H + gy) * W + gx;
          tv0 = reinterpret_cast<const unsigned*>(ep.res + rp * QI)[0];
        }
      }
      const int t2 = t + nbx;
      if (kP32Touch == 1 && t2 < hi && i < NPIX) {  // (mode 2: the residual lines only)
        const int n2 = t2 / tiles, tt2 = t2 - n2 * tiles;
        const int gy = (tt2 / tiles_x) * TY + i / HX - 1, gx = (tt2 % tiles_x) * TX + i % HX - 1;
        if ((unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W)
          tv1 = reinterpret_cast<const unsigned*>(in + ((long long)n2 * H * W + gy * W + gx) * QI)[0];
      }
    }
    // opaque per tile: keeps the compiler from hoisting every tap's fragment addresses out of the
    // tile loop (they would stay live across the epilogue: spills)
    int hpb = hp0, aSb = aS;
    asm volatile("" : "+v"(hpb), "+v"(aSb));
    f32x16 acc0[1][1], acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc0[0][0][r] = 0.0f;
      acc1[r] = 0.0f;
    }
#pragma unroll 1
    for (int s = 0; s < NCH; ++s) {
#pragma unroll
      for (int tap = 0; tap < T; ++tap) {
        const int ky = tap / 3, kx = tap % 3;
        const uint4* swt = smem + s * SW + tap * BM * 4;
        const f16x8 ah = __builtin_bit_cast(f16x8, swt[aSb]);
        const f16x8 al = __builtin_bit_cast(f16x8, swt[aSb ^ 2]);
        const int hp = hpb + ky * HX + kx;
        const int bs = s * SI + hp * 4 + (h ^ swz4(hp));
        const f16x8 bh = __builtin_bit_cast(f16x8, sx[bs]);
        const f16x8 bl = __builtin_bit_cast(f16x8, sx[bs ^ 2]);
        acc0[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc0[0][0], 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc1, 0, 0, 0);
      }
      x3_sched();
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[0][0][r] += acc1[r] * kLoInv;  // exact product, one rounding
    __syncthreads();  // every halo read done: the epilogue stages its tile over the halo
    // per-tile copies of the epilogue's table pointers behind an opaque zero: without it the
    // compiler hoists the lane's bias / scale / shift / head loads out of the tile loop and keeps
    // them live across the MFMAs (spills)
    X3Epi et = ep;
    int zo = 0;
    asm volatile("" : "+s"(zo));
    et.bias = et.bias ? et.bias + zo : nullptr;
    et.scale = et.scale ? et.scale + zo : nullptr;
    et.shift = et.shift ? et.shift + zo : nullptr;
    et.style = et.style ? et.style + zo : nullptr;
    et.head_w = et.head_w ? et.head_w + zo : nullptr;
    et.head_b = et.head_b ? et.head_b + zo : nullptr;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    x3_epilogue<32, BM, TY, TX, 1, 1>(acc0, et, sx, n, 0, ty0, tx0, H, W, 0, wid, 1, tid);
    touch ^= tv0 ^ tv1;
    __syncthreads();  // staging reads done before the next tile's halo lands
  }
  if (kP32Touch && N < 0 && touch == 0x9e3779b9u) ep.ovf[0] = 1;  // never true: keeps the loads
}

struct X3Cfg {
  int bm, ty, tx;
};

// tile configuration per (KS, CIN, COUT, variant); must match the instances in x3_launch().
// Variant 0 (default) is the faster one per level on the box (tools/conv_bench_x3.py, r03):
// 224^2 BM 32 on 8 x 32 tiles, deeper levels BM 32 with 2 blocks per CU; variant 1 the others.
bool x3_cfg(int ks, int cin, int cout, int variant, X3Cfg* c) {
  if (!((cin == 32 || cin == 64 || cin == 128 || cin == 256) && (cout == 32 || cout == 64 || cout == 128 || cout == 256)))
    return false;
  if (ks == 1) {
    *c = {32, 16, 16};
    return true;
  }
  if (ks != 3) return false;
  // variant 2 (development): BM 32, two subtiles per wave, one slab buffer (k_conv_x3 NBUF 1)
  if (cout == 32) *c = variant == 1 ? X3Cfg{32, 16, 32} : X3Cfg{32, 8, 32};
  // variant 3 (development): BM 64, two channel slices per wave, one slab buffer
  else if (cout == 64) *c = variant == 1 ? X3Cfg{64, 16, 16} : variant == 2 ? X3Cfg{32, 16, 32}
                          : variant == 3 ? X3Cfg{64, 16, 16} : X3Cfg{32, 16, 16};
  else *c = variant == 1 ? X3Cfg{64, 14, 28} : variant == 2 ? X3Cfg{32, 16, 28}
          : variant == 3 ? X3Cfg{64, 8, 28} : X3Cfg{32, 8, 28};
  return true;
}

template <int KS, int CIN, int COUT, int BM, int TY, int TX, int WM, int WN, int WPE, int CIN2 = 0, int NBUF = 2>
int x3_run(cpx_ctx* ctx, const void* in, const void* wpk, const X3Epi& ep, int N, int H, int W) {
  const int tx = cpx_div_up(W, TX), ty = cpx_div_up(H, TY);
  const long long blocks = (long long)N * tx * ty * (COUT / BM);  // (tile, output-channel block) items
  CPX_REQUIRE(blocks < (1LL << 31), CPX_ERR_ARG, "cpx_cpnet_x3_conv: too many tiles");
  hipLaunchKernelGGL((k_conv_x3<KS, CIN, COUT, BM, TY, TX, WM, WN, WPE, CIN2, NBUF>), dim3((unsigned)blocks),
                     dim3(512), 0, ctx->stream, (const uint4*)in, (const uint4*)wpk, ep, N, H, W, tx, ty);
  CPX_CHECK_LAUNCH("k_conv_x3");
  return CPX_OK;
}

// 3x3 convolution + folded block projection (cin2 > 0): the instances the CPnet schedule uses
// (each down block's second convolution, whose residual is the projection of the pooled block
// input, and the deepest up block's, at the same resolution); tile configurations as x3_cfg
int x3_launch_proj(cpx_ctx* ctx, int cin, int cout, int cin2, int variant, const void* in, const void* wpk,
                   const X3Epi& ep, int N, int H, int W) {
#define X3_P(CI, CO, C2, V, BM_, TY_, TX_, WM_, WN_, WPE_)                                \
  if (cin == CI && cout == CO && cin2 == C2 && variant == V)                               \
    return x3_run<3, CI, CO, BM_, TY_, TX_, WM_, WN_, WPE_, C2>(ctx, in, wpk, ep, N, H, W);
  X3_P(64, 64, 32, 0, 32, 16, 16, 1, 1, 4)
  X3_P(128, 128, 64, 0, 32, 8, 28, 1, 1, 4)
  X3_P(256, 256, 128, 0, 32, 8, 28, 1, 1, 4)
  X3_P(256, 256, 256, 0, 32, 8, 28, 1, 1, 4)
#define X3_P1(CI, CO, C2, V, BM_, TY_, TX_, WM_, WN_, WPE_)                               \
  if (cin == CI && cout == CO && cin2 == C2 && variant == V)                               \
    return x3_run<3, CI, CO, BM_, TY_, TX_, WM_, WN_, WPE_, C2, 1>(ctx, in, wpk, ep, N, H, W);
  X3_P1(64, 64, 32, 2, 32, 16, 32, 1, 2, 4)
  X3_P1(128, 128, 64, 2, 32, 16, 28, 1, 2, 4)
  X3_P1(256, 256, 128, 2, 32, 16, 28, 1, 2, 4)
  X3_P1(256, 256, 256, 2, 32, 16, 28, 1, 2, 4)
  X3_P1(64, 64, 32, 3, 64, 16, 16, 2, 1, 4)
  X3_P1(128, 128, 64, 3, 64, 8, 28, 2, 1, 4)
  X3_P1(256, 256, 128, 3, 64, 8, 28, 2, 1, 4)
  X3_P1(256, 256, 256, 3, 64, 8, 28, 2, 1, 4)
#undef X3_P1
#undef X3_P
  cpx_set_error("cpx_cpnet_x3_conv_proj: no instance for %d -> %d channels + projection of %d (variant %d)",
                cin, cout, cin2, variant);
  return CPX_ERR_SHAPE;
}

int x3_launch(cpx_ctx* ctx, int ks, int cin, int cout, int variant, const void* in, const void* wpk,
              const X3Epi& ep, int N, int H, int W) {
#define X3_3(CI, CO, V, BM_, TY_, TX_, WM_, WN_, WPE_)                                  \
  if (ks == 3 && cin == CI && cout == CO && variant == V)                                \
    return x3_run<3, CI, CO, BM_, TY_, TX_, WM_, WN_, WPE_>(ctx, in, wpk, ep, N, H, W);
#define X3_1(CI, CO)                                                                     \
  if (ks == 1 && cin == CI && cout == CO)                                                \
    return x3_run<1, CI, CO, 32, 16, 16, 1, 1, 4>(ctx, in, wpk, ep, N, H, W);
  // 224^2 level (32 -> 32 without in_up): the persistent weights-resident kernel, with the L2
  // prefetch of each tile's residual lines (mode 2; also touching the block's next halo, mode 1,
  // measured 443.1 against 444.1 FOV/s and +12.7 GB of PMC traffic per step, none 440.0 —
  // two-pipeline benches of 60 steps, `gpurun_out/r05w`)
  if ((variant == 2 || variant == 3) && cout == 32) variant = 0;  // (224^2: variant 0's kernels)
  if (ks == 3 && cin == 32 && cout == 32 && variant == 0 && !ep.in_up) {
    const int tx = cpx_div_up(W, 32), ty = cpx_div_up(H, 8);
    const long long tiles = (long long)N * tx * ty;
    CPX_REQUIRE(tiles < (1LL << 31), CPX_ERR_ARG, "cpx_cpnet_x3_conv: too many tiles");
    const int grid = (int)std::max(1LL, std::min(tiles, 2LL * ctx->n_cu));
    hipLaunchKernelGGL(k_conv_x3_p32<2>, dim3(grid), dim3(512), 0, ctx->stream, (const uint4*)in, (const uint4*)wpk, ep, N,
                       H, W, tx, ty);
    CPX_CHECK_LAUNCH("k_conv_x3_p32");
    return CPX_OK;
  }
#define X3_3B(CI, CO, V, BM_, TY_, TX_, WM_, WN_, WPE_)                                  \
  if (ks == 3 && cin == CI && cout == CO && variant == V)                                \
    return x3_run<3, CI, CO, BM_, TY_, TX_, WM_, WN_, WPE_, 0, 1>(ctx, in, wpk, ep, N, H, W);
  X3_3B(32, 64, 2, 32, 16, 32, 1, 2, 4)
  X3_3B(64, 64, 2, 32, 16, 32, 1, 2, 4)
  X3_3B(128, 64, 2, 32, 16, 32, 1, 2, 4)
  X3_3B(64, 128, 2, 32, 16, 28, 1, 2, 4)
  X3_3B(128, 128, 2, 32, 16, 28, 1, 2, 4)
  X3_3B(256, 128, 2, 32, 16, 28, 1, 2, 4)
  X3_3B(128, 256, 2, 32, 16, 28, 1, 2, 4)
  X3_3B(256, 256, 2, 32, 16, 28, 1, 2, 4)
  X3_3B(32, 64, 3, 64, 16, 16, 2, 1, 4)
  X3_3B(64, 64, 3, 64, 16, 16, 2, 1, 4)
  X3_3B(128, 64, 3, 64, 16, 16, 2, 1, 4)
  X3_3B(64, 128, 3, 64, 8, 28, 2, 1, 4)
  X3_3B(128, 128, 3, 64, 8, 28, 2, 1, 4)
  X3_3B(256, 128, 3, 64, 8, 28, 2, 1, 4)
  X3_3B(128, 256, 3, 64, 8, 28, 2, 1, 4)
  X3_3B(256, 256, 3, 64, 8, 28, 2, 1, 4)
#undef X3_3B
  X3_3(32, 32, 0, 32, 8, 32, 1, 1, 4)
  X3_3(64, 32, 0, 32, 8, 32, 1, 1, 4)
  X3_3(32, 32, 1, 32, 16, 32, 1, 2, 2)
  X3_3(64, 32, 1, 32, 16, 32, 1, 2, 2)
  // 112^2 level
  X3_3(32, 64, 1, 64, 16, 16, 2, 1, 2)
  X3_3(64, 64, 1, 64, 16, 16, 2, 1, 2)
  X3_3(128, 64, 1, 64, 16, 16, 2, 1, 2)
  X3_3(32, 64, 0, 32, 16, 16, 1, 1, 4)
  X3_3(64, 64, 0, 32, 16, 16, 1, 1, 4)
  X3_3(128, 64, 0, 32, 16, 16, 1, 1, 4)
  // 56^2 / 28^2 levels
  X3_3(64, 128, 1, 64, 14, 28, 2, 2, 2)
  X3_3(128, 128, 1, 64, 14, 28, 2, 2, 2)
  X3_3(256, 128, 1, 64, 14, 28, 2, 2, 2)
  X3_3(128, 256, 1, 64, 14, 28, 2, 2, 2)
  X3_3(256, 256, 1, 64, 14, 28, 2, 2, 2)
  X3_3(64, 128, 0, 32, 8, 28, 1, 1, 4)
  X3_3(128, 128, 0, 32, 8, 28, 1, 1, 4)
  X3_3(256, 128, 0, 32, 8, 28, 1, 1, 4)
  X3_3(128, 256, 0, 32, 8, 28, 1, 1, 4)
  X3_3(256, 256, 0, 32, 8, 28, 1, 1, 4)
  // 1x1 block projections (BatchNorm folded into the weights)
  X3_1(32, 64)
  X3_1(64, 128)
  X3_1(128, 256)
  X3_1(256, 256)
  X3_1(256, 128)
  X3_1(128, 64)
  X3_1(64, 32)
#undef X3_3
#undef X3_1
  cpx_set_error("cpx_cpnet_x3_conv: no instance for ks %d, %d -> %d channels (variant %d)", ks, cin, cout, variant);
  return CPX_ERR_SHAPE;
}

// ---------------------------------------------------------------------------------------------
// stem (first down block's entry) on the fp32 network input x [N][H][W][2]:
//   z0 = relu(scale0 x + shift0) (fp32, zero-padded), z = relu(scale1 (conv3x3(z0, w0) + bias0)
//   + shift1) and p = conv1x1(x, wp) (BatchNorm folded), both stored split.
constexpr int kSTY = 16, kSTX = 16;

__global__ __launch_bounds__(kSTY * kSTX) void k_cpnet_stem_x3(
    const float* __restrict__ x, int N, int H, int W, const float* __restrict__ scale0,
    const float* __restrict__ shift0, const float* __restrict__ w0, const float* __restrict__ bias0,
    const float* __restrict__ scale1, const float* __restrict__ shift1, const float* __restrict__ wp,
    uint4* __restrict__ p_out, uint4* __restrict__ z_out, int tiles_x, int tiles_y, int* ovf) {
  constexpr int NP = kSTY * kSTX;  // pixels (threads) per block
  __shared__ float sz[2][kSTY + 2][kSTX + 2];
  __shared__ uint4 so[2][NP * 8];   // z and p tiles: 8 chunks (2 slabs x hi/lo x 2) per pixel
  const int tiles = tiles_x * tiles_y;
  const int n = blockIdx.x / tiles, t = blockIdx.x - n * tiles;
  const int ty0 = (t / tiles_x) * kSTY, tx0 = (t % tiles_x) * kSTX;
  const float s00 = scale0[0], s01 = scale0[1], h00 = shift0[0], h01 = shift0[1];
  for (int i = threadIdx.x; i < (kSTY + 2) * (kSTX + 2); i += NP) {
    const int hy = i / (kSTX + 2), hx = i - hy * (kSTX + 2);
    const int gy = ty0 + hy - 1, gx = tx0 + hx - 1;
    float a = 0.0f, b = 0.0f;
    if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
      const float2 v = *reinterpret_cast<const float2*>(x + (((long long)n * H + gy) * W + gx) * 2);
      a = fmaxf(s00 * v.x + h00, 0.0f);
      b = fmaxf(s01 * v.y + h01, 0.0f);
    }
    sz[0][hy][hx] = a;
    sz[1][hy][hx] = b;
  }
  __syncthreads();
  const int ly = threadIdx.x / kSTX, lx = threadIdx.x - ly * kSTX;
  const int gy = ty0 + ly, gx = tx0 + lx;
  bool bad = false;
  const int px = threadIdx.x;
  if (gy < H && gx < W) {
    const long long pix = ((long long)n * H + gy) * W + gx;
    float in[18];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < 9; ++k) in[c * 9 + k] = sz[c][ly + k / 3][lx + k % 3];
    const float2 xv = *reinterpret_cast<const float2*>(x + pix * 2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // 8 channels per q: slab q >> 1, chunk q & 1
      float zf[8], pf[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int co = q * 8 + e;
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < 18; ++k) acc = __builtin_fmaf(w0[co * 18 + k], in[k], acc);
        zf[e] = fmaxf(__builtin_fmaf(scale1[co], acc + bias0[co], shift1[co]), 0.0f);
        pf[e] = __builtin_fmaf(wp[co * 2], xv.x, wp[co * 2 + 1] * xv.y);
      }
      uint4 hi, lo;
      const int base = (q >> 1) * 4 + (q & 1);
      // chunk slots swizzled by pixel (8 chunks = 128 B per pixel row)
      split8(zf, hi, lo, bad);
      so[0][px * 8 + (base ^ (px & 7))] = hi;
      so[0][px * 8 + ((base + 2) ^ (px & 7))] = lo;
      split8(pf, hi, lo, bad);
      so[1][px * 8 + (base ^ (px & 7))] = hi;
      so[1][px * 8 + ((base + 2) ^ (px & 7))] = lo;
    }
  }
  __syncthreads();
  // whole 16-byte chunks, consecutive threads -> consecutive chunks of a tile row (2 KiB runs)
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int i = threadIdx.x + r * NP;
    const int p = i >> 3, k = i & 7;
    const int py = ty0 + p / kSTX, pxg = tx0 + p % kSTX;
    if (py < H && pxg < W) {
      const long long g = (((long long)n * H + py) * W + pxg) * 8 + k;
      z_out[g] = so[0][p * 8 + (k ^ (p & 7))];
      p_out[g] = so[1][p * 8 + (k ^ (p & 7))];
    }
  }
  if (ovf && __ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(ovf + n, 1);
}

// 2x2/2 max-pool of split [N][2Hh][2Ww][Cn] -> x_out (the maximum's own hi/lo pair, exact) and
// z_out = split(relu?(scale x + shift)); one thread per (pixel, 8-channel group)
__global__ __launch_bounds__(256) void k_cpnet_pool_x3(const uint4* __restrict__ in,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int relu,
                                                       int N, int Hh, int Ww, int Cn,
                                                       uint4* __restrict__ xo, uint4* __restrict__ zo,
                                                       int* ovf) {
  const long long P = (long long)Hh * Ww;
  const int G = Cn / 8;         // 8-channel groups per pixel
  const int Q = Cn / 4;         // chunks per pixel
  const long long ng = (long long)N * P * G;
  const long long W2 = 2LL * Ww;
  bool bad = false;
  for (long long v = (long long)blockIdx.x * 256 + threadIdx.x; v < ng; v += (long long)gridDim.x * 256) {
    const long long pix = v / G;
    const int gi = (int)(v - pix * G);
    const int q = (gi >> 1) * 4 + (gi & 1);  // hi chunk; lo chunk = q + 2
    const long long n = pix / P;
    const long long rem = pix - n * P;
    const int hh = (int)(rem / Ww), ww = (int)(rem - (long long)hh * Ww);
    const long long base = (n * 2LL * Hh + 2LL * hh) * W2 + 2LL * ww;
    const long long src[4] = {base, base + 1, base + W2, base + W2 + 1};
    uint4 bh = in[src[0] * Q + q], bl = in[src[0] * Q + q + 2];
    float best[8];
    join8(bh, bl, best);
    f16x8 mh = __builtin_bit_cast(f16x8, bh), ml = __builtin_bit_cast(f16x8, bl);
#pragma unroll
    for (int s = 1; s < 4; ++s) {
      const uint4 ch = in[src[s] * Q + q], cl = in[src[s] * Q + q + 2];
      float f[8];
      join8(ch, cl, f);
      const f16x8 fh = __builtin_bit_cast(f16x8, ch), fl = __builtin_bit_cast(f16x8, cl);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (f[k] > best[k]) {  // max_pool2d: first maximum (NaN-free activations)
          best[k] = f[k];
          mh[k] = fh[k];
          ml[k] = fl[k];
        }
    }
    if (xo) {
      xo[pix * Q + q] = __builtin_bit_cast(uint4, mh);
      xo[pix * Q + q + 2] = __builtin_bit_cast(uint4, ml);
    }
    if (zo) {
      const int c0 = gi * 8;
      float z[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float tv = scale ? scale[c0 + k] * best[k] + shift[c0 + k] : best[k];
        z[k] = relu ? fmaxf(tv, 0.0f) : tv;
      }
      uint4 hi, lo;
      split8(z, hi, lo, bad);
      zo[pix * Q + q] = hi;
      zo[pix * Q + q + 2] = lo;
    }
    if (bad && ovf) atomicOr(ovf + n, 1);  // rare: one atomic per offending element
    bad = false;
  }
}

// style vector (CPnet.forward: avg_pool2d over the deepest feature map, L2-normalised) and the
// up path's style Linear layers, one block per image:
//   s[c] = mean over pixels of x[., c] (fp64 sum, fp32 result), s /= ||s||_2,
//   out[n][j] = lin_b[j] + sum_c lin_w[j][c] s[c]  (fp64 accumulation)
__global__ __launch_bounds__(256) void k_cpnet_style_x3(const uint4* __restrict__ x, int H, int W,
                                                        int C, const float* __restrict__ lin_w,
                                                        const float* __restrict__ lin_b, int J,
                                                        float* __restrict__ out) {
  __shared__ float s[256];
  __shared__ double red[256];
  const int n = blockIdx.x;
  const int Q = C / 4;
  const long long P = (long long)H * W;
  const uint4* xb = x + (long long)n * P * Q;
  const int c = threadIdx.x;
  float mean = 0.0f;
  if (c < C) {
    const int q = (c / 16) * 4 + ((c % 16) >> 3), e = c & 7;
    // four interleaved fp64 partial sums (fixed order: deterministic), their loads in flight
    // together: one dependent add chain over the map's 784 pixels made this one-block-per-image
    // kernel latency-bound
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    long long p = 0;
    for (; p + 4 <= P; p += 4) {
      f16x8 hi[4], lo[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        hi[u] = __builtin_bit_cast(f16x8, xb[(p + u) * Q + q]);
        lo[u] = __builtin_bit_cast(f16x8, xb[(p + u) * Q + q + 2]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += (double)((float)hi[u][e] + (float)lo[u][e] * kLoInv);
    }
    for (; p < P; ++p) {
      const f16x8 hi = __builtin_bit_cast(f16x8, xb[p * Q + q]);
      const f16x8 lo = __builtin_bit_cast(f16x8, xb[p * Q + q + 2]);
      acc[0] += (double)((float)hi[e] + (float)lo[e] * kLoInv);
    }
    mean = (float)(((acc[0] + acc[1]) + (acc[2] + acc[3])) / (double)P);
  }
  red[c] = c < C ? (double)mean * (double)mean : 0.0;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (c < o) red[c] += red[c + o];
    __syncthreads();
  }
  const float nrm = (float)sqrt(red[0]);
  if (c < C) s[c] = mean / nrm;
  __syncthreads();
  for (int j = c; j < J; j += 256) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    const float* wj = lin_w + (long long)j * C;
    int k = 0;
    for (; k + 4 <= C; k += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += (double)wj[k + u] * (double)s[k + u];
    }
    for (; k < C; ++k) acc[0] += (double)wj[k] * (double)s[k];
    out[(long long)n * J + j] = (float)(((acc[0] + acc[1]) + (acc[2] + acc[3])) + (double)lin_b[j]);
  }
}

// Network output of an image whose split activations overflowed (ovf[n] != 0): the values are
// garbage (saturated), so they are replaced by "no cell anywhere" (flows 0, cell probability
// -1 < the 0.0 threshold) before the post-processing sees them; the host re-runs that FOV with
// the fp32 network.  One block per (image, chunk of pixels); unflagged images return at once.
__global__ __launch_bounds__(256) void k_cpnet_x3_mask_overflow(float* __restrict__ out, long long P, int nout,
                                                                const int* __restrict__ ovf) {
  const int n = blockIdx.y;
  if (ovf[n] == 0) return;
  float* o = out + (long long)n * P * nout;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < P; i += (long long)gridDim.x * 256)
    for (int q = 0; q < nout; ++q) o[i * nout + q] = q == nout - 1 ? -1.0f : 0.0f;
}

}  // namespace

extern "C" int cpx_cpnet_x3_mask_overflow(cpx_ctx* ctx, float* out, int N, int H, int W, int nout, const int* ovf) {
  CPX_REQUIRE(ctx && out && ovf, CPX_ERR_ARG, "cpx_cpnet_x3_mask_overflow: null argument");
  CPX_REQUIRE(N > 0 && N < 65536 && H > 0 && W > 0 && nout > 0, CPX_ERR_ARG, "cpx_cpnet_x3_mask_overflow: bad sizes");
  const long long P = (long long)H * W;
  const unsigned gx = (unsigned)std::min<long long>((P + 255) / 256, 64);
  hipLaunchKernelGGL(k_cpnet_x3_mask_overflow, dim3(gx, (unsigned)N), dim3(256), 0, ctx->stream, out, P, nout, ovf);
  CPX_CHECK_LAUNCH("k_cpnet_x3_mask_overflow");
  return CPX_OK;
}

extern "C" int cpx_cpnet_x3_cfg(int ks, int cin, int cout, int variant, int* bm) {
  X3Cfg c;
  if (!x3_cfg(ks, cin, cout, variant, &c)) return CPX_ERR_SHAPE;
  if (bm) *bm = c.bm;
  return CPX_OK;
}

extern "C" int cpx_cpnet_x3_conv(cpx_ctx* ctx, int ks, int variant, const void* in, int in_up, int N,
                                 int H, int W, int cin, int cout, const void* wpk, const float* bias,
                                 const void* res, int res_up, const float* style, int style_stride,
                                 const float* scale, const float* shift, int relu, void* y_out,
                                 void* z_out, int z_up, const float* head_w, const float* head_b,
                                 int n_head, float* head_out, int* ovf) {
  CPX_REQUIRE(ctx && in && wpk && (y_out || z_out || head_out), CPX_ERR_ARG,
              "cpx_cpnet_x3_conv: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0, CPX_ERR_ARG, "cpx_cpnet_x3_conv: bad sizes");
  CPX_REQUIRE(!(scale == nullptr) == !(shift == nullptr), CPX_ERR_ARG,
              "cpx_cpnet_x3_conv: scale and shift go together");
  CPX_REQUIRE(!(res_up || in_up) || ((H % 2) == 0 && (W % 2) == 0), CPX_ERR_ARG,
              "cpx_cpnet_x3_conv: res_up / in_up need even sizes");
  CPX_REQUIRE(in_up == 0 || in_up == 1, CPX_ERR_ARG, "cpx_cpnet_x3_conv: in_up is 0 or 1");
  CPX_REQUIRE(((uintptr_t)in | (uintptr_t)wpk | (uintptr_t)res | (uintptr_t)y_out | (uintptr_t)z_out) % 16 == 0,
              CPX_ERR_ARG, "cpx_cpnet_x3_conv: misaligned buffers");
  CPX_REQUIRE(!style || (style_stride >= cout && style_stride % 4 == 0 && ((uintptr_t)style % 16) == 0),
              CPX_ERR_ARG, "cpx_cpnet_x3_conv: style needs a 16-byte aligned [N][stride >= cout] table");
  CPX_REQUIRE(!head_out || (ks == 3 && cout == 32 && !z_out && head_w && head_b && n_head >= 1 && n_head <= 4),
              CPX_ERR_ARG, "cpx_cpnet_x3_conv: head needs a 3x3 conv with cout 32, no z_out, 1..4 outputs");
  CPX_REQUIRE(!z_up || z_out, CPX_ERR_ARG, "cpx_cpnet_x3_conv: z_up without z_out");
  X3Epi ep{bias, (const uint4*)res, style, scale, shift, (uint4*)y_out, (uint4*)z_out, res_up, relu,
           z_up, style_stride, head_w, head_b, head_out, n_head, ovf, in_up, nullptr, nullptr,
           nullptr, nullptr, nullptr, nullptr};
  return x3_launch(ctx, ks, cin, cout, variant, in, wpk, ep, N, H, W);
}

extern "C" int cpx_cpnet_x3_conv_pool(cpx_ctx* ctx, int variant, const void* in, int N, int H, int W, int cin,
                                      int cout, const void* wpk, const float* bias, const void* res,
                                      void* y_out, void* pool_x, void* pool_z, const float* pool_scale,
                                      const float* pool_shift, int* ovf) {
  CPX_REQUIRE(ctx && in && wpk && res && y_out && pool_x && pool_z && pool_scale && pool_shift, CPX_ERR_ARG,
              "cpx_cpnet_x3_conv_pool: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0 && H % 2 == 0 && W % 2 == 0, CPX_ERR_ARG,
              "cpx_cpnet_x3_conv_pool: bad sizes (even H, W)");
  CPX_REQUIRE(((uintptr_t)in | (uintptr_t)wpk | (uintptr_t)res | (uintptr_t)y_out | (uintptr_t)pool_x |
               (uintptr_t)pool_z) % 16 == 0, CPX_ERR_ARG, "cpx_cpnet_x3_conv_pool: misaligned buffers");
  X3Epi ep{bias, (const uint4*)res, nullptr, nullptr, nullptr, (uint4*)y_out, nullptr, 0, 0, 0, 0,
           nullptr, nullptr, nullptr, 0, ovf, 0, nullptr, nullptr,
           (uint4*)pool_x, (uint4*)pool_z, pool_scale, pool_shift};
  return x3_launch(ctx, 3, cin, cout, variant, in, wpk, ep, N, H, W);
}

extern "C" int cpx_cpnet_x3_conv_proj(cpx_ctx* ctx, int variant, const void* in, int N, int H, int W,
                                      int cin, int cout, const void* wpk, const void* in2, int cin2,
                                      const void* wpk2, const float* bias, const float* style,
                                      int style_stride, const float* scale, const float* shift, int relu,
                                      void* y_out, void* z_out, int z_up, int* ovf) {
  CPX_REQUIRE(ctx && in && wpk && in2 && wpk2 && (y_out || z_out), CPX_ERR_ARG,
              "cpx_cpnet_x3_conv_proj: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0 && cin2 > 0 && cin2 % 16 == 0, CPX_ERR_ARG, "cpx_cpnet_x3_conv_proj: bad sizes");
  CPX_REQUIRE(!(scale == nullptr) == !(shift == nullptr), CPX_ERR_ARG,
              "cpx_cpnet_x3_conv_proj: scale and shift go together");
  CPX_REQUIRE(((uintptr_t)in | (uintptr_t)wpk | (uintptr_t)in2 | (uintptr_t)wpk2 | (uintptr_t)y_out |
               (uintptr_t)z_out) % 16 == 0, CPX_ERR_ARG, "cpx_cpnet_x3_conv_proj: misaligned buffers");
  CPX_REQUIRE(!style || (style_stride >= cout && style_stride % 4 == 0 && ((uintptr_t)style % 16) == 0),
              CPX_ERR_ARG, "cpx_cpnet_x3_conv_proj: style needs a 16-byte aligned [N][stride >= cout] table");
  CPX_REQUIRE(!z_up || z_out, CPX_ERR_ARG, "cpx_cpnet_x3_conv_proj: z_up without z_out");
  X3Epi ep{bias, nullptr, style, scale, shift, (uint4*)y_out, (uint4*)z_out, 0, relu, z_up, style_stride,
           nullptr, nullptr, nullptr, 0, ovf, 0, (const uint4*)in2, (const uint4*)wpk2,
           nullptr, nullptr, nullptr, nullptr};
  return x3_launch_proj(ctx, cin, cout, cin2, variant, in, wpk, ep, N, H, W);
}

extern "C" int cpx_cpnet_x3_stem(cpx_ctx* ctx, const float* x, int N, int H, int W,
                                 const float* scale0, const float* shift0, const float* w0,
                                 const float* bias0, const float* scale1, const float* shift1,
                                 const float* wp, void* p_out, void* z_out, int* ovf) {
  CPX_REQUIRE(ctx && x && scale0 && shift0 && w0 && bias0 && scale1 && shift1 && wp && p_out && z_out,
              CPX_ERR_ARG, "cpx_cpnet_x3_stem: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0, CPX_ERR_ARG, "cpx_cpnet_x3_stem: bad sizes");
  CPX_REQUIRE(((uintptr_t)x % 8) == 0 && ((uintptr_t)p_out | (uintptr_t)z_out) % 16 == 0,
              CPX_ERR_ARG, "cpx_cpnet_x3_stem: misaligned buffers");
  const int tx = cpx_div_up(W, kSTX), ty = cpx_div_up(H, kSTY);
  const long long blocks = (long long)N * tx * ty;
  CPX_REQUIRE(blocks < (1LL << 31), CPX_ERR_ARG, "cpx_cpnet_x3_stem: too many tiles");
  hipLaunchKernelGGL(k_cpnet_stem_x3, dim3((unsigned)blocks), dim3(kSTY * kSTX), 0, ctx->stream, x, N, H,
                     W, scale0, shift0, w0, bias0, scale1, shift1, wp, (uint4*)p_out, (uint4*)z_out, tx,
                     ty, ovf);
  CPX_CHECK_LAUNCH("k_cpnet_stem_x3");
  return CPX_OK;
}

extern "C" int cpx_cpnet_x3_pool(cpx_ctx* ctx, const void* in, const float* scale,
                                 const float* shift, int relu, int N, int Hh, int Ww, int Cn,
                                 void* x_out, void* z_out, int* ovf) {
  CPX_REQUIRE(ctx && in && (x_out || z_out), CPX_ERR_ARG, "cpx_cpnet_x3_pool: null argument");
  CPX_REQUIRE(N > 0 && Hh > 0 && Ww > 0 && Cn > 0 && Cn % 16 == 0, CPX_ERR_ARG,
              "cpx_cpnet_x3_pool: bad sizes (channels must be a multiple of 16)");
  CPX_REQUIRE(!(scale == nullptr) == !(shift == nullptr), CPX_ERR_ARG,
              "cpx_cpnet_x3_pool: scale and shift go together");
  CPX_REQUIRE(((uintptr_t)in | (uintptr_t)x_out | (uintptr_t)z_out) % 16 == 0, CPX_ERR_ARG,
              "cpx_cpnet_x3_pool: buffers must be 16-byte aligned");
  const long long ng = (long long)N * Hh * Ww * Cn / 8;
  const long long g = std::max(1LL, std::min((ng + 255) / 256, 32LL * ctx->n_cu));
  hipLaunchKernelGGL(k_cpnet_pool_x3, dim3((unsigned)g), dim3(256), 0, ctx->stream, (const uint4*)in,
                     scale, shift, relu, N, Hh, Ww, Cn, (uint4*)x_out, (uint4*)z_out, ovf);
  CPX_CHECK_LAUNCH("k_cpnet_pool_x3");
  return CPX_OK;
}

extern "C" int cpx_cpnet_x3_style(cpx_ctx* ctx, const void* x, int N, int H, int W, int C,
                                  const float* lin_w, const float* lin_b, int J, float* out) {
  CPX_REQUIRE(ctx && x && lin_w && lin_b && out, CPX_ERR_ARG, "cpx_cpnet_x3_style: null argument");
  CPX_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C <= 256 && C % 16 == 0 && J > 0, CPX_ERR_ARG,
              "cpx_cpnet_x3_style: bad sizes");
  hipLaunchKernelGGL(k_cpnet_style_x3, dim3(N), dim3(256), 0, ctx->stream, (const uint4*)x, H, W, C,
                     lin_w, lin_b, J, out);
  CPX_CHECK_LAUNCH("k_cpnet_style_x3");
  return CPX_OK;
}
