// a6: Cellpose (<= v3) evaluation around the CPnet forward — normalisation, resize, tiling, tile
// averaging, flow dynamics and mask assembly — restated for gfx950.  The reference runs all of
// this inside `cell_model.eval(image_4ch, diameter=100)` (Cellpose_GPU_s3fs.py:143); the exact
// semantics pinned here (and in oracle/seg_oracle.py, which these kernels match bit-exactly on
// identical network outputs) are listed in DESIGN.md §Segmentation.
//
// Data layout in HBM (per FOV): corrected fp32 planes [C][H][W] -> tiles (bf16 NHWC for the MFMA
// U-Net) -> yf fp32 [3][Ly][Lx] -> dPs/p fp32 [2][Ly][Lx] -> histogram h / seed map M int32
// [Ly+40][Lx+40] -> net-resolution labels [Ly][Lx] -> full-resolution labels int32 [H][W].
// Every reduction is integer (exact) or fixed-order, so masks are bit-reproducible.
#include "cpx_internal.h"
#include <stdlib.h>
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <type_traits>
#include <vector>

#pragma clang fp contract(off)

namespace {

constexpr int kT = 256;
constexpr int kRpad = 20;

__device__ __forceinline__ unsigned int f2key(float f) {
  unsigned int u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned int k) {
  unsigned int u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}
__device__ __forceinline__ unsigned short f2bf16(float f) {
  unsigned int u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf162f(unsigned short h) {
  return __uint_as_float(((unsigned int)h) << 16);
}

// ---------------------------------------------------------------------------------------------
// normalize99: exact order statistics by a 3-pass (11/11/10-bit) radix histogram selection
struct PctState {
  unsigned int pre[4];
  long long rank[4];
  double vi[2];
};

// Each thread takes runs of 16 consecutive pixels (four 16-byte loads) and adds a run of equal
// (rank-set, bin) keys with one LDS atomic: image planes are smooth at the coarse levels, so
// most of a run shares one bin and the same-address atomic contention (the cost of a per-pixel
// histogram on a few hot bins) drops by ~16x.
__device__ __forceinline__ void pct_flush(unsigned int (*h)[2048], unsigned int m, unsigned int bin,
                                          unsigned int cnt) {
  for (int r = 0; r < 4; ++r)
    if ((m >> r) & 1u) atomicAdd(&h[r][bin], cnt);
}

__global__ __launch_bounds__(kT) void k_pct_hist(const float* __restrict__ corr, int C, long long N,
                                                 int nchan, int pass,
                                                 const PctState* __restrict__ st,
                                                 unsigned int* __restrict__ hist) {
  __shared__ unsigned int h[4][2048];
  const int pl = blockIdx.y;  // fov * nchan + ch
  const int fov = pl / nchan, ch = pl % nchan;
  const float* src = corr + ((long long)fov * C + ch) * N;
  const int nr = pass == 0 ? 1 : 4;
  for (int i = threadIdx.x; i < nr * 2048; i += kT) (&h[0][0])[i] = 0u;
  unsigned int pre[4] = {0, 0, 0, 0};
  if (pass > 0)
    for (int r = 0; r < 4; ++r) pre[r] = st[pl].pre[r];
  __syncthreads();
  // (rank mask, bin) of one key for this pass; mask 0 = not counted
  auto classify = [&](unsigned int k, unsigned int& m, unsigned int& bin) {
    if (pass == 0) {
      m = 1u;
      bin = k >> 21;
    } else if (pass == 1) {
      m = 0u;
      for (int r = 0; r < 4; ++r) m |= ((k >> 21) == pre[r]) ? (1u << r) : 0u;
      bin = (k >> 10) & 0x7ffu;
    } else {
      m = 0u;
      for (int r = 0; r < 4; ++r) m |= ((k >> 10) == pre[r]) ? (1u << r) : 0u;
      bin = k & 0x3ffu;
    }
  };
  const long long nrun = (N + 15) / 16;
  const long long per = (nrun + gridDim.x - 1) / gridDim.x;
  const long long rb = per * blockIdx.x, re = min(nrun, rb + per);
  unsigned int cm = 0u, cb = 0u, cnt = 0u;
  const bool vec = (((uintptr_t)src) & 15u) == 0u;
  for (long long run = rb + threadIdx.x; run < re; run += kT) {
    const long long i0 = run * 16;
    float v[16];
    if (vec && i0 + 16 <= N) {
      const float4* s4 = reinterpret_cast<const float4*>(src + i0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 t = s4[q];
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = i0 + q < N ? src[i0 + q] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (i0 + q >= N) break;
      unsigned int m, bin;
      classify(f2key(v[q]), m, bin);
      if (m != cm || bin != cb) {
        if (cnt && cm) pct_flush(h, cm, cb, cnt);
        cm = m;
        cb = bin;
        cnt = 0u;
      }
      ++cnt;
    }
  }
  if (cnt && cm) pct_flush(h, cm, cb, cnt);
  __syncthreads();
  unsigned int* g = hist + (long long)pl * 4 * 2048;
  for (int i = threadIdx.x; i < nr * 2048; i += kT) {
    const unsigned int v = (&h[0][0])[i];
    if (v) atomicAdd(&g[i], v);
  }
}

__device__ __forceinline__ double lerp_np(double a, double b, double t) {
  const double d = b - a;
  return t >= 0.5 ? b - d * (1.0 - t) : a + d * t;
}

// one block (256 threads) per plane; wave r owns rank r: each lane sums 32 consecutive bins,
// a wave prefix sum finds the lane whose bins hold the rank, that lane walks its 32 bins
__global__ __launch_bounds__(256) void k_pct_find(long long N, int pass, PctState* __restrict__ st,
                                                  const unsigned int* __restrict__ hist,
                                                  double* __restrict__ pct) {
  const int pl = blockIdx.x;
  PctState& s = st[pl];
  if (pass == 0 && threadIdx.x == 0) {
    const double q[2] = {1.0, 99.0};
    for (int a = 0; a < 2; ++a) {
      const double vi = (double)(N - 1) * (q[a] / 100.0);
      const long long lo = (long long)floor(vi);
      s.vi[a] = vi;
      s.rank[2 * a] = lo;
      s.rank[2 * a + 1] = min(lo + 1, N - 1);
    }
  }
  __syncthreads();
  const int r = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nb = pass == 2 ? 1024 : 2048;
  const int per = nb / 64;  // 32 or 16 bins per lane
  const unsigned int* h = hist + ((long long)pl * 4 + (pass == 0 ? 0 : r)) * 2048 + lane * per;
  unsigned int c[32];
  long long tot = 0;
#pragma unroll
  for (int b = 0; b < 32; ++b) {
    c[b] = b < per ? h[b] : 0u;
    tot += c[b];
  }
  // inclusive prefix over lanes
  long long inc = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  const long long rank = s.rank[r];
  const long long exc = inc - tot;
  const unsigned long long hit = __ballot(inc > rank);
  const int owner = hit ? (__builtin_ffsll((long long)hit) - 1) : 63;  // 63: NaN-only planes
  __syncthreads();  // every wave has read s.rank before it is rewritten
  if (lane == owner) {
    long long cum = exc;
    int b = 0;
    for (; b < per - 1; ++b) {
      if (cum + (long long)c[b] > rank) break;
      cum += c[b];
    }
    const unsigned int bin = (unsigned int)(owner * per + b);
    s.rank[r] = rank - cum;
    s.pre[r] = pass == 0 ? bin : (pass == 1 ? (s.pre[r] << 11) | bin : (s.pre[r] << 10) | bin);
  }
  __syncthreads();
  if (pass == 2 && threadIdx.x == 0) {
    for (int a = 0; a < 2; ++a) {
      const double lo = (double)key2f(s.pre[2 * a]), hi = (double)key2f(s.pre[2 * a + 1]);
      const double t = s.vi[a] - floor(s.vi[a]);
      pct[2 * pl + a] = lerp_np(lo, hi, t);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// tiles: normalise -> bilinear resize -> zero pad -> tile cut (one thread per tile pixel)
struct AxisTab {
  const int* i0;   // [L]
  const int* i1;   // [L]
  const float* w;  // [L]
};

__device__ __forceinline__ float norm_px(float v, double p1, double den) {
  return (float)(((double)v - p1) / den);
}

__global__ __launch_bounds__(kT) void k_seg_tiles(const float* __restrict__ corr, int C, int H,
                                                  int W, int nchan, const double* __restrict__ pct,
                                                  cpx_seg_geom g, AxisTab ty_, AxisTab tx_,
                                                  int layout, void* __restrict__ tiles) {
  const int fov = blockIdx.z, t = blockIdx.y;
  const int npx = g.by * g.bx;
  const int q = blockIdx.x * kT + threadIdx.x;
  if (q >= npx) return;
  const int ty = q / g.bx, tx = q - ty * g.bx;
  const int jy = t / g.nx, jx = t - jy * g.nx;
  const int iy = g.ys[jy] + ty - g.py0, ix = g.xs[jx] + tx - g.px0;
  const bool inside = iy >= 0 && iy < g.Ly && ix >= 0 && ix < g.Lx;
  const long long ntile = (long long)fov * g.ny * g.nx + t;
  const long long N = (long long)H * W;
  for (int ch = 0; ch < nchan; ++ch) {
    float out = 0.0f;
    if (inside) {
      const double p1 = pct[((long long)fov * nchan + ch) * 2], p99 = pct[((long long)fov * nchan + ch) * 2 + 1];
      double den = p99 - p1;
      if (den == 0.0) den = 1.0;
      const float* src = corr + ((long long)fov * C + ch) * N;
      const int y0 = ty_.i0[iy], y1 = ty_.i1[iy], x0 = tx_.i0[ix], x1 = tx_.i1[ix];
      const float wy = ty_.w[iy], wx = tx_.w[ix];
      const float a00 = norm_px(src[(long long)y0 * W + x0], p1, den);
      const float a01 = norm_px(src[(long long)y0 * W + x1], p1, den);
      const float a10 = norm_px(src[(long long)y1 * W + x0], p1, den);
      const float a11 = norm_px(src[(long long)y1 * W + x1], p1, den);
      const float r0 = a00 * (1.0f - wx) + a01 * wx;
      const float r1 = a10 * (1.0f - wx) + a11 * wx;
      out = r0 * (1.0f - wy) + r1 * wy;
    }
    if (layout == CPX_TILE_F32_NCHW)
      static_cast<float*>(tiles)[(ntile * nchan + ch) * npx + q] = out;
    else if (layout == CPX_TILE_F32_NHWC)
      static_cast<float*>(tiles)[(ntile * npx + q) * nchan + ch] = out;
    else
      static_cast<unsigned short*>(tiles)[(ntile * npx + q) * nchan + ch] = f2bf16(out);
  }
}

// ---------------------------------------------------------------------------------------------
// average_tiles (taper-weighted, tile order), pad cropped
__global__ __launch_bounds__(kT) void k_seg_average(const void* __restrict__ net, int layout, int nout,
                                                    cpx_seg_geom g, const float* __restrict__ taper,
                                                    float* __restrict__ yf) {
  const int fov = blockIdx.y;
  const int q = blockIdx.x * kT + threadIdx.x;
  if (q >= g.Ly * g.Lx) return;
  const int y = q / g.Lx, x = q - y * g.Lx;
  const int py = y + g.py0, px = x + g.px0;
  const int npx = g.by * g.bx;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float nav = 0.0f;
  for (int jy = 0; jy < g.ny; ++jy) {
    const int ty = py - g.ys[jy];
    if (ty < 0 || ty >= g.by) continue;
    for (int jx = 0; jx < g.nx; ++jx) {
      const int tx = px - g.xs[jx];
      if (tx < 0 || tx >= g.bx) continue;
      const long long t = (long long)fov * g.ny * g.nx + jy * g.nx + jx;
      const int o = ty * g.bx + tx;
      const float m = taper[o];
      for (int c = 0; c < nout && c < 4; ++c) {
        float v;
        if (layout == CPX_TILE_F32_NCHW) v = static_cast<const float*>(net)[(t * nout + c) * npx + o];
        else if (layout == CPX_TILE_F32_NHWC) v = static_cast<const float*>(net)[(t * npx + o) * nout + c];
        else v = bf162f(static_cast<const unsigned short*>(net)[(t * npx + o) * nout + c]);
        acc[c] = acc[c] + v * m;
      }
      nav = nav + m;
    }
  }
  for (int c = 0; c < nout && c < 4; ++c)
    yf[(((long long)fov * nout + c) * g.Ly + y) * g.Lx + x] = acc[c] / nav;
}

// ---------------------------------------------------------------------------------------------
// dynamics (dynamics.compute_masks) at the dynamics resolution Dy x Dx: the full H x W with
// resample=True (CellposeModel.eval's default, the reference call), Ly x Lx with resample=False.
struct DynBufs {
  float2* dps;           // [B][n] (dY, dX) * cp_mask / 5: the follow_flows field (fp32; the step
                         // converts the four gathered values to fp64 exactly: half the gather
                         // bytes of an fp64 copy, and the early rounds are L2-bandwidth bound)
  float2* dpf;           // [B][n] (dY, dX) network flows (flow-error input)
  float2* p;             // [B][n] final positions (written for moving pixels only)
  unsigned char* mov;    // [B][n] pixel follows the flow (|dY * cp / 5| > 1e-3)
  int* h;                // [B][nh] histogram of final positions, padded by kRpad
  unsigned int* M;       // [B][nh] seed-expansion label map
  unsigned char* sflag;  // [B][nh] seed flags
  int* m0;               // [B][n] get_masks labels (the caller's labels buffer at full res)
  int ms;                // seed capacity per FOV (= max_objects: masks <= seeds, so every mask fits
                         // the object tables; more seeds set CPX_SEG_OVF_SEEDS)
  int* seeds;            // [B][ms] seed pixels (padded grid), row-major
  int* cnt;              // [B][ms + 1] pixels per seed label
  int* first;            // [B][ms + 1] first pixel (raster order) per seed label
  int* newlab;           // [B][ms + 1] renumbered label (0: removed)
  unsigned char* mark;   // [B][n] first-occurrence pixels of the kept labels
  int* marklist;         // [B][ms] marked pixels in raster order
  int* act;              // [B][n] moving pixels (first n_moving entries per FOV, any order)
  void* fitems0;         // [B][n] FollowItem ping
  void* fitems1;         // [B][n] FollowItem pong
  int* fcnt;             // [rounds + 1][B] items per FOV entering each follow round
  int* tiles;            // [B][ntile] ordered-compaction tile counts -> offsets
  int* totals;           // [B] ordered-compaction totals
  cpx_seg_stats* st;
};

// Dynamics pixels -> dps, dpf, moving flag; the moving pixels are compacted into `act` in
// tile order (one atomic per block; inside a tile the raster order is kept) so a wave of
// k_dyn_follow starts on 64 neighbouring pixels.  RESAMPLE: cv2 INTER_LINEAR of the Ly x Lx
// averaged output to Dy x Dx (transforms.resize_image), fp32, row pass then column pass.
constexpr int kPrepPer = 8;  // pixels per thread (thread t: pixels t, t + kT, ...)

template <bool RESAMPLE>
__global__ __launch_bounds__(kT) void k_dyn_prep(const float* __restrict__ yf, int Ly, int Lx,
                                                 int Dy, int Dx, AxisTab uy, AxisTab ux,
                                                 DynBufs d) {
  const int fov = blockIdx.y;
  const long long n = (long long)Dy * Dx;
  const long long nl = (long long)Ly * Lx;
  const long long q0 = (long long)blockIdx.x * kT * kPrepPer;
  const float* f = yf + (long long)fov * 3 * nl;
  unsigned int movbits = 0;
#pragma unroll
  for (int k = 0; k < kPrepPer; ++k) {
    const long long q = q0 + k * kT + threadIdx.x;
    if (q >= n) break;
    float v[3];
    if (RESAMPLE) {
      const int qi = (int)q;  // n < 2^29 (cpx_seg_masks): 32-bit division
      const int y = qi / Dx, x = qi - y * Dx;
      const int y0 = uy.i0[y], y1 = uy.i1[y], x0 = ux.i0[x], x1 = ux.i1[x];
      const float wy = uy.w[y], wx = ux.w[x];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float* P = f + c * nl;
        const float r0 = P[y0 * Lx + x0] * (1.0f - wx) + P[y0 * Lx + x1] * wx;
        const float r1 = P[y1 * Lx + x0] * (1.0f - wx) + P[y1 * Lx + x1] * wx;
        v[c] = r0 * (1.0f - wy) + r1 * wy;
      }
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = f[c * nl + q];
    }
    const float cp = v[2] > 0.0f ? 1.0f : 0.0f;  // cellprob > cellprob_threshold (0.0)
    const float dy = (v[0] * cp) / 5.0f, dx = (v[1] * cp) / 5.0f;
    d.dps[(long long)fov * n + q] = make_float2(dy, dx);
    d.dpf[(long long)fov * n + q] = make_float2(v[0], v[1]);
    // np.abs(dP[0]) > 1e-3: numpy compares the float32 array with the scalar cast to float32
    const bool moving = fabsf(dy) > 1e-3f;
    d.mov[(long long)fov * n + q] = (unsigned char)moving;
    movbits |= (unsigned int)moving << k;
  }
  // block-wide exclusive ranks in (k, thread) order, one atomic per block
  __shared__ int wsum[kPrepPer][kT / 64];
  __shared__ int sbase;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long bal[kPrepPer];
#pragma unroll
  for (int k = 0; k < kPrepPer; ++k) {
    bal[k] = __ballot((movbits >> k) & 1u);
    if (lane == 0) wsum[k][wid] = __popcll(bal[k]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int k = 0; k < kPrepPer; ++k)
      for (int w = 0; w < kT / 64; ++w) {
        const int c = wsum[k][w];
        wsum[k][w] = s;
        s += c;
      }
    sbase = s ? atomicAdd(&d.st[fov].n_moving, s) : 0;
  }
  __syncthreads();
  const unsigned long long lower = (1ull << lane) - 1ull;
#pragma unroll
  for (int k = 0; k < kPrepPer; ++k)
    if ((movbits >> k) & 1u)
      d.act[(long long)fov * n + sbase + wsum[k][wid] + __popcll(bal[k] & lower)] =
          (int)(q0 + k * kT + threadIdx.x);
}

// follow_flows: every moving pixel runs niter Euler steps of the map_coordinates update (fp64
// bilinear expression of the fp32 field, rounded to fp32, fp32 add, clamp).  The update depends
// on the position alone, so a pixel whose position does not change in a step sits on an exact
// fixed point and keeps it for the remaining steps: it stops there and its final position is
// bit-identical to the full loop (>= 99.9 % of the synthetic plates' pixels reach one within a
// few hundred of the 1176 steps, 82 on average).  The steps run in rounds of K: round r takes
// the pixels still moving after r rounds (positions carried in a compact item list), runs K
// steps, writes the finished ones and appends the rest to the next round's list in block order
// — so the 64 lanes of a wave stay spatial neighbours and their bilinear gathers share lines.
// wave-aggregated histogram add (lanes with equal keys: one atomic)
__device__ __forceinline__ void agg_add(int* base, int key, bool valid) {
  const int lane = threadIdx.x & 63;
  unsigned long long pend = __ballot(valid);
  while (pend) {
    const int leader = __ffsll((long long)pend) - 1;
    const int k0 = __shfl(key, leader);
    const unsigned long long m = __ballot(valid && key == k0);
    if (lane == leader) atomicAdd(&base[k0], __popcll(m));
    pend &= ~m;
  }
}

struct FollowItem {
  int q;
  float py, px;
  int pad;
};

// NI items per thread (items i0 + j kT + t, j < NI): NI independent trajectories per lane, all
// their gathers issued before any is used, so a wave keeps NI times the gathers in flight (the
// kernel is bound by the latency of each trajectory's dependent gather chain, not by issue).
// Per item the arithmetic and the order of the next round's list are those of NI = 1.
// V4: the two horizontal neighbours of a row in one 16-byte load (two gathers per step instead
// of four; the gathers' address processing, not their bytes, bounds the kernel): (x0, x0 + 1),
// or at the right edge (x0 - 1, x0) with the upper half taken for both.
template <int NI, bool V4>
__global__ __launch_bounds__(kT) void k_dyn_follow(int Dy, int Dx, int niter, int step0, int K,
                                                   int from_act, const FollowItem* __restrict__ in,
                                                   const int* __restrict__ in_cnt,
                                                   FollowItem* __restrict__ out,
                                                   int* __restrict__ out_cnt, DynBufs d) {
  const int fov = blockIdx.y;
  const long long n = (long long)Dy * Dx;
  const int n_moving = d.st[fov].n_moving;
  if (n_moving < 5) return;  // follow_flows returns inds=None -> no masks
  const int n_in = from_act ? n_moving : in_cnt[fov];
  const int steps = min(K, niter - step0);
  const float2* __restrict__ I = d.dps + (long long)fov * n;
  float2* __restrict__ P = d.p + (long long)fov * n;
  const FollowItem* src = in + (long long)fov * n;
  FollowItem* dst = out + (long long)fov * n;
  const float fLy = (float)(Dy - 1), fLx = (float)(Dx - 1);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int Dxh = Dx + 2 * kRpad;
  int* Hh = d.h + (long long)fov * (Dy + 2 * kRpad) * Dxh;
  const unsigned char* Ib = reinterpret_cast<const unsigned char*>(I);
  // V4: the FOV's field as a buffer resource (8 n < 2^31 bytes, checked by the host)
  const __amdgpu_buffer_rsrc_t rsI =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(I), (short)0, (int)(8 * n), 0x00020000);
  (void)rsI;
  __shared__ int wsum[NI][kT / 64];
  __shared__ int sbase;
  for (int i0 = blockIdx.x * kT * NI; i0 < n_in; i0 += gridDim.x * kT * NI) {  // block-uniform
    bool active[NI], done[NI];
    int q[NI];
    float py[NI], px[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int i = i0 + j * kT + threadIdx.x;
      active[j] = i < n_in;
      q[j] = 0;
      py[j] = 0.0f;
      px[j] = 0.0f;
      if (active[j]) {
        if (from_act) {
          q[j] = d.act[(long long)fov * n + i];
          py[j] = (float)(q[j] / Dx);
          px[j] = (float)(q[j] % Dx);
        } else {
          const FollowItem it = src[i];
          q[j] = it.q;
          py[j] = it.py;
          px[j] = it.px;
        }
      }
      done[j] = !active[j];
    }
    // the cell (integer position) of each item's last gathers and their values: a step that
    // stays in the same cell — most of them once a trajectory slows near its sink — reuses them
    // instead of gathering again (the field is read-only here: the same values, bit-identical)
    float2 af[NI], bf[NI], cf[NI], ef[NI];
    int cy[NI], cx[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      cy[j] = -1;
      cx[j] = -1;
      af[j] = bf[j] = cf[j] = ef[j] = make_float2(0.0f, 0.0f);
    }
    for (int s = 0; s < steps; ++s) {
      bool all = true;
#pragma unroll
      for (int j = 0; j < NI; ++j) all = all && done[j];
      if (all) break;
      // every item's gathers first (a finished item keeps its cell: no gather, its update is
      // discarded below)
      int yi[NI], xi[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        yi[j] = (int)py[j];
        xi[j] = (int)px[j];
        if (yi[j] == cy[j] && xi[j] == cx[j]) continue;
        cy[j] = yi[j];
        cx[j] = xi[j];
        const int y0 = min(Dy - 1, max(0, yi[j])), x0 = min(Dx - 1, max(0, xi[j]));
        // 32-bit byte offsets from the FOV's (block-uniform) field base: SGPR-base + VGPR-offset
        // loads, no 64-bit address arithmetic per step (the field is < 4 GiB per FOV)
        const unsigned int b00 = 8u * (unsigned int)(y0 * Dx + x0);
        const unsigned int bdx = x0 + 1 < Dx ? 8u : 0u, bdy = y0 + 1 < Dy ? 8u * (unsigned int)Dx : 0u;
        if constexpr (V4) {
          // raw buffer loads: one 16-byte access each (a plain float4 load of an 8-byte aligned
          // address is split into two 8-byte loads by the compiler)
          const unsigned int o = bdx ? b00 : b00 - 8u;  // x0 = Dx - 1 >= 1 when bdx == 0
          const float4 r0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsI, o, 0, 0));
          const float4 r1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsI, o + bdy, 0, 0));
          af[j] = bdx ? make_float2(r0.x, r0.y) : make_float2(r0.z, r0.w);
          bf[j] = make_float2(r0.z, r0.w);
          cf[j] = bdx ? make_float2(r1.x, r1.y) : make_float2(r1.z, r1.w);
          ef[j] = make_float2(r1.z, r1.w);
        } else {
          af[j] = *reinterpret_cast<const float2*>(Ib + b00);
          bf[j] = *reinterpret_cast<const float2*>(Ib + (b00 + bdx));
          cf[j] = *reinterpret_cast<const float2*>(Ib + (b00 + bdy));
          ef[j] = *reinterpret_cast<const float2*>(Ib + (b00 + bdy + bdx));
        }
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const double2 a = {(double)af[j].x, (double)af[j].y}, b = {(double)bf[j].x, (double)bf[j].y},
                      c = {(double)cf[j].x, (double)cf[j].y}, e = {(double)ef[j].x, (double)ef[j].y};
        double vy, vx;
        if (py[j] >= 1.0f && px[j] >= 1.0f) {
          // yy = frac(py) and 1 - yy are exact in fp32 (multiples of 2^-23 in [0, 1]), so
          // I * (1 - yy) is exact in fp64 and (I * (1 - yy)) * (1 - xx) == I * w00 with
          // w00 = (1 - yy) * (1 - xx) exact: the same single rounding, four fewer multiplies
          const float yf = py[j] - (float)yi[j], xf = px[j] - (float)xi[j];
          const double y1 = (double)yf, x1 = (double)xf, y0d = (double)(1.0f - yf), x0d = (double)(1.0f - xf);
          const double w00 = y0d * x0d, w01 = y0d * x1, w10 = y1 * x0d, w11 = y1 * x1;
          vy = a.x * w00 + b.x * w01 + c.x * w10 + e.x * w11;
          vx = a.y * w00 + b.y * w01 + c.y * w10 + e.y * w11;
        } else {  // within one pixel of the top / left edge: the literal expression
          const double yy = (double)py[j] - (double)yi[j], xx = (double)px[j] - (double)xi[j];
          vy = a.x * (1.0 - yy) * (1.0 - xx) + b.x * (1.0 - yy) * xx + c.x * yy * (1.0 - xx) + e.x * yy * xx;
          vx = a.y * (1.0 - yy) * (1.0 - xx) + b.y * (1.0 - yy) * xx + c.y * yy * (1.0 - xx) + e.y * yy * xx;
        }
        // clamp to [0, L - 1] in one v_med3_f32 (= fminf(L, fmaxf(0, .)) for the finite values here)
        const float ny = __builtin_amdgcn_fmed3f(py[j] + (float)vy, 0.0f, fLy);
        const float nx = __builtin_amdgcn_fmed3f(px[j] + (float)vx, 0.0f, fLx);
        if (!done[j]) {
          if (ny == py[j] && nx == px[j]) done[j] = true;  // exact fixed point
          py[j] = ny;
          px[j] = nx;
        }
      }
    }
    const bool last = step0 + steps >= niter;
    bool carry[NI];
    unsigned long long bal[NI];
    // a finished item's final position goes straight into get_masks' histogram (initialised by
    // k_hist_init before the rounds) instead of a second pass over the moving pixels
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const bool fin = active[j] && (done[j] || last);
      agg_add(Hh, ((int)py[j] + kRpad) * Dxh + (int)px[j] + kRpad, fin);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      if (active[j] && (done[j] || last)) P[q[j]] = make_float2(py[j], px[j]);
      carry[j] = active[j] && !done[j] && !last;
      bal[j] = __ballot(carry[j]);
      if (lane == 0) wsum[j][wid] = __popcll(bal[j]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int j = 0; j < NI; ++j)
        for (int w = 0; w < kT / 64; ++w) {
          const int c = wsum[j][w];
          wsum[j][w] = t;
          t += c;
        }
      sbase = t ? atomicAdd(&out_cnt[fov], t) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NI; ++j)
      if (carry[j]) {
        FollowItem it;
        it.q = q[j];
        it.py = py[j];
        it.px = px[j];
        it.pad = 0;
        dst[sbase + wsum[j][wid] + __popcll(bal[j] & ((1ull << lane) - 1ull))] = it;
      }
    __syncthreads();
  }
}

// histogram of final positions (get_masks: np.add.at(h, (p + rpad)), padded grid Dyh x Dxh).
// Pixels that did not move sit at their own coordinate: one plain store per padded cell covers
// them (and clears the rest); the moving pixels then add with wave-aggregated atomics (the
// pixels of one cell mostly end in the same bin).
// Four cells per thread (kPx4): one 16-byte store when the FOV's grid allows (nh % 4 == 0), the
// per-pixel kernels below likewise — one element per thread held these full-image passes at
// ~2 TB/s
constexpr int kPx4 = 4;

__global__ __launch_bounds__(kT) void k_hist_init(int Dy, int Dx, DynBufs d) {
  const int fov = blockIdx.y;
  const int Dxh = Dx + 2 * kRpad, Dyh = Dy + 2 * kRpad;
  const long long nh = (long long)Dyh * Dxh;
  const long long b0 = ((long long)blockIdx.x * kT + threadIdx.x) * kPx4;
  if (b0 >= nh) return;
  const unsigned char* mov = d.mov + (long long)fov * Dy * Dx;
  int v[kPx4];
#pragma unroll
  for (int u = 0; u < kPx4; ++u) {
    const long long b = b0 + u;
    v[u] = 0;
    if (b < nh) {
      const int bi = (int)b;  // nh < 2^31 (cpx_seg_masks): 32-bit division
      const int y = bi / Dxh - kRpad, x = bi - (bi / Dxh) * Dxh - kRpad;
      if (y >= 0 && y < Dy && x >= 0 && x < Dx) v[u] = mov[(long long)y * Dx + x] ? 0 : 1;
    }
  }
  int* h = d.h + (long long)fov * nh;
  if ((nh & 3) == 0) {
    *reinterpret_cast<int4*>(h + b0) = make_int4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int u = 0; u < kPx4; ++u)
      if (b0 + u < nh) h[b0 + u] = v[u];
  }
}

__global__ __launch_bounds__(kT) void k_hist_moving(int Dy, int Dx, DynBufs d) {
  const int fov = blockIdx.y;
  const long long n = (long long)Dy * Dx;
  const int i = blockIdx.x * kT + threadIdx.x;
  const int n_moving = d.st[fov].n_moving;
  // (FOVs with >= 5 moving pixels: k_dyn_follow added their final positions)
  if (n_moving >= 5 || (long long)blockIdx.x * kT >= n_moving) return;  // block-uniform
  const int Dxh = Dx + 2 * kRpad;
  const bool valid = i < n_moving;
  int key = 0;
  if (valid) {
    const int q = d.act[(long long)fov * n + i];
    // moving pixels of an FOV with < 5 of them never followed: their own coordinate
    float2 pp = n_moving >= 5 ? d.p[(long long)fov * n + q] : make_float2((float)(q / Dx), (float)(q % Dx));
    key = ((int)pp.x + kRpad) * Dxh + (int)pp.y + kRpad;
  }
  agg_add(d.h + (long long)fov * (Dy + 2 * kRpad) * Dxh, key, valid);
}

// seeds: h > 10 and h == 5x5 max (maximum_filter1d size 5 on both axes); kPx4 cells per thread
__global__ __launch_bounds__(kT) void k_seed_flags(int Dyh, int Dxh, DynBufs d) {
  const int fov = blockIdx.y;
  const long long nh = (long long)Dyh * Dxh;
  const long long q0 = ((long long)blockIdx.x * kT + threadIdx.x) * kPx4;
  if (q0 >= nh) return;
  const int* h = d.h + (long long)fov * nh;
  const bool vec = (nh & 3) == 0;
  int v[kPx4];
  if (vec) {
    const int4 t = *reinterpret_cast<const int4*>(h + q0);
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
    v[3] = t.w;
  } else {
#pragma unroll
    for (int u = 0; u < kPx4; ++u) v[u] = q0 + u < nh ? h[q0 + u] : 0;
  }
  unsigned int fw = 0;
#pragma unroll
  for (int u = 0; u < kPx4; ++u) {
    if (v[u] <= 10) continue;
    const long long q = q0 + u;
    const int y = (int)(q / Dxh), x = (int)(q % Dxh);
    int mx = v[u];
    for (int dy = -2; dy <= 2; ++dy)
      for (int dx = -2; dx <= 2; ++dx) {
        int yy = y + dy, xx = x + dx;  // scipy 'reflect' boundary (never reached by seeds)
        yy = yy < 0 ? -yy - 1 : (yy >= Dyh ? 2 * Dyh - yy - 1 : yy);
        xx = xx < 0 ? -xx - 1 : (xx >= Dxh ? 2 * Dxh - xx - 1 : xx);
        mx = max(mx, h[(long long)yy * Dxh + xx]);
      }
    fw |= (unsigned int)(v[u] >= mx) << (8 * u);
  }
  unsigned char* f = d.sflag + (long long)fov * nh;
  if (vec && ((((uintptr_t)(f + q0)) & 3u) == 0)) {
    *reinterpret_cast<unsigned int*>(f + q0) = fw;
  } else {
#pragma unroll
    for (int u = 0; u < kPx4; ++u)
      if (q0 + u < nh) f[q0 + u] = (unsigned char)((fw >> (8 * u)) & 1u);
  }
}

// ---- ordered compaction of byte flags: indices of the set flags in increasing order ---------
// (tile counts -> per-FOV exclusive scan -> in-tile ranks).  Three launches; every block works
// on one 8 KiB tile, so a 2080^2 FOV's flags spread over ~550 blocks instead of one.
constexpr int kOcThreads = 256;
constexpr int kOcPer = 32;                       // flags per thread (two 16-byte loads)
constexpr int kOcTile = kOcThreads * kOcPer;     // 8192

__device__ __forceinline__ int oc_load(const unsigned char* f, long long n, long long i0,
                                       unsigned int* bits) {
  // bit j of *bits = flag i0 + j (j < 32); returns the count
  unsigned int b = 0;
  if (i0 + kOcPer <= n && (((uintptr_t)(f + i0)) & 15u) == 0) {
    const uint4* v = reinterpret_cast<const uint4*>(f + i0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint4 t = v[h];
      const unsigned int w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int by = 0; by < 4; ++by)
          b |= (((w[k] >> (8 * by)) & 0xffu) ? 1u : 0u) << (h * 16 + k * 4 + by);
    }
  } else {
    for (int j = 0; j < kOcPer; ++j)
      if (i0 + j < n && f[i0 + j]) b |= 1u << j;
  }
  *bits = b;
  return __popc(b);
}

__global__ __launch_bounds__(kOcThreads) void k_oc_count(const unsigned char* __restrict__ flags,
                                                         long long n, int ntile, int* __restrict__ tiles) {
  const int fov = blockIdx.y, t = blockIdx.x;
  const unsigned char* f = flags + (long long)fov * n;
  unsigned int bits;
  int c = oc_load(f, n, (long long)t * kOcTile + (long long)threadIdx.x * kOcPer, &bits);
  c = wave_sum(c);
  __shared__ int ws[kOcThreads / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < kOcThreads / 64; ++w) s += ws[w];
    tiles[(long long)fov * ntile + t] = s;
  }
}

// one block per FOV: exclusive scan of the tile counts in place; total -> totals[fov]
__global__ __launch_bounds__(1024) void k_oc_scan(int ntile, int* __restrict__ tiles,
                                                  int* __restrict__ totals) {
  const int fov = blockIdx.x;
  int* t = tiles + (long long)fov * ntile;
  __shared__ int wsum[16];
  __shared__ int base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i0 = 0; i0 < ntile; i0 += 1024) {
    const int i = i0 + threadIdx.x;
    const int v = i < ntile ? t[i] : 0;
    int inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    int off = base;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    if (i < ntile) t[i] = off + inc - v;
    __syncthreads();
    if (threadIdx.x == 0) {
      int s = 0;
      for (int w = 0; w < 16; ++w) s += wsum[w];
      base += s;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) totals[fov] = base;
}

__global__ __launch_bounds__(kOcThreads) void k_oc_emit(const unsigned char* __restrict__ flags,
                                                        long long n, int ntile,
                                                        const int* __restrict__ tiles, int cap,
                                                        int* __restrict__ out, long long out_stride) {
  const int fov = blockIdx.y, t = blockIdx.x;
  const int off0 = tiles[(long long)fov * ntile + t];
  if (off0 >= cap) return;
  const unsigned char* f = flags + (long long)fov * n;
  const long long i0 = (long long)t * kOcTile + (long long)threadIdx.x * kOcPer;
  unsigned int bits;
  const int c = oc_load(f, n, i0, &bits);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  __shared__ int wsum[kOcThreads / 64];
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  int k = off0 + inc - c;
  for (int w = 0; w < wid; ++w) k += wsum[w];
  int* o = out + (long long)fov * out_stride;
  while (bits) {
    const int j = __ffs(bits) - 1;
    bits &= bits - 1;
    if (k < cap) o[k] = (int)(i0 + j);
    ++k;
  }
}

// one wave per seed: geodesic 8-connected ball of radius 5 through h > 2 (get_masks expansion)
__global__ __launch_bounds__(kT) void k_seed_expand(int Dyh, int Dxh, DynBufs d) {
  const int fov = blockIdx.y;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __shared__ unsigned char cur[kT / 64][2][169];
  const int ns = d.st[fov].n_seeds;
  const long long nh = (long long)Dyh * Dxh;
  for (int kb = blockIdx.x * (kT / 64); kb < ns; kb += gridDim.x * (kT / 64)) {  // block-uniform
  const int k = kb + wid;
  const bool active = k < ns;
  const int s = active ? d.seeds[(long long)fov * d.ms + k] : 0;
  const int sy = s / Dxh, sx = s - sy * Dxh;
  const int* h = d.h + (long long)fov * nh;
  bool good[3];
  for (int u = 0; u < 3; ++u) {
    const int c = lane + 64 * u;
    good[u] = false;
    if (c < 169 && active) {
      const int yy = sy - 6 + c / 13, xx = sx - 6 + c % 13;
      good[u] = yy >= 0 && yy < Dyh && xx >= 0 && xx < Dxh && h[(long long)yy * Dxh + xx] > 2;
      cur[wid][0][c] = (c == 84);  // the seed (window centre)
    }
  }
  __syncthreads();
  int src = 0;
  for (int it = 0; it < 5; ++it) {
    for (int u = 0; u < 3; ++u) {
      const int c = lane + 64 * u;
      if (c >= 169) continue;
      const int cy = c / 13, cx = c % 13;
      bool any = false;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int ny = cy + dy, nx = cx + dx;
          if (ny >= 0 && ny < 13 && nx >= 0 && nx < 13) any |= cur[wid][src][ny * 13 + nx] != 0;
        }
      cur[wid][src ^ 1][c] = (any && good[u]) ? 1 : 0;
    }
    __syncthreads();
    src ^= 1;
  }
  if (active) {
    unsigned int* M = d.M + (long long)fov * nh;
    for (int u = 0; u < 3; ++u) {
      const int c = lane + 64 * u;
      if (c < 169 && cur[wid][src][c]) {
        const int yy = sy - 6 + c / 13, xx = sx - 6 + c % 13;
        atomicMax(&M[(long long)yy * Dxh + xx], (unsigned int)(k + 1));  // later seeds win (M[pix[k]] = 1+k)
      }
    }
  }
  __syncthreads();
  }  // seed loop
}

// M0 = M[pflows]: every pixel's label at its final position; per label its pixel count and
// first pixel, aggregated per wave (lanes are consecutive pixels, mostly of one label).  kAsg
// pixels per thread (q = block base + k kT + thread), each step's loads for all of them issued
// before any is used: one pixel per thread left the three dependent loads (moving flag, final
// position, label map) exposed per pixel
constexpr int kAsg = 4;
__global__ __launch_bounds__(kT) void k_assign(int Dy, int Dx, DynBufs d) {
  const int fov = blockIdx.y;
  const long long n = (long long)Dy * Dx;
  const int q0 = blockIdx.x * kT * kAsg + threadIdx.x;
  const int Dxh = Dx + 2 * kRpad;
  const bool follow = d.st[fov].n_moving >= 5;
  const unsigned char* mov = d.mov + (long long)fov * n;
  const float2* P = d.p + (long long)fov * n;
  const unsigned int* M = d.M + (long long)fov * (Dy + 2 * kRpad) * Dxh;
  unsigned char mv[kAsg];
#pragma unroll
  for (int k = 0; k < kAsg; ++k) {
    const int q = q0 + k * kT;
    mv[k] = q < n ? mov[q] : 0;
  }
  float2 pp[kAsg];
#pragma unroll
  for (int k = 0; k < kAsg; ++k) {
    const int q = q0 + k * kT;
    pp[k] = make_float2(0.0f, 0.0f);
    if (follow && mv[k]) pp[k] = P[q];
  }
  int l[kAsg];
#pragma unroll
  for (int k = 0; k < kAsg; ++k) {
    const int q = q0 + k * kT;
    l[k] = 0;
    if (q < n) {
      int iy = q / Dx, ix = q - iy * Dx;
      if (follow && mv[k]) {
        iy = (int)pp[k].x;
        ix = (int)pp[k].y;
      }
      l[k] = (int)M[(long long)(iy + kRpad) * Dxh + ix + kRpad];
    }
  }
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < kAsg; ++k) {
    const int q = q0 + k * kT;
    if (q < n) d.m0[(long long)fov * n + q] = l[k];
    unsigned long long pend = __ballot(l[k] != 0);
    while (pend) {
      const int leader = __ffsll((long long)pend) - 1;
      const int l0 = __shfl(l[k], leader);
      const unsigned long long m = __ballot(l[k] == l0);
      if (lane == leader) {
        atomicAdd(&d.cnt[(long long)fov * (d.ms + 1) + l0], __popcll(m));
        atomicMin(&d.first[(long long)fov * (d.ms + 1) + l0], q);  // lowest lane = first pixel
      }
      pend &= ~m;
    }
  }
}

// big-mask removal (> 40 % of the image) + first-occurrence marks for fastremap.renumber
__global__ __launch_bounds__(kT) void k_relabel_mark(int Dy, int Dx, DynBufs d) {
  const int fov = blockIdx.y;
  const int l = blockIdx.x * kT + threadIdx.x + 1;
  if (l > d.st[fov].n_seeds) return;
  const long long o = (long long)fov * (d.ms + 1) + l;
  const int c = d.cnt[o];
  const double big = (double)Dy * (double)Dx * 0.4;
  if (c > 0 && !((double)c > big)) d.mark[(long long)fov * Dy * Dx + d.first[o]] = 1;
}

// the j-th marked pixel (raster order) carries the label that becomes j + 1
__global__ __launch_bounds__(kT) void k_relabel_apply(int Dy, int Dx, DynBufs d) {
  const int fov = blockIdx.y;
  const int n_masks = min(d.totals[fov], d.ms);
  const long long n = (long long)Dy * Dx;
  for (int j = blockIdx.x * kT + threadIdx.x; j < n_masks; j += gridDim.x * kT) {
    const int pix = d.marklist[(long long)fov * d.ms + j];
    d.mark[(long long)fov * n + pix] = 0;
    d.newlab[(long long)fov * (d.ms + 1) + d.m0[(long long)fov * n + pix]] = j + 1;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) d.st[fov].n_masks = n_masks;
}

__global__ __launch_bounds__(kT) void k_apply_newlab(int Dy, int Dx, DynBufs d) {
  const int fov = blockIdx.y;
  const long long n = (long long)Dy * Dx;
  const long long q0 = ((long long)blockIdx.x * kT + threadIdx.x) * kPx4;
  if (q0 >= n) return;
  int* m = d.m0 + (long long)fov * n;
  const int* nl = d.newlab + (long long)fov * (d.ms + 1);
  if ((n & 3) == 0 && (((uintptr_t)d.m0) & 15u) == 0) {  // (m0 may be the caller's buffer)
    const int4 t = *reinterpret_cast<const int4*>(m + q0);
    int4 o;
    o.x = t.x ? nl[t.x] : 0;  // big masks map to 0
    o.y = t.y ? nl[t.y] : 0;
    o.z = t.z ? nl[t.z] : 0;
    o.w = t.w ? nl[t.w] : 0;
    *reinterpret_cast<int4*>(m + q0) = o;
  } else {
#pragma unroll
    for (int u = 0; u < kPx4; ++u)
      if (q0 + u < n) {
        const int l = m[q0 + u];
        m[q0 + u] = l ? nl[l] : 0;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// flow-error filter (dynamics.remove_bad_flow_masks / metrics.flow_error): per mask the 2.x CPU
// masks_to_flows heat diffusion from the pixel nearest the median, 2 * (ptp x + ptp y) Jacobi
// iterations in fp64, normalised central differences, mean squared difference to dP / 5.
//
// k_flow_error_lds: one block per mask (dynamic queue over all masks of the batch).  The
// diffusion grid T ((bh+2) x (bw+2) fp64 at an even row stride, zero outside the mask) lives in
// LDS as ONE buffer: a work unit is kFeKS consecutive rows of two adjacent columns (X, X + 1),
// X odd; the thread that owns it slides a 3 x 4 window down the unit (two 16-byte LDS reads per
// row for two cells, instead of three 8-byte reads per cell), keeps the new values in registers
// and writes them back after a barrier.  Every thread owns up to U units (consecutive threads:
// consecutive column pairs).
// Sums keep the reference's term order; rows are computed unconditionally (compile-time loop)
// and only mask cells are written.
// The two cells of a column pair (X, X + 1) from the 3 x 4 window (rows u, c, d; words a =
// columns X - 1, X and b = X + 1, X + 2): the reference's 9-term sums in its own order, the two
// dependent fp64 chains interleaved so each wave has two additions in flight (the adds of one
// chain wait on each other's results)
template <typename E, typename E2>
__device__ __forceinline__ void fe_pair(const E2& ua, const E2& ub, const E2& ca, const E2& cb, const E2& da,
                                        const E2& db, E& n0, E& n1) {
  E s0 = ca.y + ua.y, s1 = cb.x + ub.x;
  s0 = s0 + da.y;
  s1 = s1 + db.x;
  s0 = s0 + ca.x;
  s1 = s1 + ca.y;
  s0 = s0 + cb.x;
  s1 = s1 + cb.y;
  s0 = s0 + ua.x;
  s1 = s1 + ua.y;
  s0 = s0 + ub.x;
  s1 = s1 + ub.y;
  s0 = s0 + da.x;
  s1 = s1 + da.y;
  s0 = s0 + db.x;
  s1 = s1 + db.y;
  n0 = (E)(1 / 9.) * s0;  // column X: c + u + d + l + r + ul + ur + dl + dr
  n1 = (E)(1 / 9.) * s1;  // column X + 1
}

constexpr int kFeKS = 12;
static_assert(kFeKS <= 32, "unit mask bits");

// the grid's row stride: bw + 2 columns (zero border) rounded up to even, so a column pair
// (2m, 2m + 1) is one 16-byte LDS word
__host__ __device__ constexpr int fe_stride(int bw) { return (bw + 3) & ~1; }
__host__ __device__ constexpr bool fe_fits(int bh, int bw, int threads, int units, int cells) {
  const int nsr = (bh + kFeKS - 1) / kFeKS;
  return (long long)(bh + 2) * fe_stride(bw) <= cells &&
         (long long)((bw + 1) / 2) * nsr <= (long long)threads * units;
}

// exclusive prefix of the per-FOV object counts (queue item -> (fov, object))
__global__ void k_obj_prefix(int B, const cpx_fov_objects* __restrict__ hdr, int* __restrict__ off) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int s = 0;
    for (int b = 0; b < B; ++b) {
      off[b] = s;
      s += hdr[b].n_objects;
    }
    off[B] = s;
  }
}

// E = double: the reference's arithmetic, the decision err > thr.  E = float (screening pass):
// the same sweeps in fp32 — half the LDS per mask, so twice the masks in flight per CU — and a
// decision only where it is certain: every operation of a sweep adds non-negative terms, so
// each fp32 cell stays within a relative (1 + 11u)^niter of the exact value (u = 2^-24; plus an
// absolute n 2^-126 for underflow), and so does the fp64 reference (u = 2^-53); from that bound
// on both grids every pixel's normalised gradient gets a bound on its error contribution (a
// pixel whose gradient is not clearly above its own uncertainty counts its whole range
// (1 + |dP/5|)^2).  A mask whose fp32 error is further from thr than the summed bound gets its
// flag (1 bad, 2 kept) — the same flag the fp64 sweeps give it; any other mask is flagged 3 and
// appended to `und` ([0] = count, then fov << 20 | object), which the fp64 pass (list = und)
// then decides exactly.
template <int THREADS, int CELLS, int U, typename E = double, int WPE = 4>
__global__ __launch_bounds__(THREADS, WPE) void k_flow_error_lds(  // WPE waves per SIMD: <= 512 / WPE VGPRs
    const int* __restrict__ m0, const float2* __restrict__ dpf, int Dy, int Dx, int B, int max_label,
    const cpx_object* __restrict__ objects, const int* __restrict__ off, int* __restrict__ ctr,
    int lo_threads, int lo_units, int lo_cells, double thr, unsigned char* __restrict__ bad,
    const int* __restrict__ list, int* __restrict__ und) {
  constexpr bool kScreen = std::is_same<E, float>::value;
  typedef typename std::conditional<kScreen, float2, double2>::type E2;
  __shared__ __attribute__((aligned(16))) E T[CELLS];
  __shared__ double sred[THREADS / 64][3];
  __shared__ unsigned long long sbest[THREADS / 64];
  __shared__ double smed[2];
  __shared__ int sitem;
  const long long n = (long long)Dy * Dx;
  const int total = list ? list[0] : off[B];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int claims = 0;; ++claims) {
    if (claims > total) {  // broken claim (cpx_internal.h kClaimBroken)
      if (tid == 0) atomicOr(ctr, kClaimBroken);
      break;
    }
    if (tid == 0) sitem = atomicAdd(ctr, 1);
    __syncthreads();
    const int item = sitem;
    __syncthreads();
    if (item >= total) break;
    int fov = 0, kobj;
    if (list) {  // the screening pass's undecided masks
      const int code = list[1 + item];
      fov = code >> 20;
      kobj = code & 0xfffff;
    } else {
      while (fov + 1 < B && off[fov + 1] <= item) ++fov;
      kobj = item - off[fov];
    }
    const cpx_object o = objects[(long long)fov * max_label + kobj];
    const int L = o.label;
    const int r0 = o.bbox[0], c0 = o.bbox[1];
    const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
    // block-uniform: objects of the smaller variant or of k_flow_error_big are skipped
    if (!fe_fits(bh, bw, THREADS, U, CELLS)) continue;
    if (lo_threads > 0 && fe_fits(bh, bw, lo_threads, lo_units, lo_cells)) continue;
    // screening: masks k_flow_error_reg already decided (or deferred) carry their flag
    if (kScreen && !list && bad[(long long)fov * (max_label + 1) + L] != 0) continue;
    // rows per unit: the one-block-per-CU variant (latency-bound: one mask at a time) takes the
    // fewest (<= kFeKS) that keep the units within the block, so a mask spreads over more lanes
    // with shorter per-iteration chains; the multi-block variants keep kFeKS (throughput-bound:
    // shorter units only add halo-row reads)
    const int ncp0 = (bw + 1) / 2;
    const int R = THREADS < 1024 ? kFeKS
                                 : min(kFeKS, max(1, (bh + max(1, THREADS * U / ncp0) - 1) / max(1, THREADS * U / ncp0)));
    const int nsr = (bh + R - 1) / R;
    const int ly = bh + 2;
    const int* lab = m0 + (long long)fov * n;
    // ---- medians of the pixel coordinates (row / column counts in the T area, as ints)
    int* rowc = reinterpret_cast<int*>(T);
    int* colc = rowc + bh;
    for (int i = tid; i < bh + bw; i += THREADS) rowc[i] = 0;
    __syncthreads();
    const int nb = bh * bw;
    for (int p = tid; p < nb; p += THREADS) {
      const int rr = p / bw, cc = p - rr * bw;
      if (lab[(long long)(r0 + rr) * Dx + c0 + cc] == L) {
        atomicAdd(&rowc[rr], 1);
        atomicAdd(&colc[cc], 1);
      }
    }
    __syncthreads();
    if (tid < 2) {
      const int* hc = tid == 0 ? rowc : colc;
      const int len = tid == 0 ? bh : bw;
      const long long cntn = o.area;
      const long long ka = (cntn - 1) / 2, kb = cntn / 2;
      long long cum = 0;
      int va = -1, vb = -1;
      for (int i = 0; i < len; ++i) {
        cum += hc[i];
        if (va < 0 && cum > ka) va = i;
        if (vb < 0 && cum > kb) { vb = i; break; }
      }
      smed[tid] = ((double)(va + 1) + (double)(vb + 1)) / 2.0;
    }
    __syncthreads();
    // ---- argmin of (x-xmed)^2 + (y-ymed)^2, first in row-major order on ties
    const double ymed = smed[0], xmed = smed[1];
    unsigned long long best = ~0ull;
    for (int p = tid; p < nb; p += THREADS) {
      const int rr = p / bw, cc = p - rr * bw;
      if (lab[(long long)(r0 + rr) * Dx + c0 + cc] != L) continue;
      const double dy = (double)(rr + 1) - ymed, dx = (double)(cc + 1) - xmed;
      const double dist = dx * dx + dy * dy;
      // medians are multiples of 1/2, so 4*dist is an exact integer: order-preserving key
      const unsigned long long key = ((unsigned long long)(dist * 4.0) << 32) | (unsigned int)p;
      best = key < best ? key : best;
    }
    best = wave_min(best);
    if (lane == 0) sbest[wid] = best;
    __syncthreads();
    unsigned long long bsel = sbest[0];
    for (int w = 1; w < THREADS / 64; ++w) bsel = sbest[w] < bsel ? sbest[w] : bsel;
    const int pbest = (int)(bsel & 0xffffffffu);
    const int ym = pbest / bw + 1, xm = pbest % bw + 1;
    const int niter = 2 * ((bw - 1) + (bh - 1));  // 2 * (ptp(x) + ptp(y))
    const int lxp = fe_stride(bw);  // row stride of T (lx = bw + 2 columns used)
    const int ncp = (bw + 1) / 2;   // column pairs (interior columns 2m + 1, 2m + 2)
    // ---- this thread's units: columns X, X + 1 (X = 2m + 1), rows Y0 .. Y0 + kFeKS - 1
    int ux[U], uy0[U], ujc[U];
    unsigned int um[U][2];
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int u = tid + i * THREADS;
      um[i][0] = um[i][1] = 0u;
      ux[i] = 1;
      uy0[i] = 1;
      ujc[i] = -1;
      if (u < ncp * nsr) {
        const int X = 2 * (u % ncp) + 1, Y0 = 1 + (u / ncp) * R;
        ux[i] = X;
        uy0[i] = Y0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (X + h > bw) continue;  // bw odd: the last pair's second column is the border
          unsigned int m = 0u;
          for (int j = 0; j < R && Y0 + j <= bh; ++j)
            if (lab[(long long)(r0 + Y0 - 1 + j) * Dx + c0 + X + h - 1] == L) m |= 1u << j;
          um[i][h] = m;
          if (X + h == xm && ym >= Y0 && ym < Y0 + R) ujc[i] = 2 * (ym - Y0) + h;
        }
      }
    }
    // Chebyshev distance of each unit from the centre: T is exactly 0.0 beyond distance it before
    // iteration it (the support grows by one cell per iteration), so a unit further than it + 1
    // would compute and store 0.0 over 0.0 — it is skipped until the support reaches it
    int ud[U];
#pragma unroll
    for (int i = 0; i < U; ++i)
      ud[i] = max(max(max(0, uy0[i] - ym), ym - (uy0[i] + R - 1)), max(max(0, ux[i] - xm), xm - (ux[i] + 1)));
    __syncthreads();  // rowc / colc / sbest reads done before T is cleared
    for (int i = tid; i < ly * lxp; i += THREADS) T[i] = (E)0;
    __syncthreads();
    if (tid == 0 && niter > 0) T[ym * lxp + xm] = (E)1;  // the first iteration's T[centre] += 1
    __syncthreads();
    E nv[U][2][kFeKS];
    const int cidx = ym * lxp + xm;
    bool cown = false;  // this thread owns the centre cell
#pragma unroll
    for (int i = 0; i < U; ++i)
      if (ujc[i] >= 0) cown = true;
    const E2* T2 = reinterpret_cast<const E2*>(T);
    for (int it = 0; it < niter; ++it) {
#pragma unroll
      for (int i = 0; i < U; ++i) {
        if (!(um[i][0] | um[i][1]) || ud[i] > it + 1) continue;  // no mask cell (or no unit), or
                                                                  // beyond the support
        // E2 offsets of the unit's rows (columns X - 1 .. X + 2 = two 16-byte words); the
        // opaque base keeps the compiler from holding every row address across the loop, and
        // rows past the object's last row read the zero border row (clamped): their sums are
        // never written
        int r = ((uy0[i] - 1) * lxp + ux[i] - 1) >> 1;
        int rmax = ((ly - 1) * lxp + ux[i] - 1) >> 1;
        const int rs = lxp >> 1;
        asm volatile("" : "+v"(r), "+v"(rmax));
        E2 ua = T2[r], ub = T2[r + 1];
        r += rs;
        E2 ca = T2[r], cb = T2[r + 1];
        r = min(r + rs, rmax);
        E2 da = T2[r], db = T2[r + 1];
#pragma unroll
        for (int j = 0; j < kFeKS; ++j) {
          // rows beyond R: predicated off (block-uniform), the loop stays unrolled so nv stays in
          // registers.  The next row's loads are issued before this row's sums (latency hidden);
          // the scheduling barrier keeps the compiler from hoisting more rows (register budget)
          if (j < R) {
            E2 na = {(E)0, (E)0}, nb = {(E)0, (E)0};
            if (j + 1 < R) {
              r = min(r + rs, rmax);
              na = T2[r];
              nb = T2[r + 1];
            }
            // column X: l = .x of a, c = .y of a, r = .x of b;  column X + 1: l = a.y, c = b.x, r = b.y
            fe_pair<E, E2>(ua, ub, ca, cb, da, db, nv[i][0][j], nv[i][1][j]);
            ua = ca; ub = cb;
            ca = da; cb = db;
            da = na; db = nb;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < U; ++i) {
        if (!(um[i][0] | um[i][1]) || ud[i] > it + 1) continue;
        int wb = uy0[i] * lxp + ux[i];
        asm volatile("" : "+v"(wb));
#pragma unroll
        for (int j = 0; j < kFeKS; ++j) {
          if ((um[i][0] >> j) & 1u) T[wb + j * lxp] = nv[i][0][j];
          if ((um[i][1] >> j) & 1u) T[wb + j * lxp + 1] = nv[i][1][j];
        }
      }
      // the next iteration's T[centre] += 1, by the centre's owner after its own store
      if (cown && it + 1 < niter) T[cidx] = T[cidx] + (E)1;
      __syncthreads();
    }
    // ---- gradients, normalisation, error vs dP/5
    const float2* F = dpf + (long long)fov * n;
    // screening: relative bound rho on |T32 - T64| per cell (both vs the exact sweeps, see above)
    // and the absolute underflow allowance alpha
    double rho = 0.0, alpha = 0.0;
    if constexpr (kScreen) {
      const double g32 = 11.0 * 0x1p-24 * (1.0 + 1e-6), g64 = 11.0 * 0x1p-53 * (1.0 + 1e-6);
      rho = (expm1((double)niter * g32) + expm1((double)niter * g64)) / (1.0 - (double)niter * g32);
      alpha = 4.0 * (double)niter * 0x1p-126;
    }
    double e0 = 0.0, e1 = 0.0, eb = 0.0;
#pragma unroll
    for (int i = 0; i < U; ++i) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        for (int j = 0; j < kFeKS; ++j) {
          if (!((um[i][h] >> j) & 1u)) continue;
          const int Y = uy0[i] + j, X = ux[i] + h;
          const double tdn = (double)T[(Y + 1) * lxp + X], tup = (double)T[(Y - 1) * lxp + X];
          const double trt = (double)T[Y * lxp + X + 1], tlf = (double)T[Y * lxp + X - 1];
          const double dy = tdn - tup;
          const double dx = trt - tlf;
          const double g = sqrt(dy * dy + dx * dx);
          const double nrm = 1e-20 + g;
          const double my = dy / nrm, mx = dx / nrm;
          const float2 f = F[(long long)(r0 + Y - 1) * Dx + c0 + X - 1];
          const double fy = (double)(f.x / 5.0f), fx = (double)(f.y / 5.0f);
          const double ty = my - fy;
          const double tx = mx - fx;
          e0 += ty * ty;
          e1 += tx * tx;
          if constexpr (kScreen) {
            // |grad32 - grad64| <= D; unit vectors then differ by <= 2 D / |grad32| (+ the 1e-20)
            const double Dy_ = rho * (tdn + tup) + 2.0 * alpha, Dx_ = rho * (trt + tlf) + 2.0 * alpha;
            const double D = sqrt(Dy_ * Dy_ + Dx_ * Dx_) * (1.0 + 1e-9);
            const double ff = sqrt(fy * fy + fx * fx);
            if (g > 3.0 * D && g > 1e-12) {
              const double ep = 2.0 * D / g + 1e-7;
              eb += ep * (2.0 * sqrt(ty * ty + tx * tx) + ep);
            } else {
              eb += (1.0 + ff) * (1.0 + ff);
            }
          }
        }
      }
    }
    e0 = wave_sum(e0);
    e1 = wave_sum(e1);
    if constexpr (kScreen) eb = wave_sum(eb);
    if (lane == 0) {
      sred[wid][0] = e0;
      sred[wid][1] = e1;
      sred[wid][2] = eb;
    }
    __syncthreads();
    if (tid == 0) {
      double s0 = 0.0, s1 = 0.0, sb = 0.0;
      for (int w = 0; w < THREADS / 64; ++w) {
        s0 += sred[w][0];
        s1 += sred[w][1];
        sb += sred[w][2];
      }
      const double err = 0.0 + s0 / (double)o.area + s1 / (double)o.area;
      unsigned char v = err > thr ? 1 : 2;
      if constexpr (kScreen) {
        // + the two fp64 error sums' own rounding (orders differ) with a wide margin
        const double bnd = sb / (double)o.area + 1e-9 * (1.0 + err);
        v = err - thr > bnd ? 1 : thr - err > bnd ? 2 : 3;
        if (v == 3) und[1 + atomicAdd(&und[0], 1)] = (fov << 20) | kobj;
      }
      bad[(long long)fov * (max_label + 1) + L] = v;
    }
    __syncthreads();
  }
}

// k_flow_error_cmp: the same per-mask diffusion for masks whose full (bh + 2) x stride grid does
// not fit the large LDS kernel (kFeLargeCells; its per-row span lookups make it slower there): T holds only each row's span of mask cells (row y keeps the
// column pairs [pb, pe] covering its mask pixels, at T2[base + p]); every cell outside a row's
// span is a non-mask cell of the reference's grid, which stays 0.0 for the whole diffusion, so
// reads there return zero.  Round masks keep ~80 % of their bbox, which takes masks up to about
// 155 x 155 px in one CU.  One unit (2 columns x kFeKS rows) per thread; masks with more units,
// more than kCmpRows rows or more cells are left to k_flow_error_big (their flag stays 0).
constexpr int kCmpRows = 256;

template <int THREADS, int CELLS, int U>
__global__ __launch_bounds__(THREADS, 1) void k_flow_error_cmp(
    const int* __restrict__ m0, const float2* __restrict__ dpf, int Dy, int Dx, int B, int max_label,
    const cpx_object* __restrict__ objects, const int* __restrict__ off, int* __restrict__ ctr,
    int lo_threads, int lo_units, int lo_cells, double thr, unsigned char* __restrict__ bad) {
  __shared__ __attribute__((aligned(16))) double T[CELLS];
  __shared__ int2 rowt[kCmpRows + 2];  // (base, pb | pe << 16) per T row; empty: pb 1, pe 0
  __shared__ double sred[THREADS / 64][2];
  __shared__ unsigned long long sbest[THREADS / 64];
  __shared__ double smed[2];
  __shared__ int sitem, stot;
  const long long n = (long long)Dy * Dx;
  const int total = off[B];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const double2 z2 = {0.0, 0.0};
  for (int claims = 0;; ++claims) {
    if (claims > total) {  // broken claim (cpx_internal.h kClaimBroken)
      if (tid == 0) atomicOr(ctr, kClaimBroken);
      break;
    }
    if (tid == 0) sitem = atomicAdd(ctr, 1);
    __syncthreads();
    const int item = sitem;
    __syncthreads();
    if (item >= total) break;
    int fov = 0;
    while (fov + 1 < B && off[fov + 1] <= item) ++fov;
    const int kobj = item - off[fov];
    const cpx_object o = objects[(long long)fov * max_label + kobj];
    const int L = o.label;
    const int r0 = o.bbox[0], c0 = o.bbox[1];
    const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
    // block-uniform: the smaller kernels' masks, and masks beyond this kernel's limits
    if (fe_fits(bh, bw, lo_threads, lo_units, lo_cells)) continue;
    const int ncp = (bw + 1) / 2;
    if (bh > kCmpRows || (long long)ncp * ((bh + kFeKS - 1) / kFeKS) > (long long)THREADS * U) continue;
    const int G = max(1, THREADS * U / ncp);  // row groups the block holds
    const int R = min(kFeKS, (bh + G - 1) / G);  // rows per unit
    const int nsr = (bh + R - 1) / R;
    const int* lab = m0 + (long long)fov * n;
    // ---- coordinate counts (medians) and per-row column extents, in the T area as ints
    int* rowc = reinterpret_cast<int*>(T);
    int* colc = rowc + bh;
    int* rmn = colc + bw;
    int* rmx = rmn + bh;
    for (int i = tid; i < bh + bw; i += THREADS) rowc[i] = 0;
    for (int i = tid; i < bh; i += THREADS) {
      rmn[i] = INT_MAX;
      rmx[i] = -1;
    }
    __syncthreads();
    const int nb = bh * bw;
    for (int p = tid; p < nb; p += THREADS) {
      const int rr = p / bw, cc = p - rr * bw;
      if (lab[(long long)(r0 + rr) * Dx + c0 + cc] == L) {
        atomicAdd(&rowc[rr], 1);
        atomicAdd(&colc[cc], 1);
        atomicMin(&rmn[rr], cc);
        atomicMax(&rmx[rr], cc);
      }
    }
    __syncthreads();
    if (tid < 2) {
      const int* hc = tid == 0 ? rowc : colc;
      const int len = tid == 0 ? bh : bw;
      const long long cntn = o.area;
      const long long ka = (cntn - 1) / 2, kb = cntn / 2;
      long long cum = 0;
      int va = -1, vb = -1;
      for (int i = 0; i < len; ++i) {
        cum += hc[i];
        if (va < 0 && cum > ka) va = i;
        if (vb < 0 && cum > kb) { vb = i; break; }
      }
      smed[tid] = ((double)(va + 1) + (double)(vb + 1)) / 2.0;
    }
    if (tid == 64) {  // row spans (T coordinates: row rr + 1, column cc + 1)
      int tot = 0;
      rowt[0] = make_int2(0, 1);
      for (int y = 1; y <= bh; ++y) {
        const int rr = y - 1;
        if (rmx[rr] < 0) {
          rowt[y] = make_int2(0, 1);
        } else {
          const int pb = (rmn[rr] + 1) >> 1, pe = (rmx[rr] + 1) >> 1;
          rowt[y] = make_int2(tot - pb, pb | (pe << 16));
          tot += pe - pb + 1;
        }
      }
      rowt[bh + 1] = make_int2(0, 1);
      stot = tot;
    }
    __syncthreads();
    const int tot2 = stot;
    if (2 * tot2 > CELLS) continue;  // block-uniform: left for k_flow_error_big
    // ---- argmin of (x-xmed)^2 + (y-ymed)^2, first in row-major order on ties
    const double ymed = smed[0], xmed = smed[1];
    unsigned long long best = ~0ull;
    for (int p = tid; p < nb; p += THREADS) {
      const int rr = p / bw, cc = p - rr * bw;
      if (lab[(long long)(r0 + rr) * Dx + c0 + cc] != L) continue;
      const double dy = (double)(rr + 1) - ymed, dx = (double)(cc + 1) - xmed;
      const double dist = dx * dx + dy * dy;
      const unsigned long long key = ((unsigned long long)(dist * 4.0) << 32) | (unsigned int)p;
      best = key < best ? key : best;
    }
    best = wave_min(best);
    if (lane == 0) sbest[wid] = best;
    __syncthreads();
    unsigned long long bsel = sbest[0];
    for (int w = 1; w < THREADS / 64; ++w) bsel = sbest[w] < bsel ? sbest[w] : bsel;
    const int pbest = (int)(bsel & 0xffffffffu);
    const int ym = pbest / bw + 1, xm = pbest % bw + 1;
    const int niter = 2 * ((bw - 1) + (bh - 1));
    // ---- this thread's units (u = tid + i THREADS): columns X, X + 1 (X = 2m + 1), rows Y0 ..
    unsigned int um[U][2];
    int X[U], Y0[U];
    bool cown = false;
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int u = tid + i * THREADS;
      um[i][0] = um[i][1] = 0u;
      X[i] = 1;
      Y0[i] = 1;
      if (u < ncp * nsr) {
        X[i] = 2 * (u % ncp) + 1;
        Y0[i] = 1 + (u / ncp) * R;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (X[i] + h > bw) continue;
          unsigned int m = 0u;
          for (int j = 0; j < R && Y0[i] + j <= bh; ++j)
            if (lab[(long long)(r0 + Y0[i] - 1 + j) * Dx + c0 + X[i] + h - 1] == L) m |= 1u << j;
          um[i][h] = m;
          if (X[i] + h == xm && ym >= Y0[i] && ym < Y0[i] + R) cown = true;
        }
      }
    }
    int ud[U];  // Chebyshev distance of the unit from the centre (see k_flow_error_lds)
#pragma unroll
    for (int i = 0; i < U; ++i)
      ud[i] = max(max(max(0, Y0[i] - ym), ym - (Y0[i] + R - 1)), max(max(0, X[i] - xm), xm - (X[i] + 1)));
    __syncthreads();  // rowc / colc / extents read: T is cleared next
    for (int i = tid; i < 2 * tot2; i += THREADS) T[i] = 0.0;
    __syncthreads();
    const int cidx = 2 * (rowt[ym].x + (xm >> 1)) + (xm & 1);
    if (tid == 0 && niter > 0) T[cidx] = 1.0;  // the first iteration's T[centre] += 1
    __syncthreads();
    const double2* T2 = reinterpret_cast<const double2*>(T);
    auto ldrow = [&](int y, int pa, double2& a, double2& b) {
      // opaque row index: keeps the compiler from hoisting every row's span lookup out of the
      // iteration loop (14 rows x U units of registers)
      asm volatile("" : "+v"(y));
      const int2 rt = rowt[y];
      const int lo = rt.y & 0xffff, hi = rt.y >> 16;
      a = (pa >= lo && pa <= hi) ? T2[rt.x + pa] : z2;
      b = (pa + 1 >= lo && pa + 1 <= hi) ? T2[rt.x + pa + 1] : z2;
    };
    double nv[U][2][kFeKS];
    for (int it = 0; it < niter; ++it) {
#pragma unroll
      for (int i = 0; i < U; ++i) {
        if (!(um[i][0] | um[i][1]) || ud[i] > it + 1) continue;
        const int pa = (X[i] - 1) >> 1;  // column pairs (X - 1, X) and (X + 1, X + 2)
        double2 ua, ub, ca, cb, da, db;
        ldrow(Y0[i] - 1, pa, ua, ub);
        ldrow(Y0[i], pa, ca, cb);
        ldrow(min(Y0[i] + 1, bh + 1), pa, da, db);
#pragma unroll
        for (int j = 0; j < kFeKS; ++j) {
          if (j < R) {  // block-uniform predicate: the loop stays unrolled, nv in registers
            double2 na = z2, nb2 = z2;
            if (j + 1 < R) ldrow(min(Y0[i] + j + 2, bh + 1), pa, na, nb2);
            // column X: l = a.x, c = a.y, r = b.x;  column X + 1: l = a.y, c = b.x, r = b.y
            fe_pair<double, double2>(ua, ub, ca, cb, da, db, nv[i][0][j], nv[i][1][j]);
            ua = ca; ub = cb;
            ca = da; cb = db;
            da = na; db = nb2;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < U; ++i) {
        if (!(um[i][0] | um[i][1]) || ud[i] > it + 1) continue;
        const int pa = (X[i] - 1) >> 1;
        // opaque copies: the per-row write predicates are not hoisted out of the iteration loop
        unsigned int m0 = um[i][0], m1 = um[i][1];
        asm volatile("" : "+v"(m0), "+v"(m1));
#pragma unroll
        for (int j = 0; j < kFeKS; ++j) {
          if (!(((m0 | m1) >> j) & 1u)) continue;
          int y = Y0[i] + j;
          asm volatile("" : "+v"(y));
          const int base = rowt[y].x;
          if ((m0 >> j) & 1u) T[2 * (base + pa) + 1] = nv[i][0][j];
          if ((m1 >> j) & 1u) T[2 * (base + pa + 1)] = nv[i][1][j];
        }
      }
      if (cown && it + 1 < niter) T[cidx] = T[cidx] + 1.0;
      __syncthreads();
    }
    // ---- gradients, normalisation, error vs dP/5
    auto ld1 = [&](int y, int x) -> double {
      const int2 rt = rowt[y];
      const int p = x >> 1;
      return (p >= (rt.y & 0xffff) && p <= (rt.y >> 16)) ? T[2 * (rt.x + p) + (x & 1)] : 0.0;
    };
    const float2* F = dpf + (long long)fov * n;
    double e0 = 0.0, e1 = 0.0;
#pragma unroll
    for (int i = 0; i < U; ++i) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        for (int j = 0; j < kFeKS; ++j) {
          if (!((um[i][h] >> j) & 1u)) continue;
          const int Y = Y0[i] + j, Xc = X[i] + h;
          const double dy = ld1(Y + 1, Xc) - ld1(Y - 1, Xc);
          const double dx = ld1(Y, Xc + 1) - ld1(Y, Xc - 1);
          const double nrm = 1e-20 + sqrt(dy * dy + dx * dx);
          const double my = dy / nrm, mx = dx / nrm;
          const float2 f = F[(long long)(r0 + Y - 1) * Dx + c0 + Xc - 1];
          const double ty = my - (double)(f.x / 5.0f);
          const double tx = mx - (double)(f.y / 5.0f);
          e0 += ty * ty;
          e1 += tx * tx;
        }
      }
    }
    e0 = wave_sum(e0);
    e1 = wave_sum(e1);
    if (lane == 0) {
      sred[wid][0] = e0;
      sred[wid][1] = e1;
    }
    __syncthreads();
    if (tid == 0) {
      double s0 = 0.0, s1 = 0.0;
      for (int w = 0; w < THREADS / 64; ++w) {
        s0 += sred[w][0];
        s1 += sred[w][1];
      }
      const double err = 0.0 + s0 / (double)o.area + s1 / (double)o.area;
      bad[(long long)fov * (max_label + 1) + L] = err > thr ? 1 : 2;
    }
    __syncthreads();
  }
}

// masks beyond the LDS kernels: one 1024-thread block per mask (dynamic queue over the batch),
// a two-buffer Jacobi over the mask's pixel list in a block-private slice of global scratch
// (L2-resident for the masks that reach here); the centre's +1 is applied by the thread that
// writes the centre, so each iteration needs one barrier.  Masks that do not fit a slice (and
// are not flagged yet) are left to k_flow_error_fov.
constexpr int kBigThreads = 1024;

__global__ __launch_bounds__(kBigThreads) void k_flow_error_big(
    const int* __restrict__ m0, const float2* __restrict__ dpf, int Dy, int Dx, int B, int max_label,
    const cpx_object* __restrict__ objects, const int* __restrict__ off, int* __restrict__ ctr,
    int lo_threads, int lo_units, int lo_cells, double thr, double* __restrict__ gscratch,
    long long slice, unsigned char* __restrict__ bad) {
  __shared__ int rowc[2112];
  __shared__ int colc[2112];
  __shared__ double sred[kBigThreads / 64][2];
  __shared__ unsigned long long sbest[kBigThreads / 64];
  __shared__ double smed[2];
  __shared__ int sitem, snpix;
  const long long n = (long long)Dy * Dx;
  const int total = off[B];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double* T0 = gscratch + (long long)blockIdx.x * slice;
  for (int claims = 0;; ++claims) {
    if (claims > total) {  // broken claim (cpx_internal.h kClaimBroken)
      if (tid == 0) atomicOr(ctr, kClaimBroken);
      break;
    }
    if (tid == 0) sitem = atomicAdd(ctr, 1);
    __syncthreads();
    const int item = sitem;
    __syncthreads();
    if (item >= total) break;
    int fov = 0;
    while (fov + 1 < B && off[fov + 1] <= item) ++fov;
    const int kobj = item - off[fov];
    const cpx_object o = objects[(long long)fov * max_label + kobj];
    const int L = o.label;
    const int r0 = o.bbox[0], c0 = o.bbox[1];
    const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
    if (fe_fits(bh, bw, lo_threads, lo_units, lo_cells)) continue;       // the small kernels'
    if (bad[(long long)fov * (max_label + 1) + L] != 0) continue;        // k_flow_error_cmp's
    const int ly = bh + 2, lx = bw + 2;
    const long long ncell = (long long)ly * lx;
    const int nb = bh * bw;
    if (bh > 2112 || bw > 2112 || 2 * ncell + (nb + 1) / 2 + 2 > slice) continue;  // k_flow_error_fov
    double* Tc = T0;
    double* Tn = T0 + ncell;
    int* plist = reinterpret_cast<int*>(T0 + 2 * ncell);
    for (long long i = tid; i < 2 * ncell; i += kBigThreads) T0[i] = 0.0;
    for (int i = tid; i < bh + bw; i += kBigThreads) (i < bh ? rowc[i] : colc[i - bh]) = 0;
    if (tid == 0) snpix = 0;
    __syncthreads();
    const int* lab = m0 + (long long)fov * n;
    for (int p = tid; p < nb; p += kBigThreads) {
      const int rr = p / bw, cc = p - rr * bw;
      const bool in = lab[(long long)(r0 + rr) * Dx + c0 + cc] == L;
      if (in) {
        atomicAdd(&rowc[rr], 1);
        atomicAdd(&colc[cc], 1);
      }
      const unsigned long long bal = __ballot(in);
      int base = 0;
      if (lane == 0 && bal) base = atomicAdd(&snpix, __popcll(bal));
      base = __shfl(base, 0);
      if (in) plist[base + __popcll(bal & ((1ull << lane) - 1ull))] = (rr + 1) * lx + cc + 1;
    }
    __syncthreads();
    const int npix = snpix;
    if (tid < 2) {
      const int* hc = tid == 0 ? rowc : colc;
      const int len = tid == 0 ? bh : bw;
      const long long cntn = o.area;
      const long long ka = (cntn - 1) / 2, kb = cntn / 2;
      long long cum = 0;
      int va = -1, vb = -1;
      for (int i = 0; i < len; ++i) {
        cum += hc[i];
        if (va < 0 && cum > ka) va = i;
        if (vb < 0 && cum > kb) { vb = i; break; }
      }
      smed[tid] = ((double)(va + 1) + (double)(vb + 1)) / 2.0;
    }
    __syncthreads();
    const double ymed = smed[0], xmed = smed[1];
    unsigned long long best = ~0ull;
    for (int p = tid; p < nb; p += kBigThreads) {
      const int rr = p / bw, cc = p - rr * bw;
      if (lab[(long long)(r0 + rr) * Dx + c0 + cc] != L) continue;
      const double dy = (double)(rr + 1) - ymed, dx = (double)(cc + 1) - xmed;
      const double dist = dx * dx + dy * dy;
      const unsigned long long key = ((unsigned long long)(dist * 4.0) << 32) | (unsigned int)p;
      best = key < best ? key : best;
    }
    best = wave_min(best);
    if (lane == 0) sbest[wid] = best;
    __syncthreads();
    unsigned long long bsel = sbest[0];
    for (int w = 1; w < kBigThreads / 64; ++w) bsel = sbest[w] < bsel ? sbest[w] : bsel;
    const int pbest = (int)(bsel & 0xffffffffu);
    const int cidx = (pbest / bw + 1) * lx + pbest % bw + 1;
    const int niter = 2 * ((bw - 1) + (bh - 1));
    if (tid == 0 && niter > 0) Tc[cidx] = 1.0;
    __syncthreads();
    for (int it = 0; it < niter; ++it) {
      const bool inc = it + 1 < niter;
      for (int i = tid; i < npix; i += kBigThreads) {
        const int q = plist[i];
        double v = 1 / 9. * (Tc[q] + Tc[q - lx] + Tc[q + lx] + Tc[q - 1] + Tc[q + 1] + Tc[q - lx - 1] +
                             Tc[q - lx + 1] + Tc[q + lx - 1] + Tc[q + lx + 1]);
        if (q == cidx && inc) v = v + 1.0;  // the next iteration's T[centre] += 1
        Tn[q] = v;
      }
      __syncthreads();
      double* t = Tc;
      Tc = Tn;
      Tn = t;
    }
    const float2* F = dpf + (long long)fov * n;
    double e0 = 0.0, e1 = 0.0;
    for (int i = tid; i < npix; i += kBigThreads) {
      const int q = plist[i];
      const int y = q / lx, x = q - (q / lx) * lx;
      const double dy = Tc[q + lx] - Tc[q - lx];
      const double dx = Tc[q + 1] - Tc[q - 1];
      const double nrm = 1e-20 + sqrt(dy * dy + dx * dx);
      const double my = dy / nrm, mx = dx / nrm;
      const float2 f = F[(long long)(r0 + y - 1) * Dx + c0 + x - 1];
      const double ty = my - (double)(f.x / 5.0f);
      const double tx = mx - (double)(f.y / 5.0f);
      e0 += ty * ty;
      e1 += tx * tx;
    }
    e0 = wave_sum(e0);
    e1 = wave_sum(e1);
    if (lane == 0) {
      sred[wid][0] = e0;
      sred[wid][1] = e1;
    }
    __syncthreads();
    if (tid == 0) {
      double s0 = 0.0, s1 = 0.0;
      for (int w = 0; w < kBigThreads / 64; ++w) {
        s0 += sred[w][0];
        s1 += sred[w][1];
      }
      const double err = 0.0 + s0 / (double)o.area + s1 / (double)o.area;
      bad[(long long)fov * (max_label + 1) + L] = err > thr ? 1 : 2;
    }
    __syncthreads();
  }
}

// last resort for masks no block slice holds: one block per FOV walks them with a two-buffer
// Jacobi in the FOV's whole scratch (no two blocks share a scratch area)
constexpr int kFlowThreads = 256;

__global__ __launch_bounds__(kFlowThreads) void k_flow_error_fov(
    const int* __restrict__ m0, const float2* __restrict__ dpf, int Dy, int Dx, int max_label,
    const cpx_object* __restrict__ objects, const cpx_fov_objects* __restrict__ hdr, int lds_threads,
    int lds_units, int lds_cells, double thr, double* __restrict__ gscratch,
    long long gscratch_per_fov, unsigned char* __restrict__ bad) {
  __shared__ int rowc[2048];
  __shared__ int colc[2048];
  __shared__ double sred[kFlowThreads / 64][2];
  __shared__ unsigned long long sbest[kFlowThreads / 64];
  __shared__ double smed[2];
  const int fov = blockIdx.x;
  const long long n = (long long)Dy * Dx;
  const int* lab = m0 + (long long)fov * n;
  const int nobj = hdr[fov].n_objects;
  for (int k = 0; k < nobj; ++k) {
  const cpx_object o = objects[(long long)fov * max_label + k];
  const int L = o.label;
  const int r0 = o.bbox[0], c0 = o.bbox[1];
  const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
  if (fe_fits(bh, bw, lds_threads, lds_units, lds_cells)) continue;  // block-uniform: an LDS kernel's
  if (bad[(long long)fov * (max_label + 1) + L] != 0) continue;      // or an earlier kernel's
  const int ly = bh + 2, lx = bw + 2;
  const int ncell = ly * lx;
  double* T0 = gscratch + (long long)fov * gscratch_per_fov;
  double* T1 = T0 + ncell;
  for (int i = threadIdx.x; i < ncell; i += kFlowThreads) {
    T0[i] = 0.0;
    T1[i] = 0.0;
  }
  for (int i = threadIdx.x; i < 2048; i += kFlowThreads) {
    rowc[i] = 0;
    colc[i] = 0;
  }
  __syncthreads();
  const int nb = bh * bw;
  for (int p = threadIdx.x; p < nb; p += kFlowThreads) {
    const int rr = p / bw, cc = p - rr * bw;
    if (lab[(long long)(r0 + rr) * Dx + c0 + cc] == L) {
      atomicAdd(&rowc[min(rr, 2047)], 1);
      atomicAdd(&colc[min(cc, 2047)], 1);
    }
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const int* hc = threadIdx.x == 0 ? rowc : colc;
    const int len = min(threadIdx.x == 0 ? bh : bw, 2048);
    const long long cntn = o.area;
    const long long ka = (cntn - 1) / 2, kb = cntn / 2;
    long long cum = 0;
    int va = -1, vb = -1;
    for (int i = 0; i < len; ++i) {
      cum += hc[i];
      if (va < 0 && cum > ka) va = i;
      if (vb < 0 && cum > kb) { vb = i; break; }
    }
    smed[threadIdx.x] = ((double)(va + 1) + (double)(vb + 1)) / 2.0;
  }
  __syncthreads();
  const double ymed = smed[0], xmed = smed[1];
  unsigned long long best = ~0ull;
  for (int p = threadIdx.x; p < nb; p += kFlowThreads) {
    const int rr = p / bw, cc = p - rr * bw;
    if (lab[(long long)(r0 + rr) * Dx + c0 + cc] != L) continue;
    const double dy = (double)(rr + 1) - ymed, dx = (double)(cc + 1) - xmed;
    const double dist = dx * dx + dy * dy;
    const unsigned long long key = ((unsigned long long)(dist * 4.0) << 32) | (unsigned int)p;
    best = key < best ? key : best;
  }
  best = wave_min(best);
  if ((threadIdx.x & 63) == 0) sbest[threadIdx.x >> 6] = best;
  __syncthreads();
  unsigned long long bsel = sbest[0];
  for (int w = 1; w < kFlowThreads / 64; ++w) bsel = sbest[w] < bsel ? sbest[w] : bsel;
  const int pbest = (int)(bsel & 0xffffffffu);
  const int ym = pbest / bw + 1, xm = pbest % bw + 1;
  const int niter = 2 * ((bw - 1) + (bh - 1));
  double* Tc = T0;
  double* Tn = T1;
  for (int it = 0; it < niter; ++it) {
    if (threadIdx.x == 0) Tc[ym * lx + xm] += 1.0;
    __syncthreads();
    for (int p = threadIdx.x; p < nb; p += kFlowThreads) {
      const int rr = p / bw, cc = p - rr * bw;
      if (lab[(long long)(r0 + rr) * Dx + c0 + cc] != L) continue;
      const int y = rr + 1, x = cc + 1;
      Tn[y * lx + x] = 1 / 9. * (Tc[y * lx + x] + Tc[(y - 1) * lx + x] + Tc[(y + 1) * lx + x] +
                                 Tc[y * lx + x - 1] + Tc[y * lx + x + 1] + Tc[(y - 1) * lx + x - 1] +
                                 Tc[(y - 1) * lx + x + 1] + Tc[(y + 1) * lx + x - 1] +
                                 Tc[(y + 1) * lx + x + 1]);
    }
    __syncthreads();
    double* t = Tc;
    Tc = Tn;
    Tn = t;
  }
  const float2* F = dpf + (long long)fov * n;
  double e0 = 0.0, e1 = 0.0;
  for (int p = threadIdx.x; p < nb; p += kFlowThreads) {
    const int rr = p / bw, cc = p - rr * bw;
    const int gy = r0 + rr, gx = c0 + cc;
    if (lab[(long long)gy * Dx + gx] != L) continue;
    const int y = rr + 1, x = cc + 1;
    const double dy = Tc[(y + 1) * lx + x] - Tc[(y - 1) * lx + x];
    const double dx = Tc[y * lx + x + 1] - Tc[y * lx + x - 1];
    const double nrm = 1e-20 + sqrt(dy * dy + dx * dx);
    const double my = dy / nrm, mx = dx / nrm;
    const float2 f = F[(long long)gy * Dx + gx];
    const double ty = my - (double)(f.x / 5.0f);
    const double tx = mx - (double)(f.y / 5.0f);
    e0 += ty * ty;
    e1 += tx * tx;
  }
  e0 = wave_sum(e0);
  e1 = wave_sum(e1);
  if ((threadIdx.x & 63) == 0) {
    sred[threadIdx.x >> 6][0] = e0;
    sred[threadIdx.x >> 6][1] = e1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s0 = 0.0, s1 = 0.0;
    for (int w = 0; w < kFlowThreads / 64; ++w) {
      s0 += sred[w][0];
      s1 += sred[w][1];
    }
    const double err = 0.0 + s0 / (double)o.area + s1 / (double)o.area;
    bad[(long long)fov * (max_label + 1) + L] = err > thr ? 1 : 2;
  }
  __syncthreads();
  }  // object loop
}

__global__ __launch_bounds__(kT) void k_apply_bad(long long n, int max_label,
                                                  const unsigned char* __restrict__ bad,
                                                  int* __restrict__ m0) {
  const int fov = blockIdx.y;
  const long long q0 = ((long long)blockIdx.x * kT + threadIdx.x) * kPx4;
  if (q0 >= n) return;
  int* m = m0 + (long long)fov * n;
  const unsigned char* bd = bad + (long long)fov * (max_label + 1);
  auto keep = [&](int l) { return (l > 0 && l <= max_label && bd[l] == 1) ? 0 : l; };
  if ((n & 3) == 0 && (((uintptr_t)m0) & 15u) == 0) {
    const int4 t = *reinterpret_cast<const int4*>(m + q0);
    const int4 o = make_int4(keep(t.x), keep(t.y), keep(t.z), keep(t.w));
    if (o.x != t.x || o.y != t.y || o.z != t.z || o.w != t.w) *reinterpret_cast<int4*>(m + q0) = o;
  } else {
#pragma unroll
    for (int u = 0; u < kPx4; ++u)
      if (q0 + u < n) {
        const int l = m[q0 + u], k = keep(l);
        if (k != l) m[q0 + u] = k;
      }
  }
}

__global__ void k_count_bad(int max_label, const unsigned char* __restrict__ bad,
                            const int* __restrict__ ctrs, int nctr, cpx_seg_stats* __restrict__ st) {
  const int fov = blockIdx.x;
  if (threadIdx.x < nctr && (ctrs[threadIdx.x] & kClaimBroken))
    atomicOr(&st[fov].overflow, CPX_SEG_ERR_INTERNAL);
  int c = 0;
  for (int l = threadIdx.x; l <= max_label; l += blockDim.x) c += bad[(long long)fov * (max_label + 1) + l] == 1;
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(&st[fov].n_bad_flow, c);
}

// nearest-neighbour resize to full resolution
constexpr int kUpRows = 8;
__global__ __launch_bounds__(kT) void k_upsample(const int* __restrict__ m0, int Ly, int Lx, int H,
                                                 int W, const int* __restrict__ ysrc,
                                                 const int* __restrict__ xsrc,
                                                 int* __restrict__ out) {
  const int fov = blockIdx.z;
  const int x = blockIdx.x * kT + threadIdx.x;
  if (x >= W) return;
  const int xs = xsrc[x];
  const int y0 = blockIdx.y * kUpRows, y1 = min(H, y0 + kUpRows);  // rows per block
  for (int y = y0; y < y1; ++y)
    out[((long long)fov * H + y) * W + x] = m0[((long long)fov * Ly + ysrc[y]) * Lx + xs];
}

// ---------------------------------------------------------------------------------------------
// fill_holes_and_remove_small_masks (parallel form; see DESIGN.md for the nesting rule)
constexpr int kFillThreads = 512;
constexpr int kFillMaxWords = 8192;  // 2 x 32 KiB bitmasks -> bbox up to 262144 px

__global__ __launch_bounds__(kT) void k_lab2idx(int max_label, const cpx_object* __restrict__ objects,
                                                const cpx_fov_objects* __restrict__ hdr,
                                                int* __restrict__ lab2idx) {
  const int fov = blockIdx.y;
  const int k = blockIdx.x * kT + threadIdx.x;
  if (k >= hdr[fov].n_objects) return;
  lab2idx[(long long)fov * (max_label + 1) + objects[(long long)fov * max_label + k].label] = k;
}

// Closure of the reached set x within one 32-pixel word over the free pixels f (x a subset of f):
// an addition carries each reached bit up to the top of its run of free bits, the bit-reversed
// addition down to its bottom, so a flood crosses any horizontal run in one step (only the turns
// and the vertical moves cost iterations; the fixed point is the same as one pixel per step).
__device__ __forceinline__ unsigned int fill_hrun(unsigned int x, unsigned int f) {
  const unsigned int up = (((f + x) ^ f) | x) & f;
  const unsigned int rf = __builtin_bitreverse32(f), rx = __builtin_bitreverse32(x);
  const unsigned int dn = __builtin_bitreverse32((((rf + rx) ^ rf) | rx) & rf);
  return up | dn;
}

// One mask k of a FOV: own / reach are its bbox bitmasks (nw words, LDS or global scratch);
// the non-object pixels reached from the bbox border (4-connectivity) are flooded, the rest are
// holes: they record the filling mask and the masks they absorb.  Block-uniform.
// G: the bitmasks are in global scratch — words are loaded and stored at agent scope (L2) and
// a device fence precedes each barrier, so no wave reads a neighbour word from a stale L1 line
template <bool G>
__device__ __forceinline__ unsigned int fill_ld(const unsigned int* p) {
  if constexpr (G) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool G>
__device__ __forceinline__ void fill_st(unsigned int* p, unsigned int v) {
  if constexpr (G) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// The bbox bitmasks of label `lab_k` (own) and the seeds of the border flood (reach: border pixels
// outside the mask); returns this thread's count of mask pixels.  L: label loads at agent scope
// (k_fill_seq re-reads pixels its own block rewrote, which a plain load could take from a stale L1 line).
template <bool G, bool L>
__device__ __forceinline__ int fill_bits(const int* __restrict__ lab, int W, int lab_k, int r0, int c0,
                                         int bh, int bw, unsigned int* own, unsigned int* reach) {
  const int wpr = (bw + 31) / 32;
  const int nw = wpr * bh;
  int cnt = 0;
  for (int w = threadIdx.x; w < nw; w += blockDim.x) {
    const int r = w / wpr, cw = w - r * wpr;
    unsigned int bits = 0, rb = 0;
    for (int b = 0; b < 32; ++b) {
      const int c = cw * 32 + b;
      if (c >= bw) break;
      const int* p = lab + (long long)(r0 + r) * W + c0 + c;
      const int v = L ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
      const bool in = v == lab_k;
      bits |= (unsigned int)in << b;
      const bool border = (r == 0 || r == bh - 1 || c == 0 || c == bw - 1);
      rb |= (unsigned int)(border && !in) << b;
    }
    fill_st<G>(own + w, bits);
    fill_st<G>(reach + w, rb);
    cnt += __popc(bits);
  }
  return cnt;
}

// Flood the bbox's non-mask pixels from the border seeds in `reach` (4-connectivity, the
// background structure of ndi.binary_fill_holes); afterwards the holes are ~own & ~reach.
// Block-uniform; starts and ends with a barrier.
template <bool G>
__device__ __forceinline__ void fill_flood(const unsigned int* own, unsigned int* reach, int bh, int bw) {
  const int wpr = (bw + 31) / 32;
  const int nw = wpr * bh;
  if (G) __threadfence();
  __syncthreads();
  // flood in place until stable (a stale neighbour read only delays a change to a later
  // iteration: every change forces another one, so the loop ends at the unique fixed point)
  for (int iter = 0; iter < bh * bw + 1; ++iter) {
    int ch = 0;
    for (int w = threadIdx.x; w < nw; w += blockDim.x) {
      const int r = w / wpr, cw = w - r * wpr;
      const unsigned int valid = (cw == wpr - 1 && (bw & 31)) ? ((1u << (bw & 31)) - 1u) : 0xffffffffu;
      const unsigned int freeb = ~fill_ld<G>(own + w) & valid;
      const unsigned int cur = fill_ld<G>(reach + w);
      unsigned int nb = (cur << 1) | (cur >> 1);
      if (cw > 0) nb |= fill_ld<G>(reach + w - 1) >> 31;
      if (cw < wpr - 1) nb |= fill_ld<G>(reach + w + 1) << 31;
      if (r > 0) nb |= fill_ld<G>(reach + w - wpr);
      if (r < bh - 1) nb |= fill_ld<G>(reach + w + wpr);
      const unsigned int nxt = fill_hrun(cur | (nb & freeb), freeb);
      if (nxt != cur) {
        fill_st<G>(reach + w, nxt);
        ch = 1;
      }
    }
    if (G) __threadfence();
    // one barrier that also returns the block-wide decision: a flag reset by thread 0 at the
    // top of the next iteration could be read as 0 by a wave still leaving this one (which then
    // broke out early: an incomplete flood, barriers out of step)
    if (!__syncthreads_or(ch)) break;
  }
}

template <bool G>
__device__ __forceinline__ void fill_one(const int* __restrict__ lab, int W, int max_label, int k,
                                         const cpx_object& o, unsigned int* own, unsigned int* reach,
                                         const int* __restrict__ l2i, int* __restrict__ fillidx,
                                         int* __restrict__ absorber) {
  const int r0 = o.bbox[0], c0 = o.bbox[1];
  const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
  const int wpr = (bw + 31) / 32;
  const int nw = wpr * bh;
  fill_bits<G, false>(lab, W, o.label, r0, c0, bh, bw, own, reach);
  fill_flood<G>(own, reach, bh, bw);
  // holes: free and unreached; mark fill owner and absorbed objects
  for (int w = threadIdx.x; w < nw; w += blockDim.x) {
    const int r = w / wpr, cw = w - r * wpr;
    const unsigned int valid = (cw == wpr - 1 && (bw & 31)) ? ((1u << (bw & 31)) - 1u) : 0xffffffffu;
    unsigned int hole = ~fill_ld<G>(own + w) & ~fill_ld<G>(reach + w) & valid;
    while (hole) {
      const int b = __ffs(hole) - 1;
      hole &= hole - 1;
      const long long gi = (long long)(r0 + r) * W + c0 + cw * 32 + b;
      atomicMax(&fillidx[gi], k + 1);
      const int l2 = lab[gi];
      if (l2 > 0 && l2 <= max_label) atomicMin(&absorber[l2i[l2]], k);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ int fill_words(const cpx_object& o) {
  return ((o.bbox[3] - o.bbox[1] + 31) / 32) * (o.bbox[2] - o.bbox[0]);
}

// masks whose bbox bitmasks fit the LDS (bbox <= 262144 px): several blocks per FOV
__global__ __launch_bounds__(kFillThreads) void k_fill_holes(
    const int* __restrict__ labels, int H, int W, int max_label, int min_size,
    const cpx_object* __restrict__ objects, const cpx_fov_objects* __restrict__ hdr,
    const int* __restrict__ lab2idx, int* __restrict__ fillidx, int* __restrict__ absorber) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned int* own = reinterpret_cast<unsigned int*>(smem);
  const int fov = blockIdx.y;
  const int nobj = hdr[fov].n_objects;
  for (int k = blockIdx.x; k < nobj; k += gridDim.x) {
    const cpx_object o = objects[(long long)fov * max_label + k];
    if (o.area < min_size || fill_words(o) > kFillMaxWords) continue;
    fill_one<false>(labels + (long long)fov * H * W, W, max_label, k, o, own, own + kFillMaxWords,
             lab2idx + (long long)fov * (max_label + 1), fillidx + (long long)fov * H * W,
             absorber + (long long)fov * max_label);
  }
}

// the larger masks (the reference has no size limit): one block per FOV, bitmasks in a global
// scratch of 2 x ceil(W / 32) x H words per FOV (L2-resident: <= 1.1 MB at 2080^2)
__global__ __launch_bounds__(1024) void k_fill_holes_big(
    const int* __restrict__ labels, int H, int W, int max_label, int min_size,
    const cpx_object* __restrict__ objects, const cpx_fov_objects* __restrict__ hdr,
    const int* __restrict__ lab2idx, int* __restrict__ fillidx, int* __restrict__ absorber,
    unsigned int* __restrict__ scratch) {
  const int fov = blockIdx.x;
  const int nobj = hdr[fov].n_objects;
  const long long per = (long long)((W + 31) / 32) * H;
  unsigned int* own = scratch + (long long)fov * 2 * per;
  for (int k = 0; k < nobj; ++k) {
    const cpx_object o = objects[(long long)fov * max_label + k];
    if (o.area < min_size || fill_words(o) <= kFillMaxWords) continue;
    fill_one<true>(labels + (long long)fov * H * W, W, max_label, k, o, own, own + per,
             lab2idx + (long long)fov * (max_label + 1), fillidx + (long long)fov * H * W,
             absorber + (long long)fov * max_label);
  }
}

// One block per FOV: kept flags + sequential new labels, and the check that the parallel fill is
// exact for this FOV.  It is when every mask is, at its turn in the reference's loop, either
// untouched or wholly overwritten by the earlier masks' fills: then each kept mask fills the holes
// of its original shape, as k_fill_holes computed them.  A mask of >= min_size pixels some of whose
// pixels lie in an earlier mask's holes (absorber < k) is checked pixel by pixel: a pixel with
// no covering fill (fillidx 0), or whose last covering fill is a later mask's (fillidx > k + 1:
// an earlier cover is then undecided), makes the FOV take k_fill_seq instead
// (CPX_SEG_OVF_FILL_PARTIAL; n_fill_partial = such masks).  Smaller masks need no check: the
// reference clears their remainder and they never fill, as here.
__global__ __launch_bounds__(1024) void k_fill_final(int max_label, int min_size,
                                                     const cpx_object* __restrict__ objects,
                                                     const cpx_fov_objects* __restrict__ hdr,
                                                     const int* __restrict__ absorber,
                                                     const int* __restrict__ labels,
                                                     const int* __restrict__ fillidx, int W, long long N,
                                                     int* __restrict__ newlab,
                                                     cpx_seg_stats* __restrict__ st) {
  const int fov = blockIdx.x;
  const int n = hdr[fov].n_objects;
  __shared__ int wsum[16];
  __shared__ int base, npart;
  if (threadIdx.x == 0) base = npart = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int* lab = labels + (long long)fov * N;
  const int* fid = fillidx + (long long)fov * N;
  for (int k0 = 0; k0 < n; k0 += blockDim.x) {
    const int k = k0 + threadIdx.x;
    int kept = 0, check = 0;
    if (k < n) {
      const cpx_object o = objects[(long long)fov * max_label + k];
      const bool absorbed = absorber[(long long)fov * max_label + k] < k;
      kept = o.area >= min_size && !absorbed;
      check = o.area >= min_size && absorbed;
    }
    // each wave checks its own absorbed masks (rare) over their bboxes, lanes across the columns
    for (unsigned long long cb = __ballot(check); cb; cb &= cb - 1) {
      const int kk = k0 + wid * 64 + __ffsll((long long)cb) - 1;
      const cpx_object o = objects[(long long)fov * max_label + kk];
      const int bw = o.bbox[3] - o.bbox[1];
      int bad = 0;
      for (int r = o.bbox[0]; r < o.bbox[2] && !bad; ++r) {
        for (int c = lane; c < bw; c += 64) {
          const long long q = (long long)r * W + o.bbox[1] + c;
          const int f = fid[q];
          bad |= lab[q] == o.label && (f == 0 || f > kk + 1);
        }
        bad = __any(bad);
      }
      if (bad && lane == 0) atomicAdd(&npart, 1);
    }
    const unsigned long long b = __ballot(kept);
    const unsigned long long lower = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (lane == 0) wsum[wid] = __popcll(b);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    if (k < n) newlab[(long long)fov * max_label + k] = kept ? off + __popcll(b & lower) + 1 : 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int w = 0; w < nw; ++w) tot += wsum[w];
      base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    st[fov].n_final = base;
    if (npart) {
      st[fov].n_fill_partial = npart;
      st[fov].overflow |= CPX_SEG_OVF_FILL_PARTIAL;
    }
  }
}

// Final labels: a pixel takes the new label of the last kept mask whose holes cover it (masks
// fill in label order, the later fill wins), else its own mask's if kept.  A filler that is not
// kept was itself inside an earlier mask's holes (absorbed), and so is everything its holes
// cover: the chain filler -> absorber[filler] leads to the mask whose fill the reference leaves
// there (tests/test_gpu_capacity.py: holes inside a mask inside a ring).  FOVs that k_fill_final
// flagged (a mask partly inside an earlier mask's holes) are left to k_fill_seq.
__global__ __launch_bounds__(kT) void k_fill_apply(int* __restrict__ labels, long long n, int max_label,
                                                   const int* __restrict__ lab2idx,
                                                   const int* __restrict__ fillidx,
                                                   const int* __restrict__ newlab,
                                                   const int* __restrict__ absorber,
                                                   const cpx_seg_stats* __restrict__ st) {
  const int fov = blockIdx.y;
  if (st[fov].overflow & CPX_SEG_OVF_FILL_PARTIAL) return;
  const int* l2i = lab2idx + (long long)fov * (max_label + 1);
  const int* nl = newlab + (long long)fov * max_label;
  const int* ab = absorber + (long long)fov * max_label;
  // four independent pixels per iteration: their dependent lookups (label -> index -> new
  // label) overlap instead of one chain of loads at a time
  const long long stride = (long long)gridDim.x * kT;
  for (long long q0 = (long long)blockIdx.x * kT + threadIdx.x; q0 < n; q0 += 4 * stride) {
    int l[4], f[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long q = q0 + u * stride;
      l[u] = q < n ? labels[(long long)fov * n + q] : 0;
      f[u] = q < n ? fillidx[(long long)fov * n + q] : 0;
    }
    int k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) k[u] = (l[u] > 0 && l[u] <= max_label) ? l2i[l[u]] : -1;
    int cand[4], fk[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      cand[u] = (k[u] >= 0 && nl[k[u]]) ? k[u] + 1 : 0;
      int c = f[u];
      while (c && !nl[c - 1]) {  // not kept: absorbed by an earlier mask (a shorter k each step)
        const int a = ab[c - 1];
        c = a < c - 1 ? a + 1 : 0;
      }
      fk[u] = c;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long q = q0 + u * stride;
      if (q >= n) continue;
      const int best = max(cand[u], fk[u]);
      labels[(long long)fov * n + q] = best ? nl[best - 1] : 0;
    }
  }
}

// The reference's own loop for the FOVs k_fill_final flagged: utils.fill_holes_and_remove_small_masks
// restated literally (oracle/seg_oracle.py:376-391, Cellpose_GPU_s3fs.py:143) — the masks in label
// order over the find_objects boxes of the pre-fill labels, each taking the pixels that still
// carry its label: fewer than min_size are cleared, otherwise its holes are filled and the mask
// relabelled j + 1 (j + 1 <= its own label, so no later mask's pixels are confused with it).  One
// block per FOV, in place; the labels are re-read at agent scope after the block's own stores.
// Bitmasks in LDS, or in the per-FOV global scratch for bboxes beyond kFillMaxWords.
__global__ __launch_bounds__(1024) void k_fill_seq(int* __restrict__ labels, int H, int W, int max_label,
                                                   int min_size, const cpx_object* __restrict__ objects,
                                                   const cpx_fov_objects* __restrict__ hdr,
                                                   unsigned int* __restrict__ scratch,
                                                   cpx_seg_stats* __restrict__ st) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int wcnt[16];
  const int fov = blockIdx.x;
  if (!(st[fov].overflow & CPX_SEG_OVF_FILL_PARTIAL)) return;
  int* lab = labels + (long long)fov * H * W;
  const long long per = (long long)((W + 31) / 32) * H;
  const int nobj = hdr[fov].n_objects;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  int j = 0;
  for (int k = 0; k < nobj; ++k) {
    const cpx_object o = objects[(long long)fov * max_label + k];
    const int r0 = o.bbox[0], c0 = o.bbox[1];
    const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
    const int wpr = (bw + 31) / 32, nw = wpr * bh;
    const bool g = nw > kFillMaxWords;
    unsigned int* own = g ? scratch + (long long)fov * 2 * per : reinterpret_cast<unsigned int*>(smem);
    unsigned int* reach = g ? own + per : own + kFillMaxWords;
    int cnt = g ? fill_bits<true, true>(lab, W, o.label, r0, c0, bh, bw, own, reach)
                : fill_bits<false, true>(lab, W, o.label, r0, c0, bh, bw, own, reach);
    cnt = wave_sum(cnt);
    if (lane == 0) wcnt[wid] = cnt;
    __syncthreads();
    int npix = 0;
    for (int w = 0; w < nwv; ++w) npix += wcnt[w];
    __syncthreads();  // (wcnt is rewritten for the next mask)
    if (npix == 0) continue;
    const bool clear = min_size > 0 && npix < min_size;
    if (!clear) {
      if (g) fill_flood<true>(own, reach, bh, bw);
      else fill_flood<false>(own, reach, bh, bw);
    } else if (g) {
      __threadfence();
    }
    __syncthreads();
    const int v = clear ? 0 : j + 1;
    for (int w = threadIdx.x; w < nw; w += blockDim.x) {
      const int r = w / wpr, cw = w - r * wpr;
      const unsigned int valid = (cw == wpr - 1 && (bw & 31)) ? ((1u << (bw & 31)) - 1u) : 0xffffffffu;
      const unsigned int ow = g ? fill_ld<true>(own + w) : own[w];
      const unsigned int rw = clear ? 0xffffffffu : (g ? fill_ld<true>(reach + w) : reach[w]);
      unsigned int set = (ow | (~ow & ~rw)) & valid;
      while (set) {
        const int b = __ffs(set) - 1;
        set &= set - 1;
        lab[(long long)(r0 + r) * W + c0 + cw * 32 + b] = v;
      }
    }
    j += !clear;
    __threadfence();
    __syncthreads();
  }
  if (threadIdx.x == 0) st[fov].n_final = j;
}

void axis_coeffs(int n_src, int n_dst, int* i0, int* i1, float* w) {
  // cv2.resize INTER_LINEAR: scale = 1 / (dst / src), fx = (float)((d + 0.5) * scale - 0.5)
  const double scale = 1.0 / ((double)n_dst / (double)n_src);
  for (int d = 0; d < n_dst; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f = f - (float)s;
    if (s < 0) {
      s = 0;
      f = 0.0f;
    }
    if (s >= n_src - 1) {
      s = n_src - 1;
      f = 0.0f;
    }
    i0[d] = s;
    i1[d] = std::min(s + 1, n_src - 1);
    w[d] = f;
  }
}

// host-side coefficient tables: bilinear H,W -> Ly,Lx (network input), bilinear Ly,Lx -> H,W
// (resample=True flows) and nearest Ly,Lx -> H,W (resample=False masks)
struct SegTabs {
  AxisTab ty, tx;
  AxisTab uy, ux;
  const int* ynear;
  const int* xnear;
};

int seg_tables(cpx_ctx* ctx, int H, int W, int Ly, int Lx, SegTabs& t) {
  const size_t words = (size_t)3 * Ly + 3 * Lx + H + W + 3 * (size_t)H + 3 * (size_t)W;
  void* buf = cpx_ws(ctx, WS_SEG_TAB, words * 4 + 256);
  if (!buf) return CPX_ERR_OOM;
  int* base = (int*)buf;
  t.ty.i0 = base;
  t.ty.i1 = base + Ly;
  t.ty.w = (const float*)(base + 2 * Ly);
  t.tx.i0 = base + 3 * Ly;
  t.tx.i1 = base + 3 * Ly + Lx;
  t.tx.w = (const float*)(base + 3 * Ly + 2 * Lx);
  t.ynear = base + 3 * Ly + 3 * Lx;
  t.xnear = base + 3 * Ly + 3 * Lx + H;
  int* up = base + 3 * Ly + 3 * Lx + H + W;
  t.uy.i0 = up;
  t.uy.i1 = up + H;
  t.uy.w = (const float*)(up + 2 * H);
  t.ux.i0 = up + 3 * H;
  t.ux.i1 = up + 3 * H + W;
  t.ux.w = (const float*)(up + 3 * H + 2 * W);
  const int key[6] = {H, W, Ly, Lx, 2, 0};
  bool same = ctx->seg_gen == ctx->ws_gen[WS_SEG_TAB];
  for (int i = 0; i < 6; ++i) same = same && ctx->seg_key[i] == key[i];
  if (same) return CPX_OK;
  std::vector<int> h(words);
  axis_coeffs(H, Ly, &h[0], &h[Ly], (float*)&h[2 * Ly]);
  axis_coeffs(W, Lx, &h[3 * Ly], &h[3 * Ly + Lx], (float*)&h[3 * Ly + 2 * Lx]);
  const double ify = 1.0 / ((double)H / (double)Ly), ifx = 1.0 / ((double)W / (double)Lx);
  for (int y = 0; y < H; ++y) h[3 * Ly + 3 * Lx + y] = std::min((int)floor(y * ify), Ly - 1);
  for (int x = 0; x < W; ++x) h[3 * Ly + 3 * Lx + H + x] = std::min((int)floor(x * ifx), Lx - 1);
  const size_t u = (size_t)3 * Ly + 3 * Lx + H + W;
  axis_coeffs(Ly, H, &h[u], &h[u + H], (float*)&h[u + 2 * H]);
  axis_coeffs(Lx, W, &h[u + 3 * H], &h[u + 3 * H + W], (float*)&h[u + 3 * H + 2 * W]);
  CPX_CHECK_HIP(hipMemcpyAsync(buf, h.data(), words * 4, hipMemcpyHostToDevice, ctx->stream));
  CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  for (int i = 0; i < 6; ++i) ctx->seg_key[i] = key[i];
  ctx->seg_gen = ctx->ws_gen[WS_SEG_TAB];
  return CPX_OK;
}

bool geom_ok(const cpx_seg_geom* g) {
  if (!g || g->Ly <= 0 || g->Lx <= 0 || g->by <= 0 || g->bx <= 0) return false;
  if (g->ny < 1 || g->nx < 1 || g->ny > CPX_SEG_MAX_TILES_AXIS || g->nx > CPX_SEG_MAX_TILES_AXIS) return false;
  for (int i = 0; i < g->ny; ++i)
    if (g->ys[i] < 0 || g->ys[i] + g->by > g->Lyp) return false;
  for (int i = 0; i < g->nx; ++i)
    if (g->xs[i] < 0 || g->xs[i] + g->bx > g->Lxp) return false;
  return g->py0 >= 0 && g->px0 >= 0 && g->py0 + g->Ly <= g->Lyp && g->px0 + g->Lx <= g->Lxp;
}

}  // namespace

extern "C" int cpx_seg_percentiles(cpx_ctx* ctx, const float* corr_dev, int B, int C, int H, int W,
                                   int nchan, double* pct_dev) {
  CPX_REQUIRE(ctx && corr_dev && pct_dev, CPX_ERR_ARG, "cpx_seg_percentiles: null argument");
  CPX_REQUIRE(B > 0 && C > 0 && nchan > 0 && nchan <= C && H > 0 && W > 0 && B * nchan <= 65535,
              CPX_ERR_ARG, "cpx_seg_percentiles: bad sizes");
  const int P = B * nchan;
  const size_t hist_bytes = (size_t)P * 4 * 2048 * 4;
  unsigned char* ws = (unsigned char*)cpx_ws(ctx, WS_SEG_PCT, hist_bytes + sizeof(PctState) * P + 256);
  if (!ws) return CPX_ERR_OOM;
  unsigned int* hist = (unsigned int*)ws;
  PctState* st = (PctState*)(ws + hist_bytes);
  const long long N = (long long)H * W;
  for (int pass = 0; pass < 3; ++pass) {
    CPX_CHECK_HIP(hipMemsetAsync(hist, 0, hist_bytes, ctx->stream));
    hipLaunchKernelGGL(k_pct_hist, dim3(48, P), dim3(kT), 0, ctx->stream, corr_dev, C, N, nchan,
                       pass, (const PctState*)st, hist);
    CPX_CHECK_LAUNCH("k_pct_hist");
    hipLaunchKernelGGL(k_pct_find, dim3(P), dim3(256), 0, ctx->stream, N, pass, st,
                       (const unsigned int*)hist, pct_dev);
    CPX_CHECK_LAUNCH("k_pct_find");
  }
  return CPX_OK;
}

extern "C" int cpx_seg_tiles(cpx_ctx* ctx, const float* corr_dev, int B, int C, int H, int W,
                             int nchan, const double* pct_dev, const cpx_seg_geom* geom, int layout,
                             void* tiles_dev) {
  CPX_REQUIRE(ctx && corr_dev && pct_dev && tiles_dev, CPX_ERR_ARG, "cpx_seg_tiles: null argument");
  CPX_REQUIRE(geom_ok(geom), CPX_ERR_ARG, "cpx_seg_tiles: bad geometry");
  CPX_REQUIRE(B > 0 && B <= 65535 && nchan > 0 && nchan <= C && H > 0 && W > 0, CPX_ERR_ARG,
              "cpx_seg_tiles: bad sizes");
  CPX_REQUIRE(layout == CPX_TILE_F32_NCHW || layout == CPX_TILE_BF16_NHWC || layout == CPX_TILE_F32_NHWC,
              CPX_ERR_ARG, "cpx_seg_tiles: bad layout %d", layout);
  SegTabs t;
  int rc = seg_tables(ctx, H, W, geom->Ly, geom->Lx, t);
  if (rc) return rc;
  const int npx = geom->by * geom->bx;
  hipLaunchKernelGGL(k_seg_tiles, dim3(cpx_div_up(npx, kT), geom->ny * geom->nx, B), dim3(kT), 0,
                     ctx->stream, corr_dev, C, H, W, nchan, pct_dev, *geom, t.ty, t.tx, layout,
                     tiles_dev);
  CPX_CHECK_LAUNCH("k_seg_tiles");
  return CPX_OK;
}

extern "C" int cpx_seg_average(cpx_ctx* ctx, const void* net_dev, int layout, int B, int nout,
                               const cpx_seg_geom* geom, const float* taper_dev, float* yf_dev) {
  CPX_REQUIRE(ctx && net_dev && taper_dev && yf_dev, CPX_ERR_ARG, "cpx_seg_average: null argument");
  CPX_REQUIRE(geom_ok(geom), CPX_ERR_ARG, "cpx_seg_average: bad geometry");
  CPX_REQUIRE(B > 0 && B <= 65535 && nout > 0 && nout <= 4, CPX_ERR_ARG, "cpx_seg_average: bad sizes");
  hipLaunchKernelGGL(k_seg_average, dim3(cpx_div_up(geom->Ly * geom->Lx, kT), B), dim3(kT), 0,
                     ctx->stream, net_dev, layout, nout, *geom, taper_dev, yf_dev);
  CPX_CHECK_LAUNCH("k_seg_average");
  return CPX_OK;
}

// ordered compaction launches (flags [B][n] bytes -> out [B][out_stride] indices, totals [B])
static int ordered_compact(cpx_ctx* ctx, const unsigned char* flags, long long n, int B, int* tiles,
                           int* totals, int cap, int* out, long long out_stride) {
  const int ntile = cpx_div_up(n, kOcTile);
  hipLaunchKernelGGL(k_oc_count, dim3(ntile, B), dim3(kOcThreads), 0, ctx->stream, flags, n, ntile, tiles);
  hipLaunchKernelGGL(k_oc_scan, dim3(B), dim3(1024), 0, ctx->stream, ntile, tiles, totals);
  hipLaunchKernelGGL(k_oc_emit, dim3(ntile, B), dim3(kOcThreads), 0, ctx->stream, flags, n, ntile,
                     (const int*)tiles, cap, out, out_stride);
  CPX_CHECK_LAUNCH("ordered_compact");
  return CPX_OK;
}

__global__ void k_seed_count(int B, int ms, const int* __restrict__ totals, cpx_seg_stats* __restrict__ st) {
  const int fov = blockIdx.x * blockDim.x + threadIdx.x;
  if (fov >= B) return;
  const int t = totals[fov];
  st[fov].n_seeds = min(t, ms);
  st[fov].n_seeds_found = t;
  if (t > ms) atomicOr(&st[fov].overflow, CPX_SEG_OVF_SEEDS);
}

constexpr int kFeSmallThreads = 256, kFeSmallCells = 5000;    // 40 KiB: 4 blocks per CU
constexpr int kFeMidThreads = 512, kFeMidCells = 10176;       // 80 KiB: 2 blocks per CU
constexpr int kFeLargeThreads = 1024, kFeLargeCells = 20224;  // 158 KiB: 1 block per CU
constexpr int kFeCmpThreads = 1024, kFeCmpU = 1, kFeCmpCells = 19968;  // compact rows: 156 KiB + rows
constexpr int kFeU = 1;                                        // 2-column x 12-row units per thread
// every register-class mask (k_flowerr_reg.hip: bbox within 128 x 120 either way) is one the
// largest fp32 screening class holds, so the LDS screening is what skips it (bad set by the
// register kernel) and no register-class mask falls to k_flow_error_cmp / k_flow_error_big
static_assert(fe_fits(kFeRegMaxLong, kFeRegMaxShort, kFeLargeThreads / 2, 2 * kFeU, kFeLargeCells) &&
                  fe_fits(kFeRegMaxShort, kFeRegMaxLong, kFeLargeThreads / 2, 2 * kFeU, kFeLargeCells),
              "register-class masks must fit the large screening class");

extern "C" int cpx_seg_masks(cpx_ctx* ctx, const float* yf_dev, int B, const cpx_seg_geom* geom,
                             int H, int W, int niter, double flow_threshold, int min_size,
                             int max_objects, int resample, int32_t* labels_dev,
                             cpx_seg_stats* stats_dev) {
  CPX_REQUIRE(ctx && yf_dev && labels_dev && stats_dev, CPX_ERR_ARG, "cpx_seg_masks: null argument");
  CPX_REQUIRE(geom_ok(geom), CPX_ERR_ARG, "cpx_seg_masks: bad geometry");
  CPX_REQUIRE(B > 0 && B <= 65535 && H > 0 && W > 0 && niter >= 0 && max_objects > 0 &&
                  (long long)(H + 2 * kRpad) * (W + 2 * kRpad) < (1LL << 31) &&
                  // k_dyn_follow addresses the float2 field with 32-bit byte offsets
                  (long long)H * W * (long long)sizeof(float2) < (1LL << 32),
              CPX_ERR_ARG, "cpx_seg_masks: bad sizes");
  const int Ly = geom->Ly, Lx = geom->Lx;
  const int Dy = resample ? H : Ly, Dx = resample ? W : Lx;  // dynamics resolution
  const int Dyh = Dy + 2 * kRpad, Dxh = Dx + 2 * kRpad;
  const long long n = (long long)Dy * Dx, nh = (long long)Dyh * Dxh;
  SegTabs tabs;
  int rc = seg_tables(ctx, H, W, Ly, Lx, tabs);
  if (rc) return rc;
  // ---- workspace carve (WS_SEG_DYN)
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const int ntile = cpx_div_up(std::max(n, nh), kOcTile);
  const size_t sz_f2 = al(sizeof(float2) * B * n);
  const size_t sz_d2 = al(sizeof(float2) * B * n);
  const size_t sz_b = al((size_t)B * n);
  const size_t sz_h = al(sizeof(int) * B * nh), sz_hb = al((size_t)B * nh);
  const size_t sz_m0 = resample ? 0 : al(sizeof(int) * B * n);
  // seeds beyond max_objects cannot all become objects of the caller's tables: the first
  // max_objects (raster order) are expanded, CPX_SEG_OVF_SEEDS is set and n_seeds_found tells
  // the caller the capacity a re-run needs (masks <= seeds, so the tables below never overflow)
  const int ms = max_objects;
  const size_t sz_seeds = al(sizeof(int) * (size_t)B * ms);
  const size_t sz_cnt = al(sizeof(int) * (size_t)B * (ms + 1));
  const size_t sz_act = al(sizeof(int) * B * n);
  const size_t sz_small = al(sizeof(int) * (size_t)B);
  // follow rounds: K = k0 steps while most pixels still move (until step sw), then k1 for the
  // long tail (k0 = 24 / 32 / 48 measured equal to 16, `gpurun_out/r06af`)
  constexpr int k0 = 16, sw = 384, k1 = 128;
  const int rounds = cpx_div_up(sw, k0) + cpx_div_up(std::max(0, niter - sw), k1) + 2;
  const size_t sz_fcnt = al(sizeof(int) * (size_t)B * (rounds + 1));
  const size_t sz_items = al((size_t)16 * B * n);
  const size_t sz_tiles = al(sizeof(int) * (size_t)B * ntile);
  const size_t total = sz_d2 + 2 * sz_f2 + 2 * sz_b + 2 * sz_h + sz_hb + sz_m0 + 2 * sz_seeds + 3 * sz_cnt +
                       sz_act + sz_small + sz_tiles + sz_fcnt + 2 * sz_items;
  unsigned char* w = (unsigned char*)cpx_ws(ctx, WS_SEG_DYN, total);
  if (!w) return CPX_ERR_OOM;
  DynBufs d;
  d.dps = (float2*)w; w += sz_d2;
  d.dpf = (float2*)w; w += sz_f2;
  d.p = (float2*)w; w += sz_f2;
  d.mov = w; w += sz_b;
  d.mark = w; w += sz_b;
  d.h = (int*)w; w += sz_h;
  d.M = (unsigned int*)w; w += sz_h;
  d.sflag = w; w += sz_hb;
  d.m0 = resample ? labels_dev : (int*)w; w += sz_m0;
  d.seeds = (int*)w; w += sz_seeds;
  d.marklist = (int*)w; w += sz_seeds;
  d.cnt = (int*)w; w += sz_cnt;
  d.first = (int*)w; w += sz_cnt;
  d.newlab = (int*)w; w += sz_cnt;
  d.act = (int*)w; w += sz_act;
  d.fcnt = (int*)w; w += sz_fcnt;
  d.fitems0 = w; w += sz_items;
  d.fitems1 = w; w += sz_items;
  d.totals = (int*)w; w += sz_small;
  d.tiles = (int*)w; w += sz_tiles;
  d.st = stats_dev;
  d.ms = ms;
  CPX_CHECK_HIP(hipMemsetAsync(stats_dev, 0, sizeof(cpx_seg_stats) * B, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.M, 0, sz_h, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.mark, 0, sz_b, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.cnt, 0, sz_cnt, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.first, 0x7f, sz_cnt, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.newlab, 0, sz_cnt, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.fcnt, 0, sz_fcnt, ctx->stream));
  const dim3 gp(cpx_div_up(n, kT), B), gh(cpx_div_up(nh, kT), B);
  const dim3 gprep(cpx_div_up(n, (long long)kT * kPrepPer), B);
  if (resample)
    hipLaunchKernelGGL(k_dyn_prep<true>, gprep, dim3(kT), 0, ctx->stream, yf_dev, Ly, Lx, Dy, Dx,
                       tabs.uy, tabs.ux, d);
  else
    hipLaunchKernelGGL(k_dyn_prep<false>, gprep, dim3(kT), 0, ctx->stream, yf_dev, Ly, Lx, Dy, Dx,
                       tabs.uy, tabs.ux, d);
  // get_masks' histogram: the cells of the pixels that do not move (the moving pixels' final
  // positions are added by the follow rounds as they finish)
  const dim3 gh4(cpx_div_up(nh, (long long)kT * kPx4), B), gp4(cpx_div_up(n, (long long)kT * kPx4), B);
  hipLaunchKernelGGL(k_hist_init, gh4, dim3(kT), 0, ctx->stream, Dy, Dx, d);
  // k_dyn_follow: two trajectories per thread and paired 16-byte gathers; per 48-FOV step
  // (`gpurun_out/r05l`, `r05m`, trajectories / gathers): 1 / scalar 12.11 ms, 2 / scalar 11.83,
  // 4 / scalar 12.54, 1 / paired 11.46, 2 / paired 11.02 (kept); every setting passed the
  // segmentation parity tests
  // (development / bench instrumentation: cpx_debug_seg_timing)
  const int sev = ctx->seg_timing && ctx->seg_nev < cpx_ctx::kSegEv ? ctx->seg_nev++ : -1;
  bool fe_timed = false;  // the register flow-error kernels were bracketed (else a zero interval)
  if (sev >= 0) CPX_CHECK_HIP(hipEventRecord(ctx->seg_ev[sev][0], ctx->stream));
  {
    const int fblk = std::max(1, std::min(cpx_div_up(n, kT), (16 * ctx->n_cu + B - 1) / B));
    int step = 0, r = 0;
    do {  // at least one round: with niter = 0 it only records the start positions
      const int K = step < sw ? k0 : k1;
      const FollowItem* in = (const FollowItem*)(r & 1 ? d.fitems1 : d.fitems0);
      FollowItem* out = (FollowItem*)(r & 1 ? d.fitems0 : d.fitems1);
      // (the right-edge form reads x0 - 1; the buffer resource holds 8 n < 2^31 bytes)
      const bool v4 = Dx >= 2 && 8LL * n < (1LL << 31);
      auto kern = v4 ? k_dyn_follow<2, true> : k_dyn_follow<2, false>;
      hipLaunchKernelGGL(kern, dim3(fblk, B), dim3(kT), 0, ctx->stream, Dy, Dx, niter, step, K,
                         r == 0 ? 1 : 0, in, (const int*)(d.fcnt + (size_t)B * r), out,
                         d.fcnt + (size_t)B * (r + 1), d);
      if (sev >= 0 && r < 64) ctx->seg_K[sev][r] = std::min(K, std::max(niter - step, 0));
      step += K;
      ++r;
    } while (step < niter);
    if (sev >= 0) {
      // items of round 0 = the moving pixels (cpx_seg_stats.n_moving, int 0 of each 48-byte
      // record), of round r >= 1 = fcnt[B r + b]
      CPX_CHECK_HIP(hipEventRecord(ctx->seg_ev[sev][1], ctx->stream));
      const int rr = std::min(r, 64);
      const int need = B * rr;
      if (ctx->seg_cnt_cap[sev] < need) {
        if (ctx->seg_cnt[sev]) CPX_CHECK_HIP(hipHostFree(ctx->seg_cnt[sev]));
        CPX_CHECK_HIP(hipHostMalloc((void**)&ctx->seg_cnt[sev], sizeof(int) * need));
        ctx->seg_cnt_cap[sev] = need;
      }
      CPX_CHECK_HIP(hipMemcpy2DAsync(ctx->seg_cnt[sev], sizeof(int), stats_dev, sizeof(cpx_seg_stats),
                                     sizeof(int), B, hipMemcpyDeviceToHost, ctx->stream));
      if (rr > 1)
        CPX_CHECK_HIP(hipMemcpyAsync(ctx->seg_cnt[sev] + B, d.fcnt + B, sizeof(int) * B * (rr - 1),
                                     hipMemcpyDeviceToHost, ctx->stream));
      ctx->seg_B[sev] = B;
      ctx->seg_rounds[sev] = rr;
    }
  }
  // (only FOVs with fewer than 5 moving pixels are left to it: one block per FOV)
  hipLaunchKernelGGL(k_hist_moving, dim3(1, B), dim3(kT), 0, ctx->stream, Dy, Dx, d);
  hipLaunchKernelGGL(k_seed_flags, gh4, dim3(kT), 0, ctx->stream, Dyh, Dxh, d);
  CPX_CHECK_LAUNCH("cpx_seg_masks follow");
  rc = ordered_compact(ctx, d.sflag, nh, B, d.tiles, d.totals, ms, d.seeds, ms);
  if (rc) return rc;
  hipLaunchKernelGGL(k_seed_count, dim3(cpx_div_up(B, 256)), dim3(256), 0, ctx->stream, B, ms,
                     (const int*)d.totals, stats_dev);
  hipLaunchKernelGGL(k_seed_expand, dim3(std::max(1, (4 * ctx->n_cu + B - 1) / B), B), dim3(kT), 0,
                     ctx->stream, Dyh, Dxh, d);
  hipLaunchKernelGGL(k_assign, dim3(cpx_div_up(n, (long long)kT * kAsg), B), dim3(kT), 0, ctx->stream, Dy, Dx, d);
  hipLaunchKernelGGL(k_relabel_mark, dim3(cpx_div_up(ms, kT), B), dim3(kT), 0, ctx->stream, Dy, Dx, d);
  CPX_CHECK_LAUNCH("cpx_seg_masks seeds");
  rc = ordered_compact(ctx, d.mark, n, B, d.tiles, d.totals, ms, d.marklist, ms);
  if (rc) return rc;
  hipLaunchKernelGGL(k_relabel_apply, dim3(4, B), dim3(kT), 0, ctx->stream, Dy, Dx, d);
  hipLaunchKernelGGL(k_apply_newlab, gp4, dim3(kT), 0, ctx->stream, Dy, Dx, d);
  CPX_CHECK_LAUNCH("cpx_seg_masks relabel");
  // ---- object workspaces (WS_SEG_OBJ): the flow-error and fill-holes object tables share it
  const int ML = max_objects;
  const size_t sz_lst = al(sizeof(cpx_label_stats) * (size_t)B * (ML + 1));
  const size_t sz_obj = al(sizeof(cpx_object) * (size_t)B * ML);
  const size_t sz_hdr = al(sizeof(cpx_fov_objects) * (size_t)B);
  const size_t sz_bad = al((size_t)B * (ML + 1));
  const size_t sz_l2i = al(sizeof(int) * (size_t)B * (ML + 1));
  const size_t sz_abs = al(sizeof(int) * (size_t)B * ML);
  const size_t sz_nl = sz_abs;
  const size_t sz_off = al(sizeof(int) * (size_t)(B + 1 + 11));  // prefix + 11 queue counters
  const size_t sz_und = al(sizeof(int) * ((size_t)B * ML + 1));  // screening: undecided masks
  const size_t gscr_per = (size_t)2 * (Dy + 2) * (Dx + 2);  // doubles per FOV (oversize masks)
  const size_t sz_gscr = al(sizeof(double) * B * gscr_per);
  unsigned char* o = (unsigned char*)cpx_ws(ctx, WS_SEG_OBJ,
      sz_lst + sz_obj + sz_hdr + sz_bad + sz_l2i + sz_abs + sz_nl + sz_off + sz_und + sz_gscr);
  if (!o) return CPX_ERR_OOM;
  cpx_label_stats* lst = (cpx_label_stats*)o; o += sz_lst;
  cpx_object* obj = (cpx_object*)o; o += sz_obj;
  cpx_fov_objects* hdr = (cpx_fov_objects*)o; o += sz_hdr;
  unsigned char* bad = o; o += sz_bad;
  int* l2i = (int*)o; o += sz_l2i;
  int* absorber = (int*)o; o += sz_abs;
  int* newlab = (int*)o; o += sz_nl;
  int* off = (int*)o; o += sz_off;
  int* und = (int*)o; o += sz_und;
  double* gscr = (double*)o;
  if (flow_threshold > 0.0) {
    rc = cpx_objects(ctx, d.m0, B, Dy, Dx, ML, 0, lst, obj, hdr);
    if (rc) return rc;
    CPX_CHECK_HIP(hipMemsetAsync(bad, 0, sz_bad, ctx->stream));
    CPX_CHECK_HIP(hipMemsetAsync(off + B + 1, 0, 11 * sizeof(int), ctx->stream));
    CPX_CHECK_HIP(hipMemsetAsync(und, 0, sizeof(int), ctx->stream));
    hipLaunchKernelGGL(k_obj_prefix, dim3(1), dim3(64), 0, ctx->stream, B,
                       (const cpx_fov_objects*)hdr, off);
    // fp32 screening of every mask the LDS kernels hold (half the LDS: twice the masks per CU),
    // then the fp64 sweeps for the masks it could not decide
    const int* lst_in = nullptr;
    if (B < 2048 && ML <= (1 << 20)) {  // list codes: fov << 20 | object
#define FE_SCREEN(TH, CE, U_, WPE, G, CTR, LT, LU, LC)                                                  \
  hipLaunchKernelGGL((k_flow_error_lds<TH, CE, U_, float, WPE>), dim3((G) * ctx->n_cu), dim3(TH), 0,    \
                     ctx->stream, (const int*)d.m0, (const float2*)d.dpf, Dy, Dx, B, ML,             \
                     (const cpx_object*)obj, (const int*)off, off + B + (CTR), LT, LU, LC, flow_threshold, \
                     bad, (const int*)nullptr, und)
      // masks of fe_reg_class 1-3 (k_flowerr_reg.hip: up to 64 x 80 one column per lane, 128 x 80 /
      // 128 x 120 in column pairs over two / four waves)
      // first, in VGPRs (k_flow_error_reg); the LDS kernels skip the masks those flagged
      if (sev >= 0) CPX_CHECK_HIP(hipEventRecord(ctx->seg_ev[sev][2], ctx->stream));
      rc = cpx_flow_error_reg_launch(ctx->n_cu, ctx->stream, d.m0, (const float2*)d.dpf, Dy, Dx, B, ML,
                                     obj, off, off + B + 9, flow_threshold, bad, und);
      if (rc) return rc;
      if (sev >= 0) {
        CPX_CHECK_HIP(hipEventRecord(ctx->seg_ev[sev][3], ctx->stream));
        fe_timed = true;
      }
      // six waves per SIMD for the small and mid classes; the large class as 512 threads with two
      // units each (the same masks as the fp64 1024 x 1 kernel), two 79 KiB blocks per CU
      FE_SCREEN(kFeSmallThreads, kFeSmallCells, kFeU, 6, 6, 6, 0, 0, 0);
      FE_SCREEN(kFeMidThreads, kFeMidCells, kFeU, 6, 3, 7, kFeSmallThreads, kFeU, kFeSmallCells);
      FE_SCREEN(kFeLargeThreads / 2, kFeLargeCells, 2 * kFeU, 4, 2, 8, kFeMidThreads, kFeU, kFeMidCells);
#undef FE_SCREEN
      lst_in = und;
      if (getenv("CPX_FE_DEBUG")) {  // profiling aid: masks the screening left undecided
        int nu = 0, nm = 0;
        CPX_CHECK_HIP(hipMemcpyAsync(&nu, und, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        CPX_CHECK_HIP(hipMemcpyAsync(&nm, off + B, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        fprintf(stderr, "flow error: %d of %d masks undecided by the fp32 screening\n", nu, nm);
      }
    }
    hipLaunchKernelGGL((k_flow_error_lds<kFeSmallThreads, kFeSmallCells, kFeU>), dim3(4 * ctx->n_cu),
                       dim3(kFeSmallThreads), 0, ctx->stream, (const int*)d.m0, (const float2*)d.dpf,
                       Dy, Dx, B, ML, (const cpx_object*)obj, (const int*)off, off + B + 1, 0, 0, 0,
                       flow_threshold, bad, lst_in, (int*)nullptr);
    hipLaunchKernelGGL((k_flow_error_lds<kFeMidThreads, kFeMidCells, kFeU>), dim3(2 * ctx->n_cu),
                       dim3(kFeMidThreads), 0, ctx->stream, (const int*)d.m0, (const float2*)d.dpf,
                       Dy, Dx, B, ML, (const cpx_object*)obj, (const int*)off, off + B + 2,
                       kFeSmallThreads, kFeU, kFeSmallCells, flow_threshold, bad, lst_in, (int*)nullptr);
    hipLaunchKernelGGL((k_flow_error_lds<kFeLargeThreads, kFeLargeCells, kFeU>), dim3(ctx->n_cu),
                       dim3(kFeLargeThreads), 0, ctx->stream, (const int*)d.m0, (const float2*)d.dpf,
                       Dy, Dx, B, ML, (const cpx_object*)obj, (const int*)off, off + B + 3,
                       kFeMidThreads, kFeU, kFeMidCells, flow_threshold, bad, lst_in, (int*)nullptr);
    hipLaunchKernelGGL((k_flow_error_cmp<kFeCmpThreads, kFeCmpCells, kFeCmpU>), dim3(ctx->n_cu),
                       dim3(kFeCmpThreads), 0, ctx->stream, (const int*)d.m0, (const float2*)d.dpf,
                       Dy, Dx, B, ML, (const cpx_object*)obj, (const int*)off, off + B + 4,
                       kFeLargeThreads, kFeU, kFeLargeCells, flow_threshold, bad);
    {
      const int nbig = std::max(1, std::min(ctx->n_cu, 4 * B));
      const long long slice = (long long)(B * gscr_per / nbig) & ~1LL;
      hipLaunchKernelGGL(k_flow_error_big, dim3(nbig), dim3(kBigThreads), 0, ctx->stream,
                         (const int*)d.m0, (const float2*)d.dpf, Dy, Dx, B, ML, (const cpx_object*)obj,
                         (const int*)off, off + B + 5, kFeLargeThreads, kFeU, kFeLargeCells, flow_threshold,
                         gscr, slice, bad);
    }
    hipLaunchKernelGGL(k_flow_error_fov, dim3(B), dim3(kFlowThreads), 0, ctx->stream,
                       (const int*)d.m0, (const float2*)d.dpf, Dy, Dx, ML, (const cpx_object*)obj,
                       (const cpx_fov_objects*)hdr, kFeLargeThreads, kFeU, kFeLargeCells,
                       flow_threshold, gscr, (long long)gscr_per, bad);
    hipLaunchKernelGGL(k_apply_bad, gp4, dim3(kT), 0, ctx->stream, n, ML,
                       (const unsigned char*)bad, d.m0);
    hipLaunchKernelGGL(k_count_bad, dim3(B), dim3(256), 0, ctx->stream, ML,
                       (const unsigned char*)bad, (const int*)(off + B + 1), 11, stats_dev);
    CPX_CHECK_LAUNCH("cpx_seg_masks flow error");
  }
  if (!resample) {
    hipLaunchKernelGGL(k_upsample, dim3(cpx_div_up(W, kT), cpx_div_up(H, kUpRows), B), dim3(kT), 0,
                       ctx->stream, (const int*)d.m0, Ly, Lx, H, W, tabs.ynear, tabs.xnear, labels_dev);
    CPX_CHECK_LAUNCH("k_upsample");
  }
  // ---- fill holes + remove small at full resolution
  rc = cpx_objects(ctx, labels_dev, B, H, W, ML, 0, lst, obj, hdr);
  if (rc) return rc;
  const long long N = (long long)H * W;
  const size_t sz_fill = al(sizeof(int) * (size_t)B * N);
  const size_t sz_fscr = al(sizeof(unsigned int) * 2 * (size_t)B * ((W + 31) / 32) * H);
  unsigned char* fw = (unsigned char*)cpx_ws(ctx, WS_SEG_FILL, sz_fill + sz_fscr);
  if (!fw) return CPX_ERR_OOM;
  int* fillidx = (int*)fw;
  unsigned int* fscr = (unsigned int*)(fw + sz_fill);
  CPX_CHECK_HIP(hipMemsetAsync(fillidx, 0, sizeof(int) * (size_t)B * N, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(absorber, 0x7f, sz_abs, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(l2i, 0, sz_l2i, ctx->stream));
  hipLaunchKernelGGL(k_lab2idx, dim3(cpx_div_up(ML, kT), B), dim3(kT), 0, ctx->stream, ML,
                     (const cpx_object*)obj, (const cpx_fov_objects*)hdr, l2i);
  static bool fattr = false;
  const size_t flds = sizeof(unsigned int) * 2 * kFillMaxWords;
  if (!fattr) {
    CPX_CHECK_HIP(hipFuncSetAttribute((const void*)k_fill_holes,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)flds));
    CPX_CHECK_HIP(hipFuncSetAttribute((const void*)k_fill_seq,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)flds));
    fattr = true;
  }
  hipLaunchKernelGGL(k_fill_holes, dim3(std::max(1, std::min(ML, (2 * ctx->n_cu + B - 1) / B)), B),
                     dim3(kFillThreads), flds, ctx->stream,
                     (const int*)labels_dev, H, W, ML, min_size, (const cpx_object*)obj,
                     (const cpx_fov_objects*)hdr, (const int*)l2i, fillidx, absorber);
  hipLaunchKernelGGL(k_fill_holes_big, dim3(B), dim3(1024), 0, ctx->stream,
                     (const int*)labels_dev, H, W, ML, min_size, (const cpx_object*)obj,
                     (const cpx_fov_objects*)hdr, (const int*)l2i, fillidx, absorber, fscr);
  if (sev >= 0 && !fe_timed) {
    CPX_CHECK_HIP(hipEventRecord(ctx->seg_ev[sev][2], ctx->stream));
    CPX_CHECK_HIP(hipEventRecord(ctx->seg_ev[sev][3], ctx->stream));
  }
  hipLaunchKernelGGL(k_fill_final, dim3(B), dim3(1024), 0, ctx->stream, ML, min_size,
                     (const cpx_object*)obj, (const cpx_fov_objects*)hdr, (const int*)absorber,
                     (const int*)labels_dev, (const int*)fillidx, W, N, newlab, stats_dev);
  // eight 256-thread blocks per CU over the batch (the kernel's full occupancy; four left its
  // loads short of the HBM rate)
  hipLaunchKernelGGL(k_fill_apply, dim3(std::max(1, std::min(cpx_div_up(N, kT), 8 * ctx->n_cu / B + 1)), B),
                     dim3(kT), 0, ctx->stream, labels_dev, N, ML, (const int*)l2i,
                     (const int*)fillidx, (const int*)newlab, (const int*)absorber,
                     (const cpx_seg_stats*)stats_dev);
  // the flagged FOVs (none on the bench plates): the reference's sequential loop, one block each;
  // the others' blocks exit at once
  hipLaunchKernelGGL(k_fill_seq, dim3(B), dim3(1024), flds, ctx->stream, labels_dev, H, W, ML, min_size,
                     (const cpx_object*)obj, (const cpx_fov_objects*)hdr, fscr, stats_dev);
  CPX_CHECK_LAUNCH("cpx_seg_masks fill holes");
  return CPX_OK;
}
