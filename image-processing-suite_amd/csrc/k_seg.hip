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
#include <limits.h>
#include <math.h>
#include <vector>

#pragma clang fp contract(off)

namespace {

constexpr int kT = 256;
constexpr int kRpad = 20;
constexpr int kMaxSeeds = 32768;

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
// dynamics
struct DynBufs {
  float* dps;      // [B][2][Ly][Lx]
  float* p;        // [B][2][Ly][Lx]
  int* h;          // [B][Lyh][Lxh]
  unsigned int* M; // [B][Lyh][Lxh]
  int* m0;         // [B][Ly][Lx]
  int* seeds;      // [B][kMaxSeeds]
  int* cnt;        // [B][kMaxSeeds + 1]
  int* first;      // [B][kMaxSeeds + 1]
  int* newlab;     // [B][kMaxSeeds + 1]
  unsigned char* mark;  // [B][Ly*Lx]
  int* act;        // [B][Ly*Lx]: indices of the moving pixels (first n_moving entries per FOV)
  cpx_seg_stats* st;
};

__global__ __launch_bounds__(kT) void k_dyn_prep(const float* __restrict__ yf, int Ly, int Lx,
                                                 DynBufs d) {
  const int fov = blockIdx.y;
  const int q = blockIdx.x * kT + threadIdx.x;
  const int n = Ly * Lx;
  int moving = 0;
  if (q < n) {
    const float* f = yf + (long long)fov * 3 * n;
    const bool cp = f[2 * n + q] > 0.0f;  // cellprob > cellprob_threshold (0.0)
    const float dy = (f[q] * (cp ? 1.0f : 0.0f)) / 5.0f;
    const float dx = (f[n + q] * (cp ? 1.0f : 0.0f)) / 5.0f;
    d.dps[(long long)fov * 2 * n + q] = dy;
    d.dps[(long long)fov * 2 * n + n + q] = dx;
    const int y = q / Lx, x = q - y * Lx;
    d.p[(long long)fov * 2 * n + q] = (float)y;
    d.p[(long long)fov * 2 * n + n + q] = (float)x;
    moving = (double)fabsf(dy) > 1e-3;
  }
  // compact the moving pixels (wave-aggregated slots; the list order does not matter, every
  // pixel writes only its own position) so k_dyn_follow runs full waves
  const unsigned long long mask = __ballot(moving);
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (lane == 0 && mask) base = atomicAdd(&d.st[fov].n_moving, __popcll(mask));
  base = __shfl(base, 0);
  if (moving) d.act[(long long)fov * n + base + __popcll(mask & ((1ull << lane) - 1ull))] = q;
}

__global__ __launch_bounds__(kT) void k_dyn_follow(int Ly, int Lx, int niter, DynBufs d) {
  const int fov = blockIdx.y;
  const int t = blockIdx.x * kT + threadIdx.x;
  const int n = Ly * Lx;
  const int n_moving = d.st[fov].n_moving;
  if (n_moving < 5) return;  // follow_flows returns inds=None -> no masks
  if (t >= n_moving) return;
  const int q = d.act[(long long)fov * n + t];  // a pixel with |dY| > 1e-3 (k_dyn_prep)
  const float* I = d.dps + (long long)fov * 2 * n;
  float py = (float)(q / Lx), px = (float)(q % Lx);
  const float fLy = (float)(Ly - 1), fLx = (float)(Lx - 1);
  for (int it = 0; it < niter; ++it) {
    const int yi = (int)py, xi = (int)px;
    const double yy = (double)py - (double)yi, xx = (double)px - (double)xi;
    const int y0 = min(Ly - 1, max(0, yi)), x0 = min(Lx - 1, max(0, xi));
    const int y1 = min(Ly - 1, y0 + 1), x1 = min(Lx - 1, x0 + 1);
    float dv[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float* Ic = I + (long long)c * n;
      const double v = (double)Ic[y0 * Lx + x0] * (1.0 - yy) * (1.0 - xx) +
                       (double)Ic[y0 * Lx + x1] * (1.0 - yy) * xx +
                       (double)Ic[y1 * Lx + x0] * yy * (1.0 - xx) +
                       (double)Ic[y1 * Lx + x1] * yy * xx;
      dv[c] = (float)v;
    }
    py = fminf(fLy, fmaxf(0.0f, py + dv[0]));
    px = fminf(fLx, fmaxf(0.0f, px + dv[1]));
  }
  d.p[(long long)fov * 2 * n + q] = py;
  d.p[(long long)fov * 2 * n + n + q] = px;
}

__global__ __launch_bounds__(kT) void k_dyn_hist(int Ly, int Lx, DynBufs d) {
  const int fov = blockIdx.y;
  const int q = blockIdx.x * kT + threadIdx.x;
  const int n = Ly * Lx;
  if (q >= n) return;
  const int Lxh = Lx + 2 * kRpad, Lyh = Ly + 2 * kRpad;
  const int iy = (int)d.p[(long long)fov * 2 * n + q] + kRpad;
  const int ix = (int)d.p[(long long)fov * 2 * n + n + q] + kRpad;
  atomicAdd(&d.h[(long long)fov * Lyh * Lxh + iy * Lxh + ix], 1);
}

// seeds: h > 10 and h == 5x5 max (maximum_filter1d size 5 on both axes)
__global__ __launch_bounds__(kT) void k_seed_flags(int Lyh, int Lxh, DynBufs d) {
  const int fov = blockIdx.y;
  const int q = blockIdx.x * kT + threadIdx.x;
  if (q >= Lyh * Lxh) return;
  const int* h = d.h + (long long)fov * Lyh * Lxh;
  const int v = h[q];
  unsigned char f = 0;
  if (v > 10) {
    const int y = q / Lxh, x = q - y * Lxh;
    int mx = v;
    for (int dy = -2; dy <= 2; ++dy)
      for (int dx = -2; dx <= 2; ++dx) {
        int yy = y + dy, xx = x + dx;  // scipy 'reflect' boundary (never reached by seeds)
        yy = yy < 0 ? -yy - 1 : (yy >= Lyh ? 2 * Lyh - yy - 1 : yy);
        xx = xx < 0 ? -xx - 1 : (xx >= Lxh ? 2 * Lxh - xx - 1 : xx);
        mx = max(mx, h[yy * Lxh + xx]);
      }
    f = (v >= mx);
  }
  // reuse the seed map M as the flag array until compaction
  d.M[(long long)fov * Lyh * Lxh + q] = f;
}

// one block per FOV: row-major compaction of seed flags into the seed list; clears M
__global__ __launch_bounds__(1024) void k_seed_compact(int Lyh, int Lxh, DynBufs d) {
  const int fov = blockIdx.x;
  unsigned int* M = d.M + (long long)fov * Lyh * Lxh;
  int* seeds = d.seeds + (long long)fov * kMaxSeeds;
  __shared__ int wsum[16];
  __shared__ int base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int n = Lyh * Lxh;
  for (int i0 = 0; i0 < n; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    const int f = (i < n) ? (int)M[i] : 0;
    if (i < n) M[i] = 0u;
    const unsigned long long b = __ballot(f);
    const unsigned long long lower = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (lane == 0) wsum[wid] = __popcll(b);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    const int k = off + __popcll(b & lower);
    if (f && k < kMaxSeeds) seeds[k] = i;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int w = 0; w < nw; ++w) tot += wsum[w];
      base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    d.st[fov].n_seeds = min(base, kMaxSeeds);
    if (base > kMaxSeeds) d.st[fov].overflow = 1;
  }
}

// one wave per seed: geodesic 8-connected ball of radius 5 through h > 2 (get_masks expansion)
__global__ __launch_bounds__(kT) void k_seed_expand(int Lyh, int Lxh, DynBufs d) {
  const int fov = blockIdx.y;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __shared__ unsigned char cur[kT / 64][2][169];
  const int ns = d.st[fov].n_seeds;
  for (int kb = blockIdx.x * (kT / 64); kb < ns; kb += gridDim.x * (kT / 64)) {  // block-uniform
  const int k = kb + wid;
  const bool active = k < ns;
  const int s = active ? d.seeds[(long long)fov * kMaxSeeds + k] : 0;
  const int sy = s / Lxh, sx = s - sy * Lxh;
  const int* h = d.h + (long long)fov * Lyh * Lxh;
  bool good[3];
  for (int u = 0; u < 3; ++u) {
    const int c = lane + 64 * u;
    good[u] = false;
    if (c < 169 && active) {
      const int yy = sy - 6 + c / 13, xx = sx - 6 + c % 13;
      good[u] = yy >= 0 && yy < Lyh && xx >= 0 && xx < Lxh && h[yy * Lxh + xx] > 2;
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
    unsigned int* M = d.M + (long long)fov * Lyh * Lxh;
    for (int u = 0; u < 3; ++u) {
      const int c = lane + 64 * u;
      if (c < 169 && cur[wid][src][c]) {
        const int yy = sy - 6 + c / 13, xx = sx - 6 + c % 13;
        atomicMax(&M[yy * Lxh + xx], (unsigned int)(k + 1));  // later seeds win (M[pix[k]] = 1+k)
      }
    }
  }
  __syncthreads();
  }  // seed loop
}

__global__ __launch_bounds__(kT) void k_assign(int Ly, int Lx, DynBufs d) {
  const int fov = blockIdx.y;
  const int q = blockIdx.x * kT + threadIdx.x;
  const int n = Ly * Lx;
  if (q >= n) return;
  const int Lxh = Lx + 2 * kRpad, Lyh = Ly + 2 * kRpad;
  const int iy = (int)d.p[(long long)fov * 2 * n + q] + kRpad;
  const int ix = (int)d.p[(long long)fov * 2 * n + n + q] + kRpad;
  const int l = (int)d.M[(long long)fov * Lyh * Lxh + iy * Lxh + ix];
  d.m0[(long long)fov * n + q] = l;
  if (l) {
    atomicAdd(&d.cnt[(long long)fov * (kMaxSeeds + 1) + l], 1);
    atomicMin(&d.first[(long long)fov * (kMaxSeeds + 1) + l], q);
  }
}

// big-mask removal + first-occurrence renumbering (fastremap.renumber)
__global__ __launch_bounds__(kT) void k_relabel_mark(int Ly, int Lx, DynBufs d) {
  const int fov = blockIdx.y;
  const int l = blockIdx.x * kT + threadIdx.x + 1;
  if (l > d.st[fov].n_seeds) return;
  const long long o = (long long)fov * (kMaxSeeds + 1) + l;
  const int c = d.cnt[o];
  const double big = (double)Ly * (double)Lx * 0.4;
  if (c > 0 && !((double)c > big)) d.mark[(long long)fov * Ly * Lx + d.first[o]] = 1;
}

// one block per FOV: exclusive scan of marks over pixel order -> rank of each label
__global__ __launch_bounds__(1024) void k_relabel_scan(int Ly, int Lx, DynBufs d) {
  const int fov = blockIdx.x;
  const int n = Ly * Lx;
  unsigned char* mark = d.mark + (long long)fov * n;
  __shared__ int wsum[16];
  __shared__ int base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // pass: rank for each marked pixel, written back as rank+1 into `first`-indexed newlab via m0
  for (int i0 = 0; i0 < n; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    const int f = (i < n) ? (int)mark[i] : 0;
    const unsigned long long b = __ballot(f);
    const unsigned long long lower = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (lane == 0) wsum[wid] = __popcll(b);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    if (f) {
      const int l = d.m0[(long long)fov * n + i];  // the label whose first pixel this is
      d.newlab[(long long)fov * (kMaxSeeds + 1) + l] = off + __popcll(b & lower) + 1;
      mark[i] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int w = 0; w < nw; ++w) tot += wsum[w];
      base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) d.st[fov].n_masks = base;
}

__global__ __launch_bounds__(kT) void k_apply_newlab(int Ly, int Lx, DynBufs d) {
  const int fov = blockIdx.y;
  const int q = blockIdx.x * kT + threadIdx.x;
  const int n = Ly * Lx;
  if (q >= n) return;
  int* m = d.m0 + (long long)fov * n + q;
  const int l = *m;
  *m = l ? d.newlab[(long long)fov * (kMaxSeeds + 1) + l] : 0;  // big masks map to 0
}

// ---------------------------------------------------------------------------------------------
// flow-error filter: masks_to_flows (heat diffusion from the pixel nearest the median, fp64)
// and per-mask mean squared difference against dP/5; one block per mask.
constexpr int kFlowThreads = 256;
constexpr int kFlowMaxCells = 2048;  // 2 x (ly+2)*(lx+2) doubles in LDS (48 KiB with the median
                                     // histograms: 3 blocks per CU); larger masks: BIG pass
constexpr int kFlowPP = 8;           // bbox pixels per thread kept in registers for the diffusion

// BIG = false: grid-stride over the masks that fit in LDS; BIG = true: one block per FOV walks
// the oversize masks with a per-FOV global scratch (no two blocks share a scratch area).
template <bool BIG>
__global__ __launch_bounds__(kFlowThreads) void k_flow_error(
    const int* __restrict__ m0, const float* __restrict__ yf, int Ly, int Lx, int max_label,
    const cpx_object* __restrict__ objects, const cpx_fov_objects* __restrict__ hdr,
    double thr, double* __restrict__ gscratch, long long gscratch_per_fov,
    unsigned char* __restrict__ bad) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* rowc = reinterpret_cast<int*>(smem + (BIG ? 0 : sizeof(double) * 2 * kFlowMaxCells));
  int* colc = rowc + 2048;
  __shared__ double sred[kFlowThreads / 64][2];
  __shared__ unsigned long long sbest[kFlowThreads / 64];
  __shared__ double smed[2];
  const int fov = blockIdx.y;
  const int n = Ly * Lx;
  const int* lab = m0 + (long long)fov * n;
  const int nobj = hdr[fov].n_objects;
  for (int k = blockIdx.x; k < nobj; k += gridDim.x) {
  const cpx_object o = objects[(long long)fov * max_label + k];
  const int L = o.label;
  const int r0 = o.bbox[0], c0 = o.bbox[1];
  const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
  const int ly = bh + 2, lx = bw + 2;
  const int ncell = ly * lx;
  if ((ncell > kFlowMaxCells) != BIG) continue;  // block-uniform
  double* T0 = BIG ? gscratch + (long long)fov * gscratch_per_fov : reinterpret_cast<double*>(smem);
  double* T1 = T0 + (BIG ? ncell : kFlowMaxCells);
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
    if (lab[(r0 + rr) * Lx + c0 + cc] == L) {
      atomicAdd(&rowc[min(rr, 2047)], 1);
      atomicAdd(&colc[min(cc, 2047)], 1);
    }
  }
  __syncthreads();
  // medians of y and x (np.median of the pixel coordinates, local +1 offset)
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
  // argmin of (x-xmed)^2 + (y-ymed)^2 over mask pixels, first in row-major order on ties
  unsigned long long best = ~0ull;
  for (int p = threadIdx.x; p < nb; p += kFlowThreads) {
    const int rr = p / bw, cc = p - rr * bw;
    if (lab[(r0 + rr) * Lx + c0 + cc] != L) continue;
    const double dy = (double)(rr + 1) - ymed, dx = (double)(cc + 1) - xmed;
    const double dist = dx * dx + dy * dy;
    // medians are multiples of 1/2, so 4*dist is an exact integer: order-preserving key
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
  const int niter = 2 * ((bw - 1) + (bh - 1));  // 2 * (ptp(x) + ptp(y))
  // Jacobi heat diffusion over mask pixels (T outside the mask stays 0).  Objects of at most
  // kFlowPP pixels per thread keep their in-mask cell indices in registers, so the iterations
  // touch LDS only (no label re-reads per iteration).
  const bool small = nb <= kFlowPP * kFlowThreads;  // block-uniform
  int myi[kFlowPP];
#pragma unroll
  for (int j = 0; j < kFlowPP; ++j) {
    const int p = threadIdx.x + j * kFlowThreads;
    myi[j] = -1;
    if (small && p < nb) {
      const int rr = p / bw, cc = p - rr * bw;
      if (lab[(r0 + rr) * Lx + c0 + cc] == L) myi[j] = (rr + 1) * lx + cc + 1;
    }
  }
  double* Tc = T0;
  double* Tn = T1;
  for (int it = 0; it < niter; ++it) {
    if (threadIdx.x == 0) Tc[ym * lx + xm] += 1.0;
    __syncthreads();
    if (small) {
#pragma unroll
      for (int j = 0; j < kFlowPP; ++j) {
        const int i = myi[j];
        if (i < 0) continue;
        Tn[i] = 1 / 9. * (Tc[i] + Tc[i - lx] + Tc[i + lx] + Tc[i - 1] + Tc[i + 1] + Tc[i - lx - 1] +
                          Tc[i - lx + 1] + Tc[i + lx - 1] + Tc[i + lx + 1]);
      }
    } else {
      for (int p = threadIdx.x; p < nb; p += kFlowThreads) {
        const int rr = p / bw, cc = p - rr * bw;
        if (lab[(r0 + rr) * Lx + c0 + cc] != L) continue;
        const int y = rr + 1, x = cc + 1;
        Tn[y * lx + x] = 1 / 9. * (Tc[y * lx + x] + Tc[(y - 1) * lx + x] + Tc[(y + 1) * lx + x] +
                                   Tc[y * lx + x - 1] + Tc[y * lx + x + 1] + Tc[(y - 1) * lx + x - 1] +
                                   Tc[(y - 1) * lx + x + 1] + Tc[(y + 1) * lx + x - 1] +
                                   Tc[(y + 1) * lx + x + 1]);
      }
    }
    __syncthreads();
    double* t = Tc;
    Tc = Tn;
    Tn = t;
  }
  // gradients, normalisation, error vs dP/5
  const float* dY = yf + (long long)fov * 3 * n;
  const float* dX = dY + n;
  double e0 = 0.0, e1 = 0.0;
  for (int p = threadIdx.x; p < nb; p += kFlowThreads) {
    const int rr = p / bw, cc = p - rr * bw;
    const int gy = r0 + rr, gx = c0 + cc;
    if (lab[gy * Lx + gx] != L) continue;
    const int y = rr + 1, x = cc + 1;
    const double dy = Tc[(y + 1) * lx + x] - Tc[(y - 1) * lx + x];
    const double dx = Tc[y * lx + x + 1] - Tc[y * lx + x - 1];
    const double nrm = 1e-20 + sqrt(dy * dy + dx * dx);
    const double my = dy / nrm, mx = dx / nrm;
    const double ty = my - (double)(dY[gy * Lx + gx] / 5.0f);
    const double tx = mx - (double)(dX[gy * Lx + gx] / 5.0f);
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
    bad[(long long)fov * (max_label + 1) + L] = err > thr ? 1 : 0;
  }
  __syncthreads();
  }  // object loop
}

__global__ __launch_bounds__(kT) void k_apply_bad(int n, int max_label,
                                                  const unsigned char* __restrict__ bad,
                                                  int* __restrict__ m0) {
  const int fov = blockIdx.y;
  const int q = blockIdx.x * kT + threadIdx.x;
  if (q >= n) return;
  int* m = m0 + (long long)fov * n + q;
  const int l = *m;
  if (l > 0 && l <= max_label && bad[(long long)fov * (max_label + 1) + l]) *m = 0;
}

__global__ void k_count_bad(int max_label, const unsigned char* __restrict__ bad,
                            cpx_seg_stats* __restrict__ st) {
  const int fov = blockIdx.x;
  int c = 0;
  for (int l = threadIdx.x; l <= max_label; l += blockDim.x) c += bad[(long long)fov * (max_label + 1) + l];
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

__global__ __launch_bounds__(kFillThreads) void k_fill_holes(
    const int* __restrict__ labels, int H, int W, int max_label, int min_size,
    const cpx_object* __restrict__ objects, const cpx_fov_objects* __restrict__ hdr,
    const int* __restrict__ lab2idx, int* __restrict__ fillidx, int* __restrict__ absorber,
    cpx_seg_stats* __restrict__ st) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned int* own = reinterpret_cast<unsigned int*>(smem);
  unsigned int* reach = own + kFillMaxWords;
  __shared__ int changed;
  const int fov = blockIdx.y;
  const int nobj = hdr[fov].n_objects;
  for (int k = blockIdx.x; k < nobj; k += gridDim.x) {
  const cpx_object o = objects[(long long)fov * max_label + k];
  if (o.area < min_size) continue;
  const int r0 = o.bbox[0], c0 = o.bbox[1];
  const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
  const int wpr = (bw + 31) / 32;
  const int nw = wpr * bh;
  if (nw > kFillMaxWords) {
    if (threadIdx.x == 0) atomicMax(&st[fov].overflow, 2);
    continue;
  }
  const int* lab = labels + (long long)fov * H * W;
  for (int w = threadIdx.x; w < nw; w += kFillThreads) {
    const int r = w / wpr, cw = w - r * wpr;
    unsigned int bits = 0, rb = 0;
    for (int b = 0; b < 32; ++b) {
      const int c = cw * 32 + b;
      if (c >= bw) break;
      const bool in = lab[(long long)(r0 + r) * W + c0 + c] == o.label;
      bits |= (unsigned int)in << b;
      const bool border = (r == 0 || r == bh - 1 || c == 0 || c == bw - 1);
      rb |= (unsigned int)(border && !in) << b;
    }
    own[w] = bits;
    reach[w] = rb;
  }
  __syncthreads();
  // flood the non-object cells from the bbox border (4-connectivity), in place until stable
  for (int iter = 0; iter < bh * bw + 1; ++iter) {
    if (threadIdx.x == 0) changed = 0;
    __syncthreads();
    int ch = 0;
    for (int w = threadIdx.x; w < nw; w += kFillThreads) {
      const int r = w / wpr, cw = w - r * wpr;
      const unsigned int valid = (cw == wpr - 1 && (bw & 31)) ? ((1u << (bw & 31)) - 1u) : 0xffffffffu;
      const unsigned int freeb = ~own[w] & valid;
      const unsigned int cur = reach[w];
      unsigned int nb = (cur << 1) | (cur >> 1);
      if (cw > 0) nb |= reach[w - 1] >> 31;
      if (cw < wpr - 1) nb |= reach[w + 1] << 31;
      if (r > 0) nb |= reach[w - wpr];
      if (r < bh - 1) nb |= reach[w + wpr];
      const unsigned int nxt = cur | (nb & freeb);
      if (nxt != cur) {
        reach[w] = nxt;
        ch = 1;
      }
    }
    if (ch) changed = 1;
    __syncthreads();
    if (!changed) break;
  }
  // holes: free and unreached; mark fill owner and absorbed objects
  for (int w = threadIdx.x; w < nw; w += kFillThreads) {
    const int r = w / wpr, cw = w - r * wpr;
    const unsigned int valid = (cw == wpr - 1 && (bw & 31)) ? ((1u << (bw & 31)) - 1u) : 0xffffffffu;
    unsigned int hole = ~own[w] & ~reach[w] & valid;
    while (hole) {
      const int b = __ffs(hole) - 1;
      hole &= hole - 1;
      const long long gi = (long long)(r0 + r) * W + c0 + cw * 32 + b;
      atomicMax(&fillidx[(long long)fov * H * W + gi], k + 1);
      const int l2 = lab[gi];
      if (l2 > 0 && l2 <= max_label) atomicMin(&absorber[(long long)fov * max_label + lab2idx[(long long)fov * (max_label + 1) + l2]], k);
    }
  }
  __syncthreads();
  }  // object loop
}

// one block per FOV: kept flags + sequential new labels
__global__ __launch_bounds__(1024) void k_fill_final(int max_label, int min_size,
                                                     const cpx_object* __restrict__ objects,
                                                     const cpx_fov_objects* __restrict__ hdr,
                                                     const int* __restrict__ absorber,
                                                     int* __restrict__ newlab,
                                                     cpx_seg_stats* __restrict__ st) {
  const int fov = blockIdx.x;
  const int n = hdr[fov].n_objects;
  __shared__ int wsum[16];
  __shared__ int base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int k0 = 0; k0 < n; k0 += blockDim.x) {
    const int k = k0 + threadIdx.x;
    int kept = 0;
    if (k < n) {
      const cpx_object o = objects[(long long)fov * max_label + k];
      kept = o.area >= min_size && !(absorber[(long long)fov * max_label + k] < k);
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
  if (threadIdx.x == 0) st[fov].n_final = base;
}

__global__ __launch_bounds__(kT) void k_fill_apply(int* __restrict__ labels, long long n, int max_label,
                                                   const int* __restrict__ lab2idx,
                                                   const int* __restrict__ fillidx,
                                                   const int* __restrict__ newlab) {
  const int fov = blockIdx.y;
  const int* l2i = lab2idx + (long long)fov * (max_label + 1);
  const int* nl = newlab + (long long)fov * max_label;
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
      fk[u] = (f[u] && nl[f[u] - 1]) ? f[u] : 0;
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

void axis_coeffs(int n_src, int n_dst, int* i0, int* i1, float* w) {
  const double scale = (double)n_src / (double)n_dst;
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

// host-side coefficient tables (bilinear for H,W -> Ly,Lx and nearest for Ly,Lx -> H,W)
struct SegTabs {
  AxisTab ty, tx;
  const int* ynear;
  const int* xnear;
};

int seg_tables(cpx_ctx* ctx, int H, int W, int Ly, int Lx, SegTabs& t) {
  const size_t words = (size_t)3 * Ly + 3 * Lx + H + W;
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
  const int key[6] = {H, W, Ly, Lx, 1, 0};
  bool same = ctx->seg_tab == buf;
  for (int i = 0; i < 6; ++i) same = same && ctx->seg_key[i] == key[i];
  if (same) return CPX_OK;
  std::vector<int> h(words);
  axis_coeffs(H, Ly, &h[0], &h[Ly], (float*)&h[2 * Ly]);
  axis_coeffs(W, Lx, &h[3 * Ly], &h[3 * Ly + Lx], (float*)&h[3 * Ly + 2 * Lx]);
  const double ify = 1.0 / ((double)H / (double)Ly), ifx = 1.0 / ((double)W / (double)Lx);
  for (int y = 0; y < H; ++y) h[3 * Ly + 3 * Lx + y] = std::min((int)floor(y * ify), Ly - 1);
  for (int x = 0; x < W; ++x) h[3 * Ly + 3 * Lx + H + x] = std::min((int)floor(x * ifx), Lx - 1);
  CPX_CHECK_HIP(hipMemcpyAsync(buf, h.data(), words * 4, hipMemcpyHostToDevice, ctx->stream));
  CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  for (int i = 0; i < 6; ++i) ctx->seg_key[i] = key[i];
  ctx->seg_tab = buf;
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
  CPX_REQUIRE(layout == CPX_TILE_F32_NCHW || layout == CPX_TILE_BF16_NHWC, CPX_ERR_ARG,
              "cpx_seg_tiles: bad layout %d", layout);
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

extern "C" int cpx_seg_masks(cpx_ctx* ctx, const float* yf_dev, int B, const cpx_seg_geom* geom,
                             int H, int W, int niter, double flow_threshold, int min_size,
                             int max_objects, int32_t* labels_dev, cpx_seg_stats* stats_dev) {
  CPX_REQUIRE(ctx && yf_dev && labels_dev && stats_dev, CPX_ERR_ARG, "cpx_seg_masks: null argument");
  CPX_REQUIRE(geom_ok(geom), CPX_ERR_ARG, "cpx_seg_masks: bad geometry");
  CPX_REQUIRE(B > 0 && B <= 65535 && H > 0 && W > 0 && niter >= 0 && max_objects > 0, CPX_ERR_ARG,
              "cpx_seg_masks: bad sizes");
  const int Ly = geom->Ly, Lx = geom->Lx;
  const int Lyh = Ly + 2 * kRpad, Lxh = Lx + 2 * kRpad;
  const long long n = (long long)Ly * Lx, nh = (long long)Lyh * Lxh;
  SegTabs tabs;
  int rc = seg_tables(ctx, H, W, Ly, Lx, tabs);
  if (rc) return rc;
  // ---- workspace carve (WS_SEG_DYN)
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t sz_dps = al(sizeof(float) * B * 2 * n), sz_p = sz_dps;
  const size_t sz_h = al(sizeof(int) * B * nh), sz_M = sz_h;
  const size_t sz_m0 = al(sizeof(int) * B * n);
  const size_t sz_seeds = al(sizeof(int) * (size_t)B * kMaxSeeds);
  const size_t sz_cnt = al(sizeof(int) * (size_t)B * (kMaxSeeds + 1));
  const size_t sz_mark = al((size_t)B * n);
  const size_t sz_act = al(sizeof(int) * B * n);
  const size_t total = sz_dps + sz_p + sz_h + sz_M + sz_m0 + sz_seeds + 3 * sz_cnt + sz_mark + sz_act;
  unsigned char* w = (unsigned char*)cpx_ws(ctx, WS_SEG_DYN, total);
  if (!w) return CPX_ERR_OOM;
  DynBufs d;
  d.dps = (float*)w; w += sz_dps;
  d.p = (float*)w; w += sz_p;
  d.h = (int*)w; w += sz_h;
  d.M = (unsigned int*)w; w += sz_M;
  d.m0 = (int*)w; w += sz_m0;
  d.seeds = (int*)w; w += sz_seeds;
  d.cnt = (int*)w; w += sz_cnt;
  d.first = (int*)w; w += sz_cnt;
  d.newlab = (int*)w; w += sz_cnt;
  d.mark = (unsigned char*)w; w += sz_mark;
  d.act = (int*)w; w += sz_act;
  d.st = stats_dev;
  CPX_CHECK_HIP(hipMemsetAsync(stats_dev, 0, sizeof(cpx_seg_stats) * B, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.h, 0, sz_h, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.cnt, 0, sz_cnt, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.first, 0x7f, sz_cnt, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.newlab, 0, sz_cnt, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(d.mark, 0, sz_mark, ctx->stream));
  const dim3 gp(cpx_div_up(n, kT), B), gh(cpx_div_up(nh, kT), B);
  hipLaunchKernelGGL(k_dyn_prep, gp, dim3(kT), 0, ctx->stream, yf_dev, Ly, Lx, d);
  hipLaunchKernelGGL(k_dyn_follow, gp, dim3(kT), 0, ctx->stream, Ly, Lx, niter, d);
  hipLaunchKernelGGL(k_dyn_hist, gp, dim3(kT), 0, ctx->stream, Ly, Lx, d);
  hipLaunchKernelGGL(k_seed_flags, gh, dim3(kT), 0, ctx->stream, Lyh, Lxh, d);
  hipLaunchKernelGGL(k_seed_compact, dim3(B), dim3(1024), 0, ctx->stream, Lyh, Lxh, d);
  hipLaunchKernelGGL(k_seed_expand, dim3(std::max(1, (4 * ctx->n_cu + B - 1) / B), B), dim3(kT), 0,
                     ctx->stream, Lyh, Lxh, d);
  hipLaunchKernelGGL(k_assign, gp, dim3(kT), 0, ctx->stream, Ly, Lx, d);
  hipLaunchKernelGGL(k_relabel_mark, dim3(cpx_div_up(kMaxSeeds, kT), B), dim3(kT), 0, ctx->stream, Ly, Lx, d);
  hipLaunchKernelGGL(k_relabel_scan, dim3(B), dim3(1024), 0, ctx->stream, Ly, Lx, d);
  hipLaunchKernelGGL(k_apply_newlab, gp, dim3(kT), 0, ctx->stream, Ly, Lx, d);
  CPX_CHECK_LAUNCH("cpx_seg_masks dynamics");
  // ---- object workspaces (WS_SEG_OBJ): net-res and full-res object tables share it
  const int ML = max_objects;
  const size_t sz_lst = al(sizeof(cpx_label_stats) * (size_t)B * (ML + 1));
  const size_t sz_obj = al(sizeof(cpx_object) * (size_t)B * ML);
  const size_t sz_hdr = al(sizeof(cpx_fov_objects) * (size_t)B);
  const size_t sz_bad = al((size_t)B * (ML + 1));
  const size_t sz_l2i = al(sizeof(int) * (size_t)B * (ML + 1));
  const size_t sz_abs = al(sizeof(int) * (size_t)B * ML);
  const size_t sz_nl = sz_abs;
  const size_t gscr_per = (size_t)2 * (Ly + 2) * (Lx + 2);  // doubles per FOV (oversize masks)
  const size_t sz_gscr = al(sizeof(double) * B * gscr_per);
  unsigned char* o = (unsigned char*)cpx_ws(ctx, WS_SEG_OBJ,
      sz_lst + sz_obj + sz_hdr + sz_bad + sz_l2i + sz_abs + sz_nl + sz_gscr);
  if (!o) return CPX_ERR_OOM;
  cpx_label_stats* lst = (cpx_label_stats*)o; o += sz_lst;
  cpx_object* obj = (cpx_object*)o; o += sz_obj;
  cpx_fov_objects* hdr = (cpx_fov_objects*)o; o += sz_hdr;
  unsigned char* bad = o; o += sz_bad;
  int* l2i = (int*)o; o += sz_l2i;
  int* absorber = (int*)o; o += sz_abs;
  int* newlab = (int*)o; o += sz_nl;
  double* gscr = (double*)o;
  if (flow_threshold > 0.0) {
    rc = cpx_objects(ctx, d.m0, B, Ly, Lx, ML, 0, lst, obj, hdr);
    if (rc) return rc;
    CPX_CHECK_HIP(hipMemsetAsync(bad, 0, sz_bad, ctx->stream));
    static bool attr = false;
    const size_t lds = sizeof(double) * 2 * kFlowMaxCells + sizeof(int) * 4096;
    if (!attr) {
      CPX_CHECK_HIP(hipFuncSetAttribute((const void*)k_flow_error<false>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      attr = true;
    }
    const int per_fov = std::max(1, std::min(ML, (6 * ctx->n_cu + B - 1) / B));
    hipLaunchKernelGGL(k_flow_error<false>, dim3(per_fov, B), dim3(kFlowThreads), lds, ctx->stream,
                       (const int*)d.m0, yf_dev, Ly, Lx, ML, (const cpx_object*)obj,
                       (const cpx_fov_objects*)hdr, flow_threshold, gscr, (long long)gscr_per, bad);
    hipLaunchKernelGGL(k_flow_error<true>, dim3(1, B), dim3(kFlowThreads), sizeof(int) * 4096,
                       ctx->stream, (const int*)d.m0, yf_dev, Ly, Lx, ML, (const cpx_object*)obj,
                       (const cpx_fov_objects*)hdr, flow_threshold, gscr, (long long)gscr_per, bad);
    hipLaunchKernelGGL(k_apply_bad, gp, dim3(kT), 0, ctx->stream, (int)n, ML,
                       (const unsigned char*)bad, d.m0);
    hipLaunchKernelGGL(k_count_bad, dim3(B), dim3(256), 0, ctx->stream, ML,
                       (const unsigned char*)bad, stats_dev);
    CPX_CHECK_LAUNCH("cpx_seg_masks flow error");
  }
  hipLaunchKernelGGL(k_upsample, dim3(cpx_div_up(W, kT), cpx_div_up(H, kUpRows), B), dim3(kT), 0, ctx->stream,
                     (const int*)d.m0, Ly, Lx, H, W, tabs.ynear, tabs.xnear, labels_dev);
  CPX_CHECK_LAUNCH("k_upsample");
  // ---- fill holes + remove small at full resolution
  rc = cpx_objects(ctx, labels_dev, B, H, W, ML, 0, lst, obj, hdr);
  if (rc) return rc;
  const long long N = (long long)H * W;
  int* fillidx = (int*)cpx_ws(ctx, WS_SEG_FILL, sizeof(int) * (size_t)B * N);
  if (!fillidx) return CPX_ERR_OOM;
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
    fattr = true;
  }
  hipLaunchKernelGGL(k_fill_holes, dim3(std::max(1, std::min(ML, (2 * ctx->n_cu + B - 1) / B)), B),
                     dim3(kFillThreads), flds, ctx->stream,
                     (const int*)labels_dev, H, W, ML, min_size, (const cpx_object*)obj,
                     (const cpx_fov_objects*)hdr, (const int*)l2i, fillidx, absorber, stats_dev);
  hipLaunchKernelGGL(k_fill_final, dim3(B), dim3(1024), 0, ctx->stream, ML, min_size,
                     (const cpx_object*)obj, (const cpx_fov_objects*)hdr, (const int*)absorber,
                     newlab, stats_dev);
  hipLaunchKernelGGL(k_fill_apply, dim3(std::max(1, std::min(cpx_div_up(N, kT), 4 * ctx->n_cu / B + 1)), B),
                     dim3(kT), 0, ctx->stream, labels_dev, N, ML, (const int*)l2i,
                     (const int*)fillidx, (const int*)newlab);
  CPX_CHECK_LAUNCH("cpx_seg_masks fill holes");
  return CPX_OK;
}
