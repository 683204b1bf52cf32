// image re-binning — Image_re-binning.py:12-22 `process_image_in_memory`,
// i.e. PIL Image.resize((out_w, out_h), LANCZOS) of a 16-bit ("I;16") plane, for G planes at
// once.  Same arithmetic as Pillow's separable resampler (libImaging/Resample.c), restated in
// oracle/rebin_oracle.py and pinned bit-exactly to the reference function's outputs:
//   * per-axis LANCZOS-3 weights (support 3 * max(in/out, 1)), normalised in fp64, computed on
//     the host with the same formula and libm as Pillow and uploaded once per geometry;
//   * horizontal pass first, over only the source rows the vertical pass reads, into a 16-bit
//     intermediate; then the vertical pass;
//   * each output: fp64 sum of pixel * weight in index order (separate multiply and add, this TU
//     is built with -ffp-contract=off), ROUND_UP, stored as low byte CLIP8(v % 256) and high
//     byte CLIP8(v >> 8) (Pillow's 16-bit store: values above 65535 keep their low byte).
// Not HBM-bound: Pillow's exact fp64 arithmetic (one multiply + one add per tap, ~2 * ksize /
// scale taps per source pixel) and the per-tap LDS reads of the horizontal pass bound it; the
// algorithmic traffic is 2 B per source pixel + 2 B per output pixel (the 16-bit intermediate
// of the rows the vertical pass reads makes one HBM round trip).
#include "cpx_internal.h"
#include <math.h>
#include <vector>
#include <type_traits>

namespace {

constexpr int kRT = 256;

__device__ __forceinline__ unsigned short pil_store16(double ss) {
  const int v = ss >= 0.0 ? (int)(ss + 0.5) : (int)(ss - 0.5);
  int lo = v % 256, hi = v >> 8;
  lo = lo < 0 ? 0 : (lo > 255 ? 255 : lo);
  hi = hi < 0 ? 0 : (hi > 255 ? 255 : hi);
  return (unsigned short)(lo | (hi << 8));
}

// Horizontal pass, generic (kernel sizes > 25, i.e. downscales by more than 4):
// out[g][r][xx] = resample of src row (y0 + r) along x; src [G][H][W],
// out [G][rows][ow].  A block owns kRT consecutive output columns for kRB consecutive rows:
// each thread loads its column's weights once (tap-major kT[x][xx], coalesced), and for every
// row the block first stages the source segment its columns read (one coalesced pass) in LDS,
// so each output's taps are LDS reads instead of kRB x ksize scattered 2-byte global loads.
// The sum keeps Pillow's order (x = 0 .. count-1).  KM = 0: generic rolled loop.
constexpr int kRB = 16;
constexpr int kSegW = 1024;  // LDS segment row capacity (source pixels per row)

template <int KM>
__global__ __launch_bounds__(kRT) void k_rebin_h(const unsigned short* __restrict__ src, int H,
                                                 int W, int y0, int rows, int ow,
                                                 const int2* __restrict__ bnd,
                                                 const double* __restrict__ kT, int ksize,
                                                 unsigned short* __restrict__ out) {
  __shared__ unsigned short seg[kRB * kSegW];
  const int x0 = blockIdx.x * kRT;
  const int xx = x0 + threadIdx.x;
  const bool act = xx < ow;
  const int g = blockIdx.z;
  const int r0 = blockIdx.y * kRB, nr = min(rows, r0 + kRB) - r0;
  // source span of this block's columns (bounds are monotone in xx)
  const int2 bf = bnd[x0];
  const int2 bl = bnd[min(ow, x0 + kRT) - 1];
  const int s0 = bf.x, span = bl.x + bl.y - s0;
  const bool staged = span <= kSegW;  // block-uniform
  const unsigned short* base = src + ((long long)g * H + y0 + r0) * W;
  if (staged) {
    // all rows' segments in one pass, 8 loads in flight per thread
    const int tot = nr * span;
    for (int i0 = 0; i0 < tot; i0 += 8 * kRT) {
      unsigned short v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * kRT + threadIdx.x;
        const int rr = i / span, c = i - rr * span;
        v[u] = i < tot ? base[(long long)rr * W + s0 + c] : (unsigned short)0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * kRT + threadIdx.x;
        const int rr = i / span, c = i - rr * span;
        if (i < tot) seg[rr * kSegW + c] = v[u];
      }
    }
    __syncthreads();
  }
  if (!act) return;
  const int2 b = bnd[xx];
  constexpr int KA = KM > 0 ? KM : 1;
  double kv[KA];
  if constexpr (KM > 0) {
#pragma unroll
    for (int x = 0; x < KM; ++x) kv[x] = x < b.y ? kT[(long long)x * ow + xx] : 0.0;
  }
  unsigned short* o = out + ((long long)g * rows + r0) * ow + xx;
  for (int r = 0; r < nr; ++r) {
    const unsigned short* row = base + (long long)r * W;
    const unsigned short* sr = seg + r * kSegW + (b.x - s0);
    double ss = 0.0;
    if constexpr (KM == 0) {
      for (int x = 0; x < b.y; ++x)
        ss += (double)(staged ? sr[x] : row[b.x + x]) * kT[(long long)x * ow + xx];
    } else {
      double pv[KM];
#pragma unroll
      for (int x = 0; x < KM; ++x) pv[x] = x < b.y ? (double)(staged ? sr[x] : row[b.x + x]) : 0.0;
#pragma unroll
      for (int x = 0; x < KM; ++x)
        if (x < b.y) ss += pv[x] * kv[x];
    }
    o[(long long)r * ow] = pil_store16(ss);
  }
}

// Vertical pass: out[g][yy][xx] = resample of column xx of src [G][rows][w] along y (bounds
// relative to row 0).  A row's weights are wave-uniform; each thread computes VW adjacent
// columns from VW-wide loads (VW = 4 when w % 4 == 0).
// EX: KM is the exact kernel size; every tap is read (rows clamped into the image) and taps
// past an output's count carry weight +0.0, which leaves the sum unchanged.
template <int KM, int VW, bool EX = false>
__global__ __launch_bounds__(kRT) void k_rebin_v(const unsigned short* __restrict__ src,
                                                 int rows, int w, int oh,
                                                 const int2* __restrict__ bnd,
                                                 const double* __restrict__ kk, int ksize,
                                                 unsigned short* __restrict__ out) {
  const int wv = w / VW;
  const long long per = (long long)oh * wv;
  const long long i = (long long)blockIdx.x * kRT + threadIdx.x;
  if (i >= per) return;
  const int g = blockIdx.y;
  const int yy = (int)(i / wv), xv = (int)(i - (long long)yy * wv);
  const int2 b = bnd[yy];
  const double* k = kk + (long long)yy * ksize;
  const unsigned short* col = src + ((long long)g * rows + b.x) * w + (long long)xv * VW;
  using VT = typename std::conditional<VW == 4, uint2, unsigned short>::type;
  double ss[VW];
#pragma unroll
  for (int v = 0; v < VW; ++v) ss[v] = 0.0;
  auto tap = [&](int y, int row) {
    const VT pv = *reinterpret_cast<const VT*>(col + (long long)row * w);
    const double ky = k[y];
    if constexpr (VW == 4) {
      ss[0] += (double)(pv.x & 0xffffu) * ky;
      ss[1] += (double)(pv.x >> 16) * ky;
      ss[2] += (double)(pv.y & 0xffffu) * ky;
      ss[3] += (double)(pv.y >> 16) * ky;
    } else {
      ss[0] += (double)pv * ky;
    }
  };
  if constexpr (EX) {
    const int ylast = rows - 1 - b.x;
#pragma unroll
    for (int y = 0; y < KM; ++y) tap(y, min(y, ylast));
  } else if constexpr (KM == 0) {
    for (int y = 0; y < b.y; ++y) tap(y, y);
  } else {
#pragma unroll
    for (int y = 0; y < KM; ++y)
      if (y < b.y) tap(y, y);
  }
  unsigned short* o = out + (long long)g * oh * w + (long long)yy * w + (long long)xv * VW;
  if constexpr (VW == 4) {
    uint2 st;
    st.x = (unsigned int)pil_store16(ss[0]) | ((unsigned int)pil_store16(ss[1]) << 16);
    st.y = (unsigned int)pil_store16(ss[2]) | ((unsigned int)pil_store16(ss[3]) << 16);
    *reinterpret_cast<uint2*>(o) = st;
  } else {
    o[0] = pil_store16(ss[0]);
  }
}

// Horizontal pass, kernel sizes up to 25 (scale <= 4): every wave works on its own: it owns
// 64 consecutive output columns and a run of rows, stages kHR source rows of its column span
// in a wave-private LDS strip (no block barrier: LDS ops of one wave complete in order), and
// issues the loads of the next kHR rows before resampling the current ones, so global latency
// hides behind the fp64 work.  K (the exact kernel size) is a template constant: all taps
// are read unconditionally — taps past an output's count have weight +0.0 and read finite
// pixels of the strip — which leaves Pillow's left-to-right sum unchanged.
constexpr int kHR = 4;      // rows per staging step
// strip chunks a kernel size needs: K = 2 ceil(3 scale) + 1 bounds scale <= (K - 1) / 6, so a
// 64-column group spans < 64 (K - 1) / 6 + K source pixels; + K pad
__host__ __device__ constexpr int hw_chunks(int K) { return (64 * (K - 1) / 6 + 2 * K + 63) / 64; }
constexpr int kHRows = 64;  // rows per block

template <int K>
__global__ __launch_bounds__(kRT) void k_rebin_hw(const unsigned short* __restrict__ src, int H,
                                                  int W, int y0, int rows, int ow,
                                                  const int2* __restrict__ bnd,
                                                  const double* __restrict__ kT,
                                                  unsigned short* __restrict__ out) {
  constexpr int NL = hw_chunks(K);
  __shared__ double strip[kRT / 64][kHR][NL * 64];  // fp64: each pixel converted once
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int xg = (blockIdx.x * (kRT / 64) + wv) * 64;
  if (xg >= ow) return;  // whole wave
  const int xx = min(xg + lane, ow - 1);
  const bool act = xg + lane < ow;
  const int2 bl = bnd[min(ow, xg + 64) - 1];
  const int s0 = bnd[xg].x, span = bl.x + bl.y - s0;
  const int bx = bnd[xx].x - s0;
  double kw[K];
#pragma unroll
  for (int x = 0; x < K; ++x) kw[x] = kT[(long long)x * ow + xx];
  const int g = blockIdx.z;
  const int r0 = blockIdx.y * kHRows, nr = min(kHRows, rows - r0);
  const unsigned short* base = src + ((long long)g * H + y0 + r0) * W + s0;
  unsigned short* o = out + ((long long)g * rows + r0) * ow + xx;
  // strip columns past the span load the span's last pixel (in bounds, finite)
  int col[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) col[l] = min(l * 64 + lane, span - 1);
  unsigned short v[kHR][NL];
  auto load = [&](int r) {
#pragma unroll
    for (int rr = 0; rr < kHR; ++rr) {
      const unsigned short* rp = base + (long long)min(r + rr, nr - 1) * W;
#pragma unroll
      for (int l = 0; l < NL; ++l) v[rr][l] = rp[col[l]];
    }
  };
  load(0);
  double(*st)[NL * 64] = strip[wv];
  for (int r = 0; r < nr; r += kHR) {
#pragma unroll
    for (int rr = 0; rr < kHR; ++rr)
#pragma unroll
      for (int l = 0; l < NL; ++l) st[rr][l * 64 + lane] = (double)v[rr][l];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (r + kHR < nr) load(r + kHR);
    double ss[kHR];
#pragma unroll
    for (int rr = 0; rr < kHR; ++rr) ss[rr] = 0.0;
#pragma unroll
    for (int x = 0; x < K; ++x)  // kHR independent chains, each in Pillow's tap order
#pragma unroll
      for (int rr = 0; rr < kHR; ++rr) ss[rr] += st[rr][bx + x] * kw[x];
#pragma unroll
    for (int rr = 0; rr < kHR; ++rr)
      if (act && r + rr < nr) o[(long long)(r + rr) * ow] = pil_store16(ss[rr]);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
}

double lanczos3(double x) {
  auto sinc = [](double t) {
    if (t == 0.0) return 1.0;
    t = t * M_PI;
    return sin(t) / t;
  };
  if (-3.0 <= x && x < 3.0) return sinc(x) * sinc(x / 3.0);
  return 0.0;
}

// Pillow precompute_coeffs for one axis: bounds (xmin, count) and ksize weights per output
int precompute(int in_size, int out_size, std::vector<int>& bounds, std::vector<double>& kk) {
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 3.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  bounds.assign(2 * (size_t)out_size, 0);
  kk.assign((size_t)out_size * ksize, 0.0);
  const double ss = 1.0 / filterscale;
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    double* k = &kk[(size_t)xx * ksize];
    for (int x = 0; x < xmax; ++x) {
      const double w = lanczos3((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    bounds[2 * (size_t)xx] = xmin;
    bounds[2 * (size_t)xx + 1] = xmax;
  }
  return ksize;
}

}  // namespace

extern "C" int cpx_rebin_u16(cpx_ctx* ctx, const uint16_t* src_dev, int G, int H, int W,
                             int out_h, int out_w, uint16_t* dst_dev) {
  CPX_REQUIRE(ctx && src_dev && dst_dev, CPX_ERR_ARG, "cpx_rebin_u16: null argument");
  CPX_REQUIRE(G > 0 && G <= 65535 && H > 0 && W > 0 && out_h > 0 && out_w > 0, CPX_ERR_ARG,
              "cpx_rebin_u16: bad sizes");
  const bool need_h = out_w != W, need_v = out_h != H;
  if (!need_h && !need_v) {
    CPX_CHECK_HIP(hipMemcpyAsync(dst_dev, src_dev, sizeof(uint16_t) * (size_t)G * H * W,
                                 hipMemcpyDeviceToDevice, ctx->stream));
    return CPX_OK;
  }
  std::vector<int> bh, bv;
  std::vector<double> kh, kv;
  const int ksh = precompute(W, out_w, bh, kh);
  const int ksv = precompute(H, out_h, bv, kv);
  {  // horizontal weights tap-major: kT[x][xx]
    std::vector<double> t((size_t)ksh * out_w);
    for (int xx = 0; xx < out_w; ++xx)
      for (int x = 0; x < ksh; ++x) t[(size_t)x * out_w + xx] = kh[(size_t)xx * ksh + x];
    kh.swap(t);
  }
  // rows of the source the vertical pass reads; vertical bounds made relative to the first
  const int y0 = need_v ? bv[0] : 0;
  const int y1 = need_v ? bv[2 * (size_t)(out_h - 1)] + bv[2 * (size_t)(out_h - 1) + 1] : H;
  if (need_h && need_v)
    for (int i = 0; i < out_h; ++i) bv[2 * (size_t)i] -= y0;
  // coefficient tables: [bh][bv][kh][kv], uploaded when the geometry changes
  const size_t nbh = bh.size() * sizeof(int), nbv = bv.size() * sizeof(int);
  const size_t nkh = kh.size() * sizeof(double), nkv = kv.size() * sizeof(double);
  const size_t o_bv = (nbh + 255) / 256 * 256, o_kh = o_bv + (nbv + 255) / 256 * 256;
  const size_t o_kv = o_kh + (nkh + 255) / 256 * 256, tab_bytes = o_kv + nkv;
  unsigned char* tab = (unsigned char*)cpx_ws(ctx, WS_REBIN, tab_bytes);
  if (!tab) return CPX_ERR_OOM;
  const int key[4] = {W, out_w, H, out_h};
  // the vertical bounds depend on whether a horizontal pass runs; H == out_h only happens
  // together with need_h, so (W, out_w, H, out_h) identifies the tables
  if (!std::equal(key, key + 4, ctx->rebin_key) || ctx->rebin_gen != ctx->ws_gen[WS_REBIN]) {
    CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));  // earlier launches may read the old tables
    CPX_CHECK_HIP(hipMemcpy(tab, bh.data(), nbh, hipMemcpyHostToDevice));
    CPX_CHECK_HIP(hipMemcpy(tab + o_bv, bv.data(), nbv, hipMemcpyHostToDevice));
    CPX_CHECK_HIP(hipMemcpy(tab + o_kh, kh.data(), nkh, hipMemcpyHostToDevice));
    CPX_CHECK_HIP(hipMemcpy(tab + o_kv, kv.data(), nkv, hipMemcpyHostToDevice));
    std::copy(key, key + 4, ctx->rebin_key);
    ctx->rebin_gen = ctx->ws_gen[WS_REBIN];
  }
  const int2* dbh = (const int2*)tab;
  const int2* dbv = (const int2*)(tab + o_bv);
  const double* dkh = (const double*)(tab + o_kh);
  const double* dkv = (const double*)(tab + o_kv);
  const unsigned short* vsrc = (const unsigned short*)src_dev;
  int vrows = H;
  if (need_h) {
    const int rows = y1 - y0;
    unsigned short* out = (unsigned short*)dst_dev;
    if (need_v) {
      out = (unsigned short*)cpx_ws(ctx, WS_REBIN_TMP, sizeof(uint16_t) * (size_t)G * rows * out_w);
      if (!out) return CPX_ERR_OOM;
    }
    // strip chunks of the widest 64-column group (+ K pad for the unconditional taps)
    int nl = 0;
    for (int a = 0; a < out_w; a += 64) {
      const int e = std::min(out_w, a + 64) - 1;
      nl = std::max(nl, cpx_div_up(bh[2 * (size_t)e] + bh[2 * (size_t)e + 1] - bh[2 * (size_t)a] + ksh, 64));
    }
    if (ksh <= 25 && nl <= hw_chunks(ksh)) {
      CPX_REQUIRE(cpx_div_up(rows, kHRows) <= 65535, CPX_ERR_ARG, "cpx_rebin_u16: plane too large");
      const dim3 grid(cpx_div_up(out_w, kRT), cpx_div_up(rows, kHRows), G);
#define CPX_REBIN_HW(KK)                                                                       \
  case KK:                                                                                     \
    hipLaunchKernelGGL(k_rebin_hw<KK>, grid, dim3(kRT), 0, ctx->stream,                         \
                       (const unsigned short*)src_dev, H, W, y0, rows, out_w, dbh, dkh, out);     \
    break;
      switch (ksh) {
        CPX_REBIN_HW(7) CPX_REBIN_HW(9) CPX_REBIN_HW(11) CPX_REBIN_HW(13) CPX_REBIN_HW(15)
        CPX_REBIN_HW(17) CPX_REBIN_HW(19) CPX_REBIN_HW(21) CPX_REBIN_HW(23) CPX_REBIN_HW(25)
        default: CPX_REQUIRE(false, CPX_ERR_ARG, "cpx_rebin_u16: kernel size");
      }
#undef CPX_REBIN_HW
      CPX_CHECK_LAUNCH("k_rebin_hw");
    } else {
    CPX_REQUIRE(cpx_div_up(rows, kRB) <= 65535, CPX_ERR_ARG, "cpx_rebin_u16: plane too large");
    const dim3 grid(cpx_div_up(out_w, kRT), cpx_div_up(rows, kRB), G);
#define CPX_REBIN_H(KM)                                                                        \
  hipLaunchKernelGGL(k_rebin_h<KM>, grid, dim3(kRT), 0, ctx->stream,                          \
                     (const unsigned short*)src_dev, H, W, y0, rows, out_w, dbh, dkh, ksh, out)
    if (ksh <= 32) CPX_REBIN_H(32);
    else CPX_REBIN_H(0);
#undef CPX_REBIN_H
    CPX_CHECK_LAUNCH("k_rebin_h");
    }
    vsrc = out;
    vrows = rows;
  }
  if (need_v) {
    const int w = need_h ? out_w : W;
    const bool v4 = (w % 4) == 0 && ((uintptr_t)vsrc % 8) == 0 && ((uintptr_t)dst_dev % 8) == 0;
    const long long per = (long long)out_h * (v4 ? w / 4 : w);
    CPX_REQUIRE((per + kRT - 1) / kRT < (1LL << 31), CPX_ERR_ARG, "cpx_rebin_u16: plane too large");
    const dim3 grid((unsigned)((per + kRT - 1) / kRT), G);
#define CPX_REBIN_V(KM, VW)                                                                    \
  hipLaunchKernelGGL((k_rebin_v<KM, VW>), grid, dim3(kRT), 0, ctx->stream, vsrc, vrows, w,    \
                     out_h, dbv, dkv, ksv, (unsigned short*)dst_dev)
#define CPX_REBIN_VX(KK)                                                                       \
  case KK:                                                                                     \
    if (v4)                                                                                    \
      hipLaunchKernelGGL((k_rebin_v<KK, 4, true>), grid, dim3(kRT), 0, ctx->stream, vsrc, vrows, \
                         w, out_h, dbv, dkv, ksv, (unsigned short*)dst_dev);                   \
    else                                                                                       \
      hipLaunchKernelGGL((k_rebin_v<KK, 1, true>), grid, dim3(kRT), 0, ctx->stream, vsrc, vrows, \
                         w, out_h, dbv, dkv, ksv, (unsigned short*)dst_dev);                   \
    break;
    switch (ksv) {  // exact kernel sizes up to 25 (scale <= 4)
      CPX_REBIN_VX(7) CPX_REBIN_VX(9) CPX_REBIN_VX(11) CPX_REBIN_VX(13) CPX_REBIN_VX(15)
      CPX_REBIN_VX(17) CPX_REBIN_VX(19) CPX_REBIN_VX(21) CPX_REBIN_VX(23) CPX_REBIN_VX(25)
      default:
        if (v4) {
          if (ksv <= 32) CPX_REBIN_V(32, 4);
          else CPX_REBIN_V(0, 4);
        } else {
          if (ksv <= 32) CPX_REBIN_V(32, 1);
          else CPX_REBIN_V(0, 1);
        }
    }
#undef CPX_REBIN_VX
#undef CPX_REBIN_V
    CPX_CHECK_LAUNCH("k_rebin_v");
  }
  return CPX_OK;
}
