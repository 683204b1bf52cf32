// a8 fast path: AreaShape + Intensity + Texture for objects whose bbox fits in LDS (the common
// case; larger objects fall back to k_shape / k_intensity_texture in k_features.hip with the same
// arithmetic).  Same definitions and bit-identical results as the fallback; see k_features.hip.
//
// Design:
//  * texture in two phases: phase A (high occupancy, one block per object-channel) makes one
//    coalesced pass over the bbox (2-D thread layout, 4 rows of loads in flight per thread)
//    for the intensity statistics and the scale_to_8bit range, then writes the 8-bit masked
//    crop to a global scratch slot (offsets from a per-FOV scan); phase B (one 1024-thread
//    block per CU with a 128 KiB LDS pair table) copies the crop to LDS and runs the four GLCM
//    angles from LDS: exact u32 pair sums in registers per run of equal keys, ASM from the
//    counts the table's atomics return, background (0,0) pairs by branch; DPP wave sums.
//  * AreaShape: bbox + 2-pixel margin bitmask in LDS; the 4-neighbour border and the
//    Benkrid-Crookes perimeter code are evaluated bit-parallel, moments are exact int64 sums.
#include "cpx_internal.h"
#include <math.h>

namespace {

typedef __int128 i128;

// Development-only phase timer of k_tex_glcm (build with -DCPX_GLCM_PROF; tools/tex_bench.py).
#ifdef CPX_GLCM_PROF
__device__ unsigned long long g_glcm_prof[8];
#define GLCM_MARK(k, pt)                                    \
  do {                                                      \
    if (threadIdx.x == 0) {                                 \
      const long long t_ = clock64();                       \
      atomicAdd(&g_glcm_prof[k], (unsigned long long)(t_ - *(pt))); \
      *(pt) = t_;                                           \
    }                                                       \
  } while (0)
#else
#define GLCM_MARK(k, pt) \
  do {                   \
  } while (0)
#endif

constexpr int kTT = 1024;            // GLCM block: 32 rows x 32 columns (16 waves)
constexpr int kRows = kTT / 32;
constexpr int kTabW = 32768;         // packed u16 pair counters (128 KiB)
constexpr int kCrop = kFastCropPx;   // u8 crop capacity (pixels)
constexpr int kMaskW = kFastMaskWords;  // membership bitmask words (bh * ceil(bw/32))
constexpr int kNW = kTT / 64;

__device__ __forceinline__ int quantize(float v, bool in, float mn, float rng, bool flat) {
  const float m = v * (in ? 1.0f : 0.0f);
  if (flat) return 0;
  float x = m - mn;  // scale_to_8bit: 255.0 * (x - min) / (max - min), fp32, truncation
  x = 255.0f * x;
  x = x / rng;
  return (int)(unsigned char)(int)x;
}

__device__ __forceinline__ bool mask_bit(const unsigned int* m, int wpr, int r, int c) {
  return (m[r * wpr + (c >> 5)] >> (c & 31)) & 1u;
}

// Wave-wide sum of a u32 on the VALU/DPP path (no LDS traffic); the result is wave-uniform.
// row_shr 1,2,4,8 = inclusive scan within each row of 16 lanes; row_bcast:15 / row_bcast:31
// carry the row totals upward, so lane 63 holds the wave total.
__device__ __forceinline__ unsigned int wave_sum_u32(unsigned int v) {
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return (unsigned int)__builtin_amdgcn_readlane((int)v, 63);
}

// The same scan for a u64 (both halves moved by DPP, 64-bit adds): no LDS round trips, where
// the generic __shfl_xor sum costs twelve ds_bpermute.
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#define CPX_U64_DPP_STEP(CTRL, ROWMASK)                                                         \
  {                                                                                            \
    const unsigned int lo_ = (unsigned int)__builtin_amdgcn_update_dpp(0, (int)(unsigned int)v, \
                                                                       CTRL, ROWMASK, 0xf, false); \
    const unsigned int hi_ = (unsigned int)__builtin_amdgcn_update_dpp(                        \
        0, (int)(unsigned int)(v >> 32), CTRL, ROWMASK, 0xf, false);                           \
    v += ((unsigned long long)hi_ << 32) | lo_;                                                \
  }
  CPX_U64_DPP_STEP(0x111, 0xf)
  CPX_U64_DPP_STEP(0x112, 0xf)
  CPX_U64_DPP_STEP(0x114, 0xf)
  CPX_U64_DPP_STEP(0x118, 0xf)
  CPX_U64_DPP_STEP(0x142, 0xa)
  CPX_U64_DPP_STEP(0x143, 0xc)
#undef CPX_U64_DPP_STEP
  const unsigned int lo = (unsigned int)__builtin_amdgcn_readlane((int)(unsigned int)v, 63);
  const unsigned int hi = (unsigned int)__builtin_amdgcn_readlane((int)(unsigned int)(v >> 32), 63);
  return ((unsigned long long)hi << 32) | lo;
}

// GLCM of one (object, channel) item: skimage graycomatrix offsets (dr, dc) for angles
// 0, pi/4, pi/2, 3pi/4 at distance 3, symmetric=False, normed, then greycoprops.
//  1. count (per angle): runs of equal keys along a thread's segment are added at once to their
//     packed-u16 counter in a 64K-key LDS table (background pairs (0, 0) only counted in a
//     register); each run also adds its exact u32 sums of c*i, c*j, c*i^2, c*j^2, c*i*j, c*d^2,
//     c*d (d = |i-j|) and a u64 fixed-point c * round(2^48 / (1 + d^2)) for homogeneity (per-term
//     relative error <= 1.2e-10), and ASM = sum c^2 grows by cnt * (2 old + cnt) from the counter
//     value its atomic returns — so counts are never read back.  With at most 65535 pairs per
//     item every total fits (sum c*d^2 <= 65535 * 255^2 < 2^32, sum c^2 <= 65535^2 < 2^32);
//  2. clear the table with 16-byte stores;
//  3. finish (once per item, all four angles): DPP wave sums, one cross-wave pass through the
//     (by then all-zero) table, greycoprops on four lanes.  All sums are integer, so the result
//     never depends on the order in which pairs or runs were visited.
struct HomTable {
  unsigned long long m[256];
  constexpr HomTable() : m() {
    for (int d = 0; d < 256; ++d) m[d] = (unsigned long long)(281474976710656.0 / (1.0 + (double)(d * d)) + 0.5);
  }
};
__constant__ HomTable kHom = HomTable();
constexpr double kHomScale = 1.0 / 281474976710656.0;  // 2^-48

struct GlcmAcc {
  unsigned int si, sj, sii, sjj, sij, asq, con, dis, bg;
  unsigned long long hom;
};
constexpr int kAccW = 11;  // 32-bit words per angle in the cross-wave reduction

__device__ __forceinline__ void glcm_key(unsigned int c, unsigned int i, unsigned int j, GlcmAcc& A) {
  const unsigned int ci = c * i, cj = c * j;
  const unsigned int d = i > j ? i - j : j - i;
  A.si += ci;
  A.sj += cj;
  A.sii += ci * i;
  A.sjj += cj * j;
  A.sij += ci * j;
  A.asq += c * c;
  A.con += c * d * d;
  A.dis += c * d;
  A.hom += (unsigned long long)c * kHom.m[d];
}

// Add a run of cnt pairs of one key: the pair sums of the run go straight into the registers
// (c*i, c*j, ..., c * hom(d) from the LDS copy of the homogeneity table), and ASM = sum c_k^2
// grows by (old + cnt)^2 - old^2 = cnt * (2*old + cnt) from the counter value the atomic returns,
// so the counts never have to be read back: the table is only cleared after the angle.
__device__ __forceinline__ void glcm_flush(unsigned int* tab, const unsigned long long* hom,
                                           unsigned int key, unsigned int cnt, GlcmAcc& A) {
  const unsigned int sh = (key & 1u) << 4;
  const unsigned int old = (atomicAdd(&tab[key >> 1], cnt << sh) >> sh) & 0xffffu;
  const unsigned int i = key >> 8, j = key & 255u;
  const unsigned int ci = cnt * i, cj = cnt * j;
  const unsigned int d = i > j ? i - j : j - i;
  A.si += ci;
  A.sj += cj;
  A.sii += ci * i;
  A.sjj += cj * j;
  A.sij += ci * j;
  A.asq += cnt * (2u * old + cnt);
  A.con += cnt * d * d;
  A.dis += cnt * d;
  A.hom += (unsigned long long)cnt * hom[d];
}

// Phase 1 of one angle over an 8-bit crop in LDS (or the global scratch slot); returns this
// thread's background-pair count.
template <bool LDS_CROP>
__device__ unsigned int glcm_count(const unsigned char* __restrict__ crop, unsigned int* tab,
                                   const unsigned long long* hom, GlcmAcc& A, int bh, int bw, int dr,
                                   int dc) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rend = bh - dr;  // dr >= 0
  const int cbeg = dc >= 0 ? 0 : -dc, cend = dc >= 0 ? bw - dc : bw;
  const long long T = (rend > 0 && cend > cbeg) ? (long long)rend * (cend - cbeg) : 0;
  // Thread = one contiguous run of the angle's T pairs (row-major); the 64 lanes of a wave
  // take runs T/64 apart (segment lane*16 + wave), so one wave-instruction touches unrelated
  // keys, and a lane adds a whole run of equal keys at once: LDS atomics to one address are
  // serialised (~2 cycles per lane), and smooth crops repeat keys along a row.
  unsigned int bg = 0;
  const int Wc = cend - cbeg;
  const int seg = (int)((T + kTT - 1) / kTT);
  int p = (lane * kNW + wid) * seg;
  const int pend = (int)min((long long)p + seg, T);
  unsigned int cur = 0, cnt = 0;
  if (p < pend) {
    const int r = p / Wc, c = p - r * Wc;
    const unsigned char* a = crop + r * bw + cbeg + c;
    const unsigned char* b = a + dr * bw + dc;
    int left = Wc - c;  // pairs left in this row
    for (; p < pend; p += 4) {
      // four keys loaded ahead (the 8 byte loads issue together), then consumed in order
      unsigned int key[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        key[u] = ((unsigned int)*a << 8) | (unsigned int)*b;
        const bool wrap = --left == 0;
        a += wrap ? (bw - Wc + 1) : 1;
        b += wrap ? (bw - Wc + 1) : 1;
        left = wrap ? Wc : left;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (p + u >= pend) break;
        if (key[u] != cur) {
          if (cur) glcm_flush(tab, hom, cur, cnt, A);
          else bg += cnt;
          cur = key[u];
          cnt = 0;
        }
        ++cnt;
      }
    }
  }
  if (cur) glcm_flush(tab, hom, cur, cnt, A);
  else bg += cnt;
  return bg;
}

// Phase 2 of one angle: clear the table for the next angle with 16-byte stores.
__device__ __forceinline__ void glcm_clear(unsigned int* tab) {
  uint4* t4 = reinterpret_cast<uint4*>(tab);
#pragma unroll
  for (int x = threadIdx.x; x < kTabW / 4; x += kTT) t4[x] = uint4{0u, 0u, 0u, 0u};
}

// Phase 3: reduce the four angles' sums over the block and write greycoprops.  `red` is
// kNW * 4 * kAccW words of the all-zero table; wave 0 zeroes them again before returning.
__device__ void glcm_finish(const GlcmAcc (&A)[4], unsigned int* red, int bh, int bw,
                            double* __restrict__ out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const unsigned int w[9] = {A[a].si, A[a].sj, A[a].sii, A[a].sjj, A[a].sij,
                               A[a].asq, A[a].con, A[a].dis, A[a].bg};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const unsigned int t = wave_sum_u32(w[k]);
      if (lane == 0) red[(wid * 4 + a) * kAccW + k] = t;
    }
    const unsigned long long hs = wave_sum_u64(A[a].hom);
    if (lane == 0) {
      red[(wid * 4 + a) * kAccW + 9] = (unsigned int)hs;
      red[(wid * 4 + a) * kAccW + 10] = (unsigned int)(hs >> 32);
    }
  }
  __syncthreads();
  if (wid == 0) {
    if (lane < 4) {
      const int a = lane;
      const int dr = a == 0 ? 0 : a == 2 ? 3 : 2;
      const int dc = a == 0 ? 3 : a == 1 ? 2 : a == 2 ? 0 : -2;
      const int rend = bh - dr;
      const int cbeg = dc >= 0 ? 0 : -dc, cend = dc >= 0 ? bw - dc : bw;
      const long long T = (rend > 0 && cend > cbeg) ? (long long)rend * (cend - cbeg) : 0;
      unsigned int v[9] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      unsigned long long hs = 0;
      for (int x = 0; x < kNW; ++x) {
        const unsigned int* r = red + (x * 4 + a) * kAccW;
#pragma unroll
        for (int k = 0; k < 9; ++k) v[k] += r[k];
        hs += (unsigned long long)r[9] | ((unsigned long long)r[10] << 32);
      }
      const unsigned int tsi = v[0], tsj = v[1], tsii = v[2], tsjj = v[3], tsij = v[4];
      const unsigned int tas = v[5], ct = v[6], dt = v[7], nbg = v[8];
      hs += (unsigned long long)nbg * kHom.m[0];  // background pairs: d = 0
      double con = 0.0, dis = 0.0, hom = 0.0, asmv = 0.0, ene = 0.0, cor = 1.0;
      if (T > 0) {
        const double Td = (double)T;
        con = (double)ct / Td;
        dis = (double)dt / Td;
        hom = ((double)hs * kHomScale) / Td;
        asmv = (double)((unsigned long long)tas + (unsigned long long)nbg * nbg) / (Td * Td);
        ene = sqrt(asmv);
        const long long vi = T * (long long)tsii - (long long)tsi * tsi;
        const long long vj = T * (long long)tsjj - (long long)tsj * tsj;
        const long long cv = T * (long long)tsij - (long long)tsi * tsj;
        const double sdi = sqrt((double)vi) / Td, sdj = sqrt((double)vj) / Td;
        cor = (sdi < 1e-15 || sdj < 1e-15) ? 1.0 : ((double)cv / (Td * Td)) / (sdi * sdj);
      }
      double* o = out + a * CPX_N_TEX_PROPS;
      o[CPX_TEX_CONTRAST] = con;
      o[CPX_TEX_DISSIMILARITY] = dis;
      o[CPX_TEX_HOMOGENEITY] = hom;
      o[CPX_TEX_ASM] = asmv;
      o[CPX_TEX_ENERGY] = ene;
      o[CPX_TEX_CORRELATION] = cor;
    }
    // re-zero the reduction words (the table must be all-zero for the next item)
    for (int x = lane; x < kNW * 4 * kAccW; x += 64) red[x] = 0u;
  }
}

// ---------------------------------------------------------------------------------------------
// Phase A (high occupancy, one block per (object, channel) item): intensity features and the
// scale_to_8bit range from one coalesced pass over the bbox, then the 8-bit masked crop is
// written to a global scratch slot (L2-resident until phase B reads it).
constexpr int kAT = 256;  // 8 rows x 32 columns

__global__ __launch_bounds__(kAT) void k_tex_stage(const int* __restrict__ labels,
                                                  const float* __restrict__ corr, int C, int H,
                                                  int W, int max_label, int F,
                                                  const cpx_object* __restrict__ objects,
                                                  const cpx_fov_objects* __restrict__ hdr,
                                                  const long long* __restrict__ crop_off,
                                                  unsigned char* __restrict__ scratch,
                                                  long long scratch_per_fov,
                                                  double* __restrict__ feats) {
  __shared__ double sd[2][kAT / 64];
  __shared__ long long sn[kAT / 64];
  __shared__ float sf[4][kAT / 64];
  const int fov = blockIdx.y;
  const int n_items = hdr[fov].n_objects * C;
  const int ty = threadIdx.x >> 5, tx = threadIdx.x & 31, lane = threadIdx.x & 63,
            wid = threadIdx.x >> 6;
  const long long N = (long long)H * W;
  const int* lab = labels + (long long)fov * N;
  for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
    const int k = item / C, ch = item - k * C;
    const long long off = crop_off[(long long)fov * max_label + k];
    if (off < 0) continue;  // not staged: fallback kernel
    const cpx_object o = objects[(long long)fov * max_label + k];
    const int r0 = o.bbox[0], c0 = o.bbox[1];
    const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
    const int L = o.label;
    const float* img = corr + ((long long)fov * C + ch) * N + (long long)r0 * W + c0;
    const int* lb = lab + (long long)r0 * W + c0;
    long long n = 0;
    double sm = 0.0, ss = 0.0;
    float omin = INFINITY, omax = -INFINITY, mmin = INFINITY, mmax = -INFINITY;
    for (int rb = 0; rb < bh; rb += 32) {  // 4 rows in flight per thread
      float vv[4];
      int ll[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + ty + 8 * u;
        vv[u] = 0.0f;
        ll[u] = -1;
        (void)r;
      }
      for (int c = tx; c < bw; c += 32) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = rb + ty + 8 * u;
          if (r < bh) {
            vv[u] = img[(long long)r * W + c];
            ll[u] = lb[(long long)r * W + c];
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = rb + ty + 8 * u;
          if (r >= bh) continue;
          const float v = vv[u];
          const bool in = ll[u] == L;
          const float m = v * (in ? 1.0f : 0.0f);
          mmin = fminf(mmin, m);
          mmax = fmaxf(mmax, m);
          if (in) {
            n += 1;
            sm += (double)v;
            ss += (double)v * (double)v;
            omin = fminf(omin, v);
            omax = fmaxf(omax, v);
          }
        }
      }
    }
    n = wave_sum(n);
    sm = wave_sum(sm);
    ss = wave_sum(ss);
    omin = wave_min(omin);
    omax = wave_max(omax);
    mmin = wave_min(mmin);
    mmax = wave_max(mmax);
    if (lane == 0) {
      sn[wid] = n;
      sd[0][wid] = sm;
      sd[1][wid] = ss;
      sf[0][wid] = omin;
      sf[1][wid] = omax;
      sf[2][wid] = mmin;
      sf[3][wid] = mmax;
    }
    __syncthreads();
    n = 0;
    sm = ss = 0.0;
    omin = mmin = INFINITY;
    omax = mmax = -INFINITY;
    for (int w = 0; w < kAT / 64; ++w) {
      n += sn[w];
      sm += sd[0][w];
      ss += sd[1][w];
      omin = fminf(omin, sf[0][w]);
      omax = fmaxf(omax, sf[1][w]);
      mmin = fminf(mmin, sf[2][w]);
      mmax = fmaxf(mmax, sf[3][w]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double* f = feats + ((long long)fov * max_label + k) * F + CPX_N_SHAPE +
                  (long long)ch * CPX_FEATURES_PER_CHANNEL;
      const double mean = n ? sm / (double)n : 0.0;
      double var = n ? (ss - sm * mean) / (double)n : 0.0;
      if (var < 0.0) var = 0.0;
      f[CPX_INT_INTEGRATED] = sm;
      f[CPX_INT_MEAN] = mean;
      f[CPX_INT_STD] = sqrt(var);
      f[CPX_INT_MIN] = (double)omin;
      f[CPX_INT_MAX] = (double)omax;
    }
    const float rng = mmax - mmin;
    const bool flat = !(mmax != mmin);
    unsigned char* dst = scratch + (long long)fov * scratch_per_fov + off +
                         (long long)ch * (((long long)bh * bw + 15) / 16 * 16);
    // the crop is written as a flat row-major byte array, four pixels per thread per step
    // packed into one 32-bit store (slots are 16-byte aligned): all lanes busy whatever bw is,
    // and a wave stores 256 contiguous bytes instead of 64 single bytes
    const int nb = bh * bw;
    for (int f0 = 4 * threadIdx.x; f0 < nb; f0 += 4 * kAT) {
      int r = f0 / bw, c = f0 - r * bw;
      float vv[4];
      int ll[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        vv[u] = 0.0f;
        ll[u] = -1;
        if (f0 + u < nb) {
          vv[u] = img[(long long)r * W + c];
          ll[u] = lb[(long long)r * W + c];
        }
        if (++c == bw) {
          c = 0;
          ++r;
        }
      }
      unsigned int word = 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        word |= (unsigned int)quantize(vv[u], ll[u] == L, mmin, rng, flat) << (8 * u);
      *reinterpret_cast<unsigned int*>(dst + f0) = word;
    }
  }
}

struct GlcmItem {
  int fov, k, ch, bh, bw, nb;  // nb <= 0: nothing to do (no slot, > 65535 px, or queue drained)
  const unsigned char* src;
};

// Work queue of k_tex_glcm (thread 0 only): items of FOV f are handed out by one atomic
// counter per FOV; a block starts on its own FOV and moves to the next FOV when that queue is
// drained, so blocks of light FOVs help heavy ones and the launch ends within about one item
// of balance.  Returns fov * 2^20 + item, or -1 when every queue has been drained (each block
// visits each FOV at most once, so every block reaches the exit).
__device__ __forceinline__ int glcm_grab(int& f, int& visited, int B, int C,
                                         const cpx_fov_objects* __restrict__ hdr,
                                         int* __restrict__ next) {
  while (visited < B) {
    const int n_items = hdr[f].n_objects * C;
    const int v = atomicAdd(&next[f], 1);
    if (v < n_items) return (f << 20) | v;
    ++visited;
    f = f + 1 == B ? 0 : f + 1;
  }
  return -1;
}

constexpr int kPre = (kCrop / 16 + kTT - 1) / kTT;  // uint4 prefetch registers per thread
static_assert(kPre == 2, "glcm_prefetch holds two uint4 per thread");

__device__ __forceinline__ GlcmItem glcm_item(int code, int C, int max_label,
                                              const cpx_object* objects,
                                              const long long* crop_off,
                                              const unsigned char* scratch,
                                              long long scratch_per_fov) {
  GlcmItem g{0, 0, 0, 0, 0, 0, nullptr};
  if (code < 0) return g;
  const int fov = code >> 20, item = code & 0xfffff;
  g.fov = fov;
  g.k = item / C;
  g.ch = item - g.k * C;
  const long long off = crop_off[(long long)fov * max_label + g.k];
  const cpx_object& o = objects[(long long)fov * max_label + g.k];
  g.bh = o.bbox[2] - o.bbox[0];
  g.bw = o.bbox[3] - o.bbox[1];
  const int nb = g.bh * g.bw;
  if (off < 0 || nb > 65535) return g;  // u32 / packed u16 sums: fallback kernel
  g.nb = nb;
  g.src = scratch + (long long)fov * scratch_per_fov + off + (long long)g.ch * ((nb + 15) / 16 * 16);
  return g;
}

__device__ __forceinline__ void glcm_prefetch(const GlcmItem& g, uint4& p0, uint4& p1) {
  if (g.nb <= 0 || g.nb > kCrop) return;
  const int n16 = (g.nb + 15) / 16;
  const uint4* s16 = reinterpret_cast<const uint4*>(g.src);
  if ((int)threadIdx.x < n16) p0 = s16[threadIdx.x];
  if ((int)threadIdx.x + kTT < n16) p1 = s16[threadIdx.x + kTT];
}

// Phase B (one 1024-thread block per CU, 128 KiB LDS pair table): GLCM of staged crops.
__global__ __launch_bounds__(kTT) void k_tex_glcm(int C, int max_label, int F,
                                                 const cpx_object* __restrict__ objects,
                                                 const cpx_fov_objects* __restrict__ hdr,
                                                 const long long* __restrict__ crop_off,
                                                 const unsigned char* __restrict__ scratch,
                                                 long long scratch_per_fov,
                                                 int* __restrict__ glcm_next,
                                                 double* __restrict__ feats) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_code[2];  // queue codes (see glcm_grab), double-buffered by iteration parity
  unsigned int* tab = reinterpret_cast<unsigned int*>(smem);
  unsigned long long* hom = reinterpret_cast<unsigned long long*>(tab + kTabW);  // 2 KiB
  unsigned char* crop = reinterpret_cast<unsigned char*>(hom + 256);
  const int B = gridDim.y;
  int q_fov = blockIdx.y, q_visited = 0;  // thread 0's queue position
  for (int x = threadIdx.x; x < kTabW; x += kTT) tab[x] = 0u;
  if (threadIdx.x < 256) hom[threadIdx.x] = kHom.m[threadIdx.x];
  if (threadIdx.x == 0) {
    s_code[0] = glcm_grab(q_fov, q_visited, B, C, hdr, glcm_next);
    s_code[1] = glcm_grab(q_fov, q_visited, B, C, hdr, glcm_next);
  }
  __syncthreads();
  // software pipeline: the next item's metadata and LDS-sized crop are loaded into registers
  // while the current item runs its four angles (the crop was written by k_tex_stage, possibly
  // on another XCD, so the loads are HBM/MALL latency); thread 0 grabs the item after that one
  // from the queue during the current item, so the atomic's latency is hidden too.
  GlcmItem cur = glcm_item(s_code[0], C, max_label, objects, crop_off, scratch, scratch_per_fov);
  uint4 p0 = {0u, 0u, 0u, 0u}, p1 = {0u, 0u, 0u, 0u};
  glcm_prefetch(cur, p0, p1);
  int ahead = -2;  // -2: nothing grabbed yet
  for (int par = 1; s_code[par ^ 1] >= 0; par ^= 1) {
    // s_code[par ^ 1] holds the current item (cur), s_code[par] receives the next one
    if (cur.nb > 0 && cur.nb <= kCrop) {
      const int n16 = (cur.nb + 15) / 16;
      if ((int)threadIdx.x < n16) reinterpret_cast<uint4*>(crop)[threadIdx.x] = p0;
      if ((int)threadIdx.x + kTT < n16) reinterpret_cast<uint4*>(crop)[threadIdx.x + kTT] = p1;
    }
    // s_code[par] was last read by the previous iteration's loop test (before its barrier); it
    // receives the item grabbed during the previous item
    if (threadIdx.x == 0 && ahead != -2) s_code[par] = ahead;
    __syncthreads();
    const GlcmItem it = cur;
    cur = glcm_item(s_code[par], C, max_label, objects, crop_off, scratch, scratch_per_fov);
    glcm_prefetch(cur, p0, p1);
    if (threadIdx.x == 0) ahead = s_code[par] >= 0 ? glcm_grab(q_fov, q_visited, B, C, hdr, glcm_next) : -1;
    if (it.nb <= 0) continue;
    double* f = feats + ((long long)it.fov * max_label + it.k) * F + CPX_N_SHAPE +
                (long long)it.ch * CPX_FEATURES_PER_CHANNEL + CPX_N_INT;
    long long pt = 0;
#ifdef CPX_GLCM_PROF
    if (threadIdx.x == 0) {
      pt = clock64();
      atomicAdd(&g_glcm_prof[5], 1ull);
      atomicAdd(&g_glcm_prof[6], (unsigned long long)it.nb);
      if (it.nb > kCrop) atomicAdd(&g_glcm_prof[7], 1ull);
    }
#endif
    // skimage offsets (dr, dc) for angles 0, pi/4, pi/2, 3pi/4 at distance 3
    GlcmAcc acc[4] = {};
#pragma unroll
    for (int a = 0; a < CPX_N_ANGLES; ++a) {
      const int dr = a == 0 ? 0 : a == 2 ? 3 : 2;
      const int dc = a == 0 ? 3 : a == 1 ? 2 : a == 2 ? 0 : -2;
      acc[a].bg = it.nb <= kCrop
                      ? glcm_count<true>(crop, tab, hom, acc[a], it.bh, it.bw, dr, dc)
                      : glcm_count<false>(it.src, tab, hom, acc[a], it.bh, it.bw, dr, dc);
      __syncthreads();
      GLCM_MARK(2, &pt);
      glcm_clear(tab);
      __syncthreads();
      GLCM_MARK(3, &pt);
    }
    glcm_finish(acc, tab, it.bh, it.bw, f);
    GLCM_MARK(4, &pt);
  }
}

// crop slots: per FOV exclusive scan of C * bbox area; objects beyond the scratch capacity or
// with bbox > 65535 px get -1 (fallback kernel).
__global__ __launch_bounds__(1024) void k_crop_offsets(int C, int max_label,
                                                      const cpx_object* __restrict__ objects,
                                                      const cpx_fov_objects* __restrict__ hdr,
                                                      long long cap, long long* __restrict__ crop_off,
                                                      int* __restrict__ glcm_next, cpx_fallback_lists fb) {
  const int fov = blockIdx.x;
  const int n = hdr[fov].n_objects;
  if (threadIdx.x == 0) glcm_next[fov] = 0;  // k_tex_glcm's work queue of this FOV
  __shared__ long long wsum[16];
  __shared__ long long base;
  __shared__ int ns, nt;
  if (threadIdx.x == 0) {
    base = 0;
    ns = nt = 0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int k0 = 0; k0 < n; k0 += blockDim.x) {
    const int k = k0 + threadIdx.x;
    long long sz = 0;
    if (k < n) {
      const cpx_object o = objects[(long long)fov * max_label + k];
      const long long nb = (long long)(o.bbox[2] - o.bbox[0]) * (o.bbox[3] - o.bbox[1]);
      sz = nb <= 65535 ? ((nb + 15) / 16) * 16 * C : 0;
    }
    // inclusive wave scan
    long long x = sz;
    for (int d = 1; d < 64; d <<= 1) {
      const long long y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    long long off = base;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    off += x - sz;
    if (k < n) {
      const bool staged = sz > 0 && off + sz <= cap;
      crop_off[(long long)fov * max_label + k] = staged ? off : -1;
      const cpx_object o = objects[(long long)fov * max_label + k];
      if (!staged) fb.tex[(long long)fov * max_label + atomicAdd(&nt, 1)] = k;
      if (!cpx_shape_fits(o.bbox[2] - o.bbox[0], o.bbox[3] - o.bbox[1]))
        fb.shape[(long long)fov * max_label + atomicAdd(&ns, 1)] = k;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      long long t = 0;
      for (int w = 0; w < nw; ++w) t += wsum[w];
      base += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    fb.n_shape[fov] = ns;
    fb.n_tex[fov] = nt;
  }
}

// ---------------------------------------------------------------------------------------------
// AreaShape fast path: bbox + 2-px margin membership bitmask in LDS
constexpr int kST = 256;
constexpr int kShapeW = kFastShapeWords;  // 8 KiB per bitmask (x2: membership + border)

__device__ __forceinline__ unsigned int getw(const unsigned int* m, int wpr, int rows, int r, int cw) {
  return (r < 0 || r >= rows || cw < 0 || cw >= wpr) ? 0u : m[r * wpr + cw];
}

__device__ __forceinline__ bool shape_fits(const cpx_object& o) {
  return cpx_shape_fits(o.bbox[2] - o.bbox[0], o.bbox[3] - o.bbox[1]);
}

__global__ __launch_bounds__(kST) void k_shape_fast(const int* __restrict__ labels, int H, int W,
                                                   int max_label, int F,
                                                   const cpx_object* __restrict__ objects,
                                                   const cpx_fov_objects* __restrict__ hdr,
                                                   double* __restrict__ feats) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned int* M = reinterpret_cast<unsigned int*>(smem);
  unsigned int* Bd = M + kShapeW;
  __shared__ long long red[6][kST / 64];
  __shared__ int redi[3][kST / 64];
  const int fov = blockIdx.y;
  const int nobj = hdr[fov].n_objects;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int ty = threadIdx.x >> 5, tx = threadIdx.x & 31;  // 8 x 32
  const int* lab = labels + (long long)fov * H * W;
  for (int k = blockIdx.x; k < nobj; k += gridDim.x) {
    const cpx_object o = objects[(long long)fov * max_label + k];
    if (!shape_fits(o)) continue;
    const int L = o.label;
    const int R0 = o.bbox[0] - 2, C0 = o.bbox[1] - 2;  // region origin (2-px margin)
    const int rows = o.bbox[2] - o.bbox[0] + 4, cols = o.bbox[3] - o.bbox[1] + 4;
    const int wpr = (cols + 31) >> 5;
    __syncthreads();
    // membership bitmask: each 32-lane half-wave builds one 32-bit word (r, cw); four words per
    // half-wave are loaded before the first ballot so the label loads overlap
    const int nw = rows * wpr;
    for (int w0 = 0; w0 < nw; w0 += 4 * (kST / 32)) {
      int lv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int w = w0 + u * (kST / 32) + ty;
        const int r = w / wpr, cw = w - r * wpr;
        const int c = cw * 32 + tx;
        const int gr = R0 + r, gc = C0 + c;
        const bool ok = w < nw && c < cols && gr >= 0 && gr < H && gc >= 0 && gc < W;
        lv[u] = ok ? lab[(long long)gr * W + gc] : -1;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int w = w0 + u * (kST / 32) + ty;
        const unsigned long long b = __ballot(lv[u] == L);
        if (w < nw) {
          if (lane == 0) M[w] = (unsigned int)b;
          if (lane == 32) M[w] = (unsigned int)(b >> 32);
        }
      }
    }
    __syncthreads();
    // border = in & !(up & down & left & right)
    for (int w = threadIdx.x; w < rows * wpr; w += kST) {
      const int r = w / wpr, cw = w - r * wpr;
      const unsigned int x = M[w];
      const unsigned int up = getw(M, wpr, rows, r - 1, cw), dn = getw(M, wpr, rows, r + 1, cw);
      const unsigned int lf = (x << 1) | (getw(M, wpr, rows, r, cw - 1) >> 31);
      const unsigned int rt = (x >> 1) | (getw(M, wpr, rows, r, cw + 1) << 31);
      Bd[w] = x & ~(up & dn & lf & rt);
    }
    __syncthreads();
    long long n = 0, sr = 0, sc = 0, srr = 0, scc = 0, src = 0;
    int n1 = 0, n2 = 0, n3 = 0;
    for (int w = threadIdx.x; w < rows * wpr; w += kST) {
      const int r = w / wpr, cw = w - r * wpr;
      unsigned int x = M[w];
      const unsigned int bx = Bd[w];
      while (x) {
        const int b = __ffs(x) - 1;
        x &= x - 1;
        const int c = cw * 32 + b;
        const long long rr = r - 2, cc = c - 2;  // bbox-local coordinates
        n += 1;
        sr += rr;
        sc += cc;
        srr += rr * rr;
        scc += cc * cc;
        src += rr * cc;
        if (!((bx >> b) & 1u)) continue;
        auto bit = [&](int rr2, int cc2) -> int {
          return (int)((getw(Bd, wpr, rows, rr2, cc2 >> 5) >> (cc2 & 31)) & 1u);
        };
        const int code = 1 + 2 * (bit(r - 1, c) + bit(r + 1, c) + bit(r, c - 1) + bit(r, c + 1)) +
                         10 * (bit(r - 1, c - 1) + bit(r - 1, c + 1) + bit(r + 1, c - 1) + bit(r + 1, c + 1));
        if (code == 5 || code == 7 || code == 15 || code == 17 || code == 25 || code == 27) n1 += 1;
        else if (code == 21 || code == 33) n2 += 1;
        else if (code == 13 || code == 23) n3 += 1;
      }
    }
    n = wave_sum(n); sr = wave_sum(sr); sc = wave_sum(sc);
    srr = wave_sum(srr); scc = wave_sum(scc); src = wave_sum(src);
    n1 = wave_sum(n1); n2 = wave_sum(n2); n3 = wave_sum(n3);
    if (lane == 0) {
      red[0][wid] = n; red[1][wid] = sr; red[2][wid] = sc;
      red[3][wid] = srr; red[4][wid] = scc; red[5][wid] = src;
      redi[0][wid] = n1; redi[1][wid] = n2; redi[2][wid] = n3;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      n = sr = sc = srr = scc = src = 0;
      n1 = n2 = n3 = 0;
      for (int w = 0; w < kST / 64; ++w) {
        n += red[0][w]; sr += red[1][w]; sc += red[2][w];
        srr += red[3][w]; scc += red[4][w]; src += red[5][w];
        n1 += redi[0][w]; n2 += redi[1][w]; n3 += redi[2][w];
      }
      double* f = feats + ((long long)fov * max_label + k) * F;
      const double SQ2 = 1.4142135623730951;
      const double area = (double)n;
      const int r0 = o.bbox[0], c0 = o.bbox[1], r1 = o.bbox[2], c1 = o.bbox[3];
      const double bba = (double)(r1 - r0) * (double)(c1 - c0);
      f[CPX_SHAPE_AREA] = area;
      f[CPX_SHAPE_PERIMETER] = (double)n1 + (double)n2 * SQ2 + (double)n3 * ((1.0 + SQ2) / 2.0);
      f[CPX_SHAPE_CENTER_Y] = o.centroid_r;
      f[CPX_SHAPE_CENTER_X] = o.centroid_c;
      f[CPX_SHAPE_BBOX_AREA] = bba;
      f[CPX_SHAPE_EXTENT] = area / bba;
      f[CPX_SHAPE_EQUIV_DIAMETER] = sqrt(4.0 * area / 3.14159265358979323846);
      const i128 NN = n;
      const i128 m20n = NN * srr - (i128)sr * sr;
      const i128 m02n = NN * scc - (i128)sc * sc;
      const i128 m11n = NN * src - (i128)sr * sc;
      const double n2d = area * area;
      const double a = (double)m02n / n2d, b = -(double)m11n / n2d, c = (double)m20n / n2d;
      const double hm = 0.5 * (a + c), hd = 0.5 * (a - c);
      const double rt = sqrt(hd * hd + b * b);
      double l1 = hm + rt;
      const i128 detn4 = m02n * m20n - m11n * m11n;
      double l2 = (l1 > 0.0) ? ((double)detn4 / (n2d * n2d)) / l1 : 0.0;
      if (l1 < 0.0) l1 = 0.0;
      if (l2 < 0.0) l2 = 0.0;
      if (l2 > l1) l2 = l1;
      f[CPX_SHAPE_MAJOR_AXIS] = 4.0 * sqrt(l1);
      f[CPX_SHAPE_MINOR_AXIS] = 4.0 * sqrt(l2);
      f[CPX_SHAPE_ECCENTRICITY] = (l1 == 0.0) ? 0.0 : sqrt(1.0 - l2 / l1);
      f[CPX_SHAPE_ORIENTATION] = (a - c == 0.0) ? ((b < 0.0) ? -3.14159265358979323846 / 4.0
                                                              : 3.14159265358979323846 / 4.0)
                                                : 0.5 * atan2(-2.0 * b, c - a);
      f[CPX_SHAPE_BBOX_MIN_Y] = r0;
      f[CPX_SHAPE_BBOX_MIN_X] = c0;
      f[CPX_SHAPE_BBOX_MAX_Y] = r1;
      f[CPX_SHAPE_BBOX_MAX_X] = c1;
    }
  }
}

}  // namespace


// internal launchers used by cpx_features (k_features.hip)
int cpx_features_fast(cpx_ctx* ctx, const int32_t* labels_dev, const float* corr_dev, int B, int C,
                      int H, int W, int max_label, int F, const cpx_object* objects_dev,
                      const cpx_fov_objects* hdr_dev, double* feats_dev, cpx_fallback_lists* fb) {
  static bool attr = false;
  const size_t lds_t = sizeof(unsigned int) * kTabW + sizeof(unsigned long long) * 256 + kCrop;
  static_assert(sizeof(unsigned int) * kTabW + sizeof(unsigned long long) * 256 + kCrop <= 160 * 1024,
                "GLCM LDS budget");
  static_assert(kNW * 4 * kAccW <= kTabW, "reduction scratch inside the table");
  const size_t lds_s = sizeof(unsigned int) * 2 * kShapeW;
  if (!attr) {
    CPX_CHECK_HIP(hipFuncSetAttribute((const void*)k_tex_glcm,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_t));
    CPX_CHECK_HIP(hipFuncSetAttribute((const void*)k_shape_fast,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_s));
    attr = true;
  }
  // workspace: crop offsets [B][max_label] + scratch (2 bytes per pixel-channel per FOV)
  const long long per_fov = ((2LL * H * W * C + 255) / 256) * 256;
  // + one GLCM work-queue counter per FOV (zeroed by k_crop_offsets) + the fallback lists
  const size_t off_bytes = ((sizeof(long long) * (size_t)B * max_label + sizeof(int) * (size_t)B * 3 +
                             sizeof(int) * 2 * (size_t)B * max_label + 255) / 256) * 256;
  unsigned char* ws = (unsigned char*)cpx_ws(ctx, WS_MISC, off_bytes + (size_t)B * per_fov + 256);  // +256: GLCM key read-ahead
  if (!ws) return CPX_ERR_OOM;
  CPX_REQUIRE(B < 2048 && (long long)max_label * C < (1 << 20), CPX_ERR_SHAPE,
              "GLCM queue codes hold fov < 2048 and items < 2^20");
  long long* crop_off = (long long*)ws;
  int* glcm_next = (int*)(crop_off + (size_t)B * max_label);
  fb->n_shape = glcm_next + B;
  fb->n_tex = fb->n_shape + B;
  fb->shape = fb->n_tex + B;
  fb->tex = fb->shape + (size_t)B * max_label;
  unsigned char* scratch = ws + off_bytes;
  hipLaunchKernelGGL(k_crop_offsets, dim3(B), dim3(1024), 0, ctx->stream, C, max_label,
                     objects_dev, hdr_dev, per_fov, crop_off, glcm_next, *fb);
  CPX_CHECK_LAUNCH("k_crop_offsets");
  const int per_fov_s = std::max(1, std::min(max_label, (8 * ctx->n_cu + B - 1) / B));
  hipLaunchKernelGGL(k_shape_fast, dim3(per_fov_s, B), dim3(kST), lds_s, ctx->stream,
                     (const int*)labels_dev, H, W, max_label, F, objects_dev, hdr_dev, feats_dev);
  CPX_CHECK_LAUNCH("k_shape_fast");
  const int per_fov_a = std::max(1, std::min(max_label * C, (16 * ctx->n_cu + B - 1) / B));
  hipLaunchKernelGGL(k_tex_stage, dim3(per_fov_a, B), dim3(kAT), 0, ctx->stream,
                     (const int*)labels_dev, corr_dev, C, H, W, max_label, F, objects_dev, hdr_dev,
                     (const long long*)crop_off, scratch, per_fov, feats_dev);
  CPX_CHECK_LAUNCH("k_tex_stage");
  const int per_fov_t = std::max(1, std::min(max_label * C, (ctx->n_cu + B - 1) / B));
  hipLaunchKernelGGL(k_tex_glcm, dim3(per_fov_t, B), dim3(kTT), lds_t, ctx->stream, C, max_label,
                     F, objects_dev, hdr_dev, (const long long*)crop_off,
                     (const unsigned char*)scratch, per_fov, glcm_next, feats_dev);
  CPX_CHECK_LAUNCH("k_tex_glcm");
  return CPX_OK;
}

#ifdef CPX_GLCM_PROF
extern "C" int cpx_debug_glcm_prof(unsigned long long* host8, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return CPX_ERR_HIP;
  if (host8 && hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_glcm_prof), 64) != hipSuccess) return CPX_ERR_HIP;
  if (reset) {
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_glcm_prof), z, 64) != hipSuccess) return CPX_ERR_HIP;
  }
  return CPX_OK;
}
#endif
