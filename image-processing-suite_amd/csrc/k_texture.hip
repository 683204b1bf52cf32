// a8 fast path: AreaShape + Intensity + Texture for objects whose bbox fits in LDS (the common
// case; larger objects fall back to k_shape / k_intensity_texture in k_features.hip with the same
// arithmetic).  Same definitions as the fallback (k_features.hip); integer sums are identical,
// fp64 intensity sums may differ in the last bits (summation order).
//
// Design:
//  * k_obj_stage (one 512-thread block per object, two per CU): the object's bbox + margin
//    membership bitmask from one read of the label image (AreaShape sums: bit-parallel border,
//    Benkrid-Crookes perimeter, exact int64 moments), then per channel one coalesced pass over the
//    bbox (values held in registers) for the Intensity columns and the scale_to_8bit range, and
//    the 8-bit masked crop written to a global scratch slot (offsets from a per-FOV scan);
//  * k_tex_glcm (one 1024-thread block per CU with a 128 KiB LDS pair table) copies a crop to LDS
//    and runs the four GLCM angles from LDS: byte-SIMD pair sums, no-return LDS atomics on a
//    diagonal-major u16 table, one scan per angle for ASM / the pair count.
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
// The same for k_obj_stage (-DCPX_STAGE_PROF): [0] queue, [1] membership masks, [2] AreaShape
// sums, [3] channel reads + Intensity sums, [4] reductions, [5] crop pass, [6] objects, [7] groups
#ifdef CPX_STAGE_PROF
__device__ unsigned long long g_stage_prof[8];
#define STAGE_MARK(k, pt)                                   \
  do {                                                      \
    if (threadIdx.x == 0) {                                 \
      const long long t_ = clock64();                       \
      atomicAdd(&g_stage_prof[k], (unsigned long long)(t_ - *(pt))); \
      *(pt) = t_;                                           \
    }                                                       \
  } while (0)
#define STAGE_COUNT(k, v) \
  do {                                                      \
    if (threadIdx.x == 0) atomicAdd(&g_stage_prof[k], (unsigned long long)(v)); \
  } while (0)
#else
#define STAGE_MARK(k, pt) \
  do {                   \
  } while (0)
#define STAGE_COUNT(k, v) \
  do {                   \
  } while (0)
#endif

constexpr int kTT = 1024;            // GLCM block (16 waves, one block per CU)
constexpr int kNW = kTT / 64;
constexpr int kTabW = 32768;         // 64K packed u16 pair counters (128 KiB), diagonal-major
constexpr int kSmall = 256 + 320 + 16 + 2048;  // LDS after the table: atomic sinks, reduction totals,
                                               // queue codes, homogeneity table
constexpr int kCrop = 160 * 1024 - 4 * kTabW - kSmall;  // u8 crop bytes held in LDS
constexpr int kSlack = 16;           // bytes the GLCM may read past a crop's last row (masked)

__device__ __forceinline__ int quantize(float v, bool in, float mn, float rng, bool flat) {
  const float m = v * (in ? 1.0f : 0.0f);
  if (flat) return 0;
  float x = m - mn;  // scale_to_8bit: 255.0 * (x - min) / (max - min), fp32, truncation
  x = 255.0f * x;
  x = x / rng;
  return (int)(unsigned char)(int)x;
}

// Staged 8-bit crops: rows padded to a multiple of 8 bytes (the GLCM reads eight pixels per
// load), kSlack bytes after the last row, slot size a multiple of 16 (uint4 copies).
__host__ __device__ __forceinline__ int crop_stride(int bw) { return (bw + 7) & ~7; }
__host__ __device__ __forceinline__ long long crop_bytes(int bh, int bw) {
  return ((long long)bh * crop_stride(bw) + kSlack + 15) / 16 * 16;
}

// GLCM of one (object, channel) item: skimage graycomatrix offsets (dr, dc) for angles
// 0, pi/4, pi/2, 3pi/4 at distance 3, symmetric=False, normed, then greycoprops.  Per angle:
//  1. count: each thread takes chunks of eight horizontally adjacent reference pixels (one
//     8-byte load of a, two of b + byte alignment), masks the columns outside the angle's
//     valid range to 0, and adds
//       - the pair sums that need no table from byte-SIMD instructions on the four-pixel words:
//         sum i, sum j and sum |i - j| by v_sad_u8, sum i^2, j^2, ij by v_dot4_u32_u8
//         (contrast = sum i^2 + j^2 - 2ij);
//       - each non-background pair (i, j) != (0, 0) to its u16 counter with a no-return LDS
//         atomic.  The table is diagonal-major: key = (dd << 8) | i with dd = (j - i) mod 256,
//         so a row dd of 256 counters holds |i - j| = dd for i <= 255 - dd and 256 - dd after;
//  2. scan (which also clears): one wave per row dd skips all-zero rows by ballot; otherwise
//     ASM = sum c^2 (v_dot2_u32_u16 on the packed counters), the non-background pair count
//     sum c, and homogeneity sum c * round(2^48 / (1 + d^2)) with d constant on each half-row
//     (per-term relative error <= 1.2e-10), then zeroes the row;
//  3. finish (once per item): background pairs = T - sum c, block reduction through LDS,
//     greycoprops on four lanes.
// Every sum is an integer (T <= 65535 pairs per item bounds them all below 2^32, the
// homogeneity below 2^64), so the result never depends on the order in which pairs are visited.
struct HomTable {
  unsigned long long m[256];
  constexpr HomTable() : m() {
    for (int d = 0; d < 256; ++d) m[d] = (unsigned long long)(281474976710656.0 / (1.0 + (double)(d * d)) + 0.5);
  }
};
__constant__ HomTable kHom = HomTable();
constexpr double kHomScale = 1.0 / 281474976710656.0;  // 2^-48

struct GlcmSums {
  unsigned int sisj;                        // count pass: sum i + (sum j << 16) (< 2^16 each per thread)
  unsigned int sii, sjj, sij, dis;
  unsigned int asq, cnt;                    // scan: sum c^2, sum c over non-background keys
  unsigned long long hom;                   // count: sum over pair slots of hom(|i - j|)
};
constexpr int kRedW = 10;  // 32-bit words per angle in the block reduction

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned int dot2_u16(unsigned int a, unsigned int b, unsigned int c) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), c, false);
}

// per-byte (x - y) mod 256 of four packed bytes (no borrow crosses a byte)
__device__ __forceinline__ unsigned int bytes_sub(unsigned int x, unsigned int y) {
  return ((x | 0x80808080u) - (y & 0x7f7f7f7fu)) ^ ((x ^ ~y) & 0x80808080u);
}

// Background and masked pairs (key 0) go to a per-lane sink word instead of a branch (a
// predicated-off atomic measured the same, tools/tex_bench.py r03).
__device__ __forceinline__ void glcm_add(unsigned int* tab, unsigned int* sink, unsigned int key) {
  atomicAdd(key ? &tab[key >> 1] : sink, (key & 1u) * 0xffffu + 1u);  // half = i & 1
}

template <int ANG, bool LDS_CROP>
__device__ __forceinline__ void glcm_count(const unsigned char* __restrict__ crop, unsigned int* tab,
                                           const unsigned long long* hom, GlcmSums& S, int bh, int bw) {
  unsigned int* sink = tab + kTabW + (threadIdx.x & 63);
  constexpr int dr = ANG == 0 ? 0 : ANG == 2 ? 3 : 2;
  constexpr int dc = ANG == 0 ? 3 : ANG == 1 ? 2 : ANG == 2 ? 0 : -2;
  constexpr int sh = dc >= 0 ? dc : dc + 8;  // byte offset of b in its aligned 16-byte window
  const int bwp = crop_stride(bw), nch = bwp >> 3;
  const int rend = bh - dr;
  const int cbeg = dc >= 0 ? 0 : -dc, cend = dc >= 0 ? bw - dc : bw;
  if (rend <= 0 || cend <= cbeg) return;
  const int nc = rend * nch;  // chunk q covers bytes 8q .. 8q + 7 of the crop (rows are whole chunks)
  // chunk q = t, t + 1024, ... of this thread is visited at crop position p = q * m mod nc (m an
  // odd prime not dividing nc): the lanes of a wave land on scattered pixels, so one LDS atomic
  // instruction rarely has two lanes on the same counter (same-address lanes serialise), which
  // neighbouring pixels of a smooth crop would.  p and its (row, chunk column) advance
  // incrementally.
  const int mul = nc % 7919 ? 7919 : 7907;
  static_assert((long long)kTT * 7919 < (1ll << 32), "32-bit products");
  unsigned p = (threadIdx.x * (unsigned)mul) % (unsigned)nc;
  const unsigned step = ((unsigned)kTT * (unsigned)mul) % (unsigned)nc;
  const int sr = step / nch, sc = step - sr * nch;
  int r = p / nch, ci = p - r * nch;
  const int boff = dr * bwp + (dc < 0 ? -8 : 0);
  for (int q = threadIdx.x; q < nc; q += kTT) {
    const unsigned char* pa = crop + 8 * (int)p;
    const uint2 A = *reinterpret_cast<const uint2*>(pa);
    unsigned int b0, b1;
    if constexpr (sh == 0) {
      const uint2 Bw = *reinterpret_cast<const uint2*>(pa + boff);
      b0 = Bw.x;
      b1 = Bw.y;
    } else {
      const uint2 L = *reinterpret_cast<const uint2*>(pa + boff);
      const uint2 R = *reinterpret_cast<const uint2*>(pa + boff + 8);
      if constexpr (sh < 4) {
        b0 = __builtin_amdgcn_alignbyte(L.y, L.x, sh);
        b1 = __builtin_amdgcn_alignbyte(R.x, L.y, sh);
      } else {
        b0 = __builtin_amdgcn_alignbyte(R.x, L.y, sh - 4);
        b1 = __builtin_amdgcn_alignbyte(R.y, R.x, sh - 4);
      }
    }
    const int c0 = 8 * ci;
    const int hi = min(cend - c0, 8), lo = max(cbeg - c0, 0);
    unsigned long long m = hi >= 8 ? ~0ull : (hi <= 0 ? 0ull : (1ull << (8 * hi)) - 1ull);
    m &= ~0ull << (8 * lo);
    const unsigned int m0 = (unsigned int)m, m1 = (unsigned int)(m >> 32);
    const unsigned int a0 = A.x & m0, a1 = A.y & m1;
    b0 &= m0;
    b1 &= m1;
    S.sisj = __builtin_amdgcn_sad_u8(a0, 0u, S.sisj);
    S.sisj = __builtin_amdgcn_sad_u8(a1, 0u, S.sisj);
    S.sisj += __builtin_amdgcn_sad_u8(b1, 0u, __builtin_amdgcn_sad_u8(b0, 0u, 0u)) << 16;
    S.dis = __builtin_amdgcn_sad_u8(a0, b0, S.dis);
    S.dis = __builtin_amdgcn_sad_u8(a1, b1, S.dis);
    S.sii = __builtin_amdgcn_udot4(a0, a0, S.sii, false);
    S.sii = __builtin_amdgcn_udot4(a1, a1, S.sii, false);
    S.sjj = __builtin_amdgcn_udot4(b0, b0, S.sjj, false);
    S.sjj = __builtin_amdgcn_udot4(b1, b1, S.sjj, false);
    S.sij = __builtin_amdgcn_udot4(a0, b0, S.sij, false);
    S.sij = __builtin_amdgcn_udot4(a1, b1, S.sij, false);
    // keys (dd << 8) | i, two per word: selectors 0-3 pick i (src1), 4-7 pick dd (src0)
    // homogeneity per pair slot from the LDS table (masked slots are (0, 0) -> hom(0); finish
    // subtracts them, background pairs stay)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned int ia = (a0 >> (8 * u)) & 255u, ib = (b0 >> (8 * u)) & 255u;
      const unsigned int ja = (a1 >> (8 * u)) & 255u, jb = (b1 >> (8 * u)) & 255u;
      S.hom += hom[ia > ib ? ia - ib : ib - ia];
      S.hom += hom[ja > jb ? ja - jb : jb - ja];
    }
    const unsigned int d0 = bytes_sub(b0, a0), d1 = bytes_sub(b1, a1);
    const unsigned int k01 = __builtin_amdgcn_perm(d0, a0, 0x05010400u);
    const unsigned int k23 = __builtin_amdgcn_perm(d0, a0, 0x07030602u);
    const unsigned int k45 = __builtin_amdgcn_perm(d1, a1, 0x05010400u);
    const unsigned int k67 = __builtin_amdgcn_perm(d1, a1, 0x07030602u);
    glcm_add(tab, sink, k01 & 0xffffu);
    glcm_add(tab, sink, k01 >> 16);
    glcm_add(tab, sink, k23 & 0xffffu);
    glcm_add(tab, sink, k23 >> 16);
    glcm_add(tab, sink, k45 & 0xffffu);
    glcm_add(tab, sink, k45 >> 16);
    glcm_add(tab, sink, k67 & 0xffffu);
    glcm_add(tab, sink, k67 >> 16);
    p += step;
    r += sr;
    ci += sc;
    if (ci >= nch) {
      ci -= nch;
      ++r;
    }
    if (p >= (unsigned)nc) {
      p -= nc;
      r -= rend;
    }
  }
}

// Scan + clear of one angle's table: ASM = sum c^2 (v_dot2_u32_u16 on the packed counters) and
// the non-background pair count sum c.  Wave w owns the row pairs w + 16k (k < 8), one 16-byte
// read per lane and pair (a wave-instruction covers two whole rows), all eight reads in flight
// before the first use; all-zero row pairs are skipped by ballot and only non-zero lanes store
// their zeros back.
__device__ __forceinline__ void glcm_scan(unsigned int* tab, GlcmSums& S) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  static_assert(kTabW == 8 * kNW * 64 * 4, "eight row pairs per wave");
  uint4* rows = reinterpret_cast<uint4*>(tab) + wid * 64 + lane;
  uint4 w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = rows[k * kNW * 64];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool nz = (w[k].x | w[k].y | w[k].z | w[k].w) != 0u;
    if (!__builtin_amdgcn_ballot_w64(nz)) continue;
    if (nz) rows[k * kNW * 64] = uint4{0u, 0u, 0u, 0u};
    S.asq = dot2_u16(w[k].x, w[k].x, S.asq);
    S.asq = dot2_u16(w[k].y, w[k].y, S.asq);
    S.asq = dot2_u16(w[k].z, w[k].z, S.asq);
    S.asq = dot2_u16(w[k].w, w[k].w, S.asq);
    S.cnt = dot2_u16(w[k].x, 0x10001u, S.cnt);
    S.cnt = dot2_u16(w[k].y, 0x10001u, S.cnt);
    S.cnt = dot2_u16(w[k].z, 0x10001u, S.cnt);
    S.cnt = dot2_u16(w[k].w, 0x10001u, S.cnt);
  }
}

// Sum of a u64 over each half-wave (lanes 0-31 -> lane 31, 32-63 -> lane 63) on the DPP path.
__device__ __forceinline__ unsigned long long half_wave_sum_u64(unsigned long long v) {
#define CPX_U64_DPP_STEP(CTRL, ROWMASK)                                                         \
  {                                                                                            \
    const unsigned int lo_ = (unsigned int)__builtin_amdgcn_update_dpp(0, (int)(unsigned int)v, \
                                                                       CTRL, ROWMASK, 0xf, false); \
    const unsigned int hi_ = (unsigned int)__builtin_amdgcn_update_dpp(                        \
        0, (int)(unsigned int)(v >> 32), CTRL, ROWMASK, 0xf, false);                           \
    v += ((unsigned long long)hi_ << 32) | lo_;                                                \
  }
  CPX_U64_DPP_STEP(0x111, 0xf)  // row_shr:1,2,4,8 -> inclusive scan within each row of 16 lanes
  CPX_U64_DPP_STEP(0x112, 0xf)
  CPX_U64_DPP_STEP(0x114, 0xf)
  CPX_U64_DPP_STEP(0x118, 0xf)
  CPX_U64_DPP_STEP(0x142, 0xa)  // row_bcast:15 -> rows 1 and 3 add the totals of rows 0 and 2
#undef CPX_U64_DPP_STEP
  return v;
}

// pair slots the dense count visits for angle a: the angle's rows x the padded row width
__device__ __forceinline__ unsigned long long glcm_slots(int a, int bh, int bw) {
  const int dr = a == 0 ? 0 : a == 2 ? 3 : 2;
  const int dc = a == 0 ? 3 : a == 1 ? 2 : a == 2 ? 0 : -2;
  const int rend = bh - dr, cbeg = dc >= 0 ? 0 : -dc, cend = dc >= 0 ? bw - dc : bw;
  return rend > 0 && cend > cbeg ? (unsigned long long)rend * crop_stride(bw) : 0ull;
}

// Finish: the four angles' per-thread sums are reduced through LDS in two rounds of two angles
// (`red` = 2 * kRedW * kTT words of the all-zero table, zeroed again before returning; `tot` =
// 4 * kRedW u64 of static LDS), then 4 * kRedW lanes store the item's totals to `raw` for
// k_glcm_props (greycoprops in fp64 on four lanes here held the block's other 1020 threads at
// the next barrier).
__device__ void glcm_finish(const GlcmSums (&S)[4], unsigned int* red, unsigned long long* tot,
                            unsigned long long* __restrict__ raw, long long* pt, int bh, int bw) {
  const int t = threadIdx.x, lane = t & 63;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2) {
      const GlcmSums& s = S[2 * h + a2];
      const unsigned int v[kRedW] = {s.sisj & 0xffffu, s.sisj >> 16, s.sii, s.sjj, s.sij, s.dis, s.asq, s.cnt,
                                     (unsigned int)s.hom, (unsigned int)(s.hom >> 32)};
#pragma unroll
      for (int k = 0; k < kRedW; ++k) red[(a2 * kRedW + k) * kTT + t] = v[k];
    }
    __syncthreads();
    unsigned long long x = 0;
    if (t < 2 * kRedW * 32) {
      // lane p sums words 32p .. 32p + 31 of its row in a lane-rotated order (bank spread)
      const uint4* src = reinterpret_cast<const uint4*>(red + (t >> 5) * kTT + (t & 31) * 32);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint4 q = src[(i + t) & 7];
        x += (unsigned long long)q.x + q.y + (unsigned long long)q.z + q.w;
      }
    }
    x = half_wave_sum_u64(x);
    if (t < 2 * kRedW * 32 && (lane & 31) == 31) tot[h * 2 * kRedW + (t >> 5)] = x;
    __syncthreads();
    GLCM_MARK(0, pt);
  }
#pragma unroll
  for (int k = 0; k < 2 * kRedW; ++k) red[k * kTT + t] = 0u;
  GLCM_MARK(1, pt);
  if (t < 4 * kRedW) {
    // homogeneity as k_tex_band reports it: over the non-background pairs (the count visited
    // every pair slot of the padded rows, each masked or background slot adding hom(0))
    const int a = t / kRedW, k = t - a * kRedW;
    unsigned long long v = tot[t];
    if (k >= 8) {
      const unsigned long long h = tot[a * kRedW + 8] + (tot[a * kRedW + 9] << 32);
      const unsigned long long hn = h - (glcm_slots(a, bh, bw) - tot[a * kRedW + 7]) * kHom.m[0];
      v = k == 8 ? (hn & 0xffffffffull) : (hn >> 32);
    }
    raw[t] = v;
  }
}

// greycoprops from k_tex_glcm's integer totals, one thread per (object, channel, angle) of the
// items the LDS path measured (staged, <= 65535 px).
__global__ __launch_bounds__(256) void k_glcm_props(int C, int max_label, int F,
                                                   const cpx_object* __restrict__ objects,
                                                   const cpx_fov_objects* __restrict__ hdr,
                                                   const long long* __restrict__ crop_off,
                                                   const unsigned long long* __restrict__ raws,
                                                   double* __restrict__ feats) {
  const int fov = blockIdx.y;
  const int id = blockIdx.x * 256 + threadIdx.x;  // (k, ch, angle)
  const int a = id & 3, item = id >> 2, k = item / C, ch = item - k * C;
  if (k >= hdr[fov].n_objects) return;
  const long long ok = (long long)fov * max_label + k;
  const cpx_object o = objects[ok];
  const int bh = o.bbox[2] - o.bbox[0], bw = o.bbox[3] - o.bbox[1];
  if (crop_off[ok] < 0 || bh * bw > 65535) return;  // the fallback kernel measures it
  const unsigned long long* v = raws + (ok * C + ch) * (4 * kRedW) + a * kRedW;
  const int dr = a == 0 ? 0 : a == 2 ? 3 : 2;
  const int dc = a == 0 ? 3 : a == 1 ? 2 : a == 2 ? 0 : -2;
  const int rend = bh - dr;
  const int cbeg = dc >= 0 ? 0 : -dc, cend = dc >= 0 ? bw - dc : bw;
  const long long T = (rend > 0 && cend > cbeg) ? (long long)rend * (cend - cbeg) : 0;
  const long long tsi = (long long)v[0], tsj = (long long)v[1], tsii = (long long)v[2],
                  tsjj = (long long)v[3], tsij = (long long)v[4];
  const unsigned long long dt = v[5], tas = v[6], ncnt = v[7];
  const unsigned long long nbg = (unsigned long long)T - ncnt;  // background pairs (0, 0)
  // v[8], v[9]: homogeneity over the non-background pairs; each background pair adds hom(0)
  const unsigned long long hs = v[8] + (v[9] << 32) + nbg * kHom.m[0];
  double con = 0.0, dis = 0.0, hom = 0.0, asmv = 0.0, ene = 0.0, cor = 1.0;
  if (T > 0) {
    const double Td = (double)T;
    con = (double)(tsii + tsjj - 2 * tsij) / Td;
    dis = (double)dt / Td;
    hom = ((double)hs * kHomScale) / Td;
    asmv = (double)(tas + nbg * nbg) / (Td * Td);
    ene = sqrt(asmv);
    const long long vi = T * tsii - tsi * tsi;
    const long long vj = T * tsjj - tsj * tsj;
    const long long cv = T * tsij - tsi * tsj;
    const double sdi = sqrt((double)vi) / Td, sdj = sqrt((double)vj) / Td;
    cor = (sdi < 1e-15 || sdj < 1e-15) ? 1.0 : ((double)cv / (Td * Td)) / (sdi * sdj);
  }
  double* out = feats + ok * F + CPX_N_SHAPE + (long long)ch * CPX_FEATURES_PER_CHANNEL + CPX_N_INT +
                a * CPX_N_TEX_PROPS;
  out[CPX_TEX_CONTRAST] = con;
  out[CPX_TEX_DISSIMILARITY] = dis;
  out[CPX_TEX_HOMOGENEITY] = hom;
  out[CPX_TEX_ASM] = asmv;
  out[CPX_TEX_ENERGY] = ene;
  out[CPX_TEX_CORRELATION] = cor;
}

struct GlcmItem {
  int fov, k, ch, bh, bw, nb;  // nb <= 0: nothing to do (no slot, > 65535 px, or queue drained)
  int bytes;                   // staged crop slot size (crop_bytes)
  const unsigned char* src;
};

// Work queue of k_tex_glcm (thread 0 only): items of FOV f are handed out by one atomic
// counter per FOV; a block starts on its own FOV and moves to the next FOV when that queue is
// drained, so blocks of light FOVs help heavy ones and the launch ends within about one item
// of balance.  Returns fov * 2^20 + item, or -1 when every queue has been drained (each block
// visits each FOV at most once, so every block reaches the exit).
__device__ __forceinline__ int glcm_grab(int& f, int& visited, int B, int C,
                                         const cpx_fov_objects* __restrict__ hdr,
                                         int* __restrict__ next, int* __restrict__ redo = nullptr) {
  if (redo) {  // k_tex_glcm over the items k_tex_band handed back: one list, one claim counter
    const int v = atomicAdd(&redo[1], 1);
    return v < redo[0] ? redo[2 + v] : -1;
  }
  while (visited < B) {
    const int n_items = hdr[f].n_objects * C;
    const int v = atomicAdd(&next[f], 1);
    if (v < n_items) return (f << 20) | v;
    ++visited;
    f = f + 1 == B ? 0 : f + 1;
  }
  return -1;
}

static_assert(kCrop / 16 <= 2 * kTT, "a crop is copied with two uint4 per thread");

__device__ __forceinline__ GlcmItem glcm_item(int code, int C, int max_label,
                                              const cpx_object* objects,
                                              const long long* crop_off,
                                              const unsigned char* scratch,
                                              long long scratch_per_fov) {
  GlcmItem g{0, 0, 0, 0, 0, 0, 0, nullptr};
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
  if (off < 0 || nb > 65535) return g;  // u16 counters / u32 sums: fallback kernel
  g.nb = nb;
  g.bytes = (int)crop_bytes(g.bh, g.bw);
  g.src = scratch + (long long)fov * scratch_per_fov + off + (long long)g.ch * g.bytes;
  return g;
}

// Touch every 128-byte line of the next item's LDS-sized crop (one dword per line): the lines
// move to this XCD's L2 while the current item runs, and the loaded word is only consumed at the
// next item (one VGPR instead of holding the crop in registers).
__device__ __forceinline__ unsigned int glcm_touch(const GlcmItem& g) {
  if (g.nb <= 0 || g.bytes > kCrop) return 0u;
  return (int)threadIdx.x * 128 < g.bytes ? *reinterpret_cast<const unsigned int*>(g.src + threadIdx.x * 128) : 0u;
}

template <int A>
__device__ __forceinline__ void glcm_angle(const GlcmItem& it, const unsigned char* crop,
                                           unsigned int* tab, const unsigned long long* hom, GlcmSums& S,
                                           long long* pt) {
  if (it.bytes <= kCrop) glcm_count<A, true>(crop, tab, hom, S, it.bh, it.bw);
  else glcm_count<A, false>(it.src, tab, hom, S, it.bh, it.bw);
  __syncthreads();
  GLCM_MARK(2, pt);
  glcm_scan(tab, S);
  __syncthreads();
  GLCM_MARK(3, pt);
}

// Phase B (one 1024-thread block per CU, 128 KiB LDS pair table): GLCM of staged crops.
__global__ __launch_bounds__(kTT) void k_tex_glcm(int C, int max_label, int F,
                                                 const cpx_object* __restrict__ objects,
                                                 const cpx_fov_objects* __restrict__ hdr,
                                                 const long long* __restrict__ crop_off,
                                                 const unsigned char* __restrict__ scratch,
                                                 long long scratch_per_fov,
                                                 int* __restrict__ glcm_next,
                                                 unsigned long long* __restrict__ glcm_raw,
                                                 int* __restrict__ redo) {
  // LDS: table at offset 0 (static, so the atomics' addresses need no base), then the
  // 64 sink words, the reduction totals, the queue codes and the crop
  __shared__ __attribute__((aligned(16))) unsigned int lds[40 * 1024];  // all 160 KiB, static
  unsigned char* smem = reinterpret_cast<unsigned char*>(lds);
  unsigned int* tab = lds;
  unsigned long long* s_tot = reinterpret_cast<unsigned long long*>(smem + 4 * kTabW + 256);
  int* s_code = reinterpret_cast<int*>(smem + 4 * kTabW + 256 + 320);  // double-buffered by parity
  unsigned long long* s_hom = reinterpret_cast<unsigned long long*>(smem + 4 * kTabW + 256 + 320 + 16);
  unsigned char* crop = smem + 4 * kTabW + kSmall;
  const int B = gridDim.y;
  int q_fov = blockIdx.y, q_visited = 0;  // thread 0's queue position
  for (int x = threadIdx.x; x < kTabW; x += kTT) tab[x] = 0u;
  if (threadIdx.x < 256) s_hom[threadIdx.x] = kHom.m[threadIdx.x];
  if (threadIdx.x == 0) {
    s_code[0] = glcm_grab(q_fov, q_visited, B, C, hdr, glcm_next, redo);
    s_code[1] = glcm_grab(q_fov, q_visited, B, C, hdr, glcm_next, redo);
  }
  __syncthreads();
  // software pipeline: the next item's metadata is loaded and its crop's lines are touched into
  // L2 while the current item runs its four angles (the crop was written by k_obj_stage, possibly
  // on another XCD, so a cold load is HBM/MALL latency); thread 0 grabs the item after that one
  // from the queue during the current item, so the atomic's latency is hidden too.
  GlcmItem cur = glcm_item(s_code[0], C, max_label, objects, crop_off, scratch, scratch_per_fov);
  unsigned int touched = glcm_touch(cur), sink_word = 0u;
  int ahead = -2;  // -2: nothing grabbed yet
  for (int par = 1; s_code[par ^ 1] >= 0; par ^= 1) {
    // s_code[par ^ 1] holds the current item (cur), s_code[par] receives the next one
    sink_word += touched;
    if (cur.nb > 0 && cur.bytes <= kCrop) {
      const int n16 = cur.bytes / 16;
      const uint4* s16 = reinterpret_cast<const uint4*>(cur.src);
      uint4 p0 = {0u, 0u, 0u, 0u}, p1 = {0u, 0u, 0u, 0u};
      if ((int)threadIdx.x < n16) p0 = s16[threadIdx.x];
      if ((int)threadIdx.x + kTT < n16) p1 = s16[threadIdx.x + kTT];
      if ((int)threadIdx.x < n16) reinterpret_cast<uint4*>(crop)[threadIdx.x] = p0;
      if ((int)threadIdx.x + kTT < n16) reinterpret_cast<uint4*>(crop)[threadIdx.x + kTT] = p1;
    }
    // s_code[par] was last read by the previous iteration's loop test (before its barrier); it
    // receives the item grabbed during the previous item
    if (threadIdx.x == 0 && ahead != -2) s_code[par] = ahead;
    __syncthreads();
    const GlcmItem it = cur;
    cur = glcm_item(s_code[par], C, max_label, objects, crop_off, scratch, scratch_per_fov);
    touched = glcm_touch(cur);
    if (threadIdx.x == 0) ahead = s_code[par] >= 0 ? glcm_grab(q_fov, q_visited, B, C, hdr, glcm_next, redo) : -1;
    if (it.nb <= 0) continue;
    unsigned long long* f = glcm_raw + (((long long)it.fov * max_label + it.k) * C + it.ch) * (4 * kRedW);
    long long pt = 0;
#ifdef CPX_GLCM_PROF
    if (threadIdx.x == 0) {
      pt = clock64();
      atomicAdd(&g_glcm_prof[5], 1ull);
      atomicAdd(&g_glcm_prof[6], (unsigned long long)it.nb);
      if (it.bytes > kCrop) atomicAdd(&g_glcm_prof[7], 1ull);
    }
#endif
    GlcmSums S[4] = {};
    glcm_angle<0>(it, crop, tab, s_hom, S[0], &pt);
    glcm_angle<1>(it, crop, tab, s_hom, S[1], &pt);
    glcm_angle<2>(it, crop, tab, s_hom, S[2], &pt);
    glcm_angle<3>(it, crop, tab, s_hom, S[3], &pt);
    glcm_finish(S, tab, s_tot, f, &pt, it.bh, it.bw);
    GLCM_MARK(4, &pt);
  }
  // keeps the touch loads alive: never true (C > 0), but the compiler cannot know that
  if (C < 0 && sink_word + touched == 0x9e3779b9u) glcm_raw[0] = 0ull;
}

// ---------------------------------------------------------------------------------------------
// k_tex_band: the GLCM of one (object, channel) item per block, three blocks per CU.
//
// On the bench plates (tools/glcm_stats.py, one FOV, 5010 items x 4 angles) half the pair slots
// are background (0, 0), an item-angle has ~1,000 distinct keys, and of the pairs with both
// values non-zero 99.76 % have |j - i| < 32.  So instead of the 128 KiB dense table (k_tex_glcm:
// one item per CU, eight block-wide barrier phases of 1024 threads per item) the counts live in
// a 33 KiB band table of u16 counters, 256 per row:
//   rows 0..62: pairs (i, i + d), d = row - 31, by i (zeros included: (0, j <= 31) is row j + 31,
//   entry 0); row 63: (0, j) and row 64: (i, 0) for the larger values; row 65: per-lane sink
//   counters (never read) that take the background pairs and the outliers, so every pair is one
//   unconditional no-return atomic;
//   a pair with both values non-zero and |j - i| > 31 is also appended to an outlier list (<=
//   kOutCap keys per angle); an item whose list overflows in any angle is handed to k_tex_glcm
//   (the dense table) through the redo list.
// The keys of four pairs come from byte-SIMD arithmetic on the packed 8-bit pixels (zero-byte
// flags, per-byte (j - i + 31) mod 256, byte selects and two byte permutes), and the count pass
// does nothing else: every sum greycoprops needs comes from the table in the scan — per group of
// 8 counters with known (d, i0): s0 = sum c, s1 = sum c i, s2 = sum c i^2, q = sum c^2, and
// sum j = s1 + d s0, sum j^2 = s2 + 2 d s1 + d^2 s0, sum ij = s2 + d s1, dissimilarity |d| s0,
// homogeneity H(|d|) s0 — the same integers as the dense kernel's.  Each sum fits 32 bits for an
// item (T <= 65535 pairs of 8-bit values: sum i^2 <= 65535 * 255^2 < 2^32), so per-thread
// partials add modulo 2^32 and the total is exact; homogeneity is a u64 fixed-point sum (kHom).
// The next item's metadata and crop (into registers) load while the current item runs.
// 256 threads per block: 512 measured 1.5 % faster with spills at the register budget three
// blocks per CU need, and no faster without them (`gpurun_out/r06h`, `r06k`)
constexpr int kBT = 256;
constexpr int kBandD = 31;                     // band half-width
constexpr int kBandScan = 2 * kBandD + 1 + 2;  // scanned rows: band + (0, j) + (i, 0)
constexpr int kSinkRow = kBandScan;            // + one row of sink counters
constexpr int kBandW = (kBandScan + 1) * 128;  // u32 words (two u16 counters each)
constexpr int kOutCap = 512;                   // outlier keys per angle
constexpr int kBandCrop = 16 * 1024;           // crops up to this many bytes staged in LDS
constexpr int kBandLds = 4 * kBandW + 2 * kOutCap + 8 * 256 + 8 * 4 * kRedW + 16 + kBandCrop;
static_assert(3 * kBandLds <= 160 * 1024, "three k_tex_band blocks per CU");
constexpr int kScanG = (kBandScan * 32 + kBT - 1) / kBT;  // 16-byte groups per thread in the scan
constexpr int kCropG = kBandCrop / 16 / kBT;              // uint4 of a staged crop per thread
static_assert(kBandCrop == kCropG * 16 * kBT, "a staged crop is whole uint4 per thread");

struct BandAcc {
  unsigned int si, sj, sii, sjj, sij, dis, asq, cnt;  // modulo 2^32 (exact totals < 2^32)
  unsigned long long hom;                             // sum c * kHom(|i - j|)
};

// per-byte 0x80 flags of the zero bytes of x (exact: no carry crosses a byte)
__device__ __forceinline__ unsigned int zero_bytes(unsigned int x) {
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}

// Counter keys (row << 8 | entry) of four pairs (a, b) given as packed bytes: klo holds pairs
// 0, 1, khi pairs 2, 3 (16 bits each); outf flags (0x80 per byte) the outliers.
__device__ __forceinline__ void band_keys(unsigned int a, unsigned int b, unsigned int sink4, unsigned int& klo,
                                          unsigned int& khi, unsigned int& outf) {
  const unsigned int za = zero_bytes(a), zb = zero_bytes(b);
  // per-byte (j - i) mod 256 (bytes_sub) and its borrow (j < i): t's bit 7 is set iff the low
  // seven bits did not borrow
  const unsigned int t = (b | 0x80808080u) - (a & 0x7f7f7f7fu);
  const unsigned int dd = t ^ ((b ^ ~a) & 0x80808080u);
  const unsigned int bor = ((~b & a) | (~(b ^ a) & ~t)) & 0x80808080u;
  const unsigned int r = ((dd & 0x7f7f7f7fu) + 0x1f1f1f1fu) ^ (dd & 0x80808080u);  // + 31
  // in the band: r <= 62 and (r >= 31, i.e. dd <= 31) exactly when j >= i — otherwise the pair
  // aliases a band key modulo 256 (|j - i| >= 225) and is out of band
  const unsigned int up = ((r & 0x7f7f7f7fu) + 0x61616161u) & 0x80808080u;  // r >= 31 (r < 128)
  const unsigned int oob = ((r | ((r | 0x80808080u) - 0x3f3f3f3fu)) | ~(up ^ bor)) & 0x80808080u;
  const unsigned int z1 = oob & za;                 // (0, j > 31)
  const unsigned int z2 = oob & zb & ~za;           // (i > 31, 0)
  outf = oob & ~za & ~zb;                           // both non-zero, |j - i| > 31
  // 0x80 flags -> 0xff byte masks (0x80 - 0x01 = 0x7f: no borrow leaves a byte)
  const unsigned int m1 = z1 | (z1 - (z1 >> 7)), m2 = z2 | (z2 - (z2 >> 7));
  const unsigned int fs = (za & zb) | outf;  // background or outlier: the sink row
  const unsigned int ms = fs | (fs - (fs >> 7));
  unsigned int row = (m1 & 0x3f3f3f3fu) | (~m1 & r);
  row = (m2 & 0x40404040u) | (~m2 & row);
  row = (ms & (0x01010101u * kSinkRow)) | (~ms & row);
  unsigned int ent = (m1 & b) | (~m1 & a);
  ent = (ms & sink4) | (~ms & ent);
  klo = __builtin_amdgcn_perm(row, ent, 0x05010400u);
  khi = __builtin_amdgcn_perm(row, ent, 0x07030602u);
}

// k: key in bits 0-15.  (Adding a wave's lanes on its first active lane's word at once — a
// flat crop's dominant key serialises its lanes on one address — measured 15 % slower: the
// ballots cost more than the conflicts, `gpurun_out/r06i`.)
__device__ __forceinline__ void band_add(unsigned int* tab, unsigned int k) {
  atomicAdd(&tab[(k & 0xffffu) >> 1], (k & 1u) * 0xffffu + 1u);
}

// One chunk of eight reference pixels: a (A) and the b bytes at the angle's offset.
template <int SH, bool SINGLE>
__device__ __forceinline__ void band_load(const unsigned char* pa, int boff, uint2& A, uint2& L, uint2& R) {
  A = *reinterpret_cast<const uint2*>(pa);
  L = *reinterpret_cast<const uint2*>(pa + boff);
  if constexpr (!SINGLE) R = *reinterpret_cast<const uint2*>(pa + boff + 8);
}

template <int ANG, bool LDS_CROP>
__device__ __forceinline__ void band_count(const unsigned char* __restrict__ crop, unsigned int* tab,
                                           unsigned short* outl, int* n_out, int bh, int bw) {
  constexpr int dr = ANG == 0 ? 0 : ANG == 2 ? 3 : 2;
  constexpr int dc = ANG == 0 ? 3 : ANG == 1 ? 2 : ANG == 2 ? 0 : -2;
  constexpr int sh = dc >= 0 ? dc : dc + 8;  // byte offset of b in its aligned 16-byte window
  const int bwp = crop_stride(bw), nch = bwp >> 3;
  const int rend = bh - dr;
  const int cbeg = dc >= 0 ? 0 : -dc, cend = dc >= 0 ? bw - dc : bw;
  if (rend <= 0 || cend <= cbeg) return;
  const int nc = rend * nch;
  // scattered visiting order (as k_tex_glcm's count): neighbouring chunks of a smooth crop share
  // keys, and same-address lanes of one atomic instruction serialise
  const int mul = nc % 7919 ? 7919 : 7907;
  unsigned p = (threadIdx.x * (unsigned)mul) % (unsigned)nc;
  const unsigned step = ((unsigned)kBT * (unsigned)mul) % (unsigned)nc;
  const int sc = step % nch;
  int ci = p % nch;
  const int boff = dr * bwp + (dc < 0 ? -8 : 0);
  const unsigned int sink4 = 0x01010101u * (2u * (threadIdx.x & 63));  // one sink word per lane
  // software pipeline: the next chunk's bytes are loaded before this chunk's atomics are issued
  uint2 A, L, R = {0u, 0u};
  if ((int)threadIdx.x < nc) band_load<sh, sh == 0>(crop + 8 * (int)p, boff, A, L, R);
  // eight no-op atomics after the first load too, so that the loop is entered with the same LDS
  // wait state as its back edge (otherwise the merge makes every iteration wait for all)
  unsigned int* sinkw = tab + kSinkRow * 128 + (threadIdx.x & 63);
#pragma unroll
  for (int u = 0; u < 8; ++u) atomicAdd(sinkw, 0u);
  for (int q = threadIdx.x; q < nc; q += kBT) {
    // every loaded dword stays live to here (also the ones this angle does not read): otherwise
    // their registers are reused right after the load, and the write-after-write forces a wait
    // for the load before this chunk's atomics — the pipeline is gone
    asm volatile("" ::"v"(A.x), "v"(A.y), "v"(L.x), "v"(L.y), "v"(R.x), "v"(R.y));
    unsigned int b0, b1;
    if constexpr (sh == 0) {
      b0 = L.x;
      b1 = L.y;
    } else if constexpr (sh < 4) {
      b0 = __builtin_amdgcn_alignbyte(L.y, L.x, sh);
      b1 = __builtin_amdgcn_alignbyte(R.x, L.y, sh);
    } else {
      b0 = __builtin_amdgcn_alignbyte(R.x, L.y, sh - 4);
      b1 = __builtin_amdgcn_alignbyte(R.y, R.x, sh - 4);
    }
    const int c0 = 8 * ci;
    const int hi = min(cend - c0, 8), lo = max(cbeg - c0, 0);
    unsigned long long m = hi >= 8 ? ~0ull : (hi <= 0 ? 0ull : (1ull << (8 * hi)) - 1ull);
    m &= ~0ull << (8 * lo);
    const unsigned int m0 = (unsigned int)m, m1 = (unsigned int)(m >> 32);
    const unsigned int a0 = A.x & m0, a1 = A.y & m1;
    b0 &= m0;
    b1 &= m1;
    unsigned int k0, k1, k2, k3, o0, o1;
    band_keys(a0, b0, sink4, k0, k1, o0);
    band_keys(a1, b1, sink4, k2, k3, o1);
    // Order matters for the LDS wait counts (LDS operations complete in order): the rare
    // outlier appends (a returning atomic) first, then the next chunk's loads, then this chunk's
    // eight atomics — every path then has the loads followed by exactly eight LDS operations, so
    // the next iteration waits for the loads only (lgkmcnt(8)), not for the atomics.  For the
    // same reason every pair is added (background and outliers to the lane's sink counter): a
    // skipped chunk would leave the wait count path-dependent, i.e. a full drain.
    if ((o0 | o1) != 0u) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int sft = 8 * (u & 3);
        if (((u < 4 ? o0 : o1) >> sft) & 0x80u) {
          const unsigned int a = ((u < 4 ? a0 : a1) >> sft) & 255u, b = ((u < 4 ? b0 : b1) >> sft) & 255u;
          const int pos = atomicAdd(n_out, 1);
          if (pos < kOutCap) outl[pos] = (unsigned short)((a << 8) | b);
        }
      }
    }
    p += step;
    ci += sc;
    if (ci >= nch) ci -= nch;
    if (p >= (unsigned)nc) p -= nc;
    band_load<sh, sh == 0>(crop + 8 * (int)p, boff, A, L, R);  // (p < nc: past the last chunk a spare valid load)
    band_add(tab, k0);
    band_add(tab, k0 >> 16);
    band_add(tab, k1);
    band_add(tab, k1 >> 16);
    band_add(tab, k2);
    band_add(tab, k2 >> 16);
    band_add(tab, k3);
    band_add(tab, k3 >> 16);
  }
}

// Scan + clear of the band table (nine 16-byte groups per thread, all loaded before the first
// use), then the outlier keys (sum c^2 from equal-key counts).
__device__ __forceinline__ void band_scan(unsigned int* tab, const unsigned short* outl, int n_out,
                                          const unsigned long long* hom, BandAcc& S) {
  uint4* t4 = reinterpret_cast<uint4*>(tab);
  constexpr int n4 = kBandScan * 32;
  uint4 w[kScanG];
#pragma unroll
  for (int k = 0; k < kScanG; ++k) {
    const int u = threadIdx.x + k * kBT;
    w[k] = u < n4 ? t4[u] : uint4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int k = 0; k < kScanG; ++k) {
    const int u = threadIdx.x + k * kBT;
    if ((w[k].x | w[k].y | w[k].z | w[k].w) == 0u) continue;
    t4[u] = uint4{0u, 0u, 0u, 0u};
    const int row = u >> 5;
    const unsigned int e0 = (unsigned int)(u & 31) << 3;
    unsigned int s0 = dot2_u16(w[k].x, 0x10001u, 0u);
    s0 = dot2_u16(w[k].y, 0x10001u, s0);
    s0 = dot2_u16(w[k].z, 0x10001u, s0);
    s0 = dot2_u16(w[k].w, 0x10001u, s0);
    unsigned int q = dot2_u16(w[k].x, w[k].x, 0u);
    q = dot2_u16(w[k].y, w[k].y, q);
    q = dot2_u16(w[k].z, w[k].z, q);
    q = dot2_u16(w[k].w, w[k].w, q);
    // sum h c_h and sum h^2 c_h over the group's counters h = 0..7 (low half first)
    unsigned int sk = dot2_u16(w[k].x, 0x00010000u, 0u);
    sk = dot2_u16(w[k].y, 0x00030002u, sk);
    sk = dot2_u16(w[k].z, 0x00050004u, sk);
    sk = dot2_u16(w[k].w, 0x00070006u, sk);
    unsigned int skk = dot2_u16(w[k].x, 0x00010000u, 0u);
    skk = dot2_u16(w[k].y, 0x00090004u, skk);
    skk = dot2_u16(w[k].z, 0x00190010u, skk);
    skk = dot2_u16(w[k].w, 0x00310024u, skk);
    const unsigned int s1 = e0 * s0 + sk, s2 = e0 * e0 * s0 + 2u * e0 * sk + skk;
    S.cnt += s0;
    S.asq += q;
    if (row < 2 * kBandD + 1) {
      const int d = row - kBandD;
      const unsigned int ud = (unsigned int)d, ad = (unsigned int)(d < 0 ? -d : d);
      S.si += s1;
      S.sj += s1 + ud * s0;
      S.sii += s2;
      S.sjj += s2 + 2u * ud * s1 + ud * ud * s0;
      S.sij += s2 + ud * s1;
      S.dis += ad * s0;
      S.hom += hom[ad] * s0;
    } else {
      // (0, j = e) or (i = e, 0): |i - j| = e
      if (row == 2 * kBandD + 1) {
        S.sj += s1;
        S.sjj += s2;
      } else {
        S.si += s1;
        S.sii += s2;
      }
      S.dis += s1;
      const unsigned int v[4] = {w[k].x, w[k].y, w[k].z, w[k].w};
#pragma unroll
      for (int h = 0; h < 8; ++h) S.hom += hom[e0 + h] * ((v[h >> 1] >> (16 * (h & 1))) & 0xffffu);
    }
  }
  for (int e = threadIdx.x; e < n_out; e += kBT) {
    const unsigned int key = outl[e];
    unsigned int c = 0;
    for (int f = 0; f < n_out; ++f) c += outl[f] == key;
    const unsigned int i = key >> 8, j = key & 255u, ad = i > j ? i - j : j - i;
    S.asq += c;
    S.cnt += 1u;
    S.si += i;
    S.sj += j;
    S.sii += i * i;
    S.sjj += j * j;
    S.sij += i * j;
    S.dis += ad;
    S.hom += hom[ad];
  }
}

// Wave totals on the DPP path (row shifts within 16 lanes, then the row broadcasts): lane 63
// holds the sum.
__device__ __forceinline__ unsigned int wave_total_u32(unsigned int v) {
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
__device__ __forceinline__ unsigned long long wave_total_u64(unsigned long long v) {
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
  return v;
}

// greycoprops totals of one angle (raw layout of k_glcm_props: si, sj, sii, sjj, sij, dis, asq,
// cnt, homogeneity split into low / high 32 bits at write-back): lane 63 of each wave adds its
// wave's totals to the block's
__device__ __forceinline__ void band_reduce(const BandAcc& S, unsigned long long* tot) {
  const unsigned int v[8] = {S.si, S.sj, S.sii, S.sjj, S.sij, S.dis, S.asq, S.cnt};
  unsigned int x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = wave_total_u32(v[k]);
  const unsigned long long h = wave_total_u64(S.hom);
  if ((threadIdx.x & 63) == 63) {
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(&tot[k], (unsigned long long)x[k]);
    atomicAdd(&tot[8], h);
  }
}

template <int A>
__device__ __forceinline__ void band_angle(const GlcmItem& it, const unsigned char* crop, unsigned int* tab,
                                           unsigned short* outl, int* n_out, const unsigned long long* hom,
                                           unsigned long long* tot, bool& overflow) {
  // the outlier counters alternate by angle: this angle's is read by every thread after the
  // barrier below, the other one (read by the previous angle before it) is reset meanwhile
  int* cnt = n_out + (A & 1);
  long long pt = 0;
#ifdef CPX_GLCM_PROF
  if (threadIdx.x == 0) pt = clock64();
#endif
  if (it.bytes <= kBandCrop) band_count<A, true>(crop, tab, outl, cnt, it.bh, it.bw);
  else band_count<A, false>(it.src, tab, outl, cnt, it.bh, it.bw);
  __syncthreads();
  GLCM_MARK(1, &pt);
  const int n = *cnt;
  if (threadIdx.x == 0) n_out[(A + 1) & 1] = 0;
  overflow |= n > kOutCap;
  BandAcc S{};
  band_scan(tab, outl, min(n, kOutCap), hom, S);
  GLCM_MARK(2, &pt);
  band_reduce(S, tot + A * kRedW);
  __syncthreads();  // the table is clear and the outlier list read before the next angle
  GLCM_MARK(3, &pt);
}

// the LDS-sized crop of an item into registers (kCropG uint4 per thread; zeros past its end)
__device__ __forceinline__ void band_crop_regs(const GlcmItem& g, uint4 (&r)[kCropG]) {
  const int n16 = (g.nb > 0 && g.bytes <= kBandCrop) ? g.bytes / 16 : 0;
  const uint4* s16 = reinterpret_cast<const uint4*>(g.src);
#pragma unroll
  for (int k = 0; k < kCropG; ++k) {
    const int x = threadIdx.x + k * kBT;
    r[k] = x < n16 ? s16[x] : uint4{0u, 0u, 0u, 0u};
  }
}

// Per-item GLCM (see above).  Items come from the per-FOV queues as in k_tex_glcm, one item
// ahead: the next item's code is claimed, its metadata loaded and its crop read into registers
// while the current item runs.  An item whose outlier list overflowed is appended to `redo`
// ([0] count, [1] claim counter, [2..] codes) for k_tex_glcm, which writes its raw sums.
__global__ __launch_bounds__(kBT) __attribute__((amdgpu_waves_per_eu(3 * kBT / 256))) void k_tex_band(int C, int max_label,
                                                 const cpx_object* __restrict__ objects,
                                                 const cpx_fov_objects* __restrict__ hdr,
                                                 const long long* __restrict__ crop_off,
                                                 const unsigned char* __restrict__ scratch,
                                                 long long scratch_per_fov, int* __restrict__ glcm_next,
                                                 unsigned long long* __restrict__ glcm_raw,
                                                 int* __restrict__ redo) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kBandLds];
  unsigned int* tab = reinterpret_cast<unsigned int*>(lds);
  unsigned short* outl = reinterpret_cast<unsigned short*>(lds + 4 * kBandW);
  unsigned long long* s_hom = reinterpret_cast<unsigned long long*>(lds + 4 * kBandW + 2 * kOutCap);
  unsigned long long* s_tot = s_hom + 256;
  int* s_cnt = reinterpret_cast<int*>(s_tot + 4 * kRedW);  // [0], [1] outlier counters
  int* s_code = s_cnt + 2;                                  // [0], [1] queue codes by parity
  unsigned char* crop = lds + kBandLds - kBandCrop;
  const int B = gridDim.y;
  int q_fov = blockIdx.y, q_visited = 0;  // thread 0's queue position
  for (int x = threadIdx.x; x < kBandW; x += kBT) tab[x] = 0u;
  for (int x = threadIdx.x; x < 256; x += kBT) s_hom[x] = kHom.m[x];
  for (int x = threadIdx.x; x < 4 * kRedW; x += kBT) s_tot[x] = 0ull;
  if (threadIdx.x == 0) {
    s_cnt[0] = s_cnt[1] = 0;
    s_code[0] = glcm_grab(q_fov, q_visited, B, C, hdr, glcm_next);
    s_code[1] = s_code[0] >= 0 ? glcm_grab(q_fov, q_visited, B, C, hdr, glcm_next) : -1;
  }
  __syncthreads();
  GlcmItem cur = glcm_item(s_code[0], C, max_label, objects, crop_off, scratch, scratch_per_fov);
  uint4 pre[kCropG];
  band_crop_regs(cur, pre);
  long long pt0 = 0;
#ifdef CPX_GLCM_PROF
  if (threadIdx.x == 0) pt0 = clock64();
#endif
  for (int par = 0; s_code[par] >= 0; par ^= 1) {
    // s_code[par]: the current item (cur), s_code[par ^ 1]: the next one; s_code[par] receives
    // the item after that before the closing barrier
    const GlcmItem it = cur;
    const int code = s_code[par];
#pragma unroll
    for (int k = 0; k < kCropG; ++k)
      if (threadIdx.x + k * kBT < it.bytes / 16 && it.bytes <= kBandCrop)
        reinterpret_cast<uint4*>(crop)[threadIdx.x + k * kBT] = pre[k];
    __syncthreads();  // crop staged
    GLCM_MARK(0, &pt0);
    const int ncode = s_code[par ^ 1];
    int ahead = -1;
    if (threadIdx.x == 0 && ncode >= 0) ahead = glcm_grab(q_fov, q_visited, B, C, hdr, glcm_next);
    cur = glcm_item(ncode, C, max_label, objects, crop_off, scratch, scratch_per_fov);
    bool overflow = false;
    if (it.nb > 0) {
#ifdef CPX_GLCM_PROF
      if (threadIdx.x == 0) {
        atomicAdd(&g_glcm_prof[5], 1ull);
        atomicAdd(&g_glcm_prof[6], (unsigned long long)it.nb);
      }
#endif
      band_angle<0>(it, crop, tab, outl, s_cnt, s_hom, s_tot, overflow);
      band_crop_regs(cur, pre);  // (the next item's metadata has arrived by now)
      band_angle<1>(it, crop, tab, outl, s_cnt, s_hom, s_tot, overflow);
      band_angle<2>(it, crop, tab, outl, s_cnt, s_hom, s_tot, overflow);
      band_angle<3>(it, crop, tab, outl, s_cnt, s_hom, s_tot, overflow);
      unsigned long long* f = glcm_raw + (((long long)it.fov * max_label + it.k) * C + it.ch) * (4 * kRedW);
      if (overflow) {
        if (threadIdx.x == 0) redo[2 + atomicAdd(&redo[0], 1)] = code;
      } else if (threadIdx.x < 4 * kRedW) {
        const int a = threadIdx.x / kRedW, k = threadIdx.x - a * kRedW;
        const unsigned long long h = s_tot[a * kRedW + 8];
        f[threadIdx.x] = k < 8 ? s_tot[threadIdx.x] : k == 8 ? (h & 0xffffffffull) : (h >> 32);
      }
    } else {
      band_crop_regs(cur, pre);
    }
    if (threadIdx.x == 0) s_code[par] = ahead;
    __syncthreads();  // totals read, the crop buffer free, the codes visible
    for (int x = threadIdx.x; x < 4 * kRedW; x += kBT) s_tot[x] = 0ull;
#ifdef CPX_GLCM_PROF
    if (threadIdx.x == 0) {
      const long long t_ = clock64();
      atomicAdd(&g_glcm_prof[4], (unsigned long long)(t_ - pt0));
      pt0 = t_;
    }
#endif
  }
}

// crop slots: per FOV exclusive scan of C * bbox area; objects beyond the scratch capacity or
// with bbox > 65535 px get -1 (fallback kernel).
__global__ __launch_bounds__(1024) void k_crop_offsets(int C, int max_label,
                                                      const cpx_object* __restrict__ objects,
                                                      const cpx_fov_objects* __restrict__ hdr,
                                                      long long cap, long long* __restrict__ crop_off,
                                                      int* __restrict__ glcm_next, cpx_fallback_lists fb,
                                                      int* __restrict__ redo) {
  const int fov = blockIdx.x;
  const int n = hdr[fov].n_objects;
  if (threadIdx.x == 0) {  // this FOV's work queues: k_tex_band [0, B), k_obj_stage [B, 2B)
    glcm_next[fov] = 0;
    glcm_next[gridDim.x + fov] = 0;
    if (fov == 0) redo[0] = redo[1] = 0;
  }
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
      const int bh = o.bbox[2] - o.bbox[0], bw = o.bbox[3] - o.bbox[1];
      // staged texture needs the fast path's membership bitmask (k_obj_stage)
      sz = ((long long)bh * bw <= 65535 && cpx_shape_fits(bh, bw)) ? crop_bytes(bh, bw) * C : 0;
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
constexpr int kShapeW = kFastShapeWords;  // 8 KiB per bitmask (x2: membership + border)

__device__ __forceinline__ unsigned int getw(const unsigned int* m, int wpr, int rows, int r, int cw) {
  return (r < 0 || r >= rows || cw < 0 || cw >= wpr) ? 0u : m[r * wpr + cw];
}

__device__ __forceinline__ bool shape_fits(const cpx_object& o) {
  return cpx_shape_fits(o.bbox[2] - o.bbox[0], o.bbox[3] - o.bbox[1]);
}

// Membership bitmask of object o over its bbox + 2-px margin (rows x wpr words in M): each
// 32-lane half-wave builds one 32-bit word (r, cw); eight words per half-wave are loaded before
// the first ballot so the label loads overlap.
// The membership words from 16-byte label loads: a lane reads 4
// consecutive labels (raw buffer load, dword-aligned; four 4-byte loads where the piece would
// cross the plane's ends), 8 lanes form a 32-pixel word, their 4-bit pieces OR-reduced over the
// 8 lanes — instead of one 4-byte load per lane and pixel and a ballot per word: features -2-3 %
// per object set (`gpurun_out/r05ab`)
template <int NT>
__device__ __forceinline__ void shape_mask16(const int* __restrict__ lab, int H, int W, const cpx_object& o,
                                             unsigned int* M) {
  constexpr int U = 4;  // words per lane group and iteration (loads in flight per lane)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int sub = lane & 7, grp = lane >> 3;  // 4-pixel piece of the word, word slot of the wave
  const int L = o.label;
  const int R0 = o.bbox[0] - 2, C0 = o.bbox[1] - 2;  // region origin (2-px margin)
  const int rows = o.bbox[2] - o.bbox[0] + 4, cols = o.bbox[3] - o.bbox[1] + 4;
  const int wpr = (cols + 31) >> 5;
  const int nw = rows * wpr;
  const bool v4ok = (long long)H * W < (1LL << 29);  // the buffer's byte range is an int
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(lab), (short)0, v4ok ? H * W * 4 : 0, 0x00020000);
  for (int w0 = wv * 8 * U; w0 < nw; w0 += (NT / 64) * 8 * U) {
    int4 lv[U];
    int cc[U], gcc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int w = w0 + u * 8 + grp;
      const int r = w / wpr, cw = w - r * wpr;
      const int c = cw * 32 + sub * 4, gr = R0 + r, gc = C0 + c;
      cc[u] = w < nw ? c : cols;  // a slot past the mask's words: no member bits
      gcc[u] = gc;
      const bool row_ok = w < nw && gr >= 0 && gr < H;
      const long long idx = (long long)gr * W + gc;
      // columns outside [0, W) are masked below; the 16 bytes must lie inside the plane (at its
      // first and last pixels, where the piece would cross the plane's ends, four 4-byte loads)
      if (v4ok && row_ok && idx >= 0 && idx + 4 <= (long long)H * W) {
        lv[u] = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(idx * 4), 0, 0));
      } else {
        int t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = (row_ok && gc + k >= 0 && gc + k < W) ? lab[idx + k] : 0;
        lv[u] = make_int4(t[0], t[1], t[2], t[3]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v[4] = {lv[u].x, lv[u].y, lv[u].z, lv[u].w};
      unsigned int bits = 0u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = cc[u] + k, gc = gcc[u] + k;
        bits |= (unsigned int)(v[k] == L && c < cols && gc >= 0 && gc < W) << k;
      }
      unsigned int word = bits << (4 * sub);
      word |= __shfl_xor(word, 1, 8);
      word |= __shfl_xor(word, 2, 8);
      word |= __shfl_xor(word, 4, 8);
      const int w = w0 + u * 8 + grp;
      if (sub == 0 && w < nw) M[w] = word;
    }
  }
}

template <int NT>
__device__ __forceinline__ void shape_mask(const int* __restrict__ lab, int H, int W, const cpx_object& o,
                                           unsigned int* M) {
  shape_mask16<NT>(lab, H, W, o, M);
}

// AreaShape sums of object o from its membership mask M (shape_mask; all threads, M complete and
// visible): border mask in Bd, Benkrid-Crookes perimeter codes, exact int64 moments -> raw[0..8]
// (n, sum r, sum c, sum r^2, sum c^2, sum rc, n1, n2, n3); k_shape_props turns them into the
// AreaShape columns (the fp64 tail runs once per object there instead of in every stage kernel,
// whose registers it would otherwise inflate).
constexpr int kShapeRaw = 9;
template <int NT>
__device__ void shape_sums(const cpx_object& o, const unsigned int* M, unsigned int* Bd,
                           long long (*red)[NT / 64], int (*redi)[NT / 64], long long* __restrict__ raw) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rows = o.bbox[2] - o.bbox[0] + 4, cols = o.bbox[3] - o.bbox[1] + 4;
  const int wpr = (cols + 31) >> 5;
  // border = in & !(up & down & left & right)
  for (int w = threadIdx.x; w < rows * wpr; w += NT) {
    const int r = w / wpr, cw = w - r * wpr;
    const unsigned int x = M[w];
    const unsigned int up = getw(M, wpr, rows, r - 1, cw), dn = getw(M, wpr, rows, r + 1, cw);
    const unsigned int lf = (x << 1) | (getw(M, wpr, rows, r, cw - 1) >> 31);
    const unsigned int rt = (x >> 1) | (getw(M, wpr, rows, r, cw + 1) << 31);
    Bd[w] = x & ~(up & dn & lf & rt);
  }
  __syncthreads();
  // per word, bit-parallel (every sum is an exact integer, so the order does not matter): the
  // column sums from popcounts of the word against the bit-index masks (sum b = sum_k 2^k
  // popc(x & m_k), sum b^2 from the pairwise products), and the Benkrid-Crookes codes
  // 1 + 2 a + 10 d (a / d = border 4- / diagonal neighbours) from bit-sliced neighbour counts:
  // n1 = codes 5, 7, 15, 17, 25, 27 (a in {2, 3}, d <= 2), n2 = 21, 33 ((a, d) = (0, 2) or
  // (1, 3)), n3 = 13, 23 (a = 1, d in {1, 2})
  constexpr unsigned int kBm[5] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u};
  long long n = 0, sr = 0, sc = 0, srr = 0, scc = 0, src = 0;
  int n1 = 0, n2 = 0, n3 = 0;
  for (int w = threadIdx.x; w < rows * wpr; w += NT) {
    const int r = w / wpr, cw = w - r * wpr;
    const unsigned int x = M[w];
    if (x) {
      const long long p = __popc(x);
      int pk[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) pk[k] = __popc(x & kBm[k]);
      long long s1 = 0, s2 = 0;
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        s1 += (long long)pk[k] << k;
        s2 += (long long)pk[k] << (2 * k);
#pragma unroll
        for (int j = k + 1; j < 5; ++j) s2 += (long long)__popc(x & kBm[k] & kBm[j]) << (k + j + 1);
      }
      const long long rr = r - 2, base = (long long)cw * 32 - 2;  // bbox-local row, column of bit 0
      const long long csum = base * p + s1;
      n += p;
      sr += rr * p;
      srr += rr * rr * p;
      sc += csum;
      scc += base * base * p + 2 * base * s1 + s2;
      src += rr * csum;
    }
    const unsigned int bx = Bd[w];
    if (bx) {
      auto lf = [&](int rw, unsigned int v) { return (v << 1) | (getw(Bd, wpr, rows, rw, cw - 1) >> 31); };
      auto rt = [&](int rw, unsigned int v) { return (v >> 1) | (getw(Bd, wpr, rows, rw, cw + 1) << 31); };
      const unsigned int U = getw(Bd, wpr, rows, r - 1, cw), D = getw(Bd, wpr, rows, r + 1, cw);
      // bit-sliced a = U + D + L + R and d = UL + UR + DL + DR (0..4 each: bits a2 a1 a0)
      auto count4 = [](unsigned int A, unsigned int B, unsigned int C, unsigned int E, unsigned int& c2,
                       unsigned int& c1, unsigned int& c0) {
        const unsigned int s0 = A ^ B, k0 = A & B, s1_ = C ^ E, k1 = C & E;
        const unsigned int cy = s0 & s1_;
        c0 = s0 ^ s1_;
        c1 = k0 ^ k1 ^ cy;
        c2 = (k0 & k1) | (cy & (k0 ^ k1));
      };
      unsigned int a2, a1, a0, d2, d1, d0;
      count4(U, D, lf(r, bx), rt(r, bx), a2, a1, a0);
      count4(lf(r - 1, U), rt(r - 1, U), lf(r + 1, D), rt(r + 1, D), d2, d1, d0);
      const unsigned int aeq0 = ~a2 & ~a1 & ~a0, aeq1 = ~a2 & ~a1 & a0, a23 = ~a2 & a1;
      const unsigned int deq1 = ~d2 & ~d1 & d0, deq2 = ~d2 & d1 & ~d0, deq3 = ~d2 & d1 & d0;
      const unsigned int dle2 = ~d2 & ~(d1 & d0);
      n1 += __popc(bx & a23 & dle2);
      n2 += __popc(bx & ((aeq0 & deq2) | (aeq1 & deq3)));
      n3 += __popc(bx & aeq1 & (deq1 | deq2));
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
  if (threadIdx.x < kShapeRaw) {
    long long t = 0;
    for (int w = 0; w < NT / 64; ++w) t += threadIdx.x < 6 ? red[threadIdx.x][w] : (long long)redi[threadIdx.x - 6][w];
    raw[threadIdx.x] = t;
  }
}

// AreaShape columns from shape_sums' raw sums, one thread per object (objects the LDS fast
// paths handled: shape_fits).
__global__ __launch_bounds__(256) void k_shape_props(int max_label, int F,
                                                    const cpx_object* __restrict__ objects,
                                                    const cpx_fov_objects* __restrict__ hdr,
                                                    const long long* __restrict__ raws,
                                                    double* __restrict__ feats) {
  const int fov = blockIdx.y, k = blockIdx.x * 256 + threadIdx.x;
  if (k >= hdr[fov].n_objects) return;
  const cpx_object o = objects[(long long)fov * max_label + k];
  if (!shape_fits(o)) return;
  const long long* raw = raws + ((long long)fov * max_label + k) * kShapeRaw;
  const long long n = raw[0], sr = raw[1], sc = raw[2], srr = raw[3], scc = raw[4], src = raw[5];
  const long long n1 = raw[6], n2 = raw[7], n3 = raw[8];
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

// Per-object staging (one block per object, objects strided over the FOV's blocks): the label
// image is read once per object into the bbox membership bitmask (AreaShape sums from it), then
// each channel's bbox is read for the Intensity columns and the scale_to_8bit range and
// quantised into the object's 8-bit crop slot for k_tex_glcm.  The first kOT * kOG 4-pixel
// groups stay in registers between the two passes; the rest of a large bbox is read twice, with
// the block's working set (one channel of one bbox, two blocks per CU) L2-resident in between.
// block size and waves per SIMD of k_obj_stage (the object-per-block staging is latency-bound:
// objects in flight per CU = blocks per CU; 3 blocks per CU at 80 VGPRs and 256-thread blocks at
// 6 / 4 and 8 / 5 measured equal or slower, `gpurun_out/r05k`)
constexpr int kOT = 512;
constexpr int stage_wpe(bool) { return 4; }
constexpr int stage_blocks_per_cu(bool twin) { return stage_wpe(twin) * 4 / (kOT / 64); }
constexpr int kOG = 1;
constexpr int kOR = 4;  // groups per iteration beyond the register-held ones

// in-bbox membership of the 4 pixels (r, c .. c + 3) from the bbox + 2-px margin bitmask
__device__ __forceinline__ unsigned int member4(const unsigned int* M, int wpr, int r, int c) {
  const int cb = c + 2, w = cb >> 5, sh = cb & 31;
  const unsigned int* row = M + (r + 2) * wpr;
  const unsigned long long two = (unsigned long long)row[w] |
                                 ((unsigned long long)(w + 1 < wpr ? row[w + 1] : 0u) << 32);
  return (unsigned int)(two >> sh) & 15u;
}

__device__ __forceinline__ unsigned int group_desc(const unsigned int* M, int wpr, int bw, int bwp, int W,
                                                   int g) {
  const int f0 = 4 * g, r = f0 / bwp, c = f0 - r * bwp;
  return (unsigned int)(r * W + c) | (member4(M, wpr, r, c) << 24) | ((unsigned int)min(4, bw - c) << 28);
}

// Intensity columns from the member count and sums (regionprops intensity_* in fp64)
__device__ __noinline__ void int_finish(double* f, long long n, double sm, double ss, float omin, float omax) {
  const double mean = n ? sm / (double)n : 0.0;
  double var = n ? (ss - sm * mean) / (double)n : 0.0;
  if (var < 0.0) var = 0.0;
  f[CPX_INT_INTEGRATED] = sm;
  f[CPX_INT_MEAN] = mean;
  f[CPX_INT_STD] = sqrt(var);
  f[CPX_INT_MIN] = (double)omin;
  f[CPX_INT_MAX] = (double)omax;
}

// load at a 32-bit byte offset from a block-uniform base (SGPR base + VGPR offset addressing)
__device__ __forceinline__ float ldg_b(const float* base, unsigned int byte_off) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(base) + byte_off);
}

// A 4-pixel group as one 16-byte raw buffer load (dword-aligned; the lanes past a row's bbox read
// pixels they then ignore, past the plane the buffer returns 0) instead of four 4-byte loads: a
// quarter of the vector-memory instructions (k_obj_stage 5.52 -> 5.28 ms per step,
// `gpurun_out/r05n`).  v4 is false for planes of 2^29 or more pixels (the buffer's byte range is
// an int): four 4-byte loads then.
__device__ __forceinline__ void ld_group(float (&dst)[4], const float* img, __amdgpu_buffer_rsrc_t rs,
                                         unsigned int img_off, unsigned int o0, unsigned int nv, bool v4) {
  if (v4) {
    const float4 t = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, 4u * (img_off + o0), 0, 0));
    dst[0] = t.x;
    dst[1] = t.y;
    dst[2] = t.z;
    dst[3] = t.w;
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) dst[u] = ldg_b(img, 4u * (o0 + min((unsigned int)u, nv - 1u)));
  }
}

struct IntAcc {
  long long n;
  double sm, ss;
  float omin, omax, mmin, mmax;
};

__device__ __forceinline__ void int_acc(IntAcc& a, float v, bool in) {
  const float m = v * (in ? 1.0f : 0.0f);
  a.mmin = fminf(a.mmin, m);
  a.mmax = fmaxf(a.mmax, m);
  if (in) {
    a.n += 1;
    a.sm += (double)v;
    a.ss += (double)v * (double)v;
    a.omin = fminf(a.omin, v);
    a.omax = fmaxf(a.omax, v);
  }
}

// The twin object set of a k_obj_stage<true> pass (Cytoplasm beside Cells: the same ObjectNumber,
// its pixels a subset of the cell's, so a Cytoplasm object whose bbox equals its cell's is staged
// from the same reads of the channels): its label image, tables and staging outputs, the Cells
// object -> twin object map, and the per-object flags of the twins staged here (the twin set's
// own k_obj_stage pass skips them).
struct StageTwin {
  const int* labels;
  const cpx_object* objects;
  const long long* crop_off;
  unsigned char* scratch;
  long long* raws;
  double* feats;
  const int* map;   // [B][max_label]: Cells object k -> twin object index, or -1
  int* done;        // [B][max_label]: twin object staged by the Cells pass
};

template <bool TWIN>
__global__ __launch_bounds__(kOT) __attribute__((amdgpu_waves_per_eu(stage_wpe(TWIN)))) void k_obj_stage(const int* __restrict__ labels,
                                                  const float* __restrict__ corr, int C, int H,
                                                  int W, int max_label, int F,
                                                  const cpx_object* __restrict__ objects,
                                                  const cpx_fov_objects* __restrict__ hdr,
                                                  const long long* __restrict__ crop_off,
                                                  unsigned char* __restrict__ scratch,
                                                  long long scratch_per_fov,
                                                  long long* __restrict__ raws,
                                                  int* __restrict__ obj_next,
                                                  double* __restrict__ feats,
                                                  const int* __restrict__ skip, StageTwin tw) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned int* M = reinterpret_cast<unsigned int*>(smem);
  unsigned int* Bd = M + kShapeW;
  unsigned int* M2 = Bd + kShapeW;  // the twin's membership mask (TWIN only)
  __shared__ long long red[6][kOT / 64];
  __shared__ int redi[3][kOT / 64];
  __shared__ double sd_[2][2][2][kOT / 64];  // [set / twin][channel parity]: no barrier before the
  __shared__ long long sn_[2][2][kOT / 64];   // next channel's partials overwrite them
  __shared__ float sf_[2][2][4][kOT / 64];
  __shared__ int s_code;
  const int fov = blockIdx.y, B = gridDim.y;
  const long long N = (long long)H * W;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int q_fov = fov, q_visited = 0;  // thread 0's queue position (glcm_grab: own FOV first, then
  long long tprof = clock64();      // (CPX_STAGE_PROF only)
  (void)tprof;
  while (true) {                    // the next ones, each FOV at most once)
    __syncthreads();  // the previous object's LDS reads are done before s_code / M change
    if (threadIdx.x == 0) s_code = glcm_grab(q_fov, q_visited, B, 1, hdr, obj_next);
    __syncthreads();
    const int code = __builtin_amdgcn_readfirstlane(s_code);  // block-uniform: scalar registers
    if (code < 0) break;
    const int fov = code >> 20, k = code & 0xfffff;
    if (skip && skip[(long long)fov * max_label + k]) continue;  // staged by the twin pass
    const int* lab = labels + (long long)fov * N;
    const cpx_object o = objects[(long long)fov * max_label + k];
    if (!shape_fits(o)) continue;  // shape and texture both in the fallback kernels
    const long long off = crop_off[(long long)fov * max_label + k];
    STAGE_MARK(0, &tprof);
    // the twin rides along when it has the same bbox and both crops are staged (block-uniform)
    int ky = -1;
    long long offy = -1;
    if constexpr (TWIN) {
      ky = tw.map[(long long)fov * max_label + k];
      if (ky >= 0) {
        const cpx_object y = tw.objects[(long long)fov * max_label + ky];
        offy = tw.crop_off[(long long)fov * max_label + ky];
        if (off < 0 || offy < 0 || y.bbox[0] != o.bbox[0] || y.bbox[1] != o.bbox[1] ||
            y.bbox[2] != o.bbox[2] || y.bbox[3] != o.bbox[3])
          ky = -1;
      }
      ky = __builtin_amdgcn_readfirstlane(ky);
    }
    shape_mask<kOT>(lab, H, W, o, M);
    if (TWIN && ky >= 0) {
      const cpx_object y = tw.objects[(long long)fov * max_label + ky];
      shape_mask<kOT>(tw.labels + (long long)fov * N, H, W, y, M2);
    }
    __syncthreads();
    STAGE_MARK(1, &tprof);
    shape_sums<kOT>(o, M, Bd, red, redi, raws + ((long long)fov * max_label + k) * kShapeRaw);
    if (TWIN && ky >= 0) {
      const cpx_object y = tw.objects[(long long)fov * max_label + ky];
      __syncthreads();  // the first sums' reads of Bd / red are done
      shape_sums<kOT>(y, M2, Bd, red, redi, tw.raws + ((long long)fov * max_label + ky) * kShapeRaw);
      if (threadIdx.x == 0) tw.done[(long long)fov * max_label + ky] = 1;
    }
    STAGE_MARK(2, &tprof);
    if (off < 0) continue;  // texture not staged: fallback kernel (block-uniform)
    const int r0 = o.bbox[0], c0 = o.bbox[1];
    const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
    const int wpr = (bw + 4 + 31) >> 5;
    const int bwp = crop_stride(bw);
    const int ng = bh * bwp / 4;  // 4-pixel groups (bwp % 4 == 0: a group never spans rows)
    const long long cbytes = crop_bytes(bh, bw);
    STAGE_COUNT(6, 1);
    STAGE_COUNT(7, ng);
    // group descriptors of the register-held groups, the same for every channel: bbox offset of
    // the group's first pixel (< 2^24: shape_fits bounds bh by 4092, and only images with
    // W <= 4096 stage crops)
    // | member bits << 24 | valid pixels (1..4) << 28
    unsigned int gd[kOG], gm2[kOG];  // gm2: the twin's member bits of the same groups
#pragma unroll
    for (int i = 0; i < kOG; ++i) {
      const int g = min((int)threadIdx.x + i * kOT, ng - 1);
      gd[i] = group_desc(M, wpr, bw, bwp, W, g);
      gm2[i] = 0u;
      if (TWIN && ky >= 0) {
        const int f0 = 4 * g, r = f0 / bwp, c = f0 - r * bwp;
        gm2[i] = member4(M2, wpr, r, c);
      }
    }
    for (int ch = 0; ch < C; ++ch) {
      const float* plane = corr + ((long long)fov * C + ch) * N;
      const float* img = plane + (long long)r0 * W + c0;
      const unsigned int img_off = (unsigned int)(r0 * W + c0);
      const bool v4 = N < (1LL << 29);  // block-uniform
      const __amdgpu_buffer_rsrc_t rsp =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(plane), (short)0, v4 ? (int)(4 * N) : 0, 0x00020000);
      IntAcc a{0, 0.0, 0.0, INFINITY, -INFINITY, INFINITY, -INFINITY};
      IntAcc a2{0, 0.0, 0.0, INFINITY, -INFINITY, INFINITY, -INFINITY};
      float v[kOG][4];
      // opaque per channel: keeps the compiler from hoisting every load's offset out of the
      // channel loop (4 * kOG more VGPRs live across it)
#pragma unroll
      for (int i = 0; i < kOG; ++i) asm volatile("" : "+v"(gd[i]));
#pragma unroll
      for (int i = 0; i < kOG; ++i) {
        const unsigned int o0 = gd[i] & 0xffffffu, nv = gd[i] >> 28;
        ld_group(v[i], img, rsp, img_off, o0, nv, v4);
      }
#pragma unroll
      for (int i = 0; i < kOG; ++i) {
        if ((int)threadIdx.x + i * kOT >= ng) continue;
        const unsigned int mb = (gd[i] >> 24) & 15u, nv = gd[i] >> 28;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if ((unsigned int)u < nv) {
            int_acc(a, v[i][u], (mb >> u) & 1u);
            if (TWIN && ky >= 0) int_acc(a2, v[i][u], (gm2[i] >> u) & 1u);
          }
      }
      // groups past the register-held ones (large bboxes) are read twice; the block's working
      // set (one channel of one bbox) stays in L2 between the two passes.  kOR groups per
      // iteration, all their loads issued before any is used (one memory latency per kOR groups)
      for (int g0 = threadIdx.x + kOG * kOT; g0 < ng; g0 += kOR * kOT) {
        unsigned int d[kOR];
        float w4[kOR][4];
#pragma unroll
        for (int r = 0; r < kOR; ++r) {
          d[r] = group_desc(M, wpr, bw, bwp, W, min(g0 + r * kOT, ng - 1));
          const unsigned int o0 = d[r] & 0xffffffu, nv = d[r] >> 28;
          ld_group(w4[r], img, rsp, img_off, o0, nv, v4);
        }
#pragma unroll
        for (int r = 0; r < kOR; ++r) {
          if (g0 + r * kOT >= ng) continue;
          const unsigned int mb = (d[r] >> 24) & 15u, nv = d[r] >> 28;
          unsigned int mb2 = 0u;
          if (TWIN && ky >= 0) {
            const int f0 = 4 * (g0 + r * kOT), rr = f0 / bwp, cc = f0 - rr * bwp;
            mb2 = member4(M2, wpr, rr, cc);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if ((unsigned int)u < nv) {
              int_acc(a, w4[r][u], (mb >> u) & 1u);
              if (TWIN && ky >= 0) int_acc(a2, w4[r][u], (mb2 >> u) & 1u);
            }
        }
      }
      STAGE_MARK(3, &tprof);
      auto reduce = [&](IntAcc& x, int t, double* fout, float& mmin, float& mmax) {
        // t: which partial slots (0: this set, 1: the twin); channel parity double-buffers them
        x.n = wave_sum(x.n);
        x.sm = wave_sum(x.sm);
        x.ss = wave_sum(x.ss);
        x.omin = wave_min(x.omin);
        x.omax = wave_max(x.omax);
        x.mmin = wave_min(x.mmin);
        x.mmax = wave_max(x.mmax);
        long long* sn = sn_[t][ch & 1];
        double(*sd)[kOT / 64] = sd_[t][ch & 1];
        float(*sf)[kOT / 64] = sf_[t][ch & 1];
        if (lane == 0) {
          sn[wid] = x.n;
          sd[0][wid] = x.sm;
          sd[1][wid] = x.ss;
          sf[0][wid] = x.omin;
          sf[1][wid] = x.omax;
          sf[2][wid] = x.mmin;
          sf[3][wid] = x.mmax;
        }
        __syncthreads();
        // every thread needs only the crop range; thread 0 finishes the Intensity columns
        mmin = sf[2][0];
        mmax = sf[3][0];
#pragma unroll
        for (int w = 1; w < kOT / 64; ++w) {
          mmin = fminf(mmin, sf[2][w]);
          mmax = fmaxf(mmax, sf[3][w]);
        }
        if (threadIdx.x == 0) {
          long long n = 0;
          double sm = 0.0, ss = 0.0;
          float omin = INFINITY, omax = -INFINITY;
          for (int w = 0; w < kOT / 64; ++w) {
            n += sn[w];
            sm += sd[0][w];
            ss += sd[1][w];
            omin = fminf(omin, sf[0][w]);
            omax = fmaxf(omax, sf[1][w]);
          }
          int_finish(fout + CPX_N_SHAPE + (long long)ch * CPX_FEATURES_PER_CHANNEL, n, sm, ss, omin, omax);
        }
      };
      float mmin, mmax, mmin2 = 0.0f, mmax2 = 0.0f;
      reduce(a, 0, feats + ((long long)fov * max_label + k) * F, mmin, mmax);
      if (TWIN && ky >= 0) reduce(a2, 1, tw.feats + ((long long)fov * max_label + ky) * F, mmin2, mmax2);
      STAGE_MARK(4, &tprof);
      const float rng = mmax - mmin;
      const bool flat = !(mmax != mmin);
      const float rng2 = mmax2 - mmin2;
      const bool flat2 = !(mmax2 != mmin2);
      unsigned char* dst = scratch + (long long)fov * scratch_per_fov + off + (long long)ch * cbytes;
      unsigned char* dst2 = TWIN && ky >= 0 ? tw.scratch + (long long)fov * scratch_per_fov + offy + (long long)ch * cbytes
                                            : nullptr;
      // the crop at the padded row stride (pad bytes 0), one 32-bit store per 4-pixel group
#pragma unroll
      for (int i = 0; i < kOG; ++i) {
        const int g = threadIdx.x + i * kOT;
        if (g >= ng) continue;
        const unsigned int mb = (gd[i] >> 24) & 15u, nv = gd[i] >> 28;
        unsigned int word = 0u, word2 = 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned int q = (unsigned int)quantize(v[i][u], (mb >> u) & 1u, mmin, rng, flat);
          word |= ((unsigned int)u < nv ? q : 0u) << (8 * u);
          if (TWIN && ky >= 0) {
            const unsigned int q2 = (unsigned int)quantize(v[i][u], (gm2[i] >> u) & 1u, mmin2, rng2, flat2);
            word2 |= ((unsigned int)u < nv ? q2 : 0u) << (8 * u);
          }
        }
        *reinterpret_cast<unsigned int*>(dst + 4 * g) = word;
        if (TWIN && ky >= 0) *reinterpret_cast<unsigned int*>(dst2 + 4 * g) = word2;
      }
      for (int g0 = threadIdx.x + kOG * kOT; g0 < ng; g0 += kOR * kOT) {
        unsigned int d[kOR];
        float w4[kOR][4];
#pragma unroll
        for (int r = 0; r < kOR; ++r) {
          d[r] = group_desc(M, wpr, bw, bwp, W, min(g0 + r * kOT, ng - 1));
          const unsigned int o0 = d[r] & 0xffffffu, nv = d[r] >> 28;
          ld_group(w4[r], img, rsp, img_off, o0, nv, v4);
        }
#pragma unroll
        for (int r = 0; r < kOR; ++r) {
          const int g = g0 + r * kOT;
          if (g >= ng) continue;
          const unsigned int mb = (d[r] >> 24) & 15u, nv = d[r] >> 28;
          unsigned int mb2 = 0u;
          if (TWIN && ky >= 0) {
            const int f0 = 4 * g, rr = f0 / bwp, cc = f0 - rr * bwp;
            mb2 = member4(M2, wpr, rr, cc);
          }
          unsigned int word = 0u, word2 = 0u;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const unsigned int q = (unsigned int)quantize(w4[r][u], (mb >> u) & 1u, mmin, rng, flat);
            word |= ((unsigned int)u < nv ? q : 0u) << (8 * u);
            if (TWIN && ky >= 0) {
              const unsigned int q2 = (unsigned int)quantize(w4[r][u], (mb2 >> u) & 1u, mmin2, rng2, flat2);
              word2 |= ((unsigned int)u < nv ? q2 : 0u) << (8 * u);
            }
          }
          *reinterpret_cast<unsigned int*>(dst + 4 * g) = word;
          if (TWIN && ky >= 0) *reinterpret_cast<unsigned int*>(dst2 + 4 * g) = word2;
        }
      }
      STAGE_MARK(5, &tprof);
    }
  }
}

}  // namespace


// internal launchers used by cpx_features (k_features.hip)
namespace {

// one object set's feature workspace (slot WS_MISC or WS_MISC2): crop offsets [B][max_label],
// the GLCM / k_obj_stage queue counters, the fallback lists, the AreaShape raw sums, the GLCM
// integer totals and the 8-bit crop scratch (2 bytes per pixel-channel per FOV)
struct FeatWs {
  long long* crop_off;
  int* glcm_next;
  cpx_fallback_lists fb;
  long long* raws;
  unsigned long long* glcm_raw;
  int* redo;  // k_tex_band -> k_tex_glcm: [0] count, [1] claim counter, [2..] item codes
  unsigned char* scratch;
  long long per_fov;
  int* twin;  // [2][B][max_label]: the twin map and done flags (cpx_features_pair only)
};

int feat_ws(cpx_ctx* ctx, int slot, int B, int C, int H, int W, int max_label, bool twin, FeatWs* w) {
  w->per_fov = ((2LL * H * W * C + 255) / 256) * 256;
  const size_t off_bytes = ((sizeof(long long) * (size_t)B * max_label + sizeof(int) * (size_t)B * 4 +
                             sizeof(int) * 2 * (size_t)B * max_label + 255) / 256) * 256;
  const size_t raw_bytes = ((sizeof(long long) * kShapeRaw * (size_t)B * max_label + 255) / 256) * 256;
  const size_t glcm_bytes = ((sizeof(unsigned long long) * 4 * kRedW * (size_t)B * max_label * C + 255) / 256) * 256;
  const size_t twin_bytes = twin ? ((sizeof(int) * 2 * (size_t)B * max_label + 255) / 256) * 256 : 0;
  const size_t redo_bytes = ((sizeof(int) * (2 + (size_t)B * max_label * C) + 255) / 256) * 256;
  unsigned char* ws = (unsigned char*)cpx_ws(ctx, slot, off_bytes + raw_bytes + glcm_bytes + twin_bytes +
                                             redo_bytes + (size_t)B * w->per_fov + 256);  // +256: crop read slack
  if (!ws) return CPX_ERR_OOM;
  w->crop_off = (long long*)ws;
  w->glcm_next = (int*)(w->crop_off + (size_t)B * max_label);  // + k_obj_stage's queues at B
  w->fb.n_shape = w->glcm_next + 2 * B;
  w->fb.n_tex = w->fb.n_shape + B;
  w->fb.shape = w->fb.n_tex + B;
  w->fb.tex = w->fb.shape + (size_t)B * max_label;
  w->raws = (long long*)(ws + off_bytes);
  w->glcm_raw = (unsigned long long*)(ws + off_bytes + raw_bytes);
  w->twin = twin ? (int*)(ws + off_bytes + raw_bytes + glcm_bytes) : nullptr;
  w->redo = (int*)(ws + off_bytes + raw_bytes + glcm_bytes + twin_bytes);
  w->scratch = ws + off_bytes + raw_bytes + glcm_bytes + twin_bytes + redo_bytes;
  return CPX_OK;
}

size_t obj_stage_lds(bool twin) { return sizeof(unsigned int) * (twin ? 3 : 2) * kShapeW; }

int obj_stage_attr() {
  static bool attr = false;
  if (!attr) {
    CPX_CHECK_HIP(hipFuncSetAttribute((const void*)k_obj_stage<false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)obj_stage_lds(false)));
    CPX_CHECK_HIP(hipFuncSetAttribute((const void*)k_obj_stage<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)obj_stage_lds(true)));
    attr = true;
  }
  return CPX_OK;
}

// Cells object k -> Cytoplasm object with the same label (both tables ascending by label), or -1;
// clears the done flags.  One block per FOV.
__global__ __launch_bounds__(256) void k_twin_map(int max_label, const cpx_object* __restrict__ objects,
                                                  const cpx_fov_objects* __restrict__ hdr,
                                                  const cpx_object* __restrict__ tobjects,
                                                  const cpx_fov_objects* __restrict__ thdr,
                                                  int* __restrict__ map, int* __restrict__ done) {
  const int fov = blockIdx.x;
  const int n = hdr[fov].n_objects, nt = thdr[fov].n_objects;
  const cpx_object* t = tobjects + (long long)fov * max_label;
  for (int k = threadIdx.x; k < max_label; k += blockDim.x) {
    int m = -1;
    if (k < n) {
      const int L = objects[(long long)fov * max_label + k].label;
      int lo = 0, hi = nt;  // first index with label >= L
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (t[mid].label < L) lo = mid + 1;
        else hi = mid;
      }
      if (lo < nt && t[lo].label == L) m = lo;
    }
    map[(long long)fov * max_label + k] = m;
    done[(long long)fov * max_label + k] = 0;
  }
}

struct SetArgs {
  const int32_t* labels;
  const cpx_object* objects;
  const cpx_fov_objects* hdr;
  double* feats;
};

int launch_offsets(cpx_ctx* ctx, const SetArgs& a, FeatWs& w, int B, int C, int W, int max_label) {
  // k_obj_stage packs a staged crop's bbox offsets (bh <= 4092) x W in 24 bits: wider images
  // measure texture in the fallback kernel (cap 0: nothing staged)
  hipLaunchKernelGGL(k_crop_offsets, dim3(B), dim3(1024), 0, ctx->stream, C, max_label,
                     a.objects, a.hdr, W <= 4096 ? w.per_fov : 0LL, w.crop_off, w.glcm_next, w.fb, w.redo);
  CPX_CHECK_LAUNCH("k_crop_offsets");
  return CPX_OK;
}

int launch_stage(cpx_ctx* ctx, const SetArgs& a, FeatWs& w, const float* corr, int B, int C, int H, int W,
                 int max_label, int F, const int* skip, const StageTwin* tw) {
  int rc = obj_stage_attr();
  if (rc) return rc;
  const int bpc = stage_blocks_per_cu(tw != nullptr);
  const int per_fov_o = std::max(1, std::min(max_label, (bpc * ctx->n_cu + B - 1) / B));  // resident
  if (tw)
    hipLaunchKernelGGL(k_obj_stage<true>, dim3(per_fov_o, B), dim3(kOT), obj_stage_lds(true), ctx->stream,
                       (const int*)a.labels, corr, C, H, W, max_label, F, a.objects, a.hdr,
                       (const long long*)w.crop_off, w.scratch, w.per_fov, w.raws, w.glcm_next + B, a.feats,
                       skip, *tw);
  else
    hipLaunchKernelGGL(k_obj_stage<false>, dim3(per_fov_o, B), dim3(kOT), obj_stage_lds(false), ctx->stream,
                       (const int*)a.labels, corr, C, H, W, max_label, F, a.objects, a.hdr,
                       (const long long*)w.crop_off, w.scratch, w.per_fov, w.raws, w.glcm_next + B, a.feats,
                       skip, StageTwin{});
  CPX_CHECK_LAUNCH("k_obj_stage");
  return CPX_OK;
}

int launch_texture(cpx_ctx* ctx, const SetArgs& a, FeatWs& w, int B, int C, int max_label, int F) {
  hipLaunchKernelGGL(k_shape_props, dim3(cpx_div_up(max_label, 256), B), dim3(256), 0, ctx->stream,
                     max_label, F, a.objects, a.hdr, (const long long*)w.raws, a.feats);
  CPX_CHECK_LAUNCH("k_shape_props");
  // three 256-thread band blocks per CU over the per-FOV queues, then the dense kernel (one block
  // per CU) over the items whose outliers overflowed the band kernel's list (none on the bench
  // plates; its blocks exit at once when the list is empty)
  const int per_fov_b = std::max(1, std::min(max_label * C, (3 * ctx->n_cu + B - 1) / B));
  const int tev = ctx->glcm_timing && ctx->glcm_nev < cpx_ctx::kGlcmEv ? ctx->glcm_nev++ : -1;
  if (tev >= 0) CPX_CHECK_HIP(hipEventRecord(ctx->glcm_ev[tev][0], ctx->stream));
  hipLaunchKernelGGL(k_tex_band, dim3(per_fov_b, B), dim3(kBT), 0, ctx->stream, C, max_label,
                     a.objects, a.hdr, (const long long*)w.crop_off, (const unsigned char*)w.scratch,
                     w.per_fov, w.glcm_next, w.glcm_raw, w.redo);
  CPX_CHECK_LAUNCH("k_tex_band");
  hipLaunchKernelGGL(k_tex_glcm, dim3(ctx->n_cu, 1), dim3(kTT), 0, ctx->stream, C, max_label,
                     F, a.objects, a.hdr, (const long long*)w.crop_off,
                     (const unsigned char*)w.scratch, w.per_fov, w.glcm_next, w.glcm_raw, w.redo);
  CPX_CHECK_LAUNCH("k_tex_glcm");
  if (tev >= 0) CPX_CHECK_HIP(hipEventRecord(ctx->glcm_ev[tev][1], ctx->stream));
  hipLaunchKernelGGL(k_glcm_props, dim3(cpx_div_up(max_label * C * 4, 256), B), dim3(256), 0, ctx->stream,
                     C, max_label, F, a.objects, a.hdr, (const long long*)w.crop_off,
                     (const unsigned long long*)w.glcm_raw, a.feats);
  CPX_CHECK_LAUNCH("k_glcm_props");
  return CPX_OK;
}

}  // namespace

int cpx_features_fast(cpx_ctx* ctx, const int32_t* labels_dev, const float* corr_dev, int B, int C,
                      int H, int W, int max_label, int F, const cpx_object* objects_dev,
                      const cpx_fov_objects* hdr_dev, double* feats_dev, cpx_fallback_lists* fb,
                      cpx_fallback_fn fallback, void* fallback_arg) {
  static_assert(sizeof(unsigned int) * kTabW + kSmall + kCrop == 160 * 1024, "GLCM LDS budget");
  static_assert(sizeof(unsigned long long) * 4 * kRedW == 320 && kCrop % 16 == 0, "GLCM LDS layout");
  static_assert(2 * kRedW * kTT <= kTabW, "reduction scratch inside the table");
  CPX_REQUIRE(B < 2048 && (long long)max_label * C < (1 << 20), CPX_ERR_SHAPE,
              "GLCM queue codes hold fov < 2048 and items < 2^20");
  FeatWs w;
  int rc = feat_ws(ctx, WS_MISC, B, C, H, W, max_label, false, &w);
  if (rc) return rc;
  *fb = w.fb;
  const SetArgs a{labels_dev, objects_dev, hdr_dev, feats_dev};
  if ((rc = launch_offsets(ctx, a, w, B, C, W, max_label))) return rc;
  if ((rc = launch_stage(ctx, a, w, corr_dev, B, C, H, W, max_label, F, nullptr, nullptr))) return rc;
  if ((rc = launch_texture(ctx, a, w, B, C, max_label, F))) return rc;
  // the fallback kernels (the few largest objects, one long block each) as the tail
  if (fallback) return fallback(ctx, ctx->stream, *fb, fallback_arg);
  return CPX_OK;
}

// Cells and Cytoplasm together: one pass over the channels of a Cells object also stages its
// Cytoplasm object when the two share the bbox (the common case: the nucleus lies inside the
// cell); the Cytoplasm pass then stages only the rest.  Same outputs as two cpx_features_fast
// calls (every sum and crop byte identical).
int cpx_features_pair_fast(cpx_ctx* ctx, const int32_t* labels_dev, const int32_t* tlabels_dev,
                           const float* corr_dev, int B, int C, int H, int W, int max_label, int F,
                           const cpx_object* objects_dev, const cpx_fov_objects* hdr_dev, double* feats_dev,
                           const cpx_object* tobjects_dev, const cpx_fov_objects* thdr_dev, double* tfeats_dev,
                           cpx_fallback_lists* fb, cpx_fallback_lists* tfb) {
  CPX_REQUIRE(B < 2048 && (long long)max_label * C < (1 << 20), CPX_ERR_SHAPE,
              "GLCM queue codes hold fov < 2048 and items < 2^20");
  FeatWs w, tw;
  int rc = feat_ws(ctx, WS_MISC, B, C, H, W, max_label, true, &w);
  if (rc) return rc;
  if ((rc = feat_ws(ctx, WS_MISC2, B, C, H, W, max_label, false, &tw))) return rc;
  *fb = w.fb;
  *tfb = tw.fb;
  const SetArgs a{labels_dev, objects_dev, hdr_dev, feats_dev};
  const SetArgs t{tlabels_dev, tobjects_dev, thdr_dev, tfeats_dev};
  int* map = w.twin;
  int* done = w.twin + (size_t)B * max_label;
  if ((rc = launch_offsets(ctx, a, w, B, C, W, max_label))) return rc;
  if ((rc = launch_offsets(ctx, t, tw, B, C, W, max_label))) return rc;
  hipLaunchKernelGGL(k_twin_map, dim3(B), dim3(256), 0, ctx->stream, max_label, objects_dev, hdr_dev,
                     tobjects_dev, thdr_dev, map, done);
  CPX_CHECK_LAUNCH("k_twin_map");
  const StageTwin st{tlabels_dev, tobjects_dev, tw.crop_off, tw.scratch, tw.raws, tfeats_dev, map, done};
  if ((rc = launch_stage(ctx, a, w, corr_dev, B, C, H, W, max_label, F, nullptr, &st))) return rc;
  if ((rc = launch_stage(ctx, t, tw, corr_dev, B, C, H, W, max_label, F, done, nullptr))) return rc;
  if ((rc = launch_texture(ctx, a, w, B, C, max_label, F))) return rc;
  return launch_texture(ctx, t, tw, B, C, max_label, F);
}

#ifdef CPX_STAGE_PROF
extern "C" int cpx_debug_stage_prof(unsigned long long* host8, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return CPX_ERR_HIP;
  if (host8 && hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_stage_prof), 64) != hipSuccess) return CPX_ERR_HIP;
  if (reset) {
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stage_prof), z, 64) != hipSuccess) return CPX_ERR_HIP;
  }
  return CPX_OK;
}
#endif

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
