// a8: per-object AreaShape / Intensity / Texture features (the CellProfiler measurement step that
// Feature_extraction_opt.py:164-167 delegates to a docker image; definitions pinned to
// scikit-image 0.18.3):
//   AreaShape: regionprops area, perimeter (Benkrid-Crookes weights, 4-neighbour border),
//              centroid, bbox, extent, equivalent diameter, inertia-tensor axes / eccentricity /
//              orientation.
//   Intensity (per channel, object pixels of the fp32 corrected plane): integrated, mean, std,
//              min, max.
//   Texture   (per channel, per angle 0/45/90/135 deg, distance 3): greycomatrix/greycoprops
//              (contrast, dissimilarity, homogeneity, ASM, energy, correlation, 256 levels,
//              symmetric=False) of the masked bbox crop quantised by scale_to_8bit
//              (Cellpose_GPU_s3fs.py:34-43).
// MI355X design: one workgroup per (object, channel) streams the object's bbox (L2-resident);
// every GLCM property except ASM is linear in the co-occurrence counts, so it is accumulated
// from exact integer pair sums; ASM = sum c_ij^2 / T^2 is accumulated without ever scanning the
// 256x256 matrix: each LDS atomic increment returns the previous count c and contributes 2c+1.
// Background pairs (0,0) dominate masked crops and are counted by ballot, not atomics.  All
// sums are integers or fixed-order fp64, so results are bit-reproducible.
#include "cpx_internal.h"
#include <math.h>

namespace {

constexpr int kShapeThreads = 256;
constexpr int kTexThreads = 512;
constexpr int kTabWords = 32768;  // 128 KiB of LDS: 65536 x u16 counters, or 32768 x u32

typedef __int128 i128;

template <typename T, int NT>
__device__ T block_sum(T v, T* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T t = 0;
  for (int w = 0; w < NT / 64; ++w) t += scratch[w];
  return t;
}
template <typename T, int NT>
__device__ T block_min(T v, T* scratch) {
  v = wave_min(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T t = scratch[0];
  for (int w = 1; w < NT / 64; ++w) t = scratch[w] < t ? scratch[w] : t;
  return t;
}
template <typename T, int NT>
__device__ T block_max(T v, T* scratch) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T t = scratch[0];
  for (int w = 1; w < NT / 64; ++w) t = scratch[w] > t ? scratch[w] : t;
  return t;
}

__device__ __forceinline__ bool in_obj(const int* lab, int H, int W, int r, int c, int L) {
  return r >= 0 && r < H && c >= 0 && c < W && lab[(long long)r * W + c] == L;
}
__device__ __forceinline__ bool is_border(const int* lab, int H, int W, int r, int c, int L) {
  return in_obj(lab, H, W, r, c, L) &&
         !(in_obj(lab, H, W, r - 1, c, L) && in_obj(lab, H, W, r + 1, c, L) &&
           in_obj(lab, H, W, r, c - 1, L) && in_obj(lab, H, W, r, c + 1, L));
}

// ---------------------------------------------------------------------------------------------
// Shape: one block per listed object (those the LDS fast path skips, k_crop_offsets' list).
__global__ __launch_bounds__(kShapeThreads) void k_shape(const int* __restrict__ labels, int H,
                                                         int W, int max_label, int F,
                                                         const cpx_object* __restrict__ objects,
                                                         const int* __restrict__ list,
                                                         const int* __restrict__ n_list,
                                                         double* __restrict__ feats) {
  const int fov = blockIdx.y;
  for (int i = blockIdx.x; i < n_list[fov]; i += gridDim.x) {
  const int k = list[(long long)fov * max_label + i];
  const cpx_object o = objects[(long long)fov * max_label + k];
  const int* lab = labels + (long long)fov * H * W;
  const int L = o.label;
  const int r0 = o.bbox[0], c0 = o.bbox[1], r1 = o.bbox[2], c1 = o.bbox[3];
  const int bw = c1 - c0;
  const long long nb = (long long)(r1 - r0) * bw;
  long long n = 0, sr = 0, sc = 0, srr = 0, scc = 0, src = 0;
  int n1 = 0, n2 = 0, n3 = 0;
  for (long long p = threadIdx.x; p < nb; p += kShapeThreads) {
    const int rr = (int)(p / bw), cc = (int)(p % bw);
    const int r = r0 + rr, c = c0 + cc;
    if (lab[(long long)r * W + c] != L) continue;
    n += 1;
    sr += rr;
    sc += cc;
    srr += (long long)rr * rr;
    scc += (long long)cc * cc;
    src += (long long)rr * cc;
    if (!is_border(lab, H, W, r, c, L)) continue;
    // skimage perimeter: code = 1 + 2 * (# 4-neighbour border px) + 10 * (# diagonal border px)
    int code = 1;
    code += 2 * (is_border(lab, H, W, r - 1, c, L) + is_border(lab, H, W, r + 1, c, L) +
                 is_border(lab, H, W, r, c - 1, L) + is_border(lab, H, W, r, c + 1, L));
    code += 10 * (is_border(lab, H, W, r - 1, c - 1, L) + is_border(lab, H, W, r - 1, c + 1, L) +
                  is_border(lab, H, W, r + 1, c - 1, L) + is_border(lab, H, W, r + 1, c + 1, L));
    if (code == 5 || code == 7 || code == 15 || code == 17 || code == 25 || code == 27) n1 += 1;
    else if (code == 21 || code == 33) n2 += 1;
    else if (code == 13 || code == 23) n3 += 1;
  }
  __shared__ long long s64[kShapeThreads / 64];
  __shared__ int s32[kShapeThreads / 64];
  n = block_sum<long long, kShapeThreads>(n, s64);
  sr = block_sum<long long, kShapeThreads>(sr, s64);
  sc = block_sum<long long, kShapeThreads>(sc, s64);
  srr = block_sum<long long, kShapeThreads>(srr, s64);
  scc = block_sum<long long, kShapeThreads>(scc, s64);
  src = block_sum<long long, kShapeThreads>(src, s64);
  n1 = block_sum<int, kShapeThreads>(n1, s32);
  n2 = block_sum<int, kShapeThreads>(n2, s32);
  n3 = block_sum<int, kShapeThreads>(n3, s32);
  if (threadIdx.x == 0) {
  double* f = feats + ((long long)fov * max_label + k) * F;
  const double SQ2 = 1.4142135623730951;
  const double area = (double)n;
  f[CPX_SHAPE_AREA] = area;
  f[CPX_SHAPE_PERIMETER] = (double)n1 + (double)n2 * SQ2 + (double)n3 * ((1.0 + SQ2) / 2.0);
  f[CPX_SHAPE_CENTER_Y] = o.centroid_r;
  f[CPX_SHAPE_CENTER_X] = o.centroid_c;
  const double bba = (double)nb;
  f[CPX_SHAPE_BBOX_AREA] = bba;
  f[CPX_SHAPE_EXTENT] = area / bba;
  f[CPX_SHAPE_EQUIV_DIAMETER] = sqrt(4.0 * area / 3.14159265358979323846);
  // exact central moments: n*mu20 = n*srr - sr^2 etc. (int128), T = [[mu02,-mu11],[-mu11,mu20]]/mu0
  const i128 N = n;
  const i128 m20n = N * srr - (i128)sr * sr;  // rows
  const i128 m02n = N * scc - (i128)sc * sc;  // cols
  const i128 m11n = N * src - (i128)sr * sc;
  const double n2d = area * area;
  const double a = (double)m02n / n2d;   // T[0,0] = mu02/mu0
  const double b = -(double)m11n / n2d;  // T[0,1] = -mu11/mu0
  const double c = (double)m20n / n2d;   // T[1,1] = mu20/mu0
  // eigenvalues: l1 = larger via stable formula, l2 = det / l1 with exact det
  const double hm = 0.5 * (a + c);
  const double hd = 0.5 * (a - c);
  const double rt = sqrt(hd * hd + b * b);
  double l1 = hm + rt;
  const i128 detn4 = m02n * m20n - m11n * m11n;  // det * n^4 (exact, >= 0)
  double l2 = (l1 > 0.0) ? ((double)detn4 / (n2d * n2d)) / l1 : 0.0;
  if (l1 < 0.0) l1 = 0.0;
  if (l2 < 0.0) l2 = 0.0;
  if (l2 > l1) l2 = l1;
  f[CPX_SHAPE_MAJOR_AXIS] = 4.0 * sqrt(l1);
  f[CPX_SHAPE_MINOR_AXIS] = 4.0 * sqrt(l2);
  f[CPX_SHAPE_ECCENTRICITY] = (l1 == 0.0) ? 0.0 : sqrt(1.0 - l2 / l1);
  double orient;
  if (a - c == 0.0) orient = (b < 0.0) ? -3.14159265358979323846 / 4.0 : 3.14159265358979323846 / 4.0;
  else orient = 0.5 * atan2(-2.0 * b, c - a);
  f[CPX_SHAPE_ORIENTATION] = orient;
  f[CPX_SHAPE_BBOX_MIN_Y] = r0;
  f[CPX_SHAPE_BBOX_MIN_X] = c0;
  f[CPX_SHAPE_BBOX_MAX_Y] = r1;
  f[CPX_SHAPE_BBOX_MAX_X] = c1;
  }
  __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Intensity + texture: one block per (object, channel) work item with a 128 KiB LDS pair table.
// The object's masked bbox is quantised once (scale_to_8bit) into an LDS crop when it fits
// (kCropBytes); the four GLCM angles then run entirely out of LDS.  Larger bboxes quantise on
// the fly from global memory (L2-resident) with the same arithmetic.
constexpr int kCropBytes = 28 * 1024;
constexpr int kNRed = 15;  // values reduced per angle
constexpr int kRedWords = kNRed * (kTexThreads / 64) + kNRed + 8 + 4 + 4;  // int64 words of scratch

struct TexCtx {
  const int* lab;
  const float* img;
  int W, L;
  float mn, rng;
  bool flat;
};

__device__ __forceinline__ int quant_val(const TexCtx& t, float v, bool in) {
  const float m = v * (in ? 1.0f : 0.0f);
  if (t.flat) return 0;
  float x = m - t.mn;  // scale_to_8bit, same fp32 operation order as numpy
  x = 255.0f * x;
  x = x / t.rng;
  return (int)(unsigned char)(int)x;
}

__device__ __forceinline__ int quant8(const TexCtx& t, int r, int c) {
  const long long i = (long long)r * t.W + c;
  return quant_val(t, t.img[i], t.lab[i] == t.L);
}

// wave-then-block reduction of kNRed int64 values; result valid in thread 0
__device__ __forceinline__ void block_reduce_n(long long* v, long long* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kNRed; ++k) v[k] = wave_sum(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < kNRed; ++k) red[k * (kTexThreads / 64) + wid] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < kNRed; ++k) {
      long long s = 0;
      for (int w = 0; w < kTexThreads / 64; ++w) s += red[k * (kTexThreads / 64) + w];
      v[k] = s;
    }
  }
}

// Turns the reduced sums (thread 0's v[]) into the six greycoprops; the 256-bin |i-j| sums are
// spread over the first 256 threads (fixed reduction tree -> deterministic).
__device__ void glcm_props(long long* v, const unsigned int* dh, long long T, double* out,
                           long long* bcast, double* redd) {
  if (threadIdx.x == 0)
    for (int k = 0; k < kNRed; ++k) bcast[k] = v[k];
  __syncthreads();
  double hterm = 0.0;
  long long cterm = 0, dterm = 0;
  const int d = threadIdx.x;
  if (d < 256) {
    long long cnt = (d < 8) ? bcast[7 + d] : (long long)dh[d];
    if (d == 0) cnt += bcast[0];
    cterm = cnt * d * d;
    dterm = cnt * d;
    hterm = (double)cnt * (1.0 / (1.0 + (double)(d * d)));
  }
  hterm = wave_sum(hterm);
  cterm = wave_sum(cterm);
  dterm = wave_sum(dterm);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0 && wid < 4) {
    redd[wid] = hterm;
    bcast[kNRed + wid] = cterm;
    bcast[kNRed + 4 + wid] = dterm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double con = 0.0, dis = 0.0, hom = 0.0, asmv = 0.0, ene = 0.0, cor = 1.0;
    if (T > 0) {
      const double Td = (double)T;
      const double hsum = (redd[0] + redd[1]) + (redd[2] + redd[3]);
      const long long cnum = bcast[kNRed] + bcast[kNRed + 1] + bcast[kNRed + 2] + bcast[kNRed + 3];
      const long long dnum = bcast[kNRed + 4] + bcast[kNRed + 5] + bcast[kNRed + 6] + bcast[kNRed + 7];
      con = (double)cnum / Td;
      dis = (double)dnum / Td;
      hom = hsum / Td;
      const long long ssq_all = v[6] + v[0] * v[0];
      asmv = (double)ssq_all / (Td * Td);
      ene = sqrt(asmv);
      const i128 vi = (i128)T * v[3] - (i128)v[1] * v[1];
      const i128 vj = (i128)T * v[4] - (i128)v[2] * v[2];
      const i128 cv = (i128)T * v[5] - (i128)v[1] * v[2];
      const double std_i = sqrt((double)vi) / Td, std_j = sqrt((double)vj) / Td;
      if (std_i < 1e-15 || std_j < 1e-15) cor = 1.0;
      else cor = ((double)cv / (Td * Td)) / (std_i * std_j);
    }
    out[CPX_TEX_CONTRAST] = con;
    out[CPX_TEX_DISSIMILARITY] = dis;
    out[CPX_TEX_HOMOGENEITY] = hom;
    out[CPX_TEX_ASM] = asmv;
    out[CPX_TEX_ENERGY] = ene;
    out[CPX_TEX_CORRELATION] = cor;
  }
}

// One angle.  STAGED: i/j come from the LDS crop (packed table, replay-zero afterwards).
// Otherwise from global; PACKED selects the u16x2 table (bbox <= 65535 px) vs two u32 passes.
template <bool STAGED, bool PACKED>
__device__ void glcm_angle(const TexCtx& t, const unsigned char* crop, int r0, int c0, int r1,
                           int c1, int dr, int dc, unsigned int* tab, unsigned int* dh,
                           long long* red, double* out) {
  const int bw = c1 - c0;
  const int ra = r0, rb = r1 - dr;  // dr >= 0
  const int ca = dc >= 0 ? c0 : c0 - dc, cb = dc >= 0 ? c1 - dc : c1;
  const int w = cb - ca;
  const int npairs = (rb > ra && w > 0) ? (rb - ra) * w : 0;
  long long v[kNRed];
#pragma unroll
  for (int k = 0; k < kNRed; ++k) v[k] = 0;
  unsigned long long dlo = 0, dhi = 0;  // 16-bit counters for |i-j| = 0..3 / 4..7
  const int passes = PACKED ? 1 : 2;
  for (int pass = 0; pass < passes; ++pass) {
    if (pass == 1) {
      __syncthreads();
      for (int x = threadIdx.x; x < kTabWords; x += kTexThreads) tab[x] = 0u;
      __syncthreads();
    }
    for (int p = threadIdx.x; p < npairs; p += kTexThreads) {
      const int rr = p / w, cc = p - rr * w;
      int i, j;
      if (STAGED) {
        const int o = (ra - r0 + rr) * bw + (ca - c0 + cc);
        i = crop[o];
        j = crop[o + dr * bw + dc];
      } else {
        i = quant8(t, ra + rr, ca + cc);
        j = quant8(t, ra + rr + dr, ca + cc + dc);
      }
      const int key = (i << 8) | j;
      if (pass == 0) {
        v[1] += i;
        v[2] += j;
        v[3] += i * i;
        v[4] += j * j;
        v[5] += i * j;
        if (key == 0) {
          v[0] += 1;
        } else {
          const int d = abs(i - j);
          if (d < 4) dlo += 1ull << (16 * d);
          else if (d < 8) dhi += 1ull << (16 * (d - 4));
          else atomicAdd(&dh[d], 1u);
        }
      }
      if (key == 0) continue;
      if (PACKED) {
        const unsigned int sh = (key & 1) * 16;
        const unsigned int old = atomicAdd(&tab[key >> 1], 1u << sh);
        v[6] += 2 * (long long)((old >> sh) & 0xffffu) + 1;
      } else {
        if ((key >> 15) != pass) continue;
        const unsigned int old = atomicAdd(&tab[key & 0x7fff], 1u);
        v[6] += 2 * (long long)old + 1;
      }
    }
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    v[7 + d] = (long long)((dlo >> (16 * d)) & 0xffffull);
    v[11 + d] = (long long)((dhi >> (16 * d)) & 0xffffull);
  }
  __syncthreads();  // all table / dh atomics done
  block_reduce_n(v, red);
  glcm_props(v, dh, npairs, out, red + kNRed * (kTexThreads / 64),
             reinterpret_cast<double*>(red + kNRed * (kTexThreads / 64) + kNRed + 8));
  __syncthreads();
  // restore the all-zero table / histogram for the next angle
  if (STAGED) {
    for (int p = threadIdx.x; p < npairs; p += kTexThreads) {
      const int rr = p / w, cc = p - rr * w;
      const int o = (ra - r0 + rr) * bw + (ca - c0 + cc);
      const int key = ((int)crop[o] << 8) | (int)crop[o + dr * bw + dc];
      tab[key >> 1] = 0u;
    }
  } else {
    for (int x = threadIdx.x; x < kTabWords; x += kTexThreads) tab[x] = 0u;
  }
  for (int x = threadIdx.x; x < 256; x += kTexThreads) dh[x] = 0u;
  __syncthreads();
}

__global__ __launch_bounds__(kTexThreads) void k_intensity_texture(
    const int* __restrict__ labels, const float* __restrict__ corr, int C, int H, int W,
    int max_label, int F, const cpx_object* __restrict__ objects,
    const int* __restrict__ list, const int* __restrict__ n_list, double* __restrict__ feats) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned int* tab = reinterpret_cast<unsigned int*>(smem);
  unsigned int* dh = tab + kTabWords;
  long long* red = reinterpret_cast<long long*>(dh + 256);          // kNRed * 8 waves
  unsigned char* crop = reinterpret_cast<unsigned char*>(red + kRedWords);
  double* redd = reinterpret_cast<double*>(red);
  float* redf = reinterpret_cast<float*>(red);
  const int fov = blockIdx.y;
  // items (object, channel, angle): the few objects the fast path did not stage are the largest,
  // so their four angles run on four blocks (the intensity pass is repeated, written once)
  const int n_items = n_list[fov] * C * CPX_N_ANGLES;
  if ((int)blockIdx.x >= n_items) return;
  for (int x = threadIdx.x; x < kTabWords; x += kTexThreads) tab[x] = 0u;
  for (int x = threadIdx.x; x < 256; x += kTexThreads) dh[x] = 0u;
  __syncthreads();
  const long long N = (long long)H * W;
  for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
    const int ang = item % CPX_N_ANGLES, kc = item / CPX_N_ANGLES;
    const int k = list[(long long)fov * max_label + kc / C], ch = kc % C;
    const cpx_object o = objects[(long long)fov * max_label + k];
    TexCtx t;
    t.lab = labels + (long long)fov * N;
    t.img = corr + ((long long)fov * C + ch) * N;
    t.W = W;
    t.L = o.label;
    const int r0 = o.bbox[0], c0 = o.bbox[1], r1 = o.bbox[2], c1 = o.bbox[3];
    const int bw = c1 - c0;
    const int nb = (r1 - r0) * bw;
    // pass 1: object intensity stats + masked-crop min/max (scale_to_8bit range)
    double s = 0.0, ss = 0.0;
    float omin = INFINITY, omax = -INFINITY, mmin = INFINITY, mmax = -INFINITY;
    long long n = 0;
    for (int p0 = threadIdx.x; p0 < nb; p0 += 4 * kTexThreads) {
      float vv[4];
      bool ii[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // issue all loads first (memory-level parallelism)
        const int p = p0 + u * kTexThreads;
        const int rr = p / bw, cc = p - rr * bw;
        const long long gi = (long long)(r0 + rr) * W + (c0 + cc);
        const bool ok = p < nb;
        vv[u] = ok ? t.img[gi] : 0.0f;
        ii[u] = ok && t.lab[gi] == t.L;
        if (!ok) vv[u] = NAN;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (p0 + u * kTexThreads >= nb) continue;
        const float v = vv[u];
        const float m = v * (ii[u] ? 1.0f : 0.0f);
        mmin = fminf(mmin, m);
        mmax = fmaxf(mmax, m);
        if (ii[u]) {
          n += 1;
          s += (double)v;
          ss += (double)v * (double)v;
          omin = fminf(omin, v);
          omax = fmaxf(omax, v);
        }
      }
    }
    n = block_sum<long long, kTexThreads>(n, red);
    s = block_sum<double, kTexThreads>(s, redd);
    ss = block_sum<double, kTexThreads>(ss, redd);
    omin = block_min<float, kTexThreads>(omin, redf);
    omax = block_max<float, kTexThreads>(omax, redf);
    mmin = block_min<float, kTexThreads>(mmin, redf);
    mmax = block_max<float, kTexThreads>(mmax, redf);
    __syncthreads();
    double* f = feats + ((long long)fov * max_label + k) * F + CPX_N_SHAPE +
                (long long)ch * CPX_FEATURES_PER_CHANNEL;
    if (threadIdx.x == 0 && ang == 0) {
      const double mean = n ? s / (double)n : 0.0;
      double var = n ? (ss - s * mean) / (double)n : 0.0;
      if (var < 0.0) var = 0.0;
      f[CPX_INT_INTEGRATED] = s;
      f[CPX_INT_MEAN] = mean;
      f[CPX_INT_STD] = sqrt(var);
      f[CPX_INT_MIN] = (double)omin;
      f[CPX_INT_MAX] = (double)omax;
    }
    t.mn = mmin;
    t.rng = mmax - mmin;
    t.flat = !(mmax != mmin);
    const bool staged = nb <= kCropBytes;
    if (staged) {
      for (int p0 = threadIdx.x; p0 < nb; p0 += 4 * kTexThreads) {
        float vv[4];
        bool ii[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int p = p0 + u * kTexThreads;
          const int rr = p / bw, cc = p - rr * bw;
          const long long gi = (long long)(r0 + rr) * W + (c0 + cc);
          const bool ok = p < nb;
          vv[u] = ok ? t.img[gi] : 0.0f;
          ii[u] = ok && t.lab[gi] == t.L;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int p = p0 + u * kTexThreads;
          if (p < nb) crop[p] = (unsigned char)quant_val(t, vv[u], ii[u]);
        }
      }
      __syncthreads();
    }
    // offsets (dr, dc) = (round(sin a * 3), round(cos a * 3)) for a = 0, 45, 90, 135 deg
    const int DR[4] = {0, 2, 3, 2}, DC[4] = {3, 2, 0, -2};
    for (int a = ang; a <= ang; ++a) {
      double* out = f + CPX_N_INT + a * CPX_N_TEX_PROPS;
      if (staged) glcm_angle<true, true>(t, crop, r0, c0, r1, c1, DR[a], DC[a], tab, dh, red, out);
      else if (nb <= 65535) glcm_angle<false, true>(t, crop, r0, c0, r1, c1, DR[a], DC[a], tab, dh, red, out);
      else glcm_angle<false, false>(t, crop, r0, c0, r1, c1, DR[a], DC[a], tab, dh, red, out);
    }
  }  // item loop
}

}  // namespace

namespace {
struct FallbackArgs {
  const int32_t* labels_dev;
  const float* corr_dev;
  int B, C, H, W, max_label, F;
  const cpx_object* objects_dev;
  double* feats_dev;
};

// fallback kernels for the objects too large for the LDS fast paths (listed per FOV), launched by
// cpx_features_fast after the fast path
int launch_fallbacks(cpx_ctx* ctx, hipStream_t stream, const cpx_fallback_lists& fb, void* arg) {
  const FallbackArgs& a = *static_cast<const FallbackArgs*>(arg);
  const int B = a.B, C = a.C, H = a.H, W = a.W, max_label = a.max_label, F = a.F;
  hipLaunchKernelGGL(k_shape, dim3(std::max(1, std::min(max_label, (4 * ctx->n_cu + B - 1) / B)), B),
                     dim3(kShapeThreads), 0, stream, (const int*)a.labels_dev, H, W, max_label, F,
                     a.objects_dev, (const int*)fb.shape, (const int*)fb.n_shape, a.feats_dev);
  CPX_CHECK_LAUNCH("k_shape");
  static bool attr = false;
  const size_t lds = sizeof(unsigned int) * (kTabWords + 256) +
                     sizeof(long long) * kRedWords + kCropBytes;
  if (!attr) {
    CPX_CHECK_HIP(hipFuncSetAttribute((const void*)k_intensity_texture,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  // blocks per FOV: enough for two listed objects' C x 4 items at once (the bench plate lists
  // ~2 objects per 48 FOVs, each a serial chain of items on the old n_cu / B blocks per FOV:
  // 0.85 ms per object set, gpurun_out/r04k); a block without an item exits at once
  const int per_fov = std::max(1, std::min(max_label * C * CPX_N_ANGLES,
                                           std::max((ctx->n_cu + B - 1) / B, 2 * C * CPX_N_ANGLES)));
  hipLaunchKernelGGL(k_intensity_texture, dim3(per_fov, B), dim3(kTexThreads), lds, stream,
                     (const int*)a.labels_dev, a.corr_dev, C, H, W, max_label, F, a.objects_dev,
                     (const int*)fb.tex, (const int*)fb.n_tex, a.feats_dev);
  CPX_CHECK_LAUNCH("k_intensity_texture");
  return CPX_OK;
}
}  // namespace

extern "C" int cpx_features(cpx_ctx* ctx, const int32_t* labels_dev, const float* corr_dev, int B,
                            int C, int H, int W, int max_label, const cpx_object* objects_dev,
                            const cpx_fov_objects* hdr_dev, double* feats_dev) {
  CPX_REQUIRE(ctx && labels_dev && corr_dev && objects_dev && hdr_dev && feats_dev, CPX_ERR_ARG,
              "cpx_features: null argument");
  CPX_REQUIRE(B > 0 && B <= 65535 && C > 0 && C <= 65535 && H > 0 && W > 0 && max_label > 0,
              CPX_ERR_ARG, "cpx_features: bad sizes");
  const int F = CPX_N_SHAPE + C * CPX_FEATURES_PER_CHANNEL;
  FallbackArgs fa{labels_dev, corr_dev, B, C, H, W, max_label, F, objects_dev, feats_dev};
  cpx_fallback_lists fb;
  return cpx_features_fast(ctx, labels_dev, corr_dev, B, C, H, W, max_label, F, objects_dev, hdr_dev,
                           feats_dev, &fb, launch_fallbacks, &fa);
}

extern "C" int cpx_features_pair(cpx_ctx* ctx, const int32_t* cells_dev, const int32_t* cyto_dev,
                                 const float* corr_dev, int B, int C, int H, int W, int max_label,
                                 const cpx_object* cells_objects_dev, const cpx_fov_objects* cells_hdr_dev,
                                 double* cells_feats_dev, const cpx_object* cyto_objects_dev,
                                 const cpx_fov_objects* cyto_hdr_dev, double* cyto_feats_dev) {
  CPX_REQUIRE(ctx && cells_dev && cyto_dev && corr_dev && cells_objects_dev && cells_hdr_dev && cells_feats_dev &&
                  cyto_objects_dev && cyto_hdr_dev && cyto_feats_dev,
              CPX_ERR_ARG, "cpx_features_pair: null argument");
  CPX_REQUIRE(B > 0 && B <= 65535 && C > 0 && C <= 65535 && H > 0 && W > 0 && max_label > 0,
              CPX_ERR_ARG, "cpx_features_pair: bad sizes");
  const int F = CPX_N_SHAPE + C * CPX_FEATURES_PER_CHANNEL;
  cpx_fallback_lists fb, tfb;
  int rc = cpx_features_pair_fast(ctx, cells_dev, cyto_dev, corr_dev, B, C, H, W, max_label, F, cells_objects_dev,
                                  cells_hdr_dev, cells_feats_dev, cyto_objects_dev, cyto_hdr_dev, cyto_feats_dev,
                                  &fb, &tfb);
  if (rc) return rc;
  FallbackArgs fa{cells_dev, corr_dev, B, C, H, W, max_label, F, cells_objects_dev, cells_feats_dev};
  FallbackArgs ta{cyto_dev, corr_dev, B, C, H, W, max_label, F, cyto_objects_dev, cyto_feats_dev};
  if ((rc = launch_fallbacks(ctx, ctx->stream, fb, &fa))) return rc;
  return launch_fallbacks(ctx, ctx->stream, tfb, &ta);
}

