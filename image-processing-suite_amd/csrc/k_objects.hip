// a7: object table — regionprops order, integer centroids, crop-box edge filter, kept index —
// and the masked 200x200 crops + scale_to_8bit (a9).
//
// Reference (Cellpose_GPU_s3fs.py):
//   :149  props = regionprops(masks)            -> labels in ascending order, absent labels skipped
//   :160  y_center, x_center = map(int, prop.centroid)   (centroid = float64 mean of coords)
//   :162  skip if y-100 < 0 or y+100 > h or x-100 < 0 or x+100 > w
//   :165-170 crop = image_4ch[y1:y2, x1:x2, :] * (masks[y1:y2, x1:x2] == label)[..., None]
//   :391-393 Cell_ID = f"{well}_{site}_cell{cell_idx}", cell_idx = rank among kept cells
//   :34-43 scale_to_8bit: uint8(255.0 * (x.astype(f32) - min) / (max - min)), zeros if max == min
// MI355X design: one streaming pass over the int32 label image accumulates exact int64 moments and
// the bbox per label (vertical runs aggregated in registers, merged per tile in an LDS hash table,
// one set of global atomics per tile and label — integer atomics, so results are order
// independent and exact); a one-block-per-FOV finisher compacts present labels in ascending
// order with a block scan.
#include "cpx_internal.h"
#include <limits.h>
#include <math.h>

namespace {

constexpr int kThreads = 256;

__global__ void k_stats_init(cpx_label_stats* __restrict__ st, long long n,
                             cpx_fov_objects* __restrict__ hdr, int B) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    cpx_label_stats s;
    s.area = s.sum_r = s.sum_c = s.sum_rr = s.sum_cc = s.sum_rc = 0;
    s.rmin = INT_MAX;
    s.rmax = -1;
    s.cmin = INT_MAX;
    s.cmax = -1;
    st[i] = s;
  }
  if (i < B) hdr[i] = cpx_fov_objects{0, 0, 0, 0};
}

// Label statistics, one block per 32-row x 256-column tile of a FOV.  A thread walks one
// column of the tile (loads coalesced across the wave), aggregates vertical runs of one label in
// registers, and merges each run into a block-private LDS hash table keyed by label (exact
// integer LDS atomics); the table is flushed with one set of global atomics per (tile, label).
// Labels are compact, so a tile holds a handful of them: global atomics drop from one set per
// run to one per tile and label.  A full table (pathological label images) spills runs
// straight to global memory, so results never depend on the table size.
constexpr int kTileR = 128;  // rows per thread: longer runs, fewer table flushes (32: 172 us, 128: 92 us per call)
constexpr int kHash = 256;

struct LdsStat {
  int key;
  unsigned int area, sum_r;
  int rmin, rmax, cmin, cmax;
  unsigned int sum_c;
  unsigned long long sum_rr, sum_cc, sum_rc;
};

__device__ __forceinline__ void lds_flush_run(LdsStat* tab, cpx_label_stats* st, int label, int c,
                                              int r0, int r1) {
  // vertical run rows r0..r1 (inclusive) in column c
  const long long cnt = r1 - r0 + 1;
  const long long sr = (long long)(r0 + r1) * cnt / 2;
  const long long srr = ((long long)r1 * (r1 + 1) * (2LL * r1 + 1) -
                         (long long)(r0 - 1) * r0 * (2LL * r0 - 1)) / 6;
  unsigned int h = ((unsigned int)label * 2654435761u) >> 24;
  for (int probe = 0; probe < kHash; ++probe, h = (h + 1) & (kHash - 1)) {
    const int k = atomicCAS(&tab[h].key, 0, label);
    if (k == 0 || k == label) {
      LdsStat* e = tab + h;
      atomicAdd(&e->area, (unsigned int)cnt);
      atomicAdd(&e->sum_r, (unsigned int)sr);
      atomicAdd(&e->sum_c, (unsigned int)(cnt * c));
      atomicAdd(&e->sum_rr, (unsigned long long)srr);
      atomicAdd(&e->sum_cc, (unsigned long long)(cnt * c * c));
      atomicAdd(&e->sum_rc, (unsigned long long)(sr * c));
      atomicMin(&e->rmin, r0);
      atomicMax(&e->rmax, r1);
      atomicMin(&e->cmin, c);
      atomicMax(&e->cmax, c);
      return;
    }
  }
  cpx_label_stats* s = st + label;  // table full: straight to global
  atomicAdd((unsigned long long*)&s->area, (unsigned long long)cnt);
  atomicAdd((unsigned long long*)&s->sum_r, (unsigned long long)sr);
  atomicAdd((unsigned long long*)&s->sum_c, (unsigned long long)(cnt * c));
  atomicAdd((unsigned long long*)&s->sum_rr, (unsigned long long)srr);
  atomicAdd((unsigned long long*)&s->sum_cc, (unsigned long long)(cnt * c * c));
  atomicAdd((unsigned long long*)&s->sum_rc, (unsigned long long)(sr * c));
  atomicMin(&s->rmin, r0);
  atomicMax(&s->rmax, r1);
  atomicMin(&s->cmin, c);
  atomicMax(&s->cmax, c);
}

// grid: (ceil(W / kThreads), ceil(H / kTileR), B)
__global__ __launch_bounds__(kThreads) void k_label_stats(const int* __restrict__ labels, int H,
                                                          int W, int max_label,
                                                          cpx_label_stats* __restrict__ stats,
                                                          cpx_fov_objects* __restrict__ hdr) {
  __shared__ LdsStat tab[kHash];
  const int fov = blockIdx.z;
  {
    LdsStat e;
    e.key = 0;
    e.area = e.sum_r = e.sum_c = 0;
    e.rmin = INT_MAX;
    e.rmax = -1;
    e.cmin = INT_MAX;
    e.cmax = -1;
    e.sum_rr = e.sum_cc = e.sum_rc = 0;
    for (int i = threadIdx.x; i < kHash; i += kThreads) tab[i] = e;
  }
  __syncthreads();
  const int c = blockIdx.x * kThreads + threadIdx.x;
  const int r0 = blockIdx.y * kTileR, r1 = min(H, r0 + kTileR);
  cpx_label_stats* st = stats + (long long)fov * (max_label + 1);
  int seen_max = 0;
  bool overflow = false;
  if (c < W) {
    const int* col = labels + (long long)fov * H * W + c;
    int cur = 0, start = 0;
    for (int rb = r0; rb < r1; rb += 8) {  // eight label loads in flight, then the run scan
      int lv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) lv[u] = rb + u < r1 ? col[(long long)(rb + u) * W] : 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = rb + u;
        if (r >= r1) break;
        int l = lv[u];
        if (l > 0) {
          seen_max = max(seen_max, l);
          if (l > max_label) {
            overflow = true;
            l = 0;
          }
        }
        if (l != cur) {
          if (cur > 0) lds_flush_run(tab, st, cur, c, start, r - 1);
          cur = l;
          start = r;
        }
      }
    }
    if (cur > 0) lds_flush_run(tab, st, cur, c, start, r1 - 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHash; i += kThreads) {
    const LdsStat e = tab[i];
    if (e.key == 0) continue;
    cpx_label_stats* s = st + e.key;
    atomicAdd((unsigned long long*)&s->area, (unsigned long long)e.area);
    atomicAdd((unsigned long long*)&s->sum_r, (unsigned long long)e.sum_r);
    atomicAdd((unsigned long long*)&s->sum_c, (unsigned long long)e.sum_c);
    atomicAdd((unsigned long long*)&s->sum_rr, e.sum_rr);
    atomicAdd((unsigned long long*)&s->sum_cc, e.sum_cc);
    atomicAdd((unsigned long long*)&s->sum_rc, e.sum_rc);
    atomicMin(&s->rmin, e.rmin);
    atomicMax(&s->rmax, e.rmax);
    atomicMin(&s->cmin, e.cmin);
    atomicMax(&s->cmax, e.cmax);
  }
  // max label / overflow (wave-aggregated)
  seen_max = wave_max(seen_max);
  int ov = wave_max((int)overflow);
  if ((threadIdx.x & 63) == 0) {
    if (seen_max) atomicMax(&hdr[fov].max_label, seen_max);
    if (ov) atomicMax(&hdr[fov].overflow, 1);
  }
}

// One block per FOV: ascending compaction, centroids, edge filter, kept rank.
__global__ __launch_bounds__(1024) void k_objects_finalize(const cpx_label_stats* __restrict__ stats,
                                                           int H, int W, int max_label, int box,
                                                           cpx_object* __restrict__ objects,
                                                           cpx_fov_objects* __restrict__ hdr) {
  const int fov = blockIdx.x;
  const cpx_label_stats* st = stats + (long long)fov * (max_label + 1);
  cpx_object* out = objects + (long long)fov * max_label;
  __shared__ int wsum_p[16], wsum_k[16];
  __shared__ int base_p, base_k;
  if (threadIdx.x == 0) {
    base_p = 0;
    base_k = 0;
  }
  __syncthreads();
  const int half = box / 2;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int l0 = 1; l0 <= max_label; l0 += blockDim.x) {
    const int l = l0 + threadIdx.x;
    int present = 0, kept = 0;
    cpx_label_stats s;
    double cr = 0, cc = 0;
    int yc = 0, xc = 0;
    if (l <= max_label) {
      s = st[l];
      present = s.area > 0;
      if (present) {
        cr = (double)s.sum_r / (double)s.area;
        cc = (double)s.sum_c / (double)s.area;
        yc = (int)cr;  // python int(): truncation toward zero (coords >= 0)
        xc = (int)cc;
        kept = !((yc - half < 0) || (yc + half > H) || (xc - half < 0) || (xc + half > W));
      }
    }
    // block-wide exclusive scans of present / kept (ballot + popcount per wave)
    const unsigned long long bp = __ballot(present), bk = __ballot(kept);
    const unsigned long long lower = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int pre_p = __popcll(bp & lower), pre_k = __popcll(bk & lower);
    if (lane == 0) {
      wsum_p[wid] = __popcll(bp);
      wsum_k[wid] = __popcll(bk);
    }
    __syncthreads();
    int off_p = base_p, off_k = base_k;
    for (int w = 0; w < wid; ++w) {
      off_p += wsum_p[w];
      off_k += wsum_k[w];
    }
    if (present) {
      cpx_object o;
      o.label = l;
      o.area = (int)s.area;
      o.bbox[0] = s.rmin;
      o.bbox[1] = s.cmin;
      o.bbox[2] = s.rmax + 1;
      o.bbox[3] = s.cmax + 1;
      o.centroid_r = cr;
      o.centroid_c = cc;
      o.yc = yc;
      o.xc = xc;
      o.kept = kept;
      o.cell_idx = kept ? off_k + pre_k : -1;
      out[off_p + pre_p] = o;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int tp = 0, tk = 0;
      for (int w = 0; w < nw; ++w) {
        tp += wsum_p[w];
        tk += wsum_k[w];
      }
      base_p += tp;
      base_k += tk;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    hdr[fov].n_objects = base_p;
    hdr[fov].n_kept = base_k;
  }
}

// One block per (crop slot, fov): masked HWC crop and per-channel 8-bit version.
__global__ __launch_bounds__(kThreads) void k_crops(const int* __restrict__ labels,
                                                    const float* __restrict__ corr, int C, int H,
                                                    int W, int max_label,
                                                    const cpx_object* __restrict__ objects,
                                                    const cpx_fov_objects* __restrict__ hdr,
                                                    int box, int max_crops,
                                                    float* __restrict__ crops,
                                                    unsigned char* __restrict__ crops8) {
  const int slot = blockIdx.x, fov = blockIdx.y;
  const cpx_fov_objects h = hdr[fov];
  if (slot >= h.n_kept) return;
  __shared__ int obj_idx;
  if (threadIdx.x == 0) obj_idx = -1;
  __syncthreads();
  const cpx_object* ob = objects + (long long)fov * max_label;
  for (int k = threadIdx.x; k < h.n_objects; k += kThreads)
    if (ob[k].cell_idx == slot) obj_idx = k;
  __syncthreads();
  if (obj_idx < 0) return;
  const cpx_object o = ob[obj_idx];
  const int half = box / 2;
  const int y1 = o.yc - half, x1 = o.xc - half;
  const long long N = (long long)H * W;
  const int* lab = labels + (long long)fov * N;
  const float* img = corr + (long long)fov * C * N;
  const long long npx = (long long)box * box;
  float* dst = crops ? crops + ((long long)fov * max_crops + slot) * npx * C : nullptr;
  __shared__ float smin[8][kThreads / 64], smax[8][kThreads / 64];
  float mn[8], mx[8];
  for (int ch = 0; ch < C && ch < 8; ++ch) {
    mn[ch] = INFINITY;
    mx[ch] = -INFINITY;
  }
  for (long long p = threadIdx.x; p < npx; p += kThreads) {
    const int yy = (int)(p / box), xx = (int)(p % box);
    const long long gi = (long long)(y1 + yy) * W + (x1 + xx);
    const bool in = lab[gi] == o.label;
    for (int ch = 0; ch < C; ++ch) {
      const float v = img[ch * N + gi] * (in ? 1.0f : 0.0f);
      if (dst) dst[p * C + ch] = v;
      if (ch < 8) {
        mn[ch] = fminf(mn[ch], v);
        mx[ch] = fmaxf(mx[ch], v);
      }
    }
  }
  if (!crops8) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int ch = 0; ch < C && ch < 8; ++ch) {
    float a = wave_min(mn[ch]), b = wave_max(mx[ch]);
    if (lane == 0) {
      smin[ch][wid] = a;
      smax[ch][wid] = b;
    }
  }
  __syncthreads();
  unsigned char* d8 = crops8 + ((long long)fov * max_crops + slot) * npx * C;
  for (int ch = 0; ch < C && ch < 8; ++ch) {
    float a = smin[ch][0], b = smax[ch][0];
    for (int w = 1; w < kThreads / 64; ++w) {
      a = fminf(a, smin[ch][w]);
      b = fmaxf(b, smax[ch][w]);
    }
    const float rng = b - a;
    for (long long p = threadIdx.x; p < npx; p += kThreads) {
      unsigned char u = 0;
      if (b != a) {
        float v;
        if (dst) {
          v = dst[p * C + ch];
        } else {  // no float crop kept: the same masked value again from the plane
          const int yy = (int)(p / box), xx = (int)(p % box);
          const long long gi = (long long)(y1 + yy) * W + (x1 + xx);
          v = img[ch * N + gi] * (lab[gi] == o.label ? 1.0f : 0.0f);
        }
        float t = v - a;
        t = 255.0f * t;
        t = t / rng;
        u = (unsigned char)(int)t;  // astype(uint8): truncation (t in [0, 255])
      }
      d8[(long long)ch * npx + p] = u;
    }
  }
}

}  // namespace

extern "C" int cpx_objects(cpx_ctx* ctx, const int32_t* labels_dev, int B, int H, int W,
                           int max_label, int box, cpx_label_stats* stats_dev,
                           cpx_object* objects_dev, cpx_fov_objects* hdr_dev) {
  CPX_REQUIRE(ctx && labels_dev && stats_dev && objects_dev && hdr_dev, CPX_ERR_ARG,
              "cpx_objects: null argument");
  CPX_REQUIRE(B > 0 && B <= 65535 && H > 0 && W > 0 && max_label > 0 && box >= 0, CPX_ERR_ARG,
              "cpx_objects: bad sizes");
  const long long nst = (long long)B * (max_label + 1);
  hipLaunchKernelGGL(k_stats_init, dim3(cpx_div_up(std::max<long long>(nst, B), kThreads)),
                     dim3(kThreads), 0, ctx->stream, stats_dev, nst, hdr_dev, B);
  CPX_CHECK_LAUNCH("k_stats_init");
  hipLaunchKernelGGL(k_label_stats, dim3(cpx_div_up(W, kThreads), cpx_div_up(H, kTileR), B),
                     dim3(kThreads), 0, ctx->stream, (const int*)labels_dev, H, W, max_label,
                     stats_dev, hdr_dev);
  CPX_CHECK_LAUNCH("k_label_stats");
  hipLaunchKernelGGL(k_objects_finalize, dim3(B), dim3(1024), 0, ctx->stream,
                     (const cpx_label_stats*)stats_dev, H, W, max_label, box, objects_dev, hdr_dev);
  CPX_CHECK_LAUNCH("k_objects_finalize");
  return CPX_OK;
}

extern "C" int cpx_crops(cpx_ctx* ctx, const int32_t* labels_dev, const float* corr_dev, int B,
                         int C, int H, int W, int max_label, const cpx_object* objects_dev,
                         const cpx_fov_objects* hdr_dev, int box, int max_crops, float* crops_dev,
                         uint8_t* crops8_dev) {
  CPX_REQUIRE(ctx && labels_dev && corr_dev && objects_dev && hdr_dev && (crops_dev || crops8_dev),
              CPX_ERR_ARG, "cpx_crops: null argument");
  CPX_REQUIRE(B > 0 && B <= 65535 && C > 0 && C <= 8 && H > 0 && W > 0 && box > 0 &&
                  max_crops > 0 && max_label > 0,
              CPX_ERR_ARG, "cpx_crops: bad sizes (C must be <= 8)");
  hipLaunchKernelGGL(k_crops, dim3(max_crops, B), dim3(kThreads), 0, ctx->stream,
                     (const int*)labels_dev, corr_dev, C, H, W, max_label, objects_dev, hdr_dev,
                     box, max_crops, crops_dev, (unsigned char*)crops8_dev);
  CPX_CHECK_LAUNCH("k_crops");
  return CPX_OK;
}
