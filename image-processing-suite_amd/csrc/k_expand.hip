// Secondary objects: Cells = expand_labels(Nuclei, distance) and Cytoplasm = Cells minus Nuclei
// (the Nuclei/Cells/Cytoplasm table set consumed by Pycyto_pertime.py:46-49, produced in the
// reference by the CellProfiler pipeline launched at Feature_extraction_opt.py:164-167).
//
// expand_labels is scikit-image 0.18.3 segmentation.expand_labels: every background pixel takes
// the label of its nearest label pixel from scipy.ndimage.distance_transform_edt(...,
// return_indices=True) when that distance is <= `distance`.  scipy's feature transform is
// separable (ni_morphology.c _ComputeFT/_VoronoiFT): pass 1 picks, in every column, the nearest
// feature row (ties -> the smaller row: `delta1 <= delta2` keeps the earlier site); pass 2 runs a
// lower envelope along every row over those per-column candidates, whose query sweep stops at the
// first site not beaten strictly (ties -> the smaller column).  The selected feature is therefore
// the lexicographic minimum of (squared distance, column, row) — which only needs the columns
// within `distance` of the pixel when the result is kept (distance <= D), so both passes are
// bounded-window here:
//   pass 1 (one thread per column and 64-row tile, coalesced): signed offset to the nearest
//          feature row in the column within D (none = -128), packed with that feature's label;
//   pass 2 (one thread per pixel, row segment + halo staged in LDS): scan the 2D+1 columns in
//          ascending order with a strict `<` (smaller column wins ties), threshold d^2 <= D^2.
// Bit-identical to skimage/scipy (tests/test_gpu_parity.py, including equidistant ties).
#include "cpx_internal.h"
#include "ws_levels.h"

namespace {

constexpr int kT = 256;
constexpr signed char kNone = -128;

// pass 1: per column and tile of kColTile rows, nearest feature row within +-D (down sweep from
// D rows above the tile, then up sweep from D rows below it).  Stored packed per pixel:
// (label of that feature << 8) | (uint8)row offset, offset kNone (label 0) when none — so pass 2
// reads the winning label from its staged row segment instead of gathering it from the labels.
constexpr int kColTile = 64;

__device__ __forceinline__ int pack_ft(int dr, int lab) { return (lab << 8) | (dr & 0xff); }
__device__ __forceinline__ int ft_dr(int v) { return (int)(signed char)(v & 0xff); }

__global__ __launch_bounds__(kT) void k_edt_cols(const int* __restrict__ labels, int H, int W,
                                                 int D, int* __restrict__ off) {
  const int fov = blockIdx.z;
  const int col = blockIdx.x * kT + threadIdx.x;
  if (col >= W) return;
  const int r0 = blockIdx.y * kColTile, r1 = min(H, r0 + kColTile);
  const long long base = (long long)fov * H * W + col;
  const int* lab = labels + base;
  int* o = off + base;
  // the tile's labels and candidates stay in registers between the two sweeps (one label read
  // and one store per pixel); the D-row halos above and below are only read
  int lv[kColTile], cur[kColTile];
#pragma unroll
  for (int u = 0; u < kColTile; ++u) lv[u] = r0 + u < r1 ? lab[(long long)(r0 + u) * W] : 0;
  // down sweep: distance to the last feature at or above, capped at D+1
  int last = -0x40000000, last_l = 0;
  for (int rb = max(0, r0 - D); rb < r0; rb += 8) {  // eight halo loads in flight
    int hv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) hv[u] = rb + u < r0 ? lab[(long long)(rb + u) * W] : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (rb + u < r0 && hv[u] != 0) {
        last = rb + u;
        last_l = hv[u];
      }
  }
#pragma unroll
  for (int u = 0; u < kColTile; ++u) {
    if (lv[u] != 0) {
      last = r0 + u;
      last_l = lv[u];
    }
    const int du = r0 + u - last;
    cur[u] = du <= D ? pack_ft(-du, last_l) : pack_ft(kNone, 0);  // feature above (or here)
  }
  // up sweep: next feature at or below; keep the above one on ties (smaller row)
  int next = 0x40000000, next_l = 0;
  for (int rb = min(H, r1 + D) - 1; rb >= r1; rb -= 8) {
    int hv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) hv[u] = rb - u >= r1 ? lab[(long long)(rb - u) * W] : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (rb - u >= r1 && hv[u] != 0) {
        next = rb - u;
        next_l = hv[u];
      }
  }
#pragma unroll
  for (int u = kColTile - 1; u >= 0; --u) {
    if (lv[u] != 0) {
      next = r0 + u;
      next_l = lv[u];
    }
    const int dd = next - (r0 + u);
    const int c = ft_dr(cur[u]);
    const int du = c == kNone ? 0x7fffffff : -c;
    if (dd <= D && dd < du) cur[u] = pack_ft(dd, next_l);
  }
#pragma unroll
  for (int u = 0; u < kColTile; ++u)
    if (r0 + u < r1) o[(long long)(r0 + u) * W] = cur[u];
}

// pass 2: per pixel, lexicographic min of (d^2, column) over the 2D+1 columns.  A block owns
// kRowsPB rows of a kT-column segment (fewer, fuller blocks: one block per row was
// dispatch-bound); all its rows' candidate segments are staged in LDS at once.
constexpr int kRowsPB = 8;
constexpr int kStageMax = (kRowsPB * (kT + 2 * 127) + kT - 1) / kT;  // staged values per thread (D <= 127)

// With `ring` (the Cells watershed, k_watershed.hip): every pixel on the border ring of its
// 32 x 32 watershed tile also stores its initial flood level (from the Nuclei label, this
// footprint label and the cell channel `corr` at plane stride `cstride`) into the tile's ring, so
// the first relax round reads its halo as four contiguous vectors.
__global__ __launch_bounds__(kT) void k_edt_rows(const int* __restrict__ nuc, int H, int W, int D,
                                                 const int* __restrict__ off,
                                                 int* __restrict__ cells, int* __restrict__ cyto,
                                                 const float* __restrict__ corr, long long cstride,
                                                 unsigned long long* __restrict__ ring, int ntx, int nty) {
  extern __shared__ int seg[];  // kRowsPB x (kT + 2D) packed candidates
  const int fov = blockIdx.z, r0 = blockIdx.y * kRowsPB;
  const int nr = min(kRowsPB, H - r0);
  const int c0 = blockIdx.x * kT;
  const int sw = kT + 2 * D;
  const int c = c0 + threadIdx.x;
  // every load of the block issued before any is used: the staged candidates (up to
  // kStageMax per thread) and this thread's Nuclei labels of its rows — one load, one LDS store
  // per loop trip and a label load per row had left a memory round trip per step exposed
  int sv[kStageMax], nv_[kRowsPB];
#pragma unroll
  for (int u = 0; u < kStageMax; ++u) {
    const int i = threadIdx.x + u * kT;
    sv[u] = pack_ft(kNone, 0);
    if (i < nr * sw) {
      const int rr = i / sw, k = i - rr * sw;
      const int cc = c0 - D + k;
      if (cc >= 0 && cc < W) sv[u] = off[((long long)fov * H + r0 + rr) * W + cc];
    }
  }
#pragma unroll
  for (int rr = 0; rr < kRowsPB; ++rr)
    nv_[rr] = (rr < nr && c < W) ? nuc[((long long)fov * H + r0 + rr) * W + c] : 0;
#pragma unroll
  for (int u = 0; u < kStageMax; ++u) {
    const int i = threadIdx.x + u * kT;
    if (i < nr * sw) seg[i] = sv[u];
  }
  __syncthreads();
  if (c >= W) return;
#pragma unroll
  for (int rr = 0; rr < kRowsPB; ++rr) {
    if (rr >= nr) break;
    const int* sr = seg + rr * sw + threadIdx.x;
    // branch-free lexicographic min of (d^2, k) as one key (d^2 << 8) | k: a column without a
    // feature has dr = kNone = -128, so its d^2 >= 16384 > D^2 (D <= 127) and it can only win
    // when no candidate is within D, which the threshold below maps to label 0 anyway
    unsigned best = 0xffffffffu;
    for (int k = 0; k <= 2 * D; ++k) {
      const int dr = ft_dr(sr[k]), dc = k - D;
      best = min(best, ((unsigned)(dr * dr + dc * dc) << 8) | (unsigned)k);
    }
    const int lab = (int)(best >> 8) <= D * D ? sr[best & 0xffu] >> 8 : 0;
    const long long px = ((long long)fov * H + r0 + rr) * W + c;
    const int nv = nv_[rr];
    if (cells) cells[px] = lab;
    if (cyto) cyto[px] = (nv == 0) ? lab : 0;
    if (ring) {
      const int y = r0 + rr, ly = y % wsl::kT, lx = c % wsl::kT;
      if (ly == 0 || ly == wsl::kT - 1 || lx == 0 || lx == wsl::kT - 1) {
        const long long pix = (long long)y * W + c;
        const unsigned long long v =
            wsl::init_level(wsl::info_of(nv, lab, corr[fov * cstride + pix]), pix);
        const long long tile = ((long long)fov * nty + y / wsl::kT) * ntx + c / wsl::kT;
        wsl::ring_store(ring, tile, ly, lx, v);
      }
    }
  }
}

}  // namespace

int cpx_expand_labels_ring(cpx_ctx* ctx, const int32_t* nuclei_dev, int B, int H, int W, int distance,
                           int32_t* cells_dev, int32_t* cyto_dev, const float* corr_cell,
                           long long corr_stride, unsigned long long* ring) {
  CPX_REQUIRE(ctx && nuclei_dev && (cells_dev || cyto_dev), CPX_ERR_ARG,
              "cpx_expand_labels: null argument");
  CPX_REQUIRE(B > 0 && B <= 65535 && H > 0 && H <= 65535 && W > 0 && distance >= 0 && distance <= 127,
              CPX_ERR_ARG, "cpx_expand_labels: bad sizes (distance must be <= 127)");
  int* off = (int*)cpx_ws(ctx, WS_FEAT, sizeof(int) * (size_t)B * H * W + 256);
  if (!off) return CPX_ERR_OOM;
  hipLaunchKernelGGL(k_edt_cols, dim3(cpx_div_up(W, kT), cpx_div_up(H, kColTile), B), dim3(kT),
                     0, ctx->stream,
                     (const int*)nuclei_dev, H, W, distance, off);
  CPX_CHECK_LAUNCH("k_edt_cols");
  hipLaunchKernelGGL(k_edt_rows, dim3(cpx_div_up(W, kT), cpx_div_up(H, kRowsPB), B), dim3(kT),
                     sizeof(int) * kRowsPB * (kT + 2 * distance), ctx->stream,
                     (const int*)nuclei_dev, H, W, distance, (const int*)off, cells_dev, cyto_dev,
                     corr_cell, corr_stride, ring, cpx_div_up(W, wsl::kT), cpx_div_up(H, wsl::kT));
  CPX_CHECK_LAUNCH("k_edt_rows");
  return CPX_OK;
}

extern "C" int cpx_expand_labels(cpx_ctx* ctx, const int32_t* nuclei_dev, int B, int H, int W,
                                 int distance, int32_t* cells_dev, int32_t* cyto_dev) {
  return cpx_expand_labels_ring(ctx, nuclei_dev, B, H, W, distance, cells_dev, cyto_dev, nullptr, 0, nullptr);
}
