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
//          feature row in the column within D (int8; none = -128);
//   pass 2 (one thread per pixel, row segment + halo staged in LDS): scan the 2D+1 columns in
//          ascending order with a strict `<` (smaller column wins ties), threshold d^2 <= D^2.
// Bit-identical to skimage/scipy (tests/test_gpu_parity.py, including equidistant ties).
#include "cpx_internal.h"

namespace {

constexpr int kT = 256;
constexpr signed char kNone = -128;

// pass 1: per column and tile of kColTile rows, nearest feature row within +-D (down sweep from
// D rows above the tile, then up sweep from D rows below it)
constexpr int kColTile = 64;

__global__ __launch_bounds__(kT) void k_edt_cols(const int* __restrict__ labels, int H, int W,
                                                 int D, signed char* __restrict__ off) {
  const int fov = blockIdx.z;
  const int col = blockIdx.x * kT + threadIdx.x;
  if (col >= W) return;
  const int r0 = blockIdx.y * kColTile, r1 = min(H, r0 + kColTile);
  const long long base = (long long)fov * H * W + col;
  const int* lab = labels + base;
  signed char* o = off + base;
  // down sweep: distance to the last feature at or above (stored), capped at D+1
  int last = -0x40000000;
  for (int r = max(0, r0 - D); r < r1; ++r) {
    if (lab[(long long)r * W] != 0) last = r;
    if (r < r0) continue;
    const int du = r - last;
    o[(long long)r * W] = du <= D ? (signed char)(-du) : kNone;  // feature above (or here)
  }
  // up sweep: next feature at or below; keep the above one on ties (smaller row)
  int next = 0x40000000;
  for (int r = min(H, r1 + D) - 1; r >= r0; --r) {
    if (lab[(long long)r * W] != 0) next = r;
    if (r >= r1) continue;
    const int dd = next - r;
    if (dd > D) continue;
    const signed char cur = o[(long long)r * W];
    const int du = cur == kNone ? 0x7fffffff : -(int)cur;
    if (dd < du) o[(long long)r * W] = (signed char)dd;
  }
}

// pass 2: per pixel, lexicographic min of (d^2, column) over the 2D+1 columns
__global__ __launch_bounds__(kT) void k_edt_rows(const int* __restrict__ nuc, int H, int W, int D,
                                                 const signed char* __restrict__ off,
                                                 int* __restrict__ cells, int* __restrict__ cyto) {
  extern __shared__ signed char seg[];  // kT + 2D
  const int fov = blockIdx.z, r = blockIdx.y;
  const int c0 = blockIdx.x * kT;
  const long long rowbase = ((long long)fov * H + r) * W;
  for (int i = threadIdx.x; i < kT + 2 * D; i += kT) {
    const int c = c0 - D + i;
    seg[i] = (c >= 0 && c < W) ? off[rowbase + c] : kNone;
  }
  __syncthreads();
  const int c = c0 + threadIdx.x;
  if (c >= W) return;
  int best = 0x7fffffff, bc = -1, br = 0;
  for (int k = 0; k <= 2 * D; ++k) {
    const signed char dr = seg[threadIdx.x + k];
    if (dr == kNone) continue;
    const int dc = k - D;
    const int d2 = (int)dr * (int)dr + dc * dc;
    if (d2 < best) {
      best = d2;
      bc = c + dc;
      br = r + dr;
    }
  }
  int lab = 0;
  if (bc >= 0 && best <= D * D) lab = nuc[((long long)fov * H + br) * W + bc];
  if (cells) cells[rowbase + c] = lab;
  if (cyto) cyto[rowbase + c] = (nuc[rowbase + c] == 0) ? lab : 0;
}

}  // namespace

extern "C" int cpx_expand_labels(cpx_ctx* ctx, const int32_t* nuclei_dev, int B, int H, int W,
                                 int distance, int32_t* cells_dev, int32_t* cyto_dev) {
  CPX_REQUIRE(ctx && nuclei_dev && (cells_dev || cyto_dev), CPX_ERR_ARG,
              "cpx_expand_labels: null argument");
  CPX_REQUIRE(B > 0 && B <= 65535 && H > 0 && H <= 65535 && W > 0 && distance >= 0 && distance <= 127,
              CPX_ERR_ARG, "cpx_expand_labels: bad sizes (distance must be <= 127)");
  signed char* off = (signed char*)cpx_ws(ctx, WS_FEAT, (size_t)B * H * W + 256);
  if (!off) return CPX_ERR_OOM;
  hipLaunchKernelGGL(k_edt_cols, dim3(cpx_div_up(W, kT), cpx_div_up(H, kColTile), B), dim3(kT),
                     0, ctx->stream,
                     (const int*)nuclei_dev, H, W, distance, off);
  CPX_CHECK_LAUNCH("k_edt_cols");
  hipLaunchKernelGGL(k_edt_rows, dim3(cpx_div_up(W, kT), H, B), dim3(kT), kT + 2 * distance,
                     ctx->stream, (const int*)nuclei_dev, H, W, distance, (const signed char*)off,
                     cells_dev, cyto_dev);
  CPX_CHECK_LAUNCH("k_edt_rows");
  return CPX_OK;
}
