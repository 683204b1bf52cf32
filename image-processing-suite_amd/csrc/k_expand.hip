// Secondary objects: Cells = expand_labels(Nuclei, distance) and Cytoplasm = Cells minus Nuclei
// (the Nuclei/Cells/Cytoplasm table set consumed by Pycyto_pertime.py:46-49, produced in the
// reference by the CellProfiler pipeline launched at Feature_extraction_opt.py:164-167).
//
// expand_labels is scikit-image 0.18.3 segmentation.expand_labels: the nearest label pixel of
// every background pixel from scipy.ndimage.distance_transform_edt(..., return_indices=True),
// kept where the distance <= `distance`.  The feature transform is scipy's separable Voronoi
// algorithm (ni_morphology.c _ComputeFT/_VoronoiFT): pass 1 runs the 1-D lower envelope down
// every column, pass 2 along every row on pass-1's features.  Tie-breaking follows the same
// comparisons (`<= 0` keeps the envelope, `delta1 <= delta2` keeps the earlier site), and all
// arithmetic is on integer coordinates in fp64 (exact), so the result is bit-identical.
// One thread per column (coalesced), then one wave per row with the row staged in LDS.
#include "cpx_internal.h"

namespace {

constexpr int kT = 256;

// Pass 1: one thread per (column, fov).  ft_r/ft_c: int32 [B][H][W] out (feature row / col).
__global__ __launch_bounds__(kT) void k_ft_cols(const int* __restrict__ labels, int H, int W,
                                                int* __restrict__ ft_r, int* __restrict__ ft_c,
                                                int* __restrict__ gbuf, int* __restrict__ sbuf) {
  const int fov = blockIdx.y;
  const int col = blockIdx.x * kT + threadIdx.x;
  if (col >= W) return;
  const long long base = (long long)fov * H * W + col;
  const int* lab = labels + base;
  int* fr = ft_r + base;
  int* fc = ft_c + base;
  int* g = gbuf + (long long)fov * H * W + col;  // envelope site rows, [l][col] (coalesced)
  // features: label pixels (input == 0 of the EDT is "label != 0" here)
  int l = -1;
  for (int ii = 0; ii < H; ++ii) {
    if (lab[(long long)ii * W] == 0) continue;
    // cross term is 0 in pass 1 (the feature lies on this column): condition reduces to
    // c*0 - b*0 - a*0 - a*b*c <= 0, i.e. a*b*c >= 0, always true for a, b >= 0 -> break
    const double fd = ii;
    while (l >= 1) {
      const double f1 = g[(long long)l * W], a = f1 - (double)g[(long long)(l - 1) * W], b = fd - f1,
                   c = a + b;
      if (-a * b * c <= 0.0) break;
      --l;
    }
    ++l;
    g[(long long)l * W] = ii;
  }
  const int maxl = l;
  if (maxl < 0) {
    for (int ii = 0; ii < H; ++ii) {
      fr[(long long)ii * W] = -1;
      fc[(long long)ii * W] = -1;
    }
    return;
  }
  l = 0;
  for (int ii = 0; ii < H; ++ii) {
    double t = (double)g[(long long)l * W] - ii;
    double d1 = t * t;
    while (l < maxl) {
      const double t2 = (double)g[(long long)(l + 1) * W] - ii;
      const double d2 = t2 * t2;
      if (d1 <= d2) break;
      d1 = d2;
      ++l;
    }
    fr[(long long)ii * W] = g[(long long)l * W];
    fc[(long long)ii * W] = col;
  }
  (void)sbuf;
}

// Pass 2: one thread per (row, fov); the row's pass-1 features are read from global.
__global__ __launch_bounds__(kT) void k_ft_rows(int H, int W, int* __restrict__ ft_r,
                                                int* __restrict__ ft_c, int* __restrict__ gbuf,
                                                int* __restrict__ fbuf) {
  const int fov = blockIdx.y;
  const int row = blockIdx.x * kT + threadIdx.x;
  if (row >= H) return;
  const long long base = ((long long)fov * H + row) * W;
  int* fr = ft_r + base;  // feature row (pass 1) at each column of this row
  int* fc = ft_c + base;  // feature col
  int* g = gbuf + ((long long)fov * H + row) * W;
  int* sr = fbuf + ((long long)fov * H + row) * W;  // saved feature rows in envelope order
  const double coor = row;
  int l = -1;
  for (int ii = 0; ii < W; ++ii) {
    const int frr = fr[ii];
    if (frr < 0) continue;
    const double fd = fc[ii];  // == ii
    const double tw = (double)frr - coor;
    const double wR = tw * tw;
    while (l >= 1) {
      const double f1 = g[l], f0 = g[l - 1];
      const double a = f1 - f0, b = fd - f1, c = a + b;
      const double tu = (double)sr[l - 1] - coor, tv = (double)sr[l] - coor;
      const double uR = tu * tu, vR = tv * tv;
      if (c * vR - b * uR - a * wR - a * b * c <= 0.0) break;
      --l;
    }
    ++l;
    g[l] = ii;
    sr[l] = frr;
  }
  const int maxl = l;
  if (maxl < 0) return;  // no features in this row after pass 1 -> stays -1
  l = 0;
  for (int ii = 0; ii < W; ++ii) {
    double t = (double)g[l] - ii, t2r = (double)sr[l] - coor;
    double d1 = t * t + t2r * t2r;
    while (l < maxl) {
      const double u = (double)g[l + 1] - ii, ur = (double)sr[l + 1] - coor;
      const double d2 = u * u + ur * ur;
      if (d1 <= d2) break;
      d1 = d2;
      ++l;
    }
    fr[ii] = sr[l];
    fc[ii] = g[l];
  }
}

// labels_out = label at the feature where squared distance <= dist^2; cyto = cells * (nuc == 0)
__global__ __launch_bounds__(kT) void k_expand_apply(const int* __restrict__ nuc, int H, int W,
                                                     const int* __restrict__ ft_r,
                                                     const int* __restrict__ ft_c, long long d2max,
                                                     int* __restrict__ cells, int* __restrict__ cyto) {
  const int fov = blockIdx.y;
  const long long n = (long long)H * W;
  for (long long q = (long long)blockIdx.x * kT + threadIdx.x; q < n; q += (long long)gridDim.x * kT) {
    const long long o = (long long)fov * n + q;
    const int r = (int)(q / W), c = (int)(q - (long long)r * W);
    const int fr = ft_r[o], fc = ft_c[o];
    int lab = 0;
    if (fr >= 0) {
      const long long dr = fr - r, dc = fc - c;
      if (dr * dr + dc * dc <= d2max) lab = nuc[(long long)fov * n + (long long)fr * W + fc];
    }
    if (cells) cells[o] = lab;
    if (cyto) cyto[o] = (nuc[o] == 0) ? lab : 0;
  }
}

}  // namespace

extern "C" int cpx_expand_labels(cpx_ctx* ctx, const int32_t* nuclei_dev, int B, int H, int W,
                                 int distance, int32_t* cells_dev, int32_t* cyto_dev) {
  CPX_REQUIRE(ctx && nuclei_dev && (cells_dev || cyto_dev), CPX_ERR_ARG,
              "cpx_expand_labels: null argument");
  CPX_REQUIRE(B > 0 && B <= 65535 && H > 0 && W > 0 && distance >= 0, CPX_ERR_ARG,
              "cpx_expand_labels: bad sizes");
  const size_t n = (size_t)B * H * W;
  int* ws = (int*)cpx_ws(ctx, WS_FEAT, sizeof(int) * n * 4 + 256);
  if (!ws) return CPX_ERR_OOM;
  int* ft_r = ws;
  int* ft_c = ws + n;
  int* g = ws + 2 * n;
  int* sr = ws + 3 * n;
  hipLaunchKernelGGL(k_ft_cols, dim3(cpx_div_up(W, kT), B), dim3(kT), 0, ctx->stream,
                     (const int*)nuclei_dev, H, W, ft_r, ft_c, g, sr);
  CPX_CHECK_LAUNCH("k_ft_cols");
  hipLaunchKernelGGL(k_ft_rows, dim3(cpx_div_up(H, kT), B), dim3(kT), 0, ctx->stream, H, W, ft_r,
                     ft_c, g, sr);
  CPX_CHECK_LAUNCH("k_ft_rows");
  const long long d2 = (long long)distance * distance;
  hipLaunchKernelGGL(k_expand_apply, dim3(std::max(1, std::min(cpx_div_up((long long)H * W, kT), 4 * ctx->n_cu / B + 1)), B),
                     dim3(kT), 0, ctx->stream, (const int*)nuclei_dev, H, W, (const int*)ft_r,
                     (const int*)ft_c, d2, cells_dev, cyto_dev);
  CPX_CHECK_LAUNCH("k_expand_apply");
  return CPX_OK;
}
