// the per-time profile step after the feature tables,
// Pycyto_pertime.py:29-172 — per-well aggregation, MAD-robustize + double sigmoid, feature
// selection statistics, and within-treatment cosine similarities.  Each kernel repeats the
// arithmetic of the library call the reference makes, in the same order, so the results are
// bit-identical to it (restated in oracle/profiles_oracle.py, pinned to pandas / scipy):
//   * cpx_group_kahan_accumulate / cpx_group_mean_finalize: pandas groupby mean
//     (_libs/groupby.pyx group_mean: Kahan sum per group and column in row order, NaN skipped);
//   * cpx_nancorr: pandas DataFrame.corr(pearson) (_libs/algos.pyx nancorr, Welford);
//   * cpx_robust_mad: pycytominer RobustMAD.fit = pandas median + scipy median_abs_deviation;
//   * cpx_mad_transform: (x - median) / (mad + eps) (RobustMAD.transform), optionally followed by
//     Pycyto_pertime.py:13-16 double_sigmoid and abs
//     (x**3 and x**6 rounded once from double-double products, as a correctly rounded pow);
//   * cpx_column_stats: value-count / nunique / NaN / extreme statistics of feature_select;
//   * cpx_cosine_groups: sklearn cosine_similarity within row groups (tolerance-level parity:
//     sklearn's BLAS Gram matrix has no fixed summation order).
// Tables are small next to the image path (wells x features), except the object tables the
// group mean reads (objects x features, HBM-bound).
#include "cpx_internal.h"
#include <math.h>

namespace {

constexpr int kGT = 64;        // group kernel: columns per block (one wave)
constexpr int kGU = 32;        // rows per pipelined chunk of the sequential Kahan chain
constexpr int kSortMax = 4096; // rows per column for the LDS sorts
constexpr int kST = 256;

// pandas group_mean accumulation: thread = (group, column); the group's rows in `order`
// (original row order), Kahan-compensated.  State persists across calls so tables can be
// streamed in row order.  The chain is sequential per group, so the wave keeps memory busy by
// software pipelining: while chunk c (kGU rows) is summed, the values of chunk c+1 and the row
// indices of chunk c+2 are in flight.
struct GroupChunk {
  int idx[kGU];
  double v[kGU];
};

__device__ __forceinline__ void load_idx(const int* order, int r, int r1, int* idx) {
#pragma unroll
  for (int u = 0; u < kGU; ++u) idx[u] = r + u < r1 ? order[r + u] : -1;
}

// value of row idx[u] (times its row scale when the column is scaled: Normalize_CP_ami's
// site scaling of integer features, one rounding as pandas' multiply)
__device__ __forceinline__ void load_vals(const double* values, long long ld, int j,
                                          const int* idx, const double* row_scale, bool scaled,
                                          double* v) {
#pragma unroll
  for (int u = 0; u < kGU; ++u) {
    v[u] = idx[u] >= 0 ? values[(long long)idx[u] * ld + j] : __builtin_nan("");
    if (scaled && idx[u] >= 0) v[u] = v[u] * row_scale[idx[u]];
  }
}

__device__ __forceinline__ void kahan_chunk(const double* v, double& s, double& c, long long& n) {
#pragma unroll
  for (int u = 0; u < kGU; ++u) {
    if (v[u] != v[u]) continue;  // NaN (and the padding) skipped
    const double y = v[u] - c;
    const double t = s + y;
    c = (t - s) - y;
    if (c != c) c = 0.0;         // GH#50367: +-inf makes the compensation NaN
    s = t;
    ++n;
  }
}

__global__ __launch_bounds__(kGT) void k_group_kahan(const double* __restrict__ values, int K,
                                                     long long ld, const int* __restrict__ order,
                                                     const int* __restrict__ offs,
                                                     const double* __restrict__ row_scale,
                                                     const unsigned char* __restrict__ col_scaled,
                                                     double* __restrict__ sumx,
                                                     double* __restrict__ comp,
                                                     long long* __restrict__ nobs) {
  const int g = blockIdx.y;
  const int j = blockIdx.x * kGT + threadIdx.x;
  if (j >= K) return;
  const bool scaled = row_scale != nullptr && col_scaled != nullptr && col_scaled[j] != 0;
  const long long sidx = (long long)g * K + j;
  double s = sumx[sidx], c = comp[sidx];
  long long n = nobs[sidx];
  const int r0 = offs[g], r1 = offs[g + 1];
  GroupChunk A, B;
  load_idx(order, r0, r1, A.idx);
  load_idx(order, r0 + kGU, r1, B.idx);
  load_vals(values, ld, j, A.idx, row_scale, scaled, A.v);
  for (int r = r0; r < r1; r += 2 * kGU) {
    // A: values of rows r.. in flight; B: indices of rows r+kGU..
    load_vals(values, ld, j, B.idx, row_scale, scaled, B.v);
    load_idx(order, r + 2 * kGU, r1, A.idx);
    kahan_chunk(A.v, s, c, n);
    if (r + kGU >= r1) break;
    load_vals(values, ld, j, A.idx, row_scale, scaled, A.v);
    load_idx(order, r + 3 * kGU, r1, B.idx);
    kahan_chunk(B.v, s, c, n);
  }
  sumx[sidx] = s;
  comp[sidx] = c;
  nobs[sidx] = n;
}

__global__ void k_group_finalize(const double* __restrict__ sumx,
                                 const long long* __restrict__ nobs, long long total,
                                 double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long long n = nobs[i];
  out[i] = n == 0 ? __builtin_nan("") : sumx[i] / (double)n;
}

// pandas nancorr: thread = one (xi, yi) pair with yi <= xi; columns are contiguous
// (mat column-major [K][N]).  1/nobs comes from an LDS table of correctly rounded reciprocals.
__global__ __launch_bounds__(kST) void k_nancorr(const double* __restrict__ mat, int N, int K,
                                                 double* __restrict__ out) {
  extern __shared__ double rcp[];
  for (int i = threadIdx.x; i < N; i += kST) rcp[i] = 1.0 / (double)(i + 1);
  __syncthreads();
  const long long p = (long long)blockIdx.x * kST + threadIdx.x;
  const long long npairs = (long long)K * (K + 1) / 2;
  if (p >= npairs) return;
  // p -> (xi, yi), yi <= xi, row-major over the lower triangle
  int xi = (int)((sqrt(8.0 * (double)p + 1.0) - 1.0) * 0.5);
  while ((long long)xi * (xi + 1) / 2 > p) --xi;
  while ((long long)(xi + 1) * (xi + 2) / 2 <= p) ++xi;
  const int yi = (int)(p - (long long)xi * (xi + 1) / 2);
  const double* cx = mat + (long long)xi * N;
  const double* cy = mat + (long long)yi * N;
  int nobs = 0;
  double meanx = 0.0, meany = 0.0, ssqdmx = 0.0, ssqdmy = 0.0, covxy = 0.0;
  for (int i = 0; i < N; ++i) {
    const double vx = cx[i], vy = cy[i];
    if (!isfinite(vx) || !isfinite(vy)) continue;
    const double r = rcp[nobs];
    ++nobs;
    const double dx = vx - meanx;
    const double dy = vy - meany;
    meanx += r * dx;
    meany += r * dy;
    ssqdmx += (vx - meanx) * dx;
    ssqdmy += (vy - meany) * dy;
    covxy += (vx - meanx) * dy;
  }
  double res = __builtin_nan("");
  if (nobs >= 1) {
    const double div = sqrt(ssqdmx * ssqdmy);
    if (div != 0.0) res = covxy / div;
  }
  out[(long long)xi * K + yi] = res;
  out[(long long)yi * K + xi] = res;
}

// Block bitonic sort of n2 (power of two <= kSortMax) doubles in LDS, ascending.
__device__ void block_sort(double* a, int n2) {
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n2; i += kST) {
        const int l = i ^ j;
        if (l > i) {
          const double x = a[i], y = a[l];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

// Gather the non-NaN values of column j at rows idx[0..n) (idx null: rows 0..n) into a,
// pad to a power of two with +inf, sort.  Returns the non-NaN count (block-uniform).
__device__ int gather_sorted(const double* col, const int* idx, int n, double* a, int* cnt,
                             int* n2out) {
  if (threadIdx.x == 0) *cnt = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += kST) {
    const double v = col[idx ? idx[i] : i];
    if (v == v) a[atomicAdd(cnt, 1)] = v;
  }
  __syncthreads();
  const int m = *cnt;
  int n2 = 1;
  while (n2 < m) n2 <<= 1;
  for (int i = m + threadIdx.x; i < n2; i += kST) a[i] = __builtin_inf();
  __syncthreads();
  block_sort(a, n2);
  *n2out = n2;
  return m;
}

__device__ __forceinline__ double median_sorted(const double* a, int m) {
  if (m == 0) return __builtin_nan("");
  return (m & 1) ? a[m / 2] : (a[m / 2 - 1] + a[m / 2]) / 2.0;
}

// pandas groupby median (well_agg_func="median", Normalize_CP_ami.py:113): one block per
// (group, column), the group's non-NaN values sorted in (dynamic) LDS.
__global__ __launch_bounds__(kST) void k_group_median(const double* __restrict__ values, int K,
                                                      long long ld,
                                                      const int* __restrict__ order,
                                                      const int* __restrict__ offs,
                                                      const double* __restrict__ row_scale,
                                                      const unsigned char* __restrict__ col_scaled,
                                                      double* __restrict__ out) {
  extern __shared__ double a_dyn[];
  __shared__ int cnt;
  const int j = blockIdx.x, g = blockIdx.y;
  const int r0 = offs[g], n = offs[g + 1] - r0;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  const bool scaled = row_scale != nullptr && col_scaled != nullptr && col_scaled[j] != 0;
  for (int i = threadIdx.x; i < n; i += kST) {
    const int row = order[r0 + i];
    double v = values[(long long)row * ld + j];
    if (scaled) v = v * row_scale[row];
    if (v == v) a_dyn[atomicAdd(&cnt, 1)] = v;
  }
  __syncthreads();
  const int m = cnt;
  int n2 = 1;
  while (n2 < m) n2 <<= 1;
  for (int i = m + threadIdx.x; i < n2; i += kST) a_dyn[i] = __builtin_inf();
  __syncthreads();
  block_sort(a_dyn, n2);
  if (threadIdx.x == 0) out[(long long)g * K + j] = median_sorted(a_dyn, m);
}

// RobustMAD.fit: one block per feature column over the fit rows.
__global__ __launch_bounds__(kST) void k_robust_mad(const double* __restrict__ mat, int N,
                                                    const int* __restrict__ fit, int n_fit,
                                                    double scale, double* __restrict__ med,
                                                    double* __restrict__ mad) {
  __shared__ double a[kSortMax];
  __shared__ int cnt;
  const int j = blockIdx.x;
  int n2;
  const int m = gather_sorted(mat + (long long)j * N, fit, n_fit, a, &cnt, &n2);
  const double md = median_sorted(a, m);
  __syncthreads();
  for (int i = threadIdx.x; i < n2; i += kST) a[i] = i < m ? fabs(a[i] - md) : __builtin_inf();
  __syncthreads();
  block_sort(a, n2);
  if (threadIdx.x == 0) {
    med[j] = md;
    mad[j] = m ? median_sorted(a, m) / scale : __builtin_nan("");
  }
}

// double-double helpers (fma-exact products)
__device__ __forceinline__ void two_prod(double a, double b, double& p, double& e) {
  p = a * b;
  e = __builtin_fma(a, b, -p);
}

// x**3 and x**6 as correctly rounded powers: exact-ish double-double products rounded once.
__device__ __forceinline__ void pow36(double t, double& p3, double& p6) {
  double s, se;
  two_prod(t, t, s, se);            // t^2 = s + se exactly
  double c, ce;
  two_prod(s, t, c, ce);            // s*t = c + ce exactly
  const double c_lo = __builtin_fma(se, t, ce);  // + se*t (rounded)
  // t^3 rounded once (to within the dd error); an overflowed product stays +-inf as pow's
  p3 = isfinite(c) ? c + c_lo : c;
  double q, qe;
  two_prod(c, c, q, qe);            // (c + c_lo)^2 = c^2 + 2 c c_lo + ...
  const double q_lo = __builtin_fma(2.0 * c, c_lo, qe);
  p6 = isfinite(q) ? q + q_lo : q;
}

// (x - median) / (mad + eps) [-> double sigmoid -> abs]; column-major [K][N].
__global__ void k_mad_transform(const double* __restrict__ mat, int N, int K,
                                const double* __restrict__ med, const double* __restrict__ mad,
                                double eps, int sigmoid, double alpha, double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)N * K) return;
  const int j = (int)(i / N);
  const double z = (mat[i] - med[j]) / (mad[j] + eps);
  if (!sigmoid) {
    out[i] = z;
    return;
  }
  const double t = z / alpha;
  double p3, p6;
  pow36(t, p3, p6);
  const double y = p3 / sqrt(1.0 + p6);
  out[i] = fabs(y);
}

// feature_select statistics per column over all N rows: NaN count, number of distinct
// values, the two largest value counts, max and min (non-NaN).
__global__ __launch_bounds__(kST) void k_column_stats(const double* __restrict__ mat, int N,
                                                      cpx_column_stat* __restrict__ st) {
  __shared__ double a[kSortMax];
  __shared__ int cnt;
  const int j = blockIdx.x;
  int n2;
  const int m = gather_sorted(mat + (long long)j * N, nullptr, N, a, &cnt, &n2);
  if (threadIdx.x == 0) {
    int runs = 0, top = 0, sec = 0, len = 0;
    for (int i = 0; i < m; ++i) {
      if (i > 0 && a[i] == a[i - 1]) {
        ++len;
      } else {
        if (len > 0) {
          if (len > top) { sec = top; top = len; } else if (len > sec) sec = len;
        }
        len = 1;
        ++runs;
      }
    }
    if (len > 0) {
      if (len > top) { sec = top; top = len; } else if (len > sec) sec = len;
    }
    cpx_column_stat s;
    s.na_count = N - m;
    s.nunique = runs;
    s.top_count = top;
    s.second_count = sec;
    s.max = m ? a[m - 1] : __builtin_nan("");
    s.min = m ? a[0] : __builtin_nan("");
    st[j] = s;
  }
}

// sklearn cosine_similarity within groups of consecutive rows (row-major [N][F], NaN read as
// 0 = the reference's fillna(0)): row norms, then one thread per upper-triangle pair.
__global__ void k_row_norms(const double* __restrict__ x, int N, int F, double* __restrict__ nrm) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  const double* row = x + (long long)r * F;
  double s = 0.0;
  for (int f = 0; f < F; ++f) {
    const double v = row[f] == row[f] ? row[f] : 0.0;
    s += v * v;
  }
  s = sqrt(s);
  nrm[r] = s == 0.0 ? 1.0 : s;
}

__global__ void k_cosine_pairs(const double* __restrict__ x, int F, const int* __restrict__ offs,
                               const long long* __restrict__ poffs, int G,
                               const double* __restrict__ nrm, double* __restrict__ out) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= poffs[G]) return;
  int lo = 0, hi = G - 1;  // group of pair p
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (poffs[mid] <= p) lo = mid; else hi = mid - 1;
  }
  const int g = lo;
  const int n = offs[g + 1] - offs[g];
  long long q = p - poffs[g];
  // np.triu_indices(n, 1) order: (0,1), (0,2), ..., (1,2), ...
  int i = 0;
  while (q >= n - 1 - i) { q -= n - 1 - i; ++i; }
  const int jj = i + 1 + (int)q;
  const int ri = offs[g] + i, rj = offs[g] + jj;
  const double* a = x + (long long)ri * F;
  const double* b = x + (long long)rj * F;
  const double na = nrm[ri], nb = nrm[rj];
  double s = 0.0;
  for (int f = 0; f < F; ++f) {
    const double va = a[f] == a[f] ? a[f] : 0.0;
    const double vb = b[f] == b[f] ? b[f] : 0.0;
    s += (va / na) * (vb / nb);
  }
  out[p] = s;
}

}  // namespace

extern "C" int cpx_group_kahan_accumulate(cpx_ctx* ctx, const double* values_dev, int n_rows,
                                          int K, long long ld, const int32_t* order_dev,
                                          const int32_t* offs_dev, int G,
                                          const double* row_scale_dev,
                                          const uint8_t* col_scaled_dev, double* sum_dev,
                                          double* comp_dev, int64_t* nobs_dev) {
  CPX_REQUIRE(ctx && values_dev && order_dev && offs_dev && sum_dev && comp_dev && nobs_dev,
              CPX_ERR_ARG, "cpx_group_kahan_accumulate: null argument");
  CPX_REQUIRE(n_rows >= 0 && K > 0 && ld >= K && G > 0 && G <= 65535, CPX_ERR_ARG,
              "cpx_group_kahan_accumulate: bad sizes");
  if (n_rows == 0) return CPX_OK;
  hipLaunchKernelGGL(k_group_kahan, dim3(cpx_div_up(K, kGT), G), dim3(kGT), 0, ctx->stream,
                     values_dev, K, ld, (const int*)order_dev, (const int*)offs_dev, row_scale_dev,
                     (const unsigned char*)col_scaled_dev, sum_dev, comp_dev, (long long*)nobs_dev);
  CPX_CHECK_LAUNCH("k_group_kahan");
  return CPX_OK;
}

extern "C" int cpx_group_median(cpx_ctx* ctx, const double* values_dev, int n_rows, int K,
                                long long ld, const int32_t* order_dev, const int32_t* offs_dev,
                                int G, int max_group_rows, const double* row_scale_dev,
                                const uint8_t* col_scaled_dev, double* out_dev) {
  CPX_REQUIRE(ctx && values_dev && order_dev && offs_dev && out_dev && n_rows >= 0 && K > 0 &&
                  ld >= K && G > 0 && G <= 65535 && max_group_rows >= 0 && max_group_rows <= 16384,
              CPX_ERR_ARG, "cpx_group_median: bad argument (at most 16384 rows per group)");
  int n2 = 1;
  while (n2 < max_group_rows) n2 <<= 1;
  hipLaunchKernelGGL(k_group_median, dim3(K, G), dim3(kST), sizeof(double) * n2, ctx->stream,
                     values_dev, K, ld, (const int*)order_dev, (const int*)offs_dev, row_scale_dev,
                     (const unsigned char*)col_scaled_dev, out_dev);
  CPX_CHECK_LAUNCH("k_group_median");
  return CPX_OK;
}

extern "C" int cpx_group_mean_finalize(cpx_ctx* ctx, const double* sum_dev,
                                       const int64_t* nobs_dev, int G, int K, double* out_dev) {
  CPX_REQUIRE(ctx && sum_dev && nobs_dev && out_dev && G > 0 && K > 0, CPX_ERR_ARG,
              "cpx_group_mean_finalize: bad argument");
  const long long total = (long long)G * K;
  hipLaunchKernelGGL(k_group_finalize, dim3(cpx_div_up(total, 256)), dim3(256), 0, ctx->stream,
                     sum_dev, (const long long*)nobs_dev, total, out_dev);
  CPX_CHECK_LAUNCH("k_group_finalize");
  return CPX_OK;
}

extern "C" int cpx_nancorr(cpx_ctx* ctx, const double* mat_dev, int N, int K, double* out_dev) {
  CPX_REQUIRE(ctx && mat_dev && out_dev && N >= 0 && N <= 8192 && K > 0 && K <= 65536,
              CPX_ERR_ARG, "cpx_nancorr: bad argument (N <= 8192 rows)");
  const long long npairs = (long long)K * (K + 1) / 2;
  hipLaunchKernelGGL(k_nancorr, dim3(cpx_div_up(npairs, kST)), dim3(kST),
                     sizeof(double) * std::max(N, 1), ctx->stream, mat_dev, N, K, out_dev);
  CPX_CHECK_LAUNCH("k_nancorr");
  return CPX_OK;
}

extern "C" int cpx_robust_mad(cpx_ctx* ctx, const double* mat_dev, int N, int K,
                              const int32_t* fit_rows_dev, int n_fit, double scale,
                              double* med_dev, double* mad_dev) {
  CPX_REQUIRE(ctx && mat_dev && fit_rows_dev && med_dev && mad_dev && K > 0 && n_fit >= 0 &&
                  n_fit <= kSortMax && K <= 2147483647,
              CPX_ERR_ARG, "cpx_robust_mad: bad argument (at most %d fit rows)", kSortMax);
  hipLaunchKernelGGL(k_robust_mad, dim3(K), dim3(kST), 0, ctx->stream, mat_dev, N,
                     (const int*)fit_rows_dev, n_fit, scale, med_dev, mad_dev);
  CPX_CHECK_LAUNCH("k_robust_mad");
  return CPX_OK;
}

extern "C" int cpx_mad_transform(cpx_ctx* ctx, const double* mat_dev, int N, int K,
                                 const double* med_dev, const double* mad_dev, double eps,
                                 int double_sigmoid, double alpha, double* out_dev) {
  CPX_REQUIRE(ctx && mat_dev && med_dev && mad_dev && out_dev && N >= 0 && K > 0, CPX_ERR_ARG,
              "cpx_mad_transform: bad argument");
  const long long total = (long long)N * K;
  if (total == 0) return CPX_OK;
  hipLaunchKernelGGL(k_mad_transform, dim3(cpx_div_up(total, 256)), dim3(256), 0, ctx->stream,
                     mat_dev, N, K, med_dev, mad_dev, eps, double_sigmoid, alpha, out_dev);
  CPX_CHECK_LAUNCH("k_mad_transform");
  return CPX_OK;
}

extern "C" int cpx_column_stats(cpx_ctx* ctx, const double* mat_dev, int N, int K,
                                cpx_column_stat* stats_dev) {
  CPX_REQUIRE(ctx && mat_dev && stats_dev && N >= 0 && N <= kSortMax && K > 0, CPX_ERR_ARG,
              "cpx_column_stats: bad argument (at most %d rows)", kSortMax);
  hipLaunchKernelGGL(k_column_stats, dim3(K), dim3(kST), 0, ctx->stream, mat_dev, N, stats_dev);
  CPX_CHECK_LAUNCH("k_column_stats");
  return CPX_OK;
}

extern "C" int cpx_cosine_groups(cpx_ctx* ctx, const double* x_dev, int N, int F,
                                 const int32_t* offs_dev, const int64_t* pair_offs_dev, int G,
                                 long long n_pairs, double* norms_dev, double* out_dev) {
  CPX_REQUIRE(ctx && x_dev && offs_dev && pair_offs_dev && norms_dev && out_dev && N >= 0 &&
                  F > 0 && G > 0 && n_pairs >= 0,
              CPX_ERR_ARG, "cpx_cosine_groups: bad argument");
  if (N == 0) return CPX_OK;
  hipLaunchKernelGGL(k_row_norms, dim3(cpx_div_up(N, 256)), dim3(256), 0, ctx->stream, x_dev, N,
                     F, norms_dev);
  CPX_CHECK_LAUNCH("k_row_norms");
  if (n_pairs == 0) return CPX_OK;
  hipLaunchKernelGGL(k_cosine_pairs, dim3(cpx_div_up(n_pairs, 256)), dim3(256), 0, ctx->stream,
                     x_dev, F, (const int*)offs_dev, (const long long*)pair_offs_dev, G, norms_dev,
                     out_dev);
  CPX_CHECK_LAUNCH("k_cosine_pairs");
  return CPX_OK;
}
