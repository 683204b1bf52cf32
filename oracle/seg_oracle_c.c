/* C restatement of the two hot loops of oracle/seg_oracle.py — TEST INFRASTRUCTURE ONLY.
 *
 * The numpy restatement in seg_oracle.py is the definition; at Cellpose's full-resolution
 * defaults (resample=True, niter = 200 / rescale = 1176 for the reference's nuclei model at
 * diameter 100, Cellpose_GPU_s3fs.py:28,143) its literal loops need minutes per 2080^2 FOV, so
 * these two are repeated here statement by statement in plain C (no FMA contraction: compiled
 * with -ffp-contract=off; x86-64 SSE arithmetic, so float stays float and double stays double):
 *
 *   follow_flows_c  — dynamics.follow_flows / steps2D_interp with the CPU map_coordinates step
 *                     (seg_oracle.follow_flows): fp64 bilinear expression of the fp32 flow,
 *                     rounded to fp32, fp32 add, clamp to [0, L-1]; every pixel runs all niter
 *                     steps (no early exit: the HIP kernel's fixed-point exit is checked against
 *                     this plain loop).
 *   flow_error_c    — dynamics.masks_to_flows (2.x CPU heat diffusion) + metrics.flow_error
 *                     (seg_oracle.masks_to_flows / remove_bad_flow_masks): per object the
 *                     median-nearest centre, 2*(ptp x + ptp y) Jacobi iterations in fp64,
 *                     central differences, normalisation by 1e-20 + sqrt(dy^2 + dx^2), and the
 *                     per-label means of the squared differences to dP/5 accumulated in raster
 *                     order (ndimage.mean = bincount sums / counts).
 *
 * tests/test_seg_oracle_c.py checks both against the numpy restatement on small inputs.
 * Objects are independent, so the per-object and per-pixel loops run under OpenMP; every
 * result is computed by exactly one thread in the sequential order above.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

/* dps: float32 [2][Ly][Lx] (dP * cp_mask / 5); py/px: float32 [n] start positions, updated. */
void follow_flows_c(const float* dps, int Ly, int Lx, int64_t n, int niter, float* py, float* px) {
  const int64_t N = (int64_t)Ly * Lx;
  const float fLy = (float)(Ly - 1), fLx = (float)(Lx - 1);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t i = 0; i < n; ++i) {
    float y = py[i], x = px[i];
    for (int it = 0; it < niter; ++it) {
      const int yf = (int)y, xf = (int)x;
      const double yy = (double)(float)(y - (float)yf);
      const double xx = (double)(float)(x - (float)xf);
      const int y0 = imin(Ly - 1, imax(0, yf)), x0 = imin(Lx - 1, imax(0, xf));
      const int y1 = imin(Ly - 1, y0 + 1), x1 = imin(Lx - 1, x0 + 1);
      float d[2];
      for (int c = 0; c < 2; ++c) {
        const float* I = dps + c * N;
        const double v = (double)I[(int64_t)y0 * Lx + x0] * (1 - yy) * (1 - xx) +
                         (double)I[(int64_t)y0 * Lx + x1] * (1 - yy) * xx +
                         (double)I[(int64_t)y1 * Lx + x0] * yy * (1 - xx) +
                         (double)I[(int64_t)y1 * Lx + x1] * yy * xx;
        d[c] = (float)v;
      }
      const float ny = y + d[0], nx = x + d[1];
      y = fminf(fLy, fmaxf(0.0f, ny));
      x = fminf(fLx, fmaxf(0.0f, nx));
    }
    py[i] = y;
    px[i] = x;
  }
}

/* masks: int32 [Ly][Lx] labels 1..nlab (0 = background); dP: float32 [2][Ly][Lx] (network
 * flows, unmasked); err_out: float64 [nlab] (NaN for absent labels, as ndimage.mean). */
void flow_error_c(const int32_t* masks, const float* dP, int Ly, int Lx, int nlab, double* err_out) {
  const int64_t N = (int64_t)Ly * Lx;
  int* bb = (int*)malloc(sizeof(int) * 4 * (size_t)(nlab + 1));
  for (int l = 0; l <= nlab; ++l) {
    bb[4 * l] = Ly; bb[4 * l + 1] = Lx; bb[4 * l + 2] = -1; bb[4 * l + 3] = -1;
  }
  for (int r = 0; r < Ly; ++r)
    for (int c = 0; c < Lx; ++c) {
      const int l = masks[(int64_t)r * Lx + c];
      if (l <= 0 || l > nlab) continue;
      int* b = bb + 4 * l;
      if (r < b[0]) b[0] = r;
      if (c < b[1]) b[1] = c;
      if (r > b[2]) b[2] = r;
      if (c > b[3]) b[3] = c;
    }
  double* mu = (double*)calloc((size_t)2 * N, sizeof(double));
#pragma omp parallel for schedule(dynamic, 1)
  for (int l = 1; l <= nlab; ++l) {
    const int* b = bb + 4 * l;
    if (b[2] < 0) continue;
    const int r0 = b[0], c0 = b[1];
    const int bh = b[2] - r0 + 1, bw = b[3] - c0 + 1;
    const int ly = bh + 2, lx = bw + 2;
    /* mask pixels of the bbox in raster order (local coordinates + 1) */
    int64_t np_ = 0;
    for (int r = 0; r < bh; ++r)
      for (int c = 0; c < bw; ++c) np_ += masks[(int64_t)(r0 + r) * Lx + c0 + c] == l;
    int* ys = (int*)malloc(sizeof(int) * np_);
    int* xs = (int*)malloc(sizeof(int) * np_);
    int64_t k = 0;
    int* rowc = (int*)calloc(bh, sizeof(int));
    int* colc = (int*)calloc(bw, sizeof(int));
    for (int r = 0; r < bh; ++r)
      for (int c = 0; c < bw; ++c)
        if (masks[(int64_t)(r0 + r) * Lx + c0 + c] == l) {
          ys[k] = r + 1; xs[k] = c + 1; ++k;
          rowc[r]++; colc[c]++;
        }
    /* np.median of the coordinates: mean of the two middle order statistics */
    double med[2];
    for (int a = 0; a < 2; ++a) {
      const int* h = a == 0 ? rowc : colc;
      const int len = a == 0 ? bh : bw;
      const int64_t ka = (np_ - 1) / 2, kb = np_ / 2;
      int64_t cum = 0;
      int va = -1, vb = -1;
      for (int i = 0; i < len; ++i) {
        cum += h[i];
        if (va < 0 && cum > ka) va = i + 1;
        if (vb < 0 && cum > kb) { vb = i + 1; break; }
      }
      med[a] = ((double)va + (double)vb) / 2.0;
    }
    int64_t best = 0;
    double bd = 0.0;
    for (int64_t i = 0; i < np_; ++i) {
      const double dx = (double)xs[i] - med[1], dy = (double)ys[i] - med[0];
      const double d = dx * dx + dy * dy;  /* (x - xmed)**2 + (y - ymed)**2 */
      if (i == 0 || d < bd) { bd = d; best = i; }
    }
    const int ym = ys[best], xm = xs[best];
    const int niter = 2 * ((bw - 1) + (bh - 1));
    double* T = (double*)calloc((size_t)ly * lx, sizeof(double));
    double* Tn = (double*)malloc(sizeof(double) * np_);
    for (int it = 0; it < niter; ++it) {
      T[ym * lx + xm] += 1;
      for (int64_t i = 0; i < np_; ++i) {
        const int y = ys[i], x = xs[i];
        Tn[i] = 1 / 9. * (T[y * lx + x] + T[(y - 1) * lx + x] + T[(y + 1) * lx + x] +
                          T[y * lx + x - 1] + T[y * lx + x + 1] +
                          T[(y - 1) * lx + x - 1] + T[(y - 1) * lx + x + 1] +
                          T[(y + 1) * lx + x - 1] + T[(y + 1) * lx + x + 1]);
      }
      for (int64_t i = 0; i < np_; ++i) T[ys[i] * lx + xs[i]] = Tn[i];
    }
    for (int64_t i = 0; i < np_; ++i) {
      const int y = ys[i], x = xs[i];
      const int64_t g = (int64_t)(r0 + y - 1) * Lx + (c0 + x - 1);
      mu[g] = T[(y + 1) * lx + x] - T[(y - 1) * lx + x];
      mu[N + g] = T[y * lx + x + 1] - T[y * lx + x - 1];
    }
    free(T); free(Tn); free(ys); free(xs); free(rowc); free(colc);
  }
  /* mu /= 1e-20 + (mu**2).sum(axis=0)**0.5 ; error sums per label in raster order */
  double* s0 = (double*)calloc((size_t)nlab + 1, sizeof(double));
  double* s1 = (double*)calloc((size_t)nlab + 1, sizeof(double));
  int64_t* cnt = (int64_t*)calloc((size_t)nlab + 1, sizeof(int64_t));
  for (int64_t g = 0; g < N; ++g) {
    const int l = masks[g];
    const double a = mu[g], b = mu[N + g];
    const double nrm = 1e-20 + sqrt(a * a + b * b);
    const double m0 = a / nrm, m1 = b / nrm;
    if (l <= 0 || l > nlab) continue;
    const double t0 = m0 - (double)(dP[g] / 5.0f);
    const double t1 = m1 - (double)(dP[N + g] / 5.0f);
    s0[l] += t0 * t0;
    s1[l] += t1 * t1;
    cnt[l] += 1;
  }
  for (int l = 1; l <= nlab; ++l) {
    const double c = (double)cnt[l];
    err_out[l - 1] = 0.0 + s0[l] / c + s1[l] / c;
  }
  free(s0); free(s1); free(cnt); free(mu); free(bb);
}
