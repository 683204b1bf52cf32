/* Dynamics probe (analysis only, not product or oracle): runs the map_coordinates follow step of
 * oracle/seg_oracle_c.c for every moving pixel and records, per pixel,
 *   fix[i]  = first step whose update leaves the position unchanged (-1 if none within niter),
 *   det[i]  = step at which Brent's cycle detection sees a repeated position (-1 if none),
 *   per[i]  = the detected period,
 *   ok[i]   = 1 if the position predicted from (det, per) equals the full-loop final position. */
#include <math.h>
#include <stdint.h>
#include <string.h>
static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline void step(const float* dps, int Ly, int Lx, float* py, float* px) {
  const int64_t N = (int64_t)Ly * Lx;
  float y = *py, x = *px;
  const int yf = (int)y, xf = (int)x;
  const double yy = (double)(float)(y - (float)yf), xx = (double)(float)(x - (float)xf);
  const int y0 = imin(Ly - 1, imax(0, yf)), x0 = imin(Lx - 1, imax(0, xf));
  const int y1 = imin(Ly - 1, y0 + 1), x1 = imin(Lx - 1, x0 + 1);
  float d[2];
  for (int c = 0; c < 2; ++c) {
    const float* I = dps + c * N;
    const double v = (double)I[(int64_t)y0 * Lx + x0] * (1 - yy) * (1 - xx) + (double)I[(int64_t)y0 * Lx + x1] * (1 - yy) * xx +
                     (double)I[(int64_t)y1 * Lx + x0] * yy * (1 - xx) + (double)I[(int64_t)y1 * Lx + x1] * yy * xx;
    d[c] = (float)v;
  }
  *py = fminf((float)(Ly - 1), fmaxf(0.0f, y + d[0]));
  *px = fminf((float)(Lx - 1), fmaxf(0.0f, x + d[1]));
}
void probe(const float* dps, int Ly, int Lx, int64_t n, int niter, const float* py0, const float* px0,
           int* fix, int* det, int* per, int* ok) {
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t i = 0; i < n; ++i) {
    float y = py0[i], x = px0[i];
    float sy = y, sx = x;
    int power = 1, lam = 0;
    int f = -1, dt = -1, pd = 0;
    float fy = 0, fx = 0;
    for (int t = 0; t < niter; ++t) {
      const float oy = y, ox = x;
      step(dps, Ly, Lx, &y, &x);
      if (f < 0 && y == oy && x == ox) f = t;
      ++lam;
      if (dt < 0) {
        if (y == sy && x == sx) {
          dt = t + 1; pd = lam;  /* positions after step t+1 repeat with period lam */
          /* predict: after niter steps = position after dt + ((niter - dt) mod pd) steps */
          float qy = y, qx = x;
          const int r = (niter - dt) % pd;
          for (int k = 0; k < r; ++k) step(dps, Ly, Lx, &qy, &qx);
          fy = qy; fx = qx;
        } else if (lam == power) {
          sy = y; sx = x; power *= 2; lam = 0;
        }
      }
    }
    fix[i] = f; det[i] = dt; per[i] = pd;
    ok[i] = dt < 0 ? -1 : (fy == y && fx == x);
  }
}
