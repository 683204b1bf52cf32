// a6 (flow-error filter, fp32 screening): the register-resident screening kernels.  The flow
// error (Cellpose 2.x dynamics.remove_bad_flow_masks / metrics.flow_error, restated in
// oracle/seg_oracle.py) diffuses heat over each mask for 2 (ptp x + ptp y) Jacobi sweeps; the
// screening pass (k_seg.hip, k_flow_error_lds<..., float>) decides a mask's flag in fp32 only where
// a certified bound puts its error clearly on one side of the threshold and defers the rest to the
// fp64 kernels.  The kernels here run the same screening with the grid in VGPRs instead of LDS for
// masks up to 128 x 120 px (fe_reg_class); they are launched first, and the LDS screening kernels skip every mask
// whose flag they set.  Compiled with -fno-slp-vectorize: pairing rows into packed adds would
// separate the DPP neighbour reads from the adds they fold into.
#include "cpx_internal.h"
#include <math.h>
#include <stdlib.h>


#pragma clang fp contract(off)

namespace {

// ---------------------------------------------------------------------------------------------
// k_flow_error_reg: the fp32 screening sweeps with the diffusion grid in VGPRs (one mask per
// block of NW waves, no LDS round trip and no barrier per sweep for NW = 1).  The grid is stored
// with its shorter side on the rows ("storage" orientation: transposed when bh > bw — the
// 9-point stencil, the centre source and the gradient pair are symmetric under a transpose, and
// every original-coordinate quantity (medians, the argmin's tie order, the flows, dy / dx) is
// formed in the original orientation): lane l holds storage grid columns 2l and 2l + 1 (a float2
// per row; column 0 and SC + 1 are the zero border, read as the DPP shifts' out-of-range zeros, so
// SC <= 128), wave w rows 1 + w RS .. RS + w RS
// (registers T[j]).  A sweep per row: vertical 3-sums of the pair (two packed adds), the
// horizontal neighbours from the adjacent lanes by DPP wave shifts, times (1/9 or 0) per cell
// (Wt: the mask and the 1/9 in one packed multiply).  The summation order differs from the
// reference's (screening only: every cell still passes through <= 6 roundings of non-negative
// terms per sweep, within the 11u of the bound k_flow_error_lds certifies); decisions, the
// `und` list and the bad flags are exactly k_flow_error_lds<..., float>'s, and a mask handled
// here is skipped by the LDS screening kernels (its flag is already set).
__device__ __forceinline__ float dpp_from_left(float v) {  // lane l gets lane l - 1's v (lane 0: 0)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_from_right(float v) {  // lane l gets lane l + 1's v (lane 63: 0)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}

// first index i < len (<= 192) with h[0] + ... + h[i] > k: one wave, three consecutive entries
// per lane
__device__ __forceinline__ int fe_hist_rank(const int* h, int len, long long k) {
  const int lane = threadIdx.x & 63;
  int e[3], s = 0;
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    e[u] = 3 * lane + u < len ? h[3 * lane + u] : 0;
    s += e[u];
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(s, d, 64);
    if (lane >= d) s += y;
  }
  // the first lane whose inclusive total exceeds k holds the index; inside it, the first entry
  const unsigned long long bb = __ballot((long long)s > k);
  const int lb = bb ? __ffsll((long long)bb) - 1 : 63;
  const long long c0 = (long long)__shfl(s - e[1] - e[2], lb, 64);  // through entry 3 lb
  const long long c1 = c0 + __shfl(e[1], lb, 64);                    // through entry 3 lb + 1
  return c0 > k ? 3 * lb : c1 > k ? 3 * lb + 1 : 3 * lb + 2;
}

constexpr int kFeRegRows = 40;  // register rows per wave (T + Wt: 4 VGPRs per row)
static_assert(3 * kFeRegRows == kFeRegMaxShort && 2 * 64 == kFeRegMaxLong, "cpx_internal.h class bounds");
typedef float fe_v2 __attribute__((ext_vector_type(2)));  // v_pk_*_f32 operands

// Row jc (wave-uniform, 0 <= jc < RW; jc == RW or beyond: no-op) of a register array without a
// dynamic index: a binary search over compile-time rows (scalar branches only).  The asm marker
// keeps the leaves distinct, so the compiler does not merge them back into an indexed access
// (which would move the whole array to scratch).
template <int OP, int RW, int LO = 0, typename V>
__device__ __forceinline__ void fe_row_op(V* T, int jc, V& v) {
  if constexpr (RW - LO == 1) {
    if (jc == LO) {
      if constexpr (OP == 0) T[LO] += v;  // add
      if constexpr (OP == 1) T[LO] = v;   // set
      if constexpr (OP == 2) v = T[LO];   // get
      asm volatile("; fe_row_op %0 %1" ::"n"(OP), "n"(LO));
    }
  } else {
    constexpr int MID = LO + (RW - LO) / 2;
    if (jc < MID) fe_row_op<OP, MID, LO, V>(T, jc, v);
    else fe_row_op<OP, RW, MID, V>(T, jc, v);
  }
}

// Which register kernel takes a mask, and its storage orientation (tr: storage rows = original
// columns).  Class 1 (k_flow_error_reg1): one column per lane, the mask's columns <= 64 lanes and
// its rows <= kFeReg1Rows registers, rows = the shorter side when both fit.  Class 2
// (k_flow_error_reg, two columns per lane over two waves): columns <= 128, rows <= 2 x kFeRegRows
// (80); class 3 the same over four waves of kFeReg3Rows, rows <= 3 x kFeRegRows (120); rows = the
// shorter side.
// Class 0: the LDS kernels.
constexpr int kFeReg1Rows = 80;
// class 3 runs as four waves of 32 rows: two 256-thread blocks per CU at the kernel's two waves
// per SIMD fill all eight wave slots, where three waves of 40 rows left two idle (3.27 -> 2.82 ms
// per 32 FOVs, `gpurun_out/r06ag`; five waves of 24 rows or eight of 16 fit fewer waves per CU)
constexpr int kFeReg3Rows = 32;
static_assert(4 * kFeReg3Rows >= kFeRegMaxShort, "class 3 rows fit four waves");
__device__ __forceinline__ int fe_reg_class(int bh, int bw, bool& tr) {
  const int mn = min(bh, bw), mx = max(bh, bw);
  if (mn < 1) return 0;
  if (mx <= 64) { tr = bh > bw; return 1; }
  if (mn <= 64 && mx <= kFeReg1Rows) { tr = bw > bh; return 1; }
  if (mx <= 128 && mn <= 2 * kFeRegRows) { tr = bh > bw; return 2; }
  if (mx <= 128 && mn <= 3 * kFeRegRows) { tr = bh > bw; return 3; }
  return 0;
}

template <int RW, int NW, int CLS>
__global__ __launch_bounds__(64 * NW, 2) void k_flow_error_reg(
    const int* __restrict__ m0, const float2* __restrict__ dpf, int Dy, int Dx, int B, int max_label,
    const cpx_object* __restrict__ objects, const int* __restrict__ off, int* __restrict__ ctr, int lo_rows,
    double thr, unsigned char* __restrict__ bad, int* __restrict__ und) {
  static_assert(RW % 8 == 0, "rows in groups of 8");
  constexpr int NT = 64 * NW;
  __shared__ fe_v2 xr[2][NW][2][64];  // boundary rows: [sweep parity][wave][first, last][lane]
  __shared__ int hrow[RW * NW], hcol[128];
  __shared__ double sred[NW][3];
  __shared__ unsigned long long sbest[NW];
  __shared__ int sitem, smed2[2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const long long n = (long long)Dy * Dx;
  const int total = off[B];
  for (int claims = 0;; ++claims) {
    if (claims > total) {  // broken claim (cpx_internal.h kClaimBroken)
      if (tid == 0) atomicOr(ctr, kClaimBroken);
      break;
    }
    if (tid == 0) sitem = atomicAdd(ctr, 1);
    __syncthreads();
    const int item = __builtin_amdgcn_readfirstlane(sitem);  // uniform control flow from here
    __syncthreads();
    if (item >= total) break;
    int fov = 0;
    while (fov + 1 < B && off[fov + 1] <= item) ++fov;
    const int kobj = item - off[fov];
    const cpx_object o = objects[(long long)fov * max_label + kobj];
    const int L = o.label;
    const int r0 = o.bbox[0], c0 = o.bbox[1];
    const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
    bool tr = false;
    if (fe_reg_class(bh, bw, tr) != CLS) continue;  // block-uniform
    const int SR = tr ? bw : bh, SC = tr ? bh : bw;  // storage rows / columns
    // rows per wave (the slabs split the mask evenly); this wave's rows 1 + wv RS .. wv RS + nrow
    const int RS = (SR + NW - 1) / NW;
    const int nrow = __builtin_amdgcn_readfirstlane(max(0, min(RS, SR - wv * RS)));
    // the bbox origin; storage grid (gr, gc), 1-based interior -> 32-bit offset from it
    const int* lab = m0 + (long long)fov * n + (long long)r0 * Dx + c0;
    for (int i = tid; i < RW * NW; i += NT) hrow[i] = 0;
    for (int i = tid; i < 128; i += NT) hcol[i] = 0;
    __syncthreads();
    // ---- mask -> Wt (1/9 on mask cells, 0 elsewhere), storage row / column counts
    fe_v2 T[RW], Wt[RW];
    const int gca = 2 * lane + 1, gcb = 2 * lane + 2;  // columns 0 and 129: implicit (DPP bound) zeros
    const bool ca_in = gca <= SC, cb_in = gcb <= SC;
    const int offa = tr ? (gca - 1) * Dx : gca - 1, offb = tr ? (gcb - 1) * Dx : gcb - 1;
    const int rstep = tr ? 1 : Dx;  // label offset per storage row
    int cnta = 0, cntb = 0;
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      const int gr = 1 + wv * RS + j;
      bool ia = false, ib = false;
      if (j < nrow) {
        const int ro = (gr - 1) * rstep;
        ia = ca_in && lab[ro + offa] == L;
        ib = cb_in && lab[ro + offb] == L;
      }
      T[j] = fe_v2{0.f, 0.f};
      Wt[j] = fe_v2{ia ? (float)(1 / 9.) : 0.f, ib ? (float)(1 / 9.) : 0.f};
      cnta += ia;
      cntb += ib;
      const int rc = __popcll(__ballot(ia)) + __popcll(__ballot(ib));
      if (lane == 0 && j < nrow) hrow[gr - 1] = rc;
      if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // at most 16 label loads in flight
    }
    if (ca_in && cnta) atomicAdd(&hcol[gca - 1], cnta);
    if (cb_in && cntb) atomicAdd(&hcol[gcb - 1], cntb);
    __syncthreads();
    // ---- medians of the original coordinates (row / column counts), as k_flow_error_lds
    if (wv == 0) {
      const long long cntn = o.area;
      const long long ka = (cntn - 1) / 2, kb = cntn / 2;
      const int* hy = tr ? hcol : hrow;  // original rows
      const int* hx = tr ? hrow : hcol;  // original columns
      const int ya = fe_hist_rank(hy, bh, ka), yb = fe_hist_rank(hy, bh, kb);
      const int xa = fe_hist_rank(hx, bw, ka), xb = fe_hist_rank(hx, bw, kb);
      if (lane == 0) {
        smed2[0] = ya + yb + 2;  // 2 * ymed (ymed = ((ya + 1) + (yb + 1)) / 2)
        smed2[1] = xa + xb + 2;
      }
    }
    __syncthreads();
    // ---- argmin of (x - xmed)^2 + (y - ymed)^2 (4x that is an exact integer), first in
    // original row-major order on ties
    const int ym2 = smed2[0], xm2 = smed2[1];
    unsigned long long best = ~0ull;
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      const int gr = 1 + wv * RS + j;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int gc = h ? gcb : gca;
        const int rr = (tr ? gc : gr) - 1, cc = (tr ? gr : gc) - 1;
        const int dy2 = 2 * (rr + 1) - ym2, dx2 = 2 * (cc + 1) - xm2;  // |.| <= 256
        const unsigned long long key = ((unsigned long long)(dy2 * dy2 + dx2 * dx2) << 32) |
                                       (unsigned int)(rr * bw + cc);
        if ((h ? Wt[j].y : Wt[j].x) != 0.f && key < best) best = key;
      }
    }
    best = wave_min(best);
    if (lane == 0) sbest[wv] = best;
    __syncthreads();
    unsigned long long bsel = sbest[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) bsel = sbest[w] < bsel ? sbest[w] : bsel;
    const int pbest = (int)(bsel & 0xffffffffu);
    const int ym = pbest / bw + 1, xm = pbest % bw + 1;  // original, 1-based in the padded grid
    const int cr = tr ? xm : ym, cgc = tr ? ym : xm;     // storage centre
    const int wc = __builtin_amdgcn_readfirstlane((cr - 1) / RS), jc = __builtin_amdgcn_readfirstlane((cr - 1) % RS);
    fe_v2 cadd = lane == ((cgc - 1) >> 1) ? (((cgc - 1) & 1) ? fe_v2{0.f, 1.f} : fe_v2{1.f, 0.f}) : fe_v2{0.f, 0.f};
    const int niter = 2 * ((bw - 1) + (bh - 1));
    if (niter > 0 && wv == wc) fe_row_op<0, RW>(T, jc, cadd);  // the first iteration's T[centre] += 1
    // ---- the sweeps (rows in groups of 8: the group branch is wave-uniform, the rows of a group
    // interleave; rows past nrow have Wt = 0 and stay 0)
    fe_v2 up = {0.f, 0.f}, dn = {0.f, 0.f};
    for (int it = 0; it < niter; ++it) {
      if constexpr (NW > 1) {  // the neighbouring slabs' boundary rows (old values)
        const int par = it & 1;
        fe_v2 last = {0.f, 0.f};
        fe_row_op<2, RW>(T, nrow - 1, last);
        xr[par][wv][0][lane] = T[0];
        xr[par][wv][1][lane] = last;
        __syncthreads();
        if (wv > 0) up = xr[par][wv - 1][1][lane];
        if (wv < NW - 1) dn = xr[par][wv + 1][0][lane];
        fe_row_op<1, RW>(T, nrow, dn);  // the row below the slab (nrow < RW)
      }
      fe_v2 po = up;
#pragma unroll
      for (int g = 0; g < RW / 8; ++g) {
        if (8 * g < nrow) {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            const int j = 8 * g + jj;
            const fe_v2 cur = T[j];
            const fe_v2 nx = j + 1 < RW ? T[j + 1] : dn;
            const fe_v2 v = (po + cur) + nx;  // packed
            const float s = v.x + v.y;
            const fe_v2 hh = fe_v2{dpp_from_left(v.y) + s, dpp_from_right(v.x) + s};
            po = cur;
            T[j] = hh * Wt[j];
          }
        }
      }
      // the next sweep's T[centre] += 1
      if (wv == wc && it + 1 < niter) fe_row_op<0, RW>(T, jc, cadd);
    }
    // ---- gradients, normalisation, error vs dP/5 (k_flow_error_lds's screening arithmetic)
    if constexpr (NW > 1) {
      const int par = niter & 1;
      fe_v2 last = {0.f, 0.f};
      fe_row_op<2, RW>(T, nrow - 1, last);
      xr[par][wv][0][lane] = T[0];
      xr[par][wv][1][lane] = last;
      __syncthreads();
      if (wv > 0) up = xr[par][wv - 1][1][lane];
      if (wv < NW - 1) dn = xr[par][wv + 1][0][lane];
    }
    fe_row_op<1, RW>(T, nrow, dn);  // the row below the slab
    const float2* F = dpf + (long long)fov * n;
    const double g32 = 11.0 * 0x1p-24 * (1.0 + 1e-6), g64 = 11.0 * 0x1p-53 * (1.0 + 1e-6);
    const double rho = (expm1((double)niter * g32) + expm1((double)niter * g64)) / (1.0 - (double)niter * g32);
    const double alpha = 4.0 * (double)niter * 0x1p-126;
    double e0 = 0.0, e1 = 0.0, eb = 0.0;
    // one row per iteration from T[0] / Wt[0], the arrays shifted down by one row after it (the
    // heavy fp64 body is emitted once; static register indices only)
    fe_v2 tu = up, dnx = nrow == RW ? dn : fe_v2{0.f, 0.f};
    // eight rows per iteration from T[0 .. 8] / Wt[0 .. 7], the arrays shifted down by eight rows
    // after it (static register indices only); the row below the slab enters at the first shift
#pragma unroll 1
    for (int j0 = 0; j0 < nrow; j0 += 8) {
#pragma unroll
     for (int jj = 0; jj < 8; ++jj) {
      const int gr = 1 + wv * RS + j0 + jj;
      const fe_v2 tc = T[jj], wc2 = Wt[jj];
      const fe_v2 td = T[jj + 1];
      // storage horizontal neighbours of columns a (2l) and b (2l + 1)
      const float la = dpp_from_left(tc.y), ra = tc.y, lb = tc.x, rb = dpp_from_right(tc.x);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if ((h ? wc2.y : wc2.x) == 0.f) continue;
        const int gc = h ? gcb : gca;
        const float sd = h ? td.y : td.x, su = h ? tu.y : tu.x, sr = h ? rb : ra, sl = h ? lb : la;
        // original orientation: down / up / right / left
        const double tdn = (double)(tr ? sr : sd), tup = (double)(tr ? sl : su);
        const double trt = (double)(tr ? sd : sr), tlf = (double)(tr ? su : sl);
        const int Y = tr ? gc : gr, X = tr ? gr : gc;
        const double dy = tdn - tup;
        const double dx = trt - tlf;
        const double g = sqrt(dy * dy + dx * dx);
        const double nrm = 1e-20 + g;
        const double my = dy / nrm, mx = dx / nrm;
        const float2 f = F[(long long)(r0 + Y - 1) * Dx + c0 + X - 1];
        const double fy = (double)(f.x / 5.0f), fx = (double)(f.y / 5.0f);
        const double ty = my - fy;
        const double tx = mx - fx;
        e0 += ty * ty;
        e1 += tx * tx;
        const double Dy_ = rho * (tdn + tup) + 2.0 * alpha, Dx_ = rho * (trt + tlf) + 2.0 * alpha;
        const double D = sqrt(Dy_ * Dy_ + Dx_ * Dx_) * (1.0 + 1e-9);
        const double ff = sqrt(fy * fy + fx * fx);
        if (g > 3.0 * D && g > 1e-12) {
          const double ep = 2.0 * D / g + 1e-7;
          eb += ep * (2.0 * sqrt(ty * ty + tx * tx) + ep);
        } else {
          eb += (1.0 + ff) * (1.0 + ff);
        }
      }
      tu = tc;
     }
#pragma unroll
      for (int k = 0; k < RW; ++k) {
        T[k] = k + 8 < RW ? T[k + 8] : k + 8 == RW ? dnx : fe_v2{0.f, 0.f};
        Wt[k] = k + 8 < RW ? Wt[k + 8] : fe_v2{0.f, 0.f};
      }
      dnx = fe_v2{0.f, 0.f};
    }
    e0 = wave_sum(e0);
    e1 = wave_sum(e1);
    eb = wave_sum(eb);
    if (lane == 0) {
      sred[wv][0] = e0;
      sred[wv][1] = e1;
      sred[wv][2] = eb;
    }
    __syncthreads();
    if (tid == 0) {
      double s0 = 0.0, s1 = 0.0, sb = 0.0;
      for (int w = 0; w < NW; ++w) {
        s0 += sred[w][0];
        s1 += sred[w][1];
        sb += sred[w][2];
      }
      const double err = 0.0 + s0 / (double)o.area + s1 / (double)o.area;
      const double bnd = sb / (double)o.area + 1e-9 * (1.0 + err);
      const unsigned char v = err - thr > bnd ? 1 : thr - err > bnd ? 2 : 3;
      if (v == 3) und[1 + atomicAdd(&und[0], 1)] = (fov << 20) | kobj;
      bad[(long long)fov * (max_label + 1) + L] = v;
    }
    __syncthreads();
  }
}

// k_flow_error_reg1: class 1 of fe_reg_class — one storage column per lane (lane l = column
// l + 1; columns 0 and SC + 1 are the DPP shifts' out-of-range zeros), the rows in registers
// (T[j], Wt[j]: 2 VGPRs per row), one wave per mask: no exchange and no barrier in the sweeps.  A
// sweep per row: the vertical 3-sum (2 adds), the horizontal 3-sum with both neighbours read by
// DPP (2 adds with the DPP folded into the operand), times 1/9 or 0 (1 mul).  Arithmetic, bound
// and decision as k_flow_error_reg.
template <int RW>
__global__ __launch_bounds__(64, 2) void k_flow_error_reg1(
    const int* __restrict__ m0, const float2* __restrict__ dpf, int Dy, int Dx, int B, int max_label,
    const cpx_object* __restrict__ objects, const int* __restrict__ off, int* __restrict__ ctr, double thr,
    unsigned char* __restrict__ bad, int* __restrict__ und) {
  static_assert(RW % 8 == 0, "rows in groups of 8");
  __shared__ int hrow[RW], hcol[64];
  const int lane = threadIdx.x;
  const long long n = (long long)Dy * Dx;
  const int total = off[B];
  for (int claims = 0;; ++claims) {
    if (claims > total) {  // broken claim (cpx_internal.h kClaimBroken); claims is wave-uniform
      if (lane == 0) atomicOr(ctr, kClaimBroken);
      break;
    }
    // the claim without a divergent branch (every lane adds, only lane 0 adds 1; its old value,
    // read into an SGPR, is the item): the item loop's control flow stays wave-uniform — with a
    // lane-0 branch and a one-wave block (whose barriers are no-ops) the compiler re-read the
    // shared item without re-claiming and the loop never ended
    const int item = __builtin_amdgcn_readfirstlane(atomicAdd(ctr, lane == 0 ? 1 : 0));
    if (item >= total) break;
    int fov = 0;
    while (fov + 1 < B && off[fov + 1] <= item) ++fov;
    const int kobj = item - off[fov];
    const cpx_object o = objects[(long long)fov * max_label + kobj];
    const int L = o.label;
    const int r0 = o.bbox[0], c0 = o.bbox[1];
    const int bh = o.bbox[2] - r0, bw = o.bbox[3] - c0;
    bool tr = false;
    if (fe_reg_class(bh, bw, tr) != 1) continue;  // wave-uniform
    const int SR = __builtin_amdgcn_readfirstlane(tr ? bw : bh), SC = tr ? bh : bw;  // storage rows / columns
    const int* lab = m0 + (long long)fov * n + (long long)r0 * Dx + c0;
    hcol[lane] = 0;
    for (int i = lane; i < RW; i += 64) hrow[i] = 0;
    __syncthreads();
    // ---- mask -> Wt (1/9 on mask cells, 0 elsewhere), storage row / column counts
    float T[RW], Wt[RW];
    const int gc = lane + 1;
    const bool c_in = gc <= SC;
    const int offc = tr ? (gc - 1) * Dx : gc - 1;
    const int rstep = tr ? 1 : Dx;  // label offset per storage row
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      bool in = false;
      if (j < SR) in = c_in && lab[j * rstep + offc] == L;
      T[j] = 0.f;
      Wt[j] = in ? (float)(1 / 9.) : 0.f;
      cnt += in;
      const int rc = __popcll(__ballot(in));
      if (lane == 0 && j < SR) hrow[j] = rc;
      if ((j & 15) == 15) __builtin_amdgcn_sched_barrier(0);  // at most 16 label loads in flight
    }
    if (c_in) hcol[gc - 1] = cnt;
    __syncthreads();
    // ---- medians of the original coordinates, as k_flow_error_lds
    const long long cntn = o.area;
    const long long ka = (cntn - 1) / 2, kb = cntn / 2;
    const int* hy = tr ? hcol : hrow;  // original rows
    const int* hx = tr ? hrow : hcol;  // original columns
    const int ym2 = fe_hist_rank(hy, bh, ka) + fe_hist_rank(hy, bh, kb) + 2;  // 2 * ymed
    const int xm2 = fe_hist_rank(hx, bw, ka) + fe_hist_rank(hx, bw, kb) + 2;
    // ---- argmin of (x - xmed)^2 + (y - ymed)^2 (4x that is an exact integer), first in
    // original row-major order on ties
    unsigned long long best = ~0ull;
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      const int gr = j + 1;
      const int rr = (tr ? gc : gr) - 1, cc = (tr ? gr : gc) - 1;
      const int dy2 = 2 * (rr + 1) - ym2, dx2 = 2 * (cc + 1) - xm2;  // |.| <= 256
      const unsigned long long key = ((unsigned long long)(dy2 * dy2 + dx2 * dx2) << 32) |
                                     (unsigned int)(rr * bw + cc);
      if (Wt[j] != 0.f && key < best) best = key;
    }
    best = wave_min(best);
    const int pbest = (int)(best & 0xffffffffu);
    const int ym = pbest / bw + 1, xm = pbest % bw + 1;  // original, 1-based in the padded grid
    const int jc = __builtin_amdgcn_readfirstlane((tr ? xm : ym) - 1), cgc = tr ? ym : xm;
    float cadd = lane == cgc - 1 ? 1.f : 0.f;
    const int niter = 2 * ((bw - 1) + (bh - 1));
    if (niter > 0) fe_row_op<0, RW>(T, jc, cadd);  // the first iteration's T[centre] += 1
    // ---- the sweeps (rows in groups of 8; rows past SR have Wt = 0 and stay 0)
    for (int it = 0; it < niter; ++it) {
      float po = 0.f;  // the old value of the row above the group
#pragma unroll
      for (int g = 0; g < RW / 8; ++g) {
        if (8 * g < SR) {
          // the group's vertical sums from the old rows, then the horizontal sums, then the
          // stores: eight rows between a sum and its DPP reads (no hazard wait states)
          float v[8];
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            const int j = 8 * g + jj;
            const float up = jj ? T[j - 1] : po;
            const float nx = j + 1 < RW ? T[j + 1] : 0.f;
            v[jj] = (up + T[j]) + nx;
          }
          po = T[8 * g + 7];
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            const int j = 8 * g + jj;
            T[j] = ((dpp_from_left(v[jj]) + v[jj]) + dpp_from_right(v[jj])) * Wt[j];
          }
        }
      }
      if (it + 1 < niter) fe_row_op<0, RW>(T, jc, cadd);  // the next sweep's T[centre] += 1
    }
    // ---- gradients, normalisation, error vs dP/5 (k_flow_error_lds's screening arithmetic); one
    // row per iteration from T[0] / Wt[0], the arrays shifted down by one row after it
    const float2* F = dpf + (long long)fov * n;
    const double g32 = 11.0 * 0x1p-24 * (1.0 + 1e-6), g64 = 11.0 * 0x1p-53 * (1.0 + 1e-6);
    const double rho = (expm1((double)niter * g32) + expm1((double)niter * g64)) / (1.0 - (double)niter * g32);
    const double alpha = 4.0 * (double)niter * 0x1p-126;
    double e0 = 0.0, e1 = 0.0, eb = 0.0;
    float tu = 0.f;
    // eight rows per iteration from T[0 .. 8] / Wt[0 .. 7], the arrays shifted down by eight rows
    // after it (static register indices only; nine moves per row instead of eighty)
#pragma unroll 1
    for (int j0 = 0; j0 < SR; j0 += 8) {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const float tc = T[jj], w = Wt[jj], td = T[jj + 1];
        const float sl = dpp_from_left(tc), sr = dpp_from_right(tc);
        if (w != 0.f) {
          const int gr = j0 + jj + 1;
          // original orientation: down / up / right / left
          const double tdn = (double)(tr ? sr : td), tup = (double)(tr ? sl : tu);
          const double trt = (double)(tr ? td : sr), tlf = (double)(tr ? tu : sl);
          const int Y = tr ? gc : gr, X = tr ? gr : gc;
          const double dy = tdn - tup;
          const double dx = trt - tlf;
          const double g = sqrt(dy * dy + dx * dx);
          const double nrm = 1e-20 + g;
          const double my = dy / nrm, mx = dx / nrm;
          const float2 f = F[(long long)(r0 + Y - 1) * Dx + c0 + X - 1];
          const double fy = (double)(f.x / 5.0f), fx = (double)(f.y / 5.0f);
          const double ty = my - fy;
          const double tx = mx - fx;
          e0 += ty * ty;
          e1 += tx * tx;
          const double Dy_ = rho * (tdn + tup) + 2.0 * alpha, Dx_ = rho * (trt + tlf) + 2.0 * alpha;
          const double D = sqrt(Dy_ * Dy_ + Dx_ * Dx_) * (1.0 + 1e-9);
          const double ff = sqrt(fy * fy + fx * fx);
          if (g > 3.0 * D && g > 1e-12) {
            const double ep = 2.0 * D / g + 1e-7;
            eb += ep * (2.0 * sqrt(ty * ty + tx * tx) + ep);
          } else {
            eb += (1.0 + ff) * (1.0 + ff);
          }
        }
        tu = tc;
      }
#pragma unroll
      for (int k = 0; k + 8 < RW; ++k) {
        T[k] = T[k + 8];
        Wt[k] = Wt[k + 8];
      }
#pragma unroll
      for (int k = RW - 8; k < RW; ++k) {
        T[k] = 0.f;
        Wt[k] = 0.f;
      }
    }
    e0 = wave_sum(e0);
    e1 = wave_sum(e1);
    eb = wave_sum(eb);
    if (lane == 0) {
      const double err = 0.0 + e0 / (double)o.area + e1 / (double)o.area;
      const double bnd = eb / (double)o.area + 1e-9 * (1.0 + err);
      const unsigned char v = err - thr > bnd ? 1 : thr - err > bnd ? 2 : 3;
      if (v == 3) und[1 + atomicAdd(&und[0], 1)] = (fov << 20) | kobj;
      bad[(long long)fov * (max_label + 1) + L] = v;
    }
  }
}


}  // namespace

int cpx_flow_error_reg_launch(int n_cu, hipStream_t stream, const int* m0, const float2* dpf, int Dy, int Dx,
                              int B, int ML, const cpx_object* obj, const int* off, int* ctr, double thr,
                              unsigned char* bad, int* und) {
  hipLaunchKernelGGL((k_flow_error_reg1<kFeReg1Rows>), dim3(8 * n_cu), dim3(64), 0, stream, m0, dpf, Dy, Dx, B,
                     ML, obj, off, ctr, thr, bad, und);
  hipLaunchKernelGGL((k_flow_error_reg<kFeRegRows, 2, 2>), dim3(4 * n_cu), dim3(128), 0, stream, m0, dpf, Dy, Dx,
                     B, ML, obj, off, ctr + 1, 0, thr, bad, und);
  hipLaunchKernelGGL((k_flow_error_reg<kFeReg3Rows, 4, 3>), dim3(2 * n_cu), dim3(256), 0, stream, m0, dpf, Dy, Dx,
                     B, ML, obj, off, ctr + 2, 0, thr, bad, und);
  CPX_CHECK_LAUNCH("k_flow_error_reg");
  return CPX_OK;
}
