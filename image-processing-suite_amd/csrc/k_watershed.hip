// a8 secondary objects: Cells by marker watershed from the Nuclei (skimage
// 0.18.3 segmentation.watershed, skimage/segmentation/_watershed.py:94), Cytoplasm = Cells minus
// Nuclei.  Stated inputs (oracle/ws_oracle.py): markers = Nuclei, mask = the
// expand_labels(Nuclei, distance) footprint, elevation key(p) = (65535 - q16(corr_cell(p))) << 23
// | (y*W + x) — all keys distinct, so skimage's heap flood (pop by (value, age), label at push)
// has one total pop order and its result has a parallel characterisation:
//
//   B(p)  = min over 4-paths marker -> p inside the mask of the max key on the path (markers:
//           B = key): the flood level at which p is popped (the running max of popped keys);
//   label = a free pixel is labelled by the first of its neighbours to pop = its neighbour with
//           the smallest B (neighbours tied on B were popped in the same "phase", opened by the
//           pass pixel whose key is that B, and carry the same label).
//
// Computed in two phases over the whole batch, with no host synchronisation:
//   k_ws_relax  (rounds) B by a label-correcting worklist per 32 x 32 tile held in LDS (one wave
//               per tile, its own LDS queue, no barrier on the hop path): every improved pixel
//               p pushes max(key(n), B(p)) to its neighbours with an LDS atomic min, so the work
//               is ~2 visits per free pixel (15 % of a FOV's pixels are free: the rings around
//               the nuclei); a tile whose border changes flags the facing neighbour, which in
//               the next round re-evaluates only its border pixels against the new halo (a
//               queue overflow re-runs the whole tile);
//   k_ws_ptr_init + k_ws_jump (rounds)  labels by pointer jumping over the converged B: a member
//               of a phase points at its pass pixel, a phase start at the pass of its minimum
//               neighbour, every chain ends at a marker (see the comment above k_ws_ptr_init).
// k_ws_status / k_ws_jump_fail fail a FOV (status -1) when the rounds enqueued did not reach the
// fixed point (the host raises).  Exactness vs the sequential heap flood: tests/test_watershed.py
// (oracle) and tests/test_gpu_watershed.py (this kernel), pinned to skimage itself by
// tests/golden/watershed_cases.npz.
#include "cpx_internal.h"
#include "ws_levels.h"
#include <stdio.h>
#include <stdlib.h>

namespace {

using namespace wsl;
constexpr int kThreads = 64;           // one wave per tile: no block barrier on the hop path,
constexpr int kWaves = kThreads / 64;  // eight independent tiles per CU (18 KiB of LDS each)
constexpr int kLS = kT + 3;            // LDS row stride (odd)
constexpr int kLRows = kT + 2;
constexpr int kPerThread = kT * kT / kThreads;
// tile flag bits (per round)
constexpr unsigned char kUp = 1, kLeft = 2, kRight = 4, kDown = 8;  // that border changed
constexpr unsigned char kSelf = 16;   // a wave queue overflowed: re-run the whole tile
constexpr int kQCap = 2048;           // per-wave LDS queue (tile-local pixel indices)
static_assert(kQCap >= kT * kT + 3 * 64, "the seeds of a whole tile plus one drain step fit");
static_assert(kWaves == 1, "one wave per tile");
constexpr unsigned kNoKey = 0xffffffffu;             // sK of a pixel without a key
constexpr unsigned long long kMarkBit = 1ull << 40;  // stored level of a marker: key | kMarkBit
static_assert(kKeyShift + 16 < 40, "keys stay below the marker bit");

struct WsArgs {
  const int* nuc;      // [B][H][W] markers
  const int* foot;     // [B][H][W] expand_labels footprint (!= 0 = in mask)
  const float* corr;   // [B][C][H][W]
  int C, ch, H, W, ntx, nty, total;
  unsigned long long* Bg;  // [B][H][W] stored levels: kBlocked | key | kMarkBit (markers) | B
  unsigned short* inv;     // [B][H][W] 65535 - q16 of free pixels (tiles with free pixels)
  unsigned char* tfree;    // [B * tiles] tile has free pixels
  unsigned long long* ring;  // [B * tiles][4][kT] border levels (ws_levels.h); initial ones from k_edt_rows
  int* last;               // [B][2] last active relax / label round
  unsigned long long* dbg; // optional counters (CPX_WS_DEBUG): [kernel][round][4]
};

__device__ __forceinline__ unsigned char border_bits(int y, int x) {
  unsigned char m = 0;
  if (y == 0) m |= kUp;
  if (y == kT - 1) m |= kDown;
  if (x == 0) m |= kLeft;
  if (x == kT - 1) m |= kRight;
  return m;
}

__device__ __forceinline__ bool neighbour_flagged(const unsigned char* Fp, int fov, int ty, int tx,
                                                  int nty, int ntx, unsigned char self_bits) {
  const int base = fov * nty * ntx;
  const int t = base + ty * ntx + tx;
  if (Fp[t] & self_bits) return true;
  if (ty > 0 && (Fp[t - ntx] & kDown)) return true;
  if (ty + 1 < nty && (Fp[t + ntx] & kUp)) return true;
  if (tx > 0 && (Fp[t - 1] & kRight)) return true;
  if (tx + 1 < ntx && (Fp[t + 1] & kLeft)) return true;
  return false;
}

// halo pixel h of 4*kT (top row, bottom row, left column, right column) -> tile-local (y, x)
__device__ __forceinline__ void halo_pos(int h, int& y, int& x) {
  const int side = h / kT, k = h % kT;
  if (side == 0) { y = -1; x = k; }
  else if (side == 1) { y = kT; x = k; }
  else if (side == 2) { y = k; x = -1; }
  else { y = k; x = kT; }
}


// stored level -> level (markers: their key); kBlocked / kUnreached are stored as themselves
__device__ __forceinline__ bool stored_marker(unsigned long long v) { return v < kUnreached && (v & kMarkBit); }
__device__ __forceinline__ unsigned long long level_of(unsigned long long v) {
  return stored_marker(v) ? (v & ~kMarkBit) : v;
}

// wave-local queue of tile pixel indices (ring of kQCap): head / tail are wave-uniform
struct WaveQueue {
  unsigned short* q;
  int head, tail;
  __device__ __forceinline__ void push(bool pred, int item, int lane) {
    const unsigned long long m = __ballot(pred);
    if (pred) {
      const int pos = tail + __popcll(m & ((1ull << lane) - 1ull));
      q[pos & (kQCap - 1)] = (unsigned short)item;
    }
    tail += __popcll(m);
  }
};

__device__ __forceinline__ int lds_off(int i) { return (1 + i / kT) * kLS + 1 + i % kT; }

// index of the k-th border pixel (k < 4*kT) of the tile
__device__ __forceinline__ int border_pixel(int k) {
  const int side = k / kT, j = k % kT;
  if (side == 0) return j;
  if (side == 1) return (kT - 1) * kT + j;
  if (side == 2) return j * kT;
  return j * kT + kT - 1;
}


// Tiles of a round: XCD x (the blocks b with b % 8 == x) owns the contiguous tile range
// [total x / 8, total (x + 1) / 8) and block b takes the tiles lo + b / 8 + k * (blocks on its
// XCD), so horizontally and vertically adjacent tiles run on one XCD at about the same time and
// the 4-byte column halos they read from each other's lines hit that XCD's L2.  Blocks get few
// tiles (kShare0 in round 0, kShare later) and the hardware dispatcher balances the rest: a free
// tile costs ~10x an empty one, and with shares of 50-100 tiles per block the average wave sat
// idle for 40 % of round 0 (SQ_WAVE_CYCLES against the kernel's duration, gpurun_out/r06o);
// shares of 4 / 16 took the relax rounds from 5.47 to 4.61 ms per 48 FOVs (gpurun_out/r06s;
// claiming chunks from per-XCD counters instead measured the same, 4.58 ms).  A block
// evaluates its tiles at once, one per lane, from the flags of the previous round: inactive ones
// get their flags written, active ones are relaxed in order.  Active: every tile in round 0,
// later a tile with free pixels whose facing neighbour's border changed (or whose own queue
// overflowed: kSelf).
constexpr int kShare0 = 4, kShare = 16;
static_assert(kShare0 <= kThreads && kShare <= kThreads, "one tile per lane");

__device__ __forceinline__ bool tile_active(const WsArgs& a, int round, const unsigned char* Fp, int t) {
  if (round == 0) return true;
  const int per = a.nty * a.ntx;
  const int fov = t / per, tt = t - fov * per, ty = tt / a.ntx, tx = tt - ty * a.ntx;
  (void)fov;
  // all flags loaded before use (clamped neighbour indices; edges masked after)
  const unsigned char fs = Fp[t], fr = a.tfree[t];
  const unsigned char fu = Fp[ty > 0 ? t - a.ntx : t], fd = Fp[ty + 1 < a.nty ? t + a.ntx : t];
  const unsigned char fl = Fp[tx > 0 ? t - 1 : t], fg = Fp[tx + 1 < a.ntx ? t + 1 : t];
  const bool nb = (ty > 0 && (fu & kDown)) || (ty + 1 < a.nty && (fd & kUp)) ||
                  (tx > 0 && (fl & kRight)) || (tx + 1 < a.ntx && (fg & kLeft));
  return fr && (nb || (fs & kSelf));
}

// border bits of a padded LDS offset (tile rows / columns 1..kT)
__device__ __forceinline__ unsigned char border_bits_off(int o) {
  return border_bits(o / kLS - 1, o % kLS - 1);
}

template <bool R0>
__global__ __launch_bounds__(kThreads, 2) void k_ws_relax(WsArgs a, int round,
                                                       const unsigned char* __restrict__ Fp,
                                                       unsigned char* __restrict__ Fn) {
  // levels of the tile + halo, and the key of every free tile pixel (kBlocked for markers,
  // blocked pixels and the halo: max(kBlocked, .) never lowers them, so the pushes need no
  // bounds or type checks); the queue holds padded LDS offsets
  // sK holds a free pixel's inverted intensity (its key without the pixel index, which follows
  // from the LDS offset) or kNoKey; the seed candidates share the queue's storage (a seed is read
  // before the queue's tail can reach its slot): 18 KiB per tile, eight tiles per CU
  __shared__ unsigned long long sB[kLRows * kLS];
  __shared__ unsigned sK[kLRows * kLS];
  __shared__ unsigned short sQ[kQCap];
  unsigned short* sS = sQ;  // seed candidates
  __shared__ unsigned s_bits;
  const int lane = threadIdx.x;
  const long long hw = (long long)a.H * a.W;
  const long long hwc = hw * a.C;
  const int G = gridDim.x, xb = blockIdx.x & 7, xi = blockIdx.x >> 3, ng = G < 8 ? G : 8;
  const int gx = (G - xb + 7) >> 3;
  const int lo = (int)((long long)a.total * xb / ng), hi = (int)((long long)a.total * (xb + 1) / ng);
  // (shares <= 64 tiles: one pass)
  for (int k = 0; lo + xi + k * gx < hi; k += kThreads) {
    const int tl = lo + xi + (k + lane) * gx;  // this lane's tile
    const bool ok = tl < hi;
    bool act = false;
    if (ok) {
      act = tile_active(a, round, Fp, tl);
      if (!act) Fn[tl] = 0;
    }
    for (unsigned long long am = __ballot(act); am; am &= am - 1) {
      const int t = __shfl(tl, __ffsll((long long)am) - 1, 64);
      const int per = a.nty * a.ntx;
      const int fov = t / per, tt = t - fov * per, ty = tt / a.ntx, tx = tt - ty * a.ntx;
      const bool full = R0 || (Fp[t] & kSelf) != 0;
      const int y0 = ty * kT, x0 = tx * kT;
      // key of the pixel at padded LDS offset o (kBlocked for markers, blocked pixels, the halo)
      auto key_at = [&](int o) -> unsigned long long {
        const unsigned v = sK[o];
        if (v == kNoKey) return kBlocked;
        const int oy = o / kLS - 1, ox = o - (o / kLS) * kLS - 1;
        return ((unsigned long long)v << kKeyShift) | (unsigned long long)((long long)(y0 + oy) * a.W + x0 + ox);
      };
      if (lane == 0) s_bits = 0;
      const int* nucf = a.nuc + fov * hw;
      const int* footf = a.foot + fov * hw;
      const float* cf = a.corr + fov * hwc + (long long)a.ch * hw;
      const unsigned long long* Bf = a.Bg + fov * hw;
      // every load of the tile and of this lane's halo pixels in flight before any is used
      // (round 0: nuclei, footprint, cell channel; later rounds: stored level, inverted key)
      unsigned long long w0_[kPerThread];
      int w1_[kPerThread];
  #pragma unroll
      for (int k = 0; k < kPerThread; ++k) {
        const int i = lane + k * kThreads, y = y0 + i / kT, x = x0 + i % kT;
        const long long pix = (y < a.H && x < a.W) ? (long long)y * a.W + x : 0;
        if (R0) {
          w0_[k] = ((unsigned long long)(unsigned)nucf[pix] << 32) | (unsigned)footf[pix];
          w1_[k] = __float_as_int(cf[pix]);
        } else {
          w0_[k] = Bf[pix];
          w1_[k] = a.inv[fov * hw + pix];
        }
      }
      // halo: the facing border vectors of the four neighbour tiles' rings (contiguous; the initial
      // rings come from k_edt_rows, later ones from the neighbours' previous visits — any of them is
      // an upper bound of the final level, and a changed border flags this tile for the next round)
      constexpr int kHalo = kRing / kThreads;
      static_assert(kRing % kThreads == 0, "whole halo per lane");
      unsigned long long hv[kHalo];
      int ho[kHalo];
  #pragma unroll
      for (int k = 0; k < kHalo; ++k) {
        const int h = lane + k * kThreads, side = h / kT, j = h % kT;
        int hy, hx;
        halo_pos(h, hy, hx);
        ho[k] = (1 + hy) * kLS + 1 + hx;
        long long src = -1;
        if (side == 0) { if (ty > 0 && x0 + j < a.W) src = (long long)(t - a.ntx) * kRing + kT + j; }
        else if (side == 1) { if (ty + 1 < a.nty && x0 + j < a.W) src = (long long)(t + a.ntx) * kRing + j; }
        else if (side == 2) { if (tx > 0 && y0 + j < a.H) src = (long long)(t - 1) * kRing + 3 * kT + j; }
        else if (tx + 1 < a.ntx && y0 + j < a.H) src = (long long)(t + 1) * kRing + 2 * kT + j;
        hv[k] = src >= 0 ? a.ring[src] : kBlocked;
      }
      int any_free = 0;
  #pragma unroll
      for (int k = 0; k < kPerThread; ++k) {
        const int i = lane + k * kThreads, y = y0 + i / kT, x = x0 + i % kT;
        unsigned long long b = kBlocked, key = kBlocked;
        if (y < a.H && x < a.W) {
          const long long pix = (long long)y * a.W + x;
          if (R0) {
            const unsigned inf = info_of((int)(w0_[k] >> 32), (int)(unsigned)w0_[k], __int_as_float(w1_[k]));
            b = init_level(inf, pix);
            if (!(inf & (kMark | kBlk))) key = key_of(inf, pix);
          } else {
            const unsigned long long v = w0_[k];
            b = level_of(v);
            if (v != kBlocked && !stored_marker(v)) key = key_of((unsigned)w1_[k], pix);
          }
        }
        any_free |= key != kBlocked;
        sB[lds_off(i)] = b;
        sK[lds_off(i)] = key != kBlocked ? (unsigned)(key >> kKeyShift) : kNoKey;
      }
  #pragma unroll
      for (int k = 0; k < kHalo; ++k) {
        sB[ho[k]] = hv[k];
        sK[ho[k]] = kNoKey;
      }
      any_free = __syncthreads_or(any_free);
      if (R0) {
        if (lane == 0) a.tfree[t] = (unsigned char)(any_free != 0);
        if (!any_free) {  // no free pixel: only the border ring is ever read (as a neighbour's halo)
          for (int k = lane; k < 4 * kT; k += kThreads) {
            const int i = border_pixel(k), y = y0 + i / kT, x = x0 + i % kT;
            if (y < a.H && x < a.W) {
              const unsigned long long b = sB[lds_off(i)];
              a.Bg[fov * hw + (long long)y * a.W + x] = b == kBlocked ? b : (b | kMarkBit);
            }
          }
          if (lane == 0) Fn[t] = 0;
          __syncthreads();
          continue;
        }
      }
      WaveQueue wq{sQ, 0, 0};
      unsigned bits = 0;
      // seeds: every free pixel (full) or the border pixels (new halo), pulled from its neighbours;
      // the candidates are compacted first (a fifth of a tile's pixels are free)
      int nseed = 0;
      if (full) {
  #pragma unroll
        for (int k = 0; k < kPerThread; ++k) {
          const int o = lds_off(lane + k * kThreads);
          const bool c = sK[o] != kNoKey;
          const unsigned long long m = __ballot(c);
          if (c) sS[nseed + __popcll(m & ((1ull << lane) - 1ull))] = (unsigned short)o;
          nseed += __popcll(m);
        }
      } else {
        for (int k = lane; k < 4 * kT; k += kThreads) sS[k] = (unsigned short)lds_off(border_pixel(k));
        nseed = 4 * kT;
      }
      __syncthreads();
      for (int base = 0; base < nseed; base += kThreads) {
        const int o = base + lane < nseed ? (int)sS[base + lane] : kLS + 1;
        const unsigned long long key = base + lane < nseed ? key_at(o) : kBlocked;
        bool imp = false;
        if (key != kBlocked) {
          const unsigned long long u = sB[o - kLS], l = sB[o - 1], r = sB[o + 1], d = sB[o + kLS];
          unsigned long long m = u < l ? u : l;
          m = r < m ? r : m;
          m = d < m ? d : m;
          const unsigned long long nv = m > key ? m : key;
          if (nv < sB[o]) imp = nv < atomicMin(&sB[o], nv);
        }
        if (imp) bits |= border_bits_off(o);
        wq.push(imp, o, lane);
      }
      // drain: push the improved level to the four neighbours (all reads of a step issued together)
      bool ovf = false;
      int dsteps = 0, ditems = 0;
      while (wq.tail != wq.head) {
        const int cnt = min(64, wq.tail - wq.head);
        ++dsteps;
        ditems += cnt;
        if (wq.tail - wq.head + 3 * cnt > kQCap) {
          ovf = true;
          break;
        }
        const bool act = lane < cnt;
        const int o = act ? (int)wq.q[(wq.head + lane) & (kQCap - 1)] : kLS + 1;
        wq.head += cnt;
        const int nb[4] = {o - kLS, o - 1, o + 1, o + kLS};
        const unsigned long long b = sB[o];
        unsigned long long kk[4], bb[4];
  #pragma unroll
        for (int d = 0; d < 4; ++d) {
          kk[d] = key_at(nb[d]);
          bb[d] = sB[nb[d]];
        }
        bool imp[4];
  #pragma unroll
        for (int d = 0; d < 4; ++d) {
          const unsigned long long nv = b > kk[d] ? b : kk[d];
          imp[d] = act && nv < bb[d];
          if (imp[d]) imp[d] = nv < atomicMin(&sB[nb[d]], nv);
        }
  #pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (imp[d]) bits |= border_bits_off(nb[d]);
          wq.push(imp[d], nb[d], lane);
        }
      }
      if (ovf) bits |= kSelf;
      if (bits) atomicOr(&s_bits, bits);
      if (a.dbg && lane == 0) {
        unsigned long long* c = a.dbg + (0 * 64 + round) * 4;
        atomicAdd(c, 1ull);
        atomicAdd(c + 1, (unsigned long long)dsteps);
        atomicAdd(c + 2, (unsigned long long)ditems);
        atomicAdd(c + 3, (unsigned long long)ovf);
      }
      __syncthreads();
      // a later-round visit that improved no seed changed nothing: its levels and ring stay as
      // stored (round 2 of 48 FOVs visits ~106 K tiles for 0.6 M worklist items)
      if (!R0 && wq.tail == 0) {
        if (lane == 0) Fn[t] = (unsigned char)s_bits;
        __syncthreads();
        continue;
      }
      for (int i = lane; i < kT * kT; i += kThreads) {
        const int y = y0 + i / kT, x = x0 + i % kT;
        if (y >= a.H || x >= a.W) continue;
        const long long pix = fov * hw + (long long)y * a.W + x;
        const int o = lds_off(i);
        const unsigned long long b = sB[o];
        const unsigned kv = sK[o];
        if (kv != kNoKey) {
          a.Bg[pix] = b;
          if (R0) a.inv[pix] = (unsigned short)kv;
        } else if (R0) {
          a.Bg[pix] = b == kBlocked ? b : (b | kMarkBit);
        }
      }
      // this tile's border levels for its neighbours' halos
      for (int h = lane; h < kRing; h += kThreads) {
        const int side = h / kT, j = h % kT;
        const int ly = side == 0 ? 0 : side == 1 ? kT - 1 : j, lx = side == 2 ? 0 : side == 3 ? kT - 1 : j;
        if (y0 + ly < a.H && x0 + lx < a.W) a.ring[(long long)t * kRing + h] = sB[(1 + ly) * kLS + 1 + lx];
      }
      if (lane == 0) {
        Fn[t] = (unsigned char)s_bits;
        a.last[fov * 2] = round;
      }
      __syncthreads();
    }
  }
}

// Labels from the converged levels, by pointer jumping.  A free reached pixel p belongs to the
// flood phase opened by its pass pixel: pass(p) = the pixel whose key is B(p) (the low 23 bits of
// B).  A member (B(p) > key(p)) has the label of its pass; a phase start (B(p) == key(p)) has the
// label of its first-popped neighbour, i.e. of the pass of its neighbours' minimum level S(p)
// (neighbours tied at S share that pass).  So ptr(p) = pass of (member ? B(p) : S(p)) — always an
// earlier-popped pass or a marker — and following ptr ends at the marker whose label p takes.
// k_ws_ptr_init resolves the pixels whose target is a marker and lists the rest; each k_ws_jump
// round resolves the listed pixels whose target is labelled and halves the others' chains.
constexpr int kJumpThreads = 256;
constexpr long long kIdxMask = (1ll << kKeyShift) - 1;

// Survivors of a block are gathered in LDS and appended to the global list with one atomic per
// block (a per-wave atomic on one counter serialises ~10^6 times per batch).
constexpr int kJumpPer = 8;                       // list items / pixels per thread
constexpr int kJumpChunk = kJumpThreads * kJumpPer;

__device__ __forceinline__ void block_append(bool pred, int item, int* s_buf, int* s_cnt) {
  const unsigned long long m = __ballot(pred);
  if (!m) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(s_cnt, __popcll(m));
  base = __shfl(base, leader, 64);
  if (pred) s_buf[base + __popcll(m & ((1ull << lane) - 1ull))] = item;
}

__device__ __forceinline__ void block_flush(const int* s_buf, int* s_cnt, int* s_base, int* list, int* cnt) {
  __syncthreads();
  if (threadIdx.x == 0) *s_base = *s_cnt ? atomicAdd(cnt, *s_cnt) : 0;
  __syncthreads();
  for (int i = threadIdx.x; i < *s_cnt; i += kJumpThreads) list[*s_base + i] = s_buf[i];
  __syncthreads();
  if (threadIdx.x == 0) *s_cnt = 0;
  __syncthreads();
}

// one block per 32 x 32 tile (tiles without free pixels stored only their border ring: nothing
// to label there)
// In-tile chain resolution: pointer chains that stay inside the tile are followed in LDS (ten
// doubling rounds cover any chain of the tile's 1024 pixels); only pixels whose chain leaves the
// tile go to the global list, their pointer compressed to the chain's first pixel outside.  (Done
// per pixel in the global rounds alone, nearly every free pixel went through 5-7 rounds of
// scattered 4-byte gathers.)
constexpr int kInTileRounds = 10;
static_assert((1 << kInTileRounds) >= kT * kT, "doubling rounds cover a whole tile");

__global__ __launch_bounds__(kJumpThreads) void k_ws_ptr_init(WsArgs a, int* __restrict__ cells,
                                                              int* __restrict__ cyto, int* __restrict__ ptr,
                                                              int* __restrict__ list, int* __restrict__ cnt) {
  __shared__ int s_buf[kT * kT];
  __shared__ int s_lab[kT * kT];  // label (> 0), 0 = unresolved, -1 = no chain (not a free reached pixel)
  __shared__ int s_tgt[kT * kT];  // FOV-global index of the pixel's current ancestor
  __shared__ short s_loc[kT * kT];  // that ancestor's index in this tile, -1 outside it
  __shared__ int s_cnt, s_base;
  constexpr int PER = kT * kT / kJumpThreads;
  // XCD-aware: each XCD labels a contiguous run of tiles (neighbour level reads stay in its L2)
  const int G = gridDim.x, xb = blockIdx.x & 7;
  const int t = xb * (G >> 3) + min(xb, G & 7) + (blockIdx.x >> 3);
  if (!a.tfree[t]) return;
  const int per = a.nty * a.ntx;
  const int fov = t / per, tt = t - fov * per, ty = tt / a.ntx, tx = tt - ty * a.ntx;
  const long long hw = (long long)a.H * a.W;
  const int y0 = ty * kT, x0 = tx * kT;
  if (threadIdx.x == 0) s_cnt = 0;
  int lab[PER], tgt[PER], loc[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = threadIdx.x + k * kJumpThreads, y = y0 + i / kT, x = x0 + i % kT;
    lab[k] = -1;
    tgt[k] = 0;
    loc[k] = -1;
    if (y < a.H && x < a.W) {
      const long long idx = (long long)y * a.W + x;
      const long long g = fov * hw + idx;
      const unsigned long long v = a.Bg[g];
      if (v != kBlocked && !stored_marker(v)) {
        if (v >= kUnreached) {  // never flooded: left unlabelled, as skimage leaves it
          cells[g] = 0;
          cyto[g] = 0;
        } else {
          const unsigned long long key = ((unsigned long long)a.inv[g] << kKeyShift) | (unsigned long long)idx;
          unsigned long long S = kBlocked;
          if (y > 0) S = min(S, level_of(a.Bg[g - a.W]));
          if (x > 0) S = min(S, level_of(a.Bg[g - 1]));
          if (x + 1 < a.W) S = min(S, level_of(a.Bg[g + 1]));
          if (y + 1 < a.H) S = min(S, level_of(a.Bg[g + a.W]));
          const int ti = (int)((v == key ? S : v) & (unsigned long long)kIdxMask);
          const long long tg = fov * hw + ti;
          lab[k] = stored_marker(a.Bg[tg]) ? a.nuc[tg] : 0;
          tgt[k] = (int)tg;
          const int ty_ = ti / a.W - y0, tx_ = ti - (ti / a.W) * a.W - x0;
          loc[k] = (ty_ >= 0 && ty_ < kT && tx_ >= 0 && tx_ < kT) ? ty_ * kT + tx_ : -1;
        }
      }
    }
    s_lab[i] = lab[k];
    s_tgt[i] = tgt[k];
    s_loc[i] = (short)loc[k];
  }
  __syncthreads();
  for (int r = 0; r < kInTileRounds; ++r) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (lab[k] != 0) continue;
      const int li = loc[k];
      if (li < 0) continue;  // the chain has left the tile
      const int l = s_lab[li];
      if (l > 0) lab[k] = l;
      else if (l == 0) {  // jump to the ancestor's ancestor
        tgt[k] = s_tgt[li];
        loc[k] = s_loc[li];
      } else continue;  // (an ancestor is always a free reached pixel or a marker)
      any = true;
    }
    __syncthreads();  // every read of this round before the writes
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + k * kJumpThreads;
      s_lab[i] = lab[k];
      s_tgt[i] = tgt[k];
      s_loc[i] = (short)loc[k];
    }
    if (!__syncthreads_or(any)) break;
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = threadIdx.x + k * kJumpThreads, y = y0 + i / kT, x = x0 + i % kT;
    const long long g = fov * hw + (long long)y * a.W + x;
    const bool app = lab[k] == 0;
    if (lab[k] >= 0) {
      cells[g] = lab[k];
      cyto[g] = lab[k];
      if (app) ptr[g] = tgt[k];
    }
    block_append(app, (int)g, s_buf, &s_cnt);
  }
  block_flush(s_buf, &s_cnt, &s_base, list, cnt);
}

__global__ __launch_bounds__(kJumpThreads) void k_ws_jump(int r, int* __restrict__ cells, int* __restrict__ cyto,
                                                          int* __restrict__ ptr, const int* __restrict__ in,
                                                          int* __restrict__ out, int* __restrict__ cnt) {
  __shared__ int s_buf[kJumpChunk];
  __shared__ int s_cnt, s_base;
  const int n = cnt[r];
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  for (int c0 = blockIdx.x * kJumpChunk; c0 < n; c0 += gridDim.x * kJumpChunk) {
    int g_[kJumpPer], q_[kJumpPer];
#pragma unroll
    for (int k = 0; k < kJumpPer; ++k) {
      const int i = c0 + threadIdx.x + k * kJumpThreads;
      g_[k] = i < n ? in[i] : -1;
    }
#pragma unroll
    for (int k = 0; k < kJumpPer; ++k) q_[k] = g_[k] >= 0 ? ptr[g_[k]] : 0;
#pragma unroll
    for (int k = 0; k < kJumpPer; ++k) {
      bool app = false;
      if (g_[k] >= 0) {
        const int l = cells[q_[k]];
        if (l > 0) {
          cells[g_[k]] = l;
          cyto[g_[k]] = l;
        } else {
          ptr[g_[k]] = ptr[q_[k]];
          app = true;
        }
      }
      block_append(app, g_[k], s_buf, &s_cnt);
    }
    block_flush(s_buf, &s_cnt, &s_base, out, cnt + r + 1);
  }
}

// a FOV whose pixels are still listed after the last jump round failed
__global__ __launch_bounds__(kJumpThreads) void k_ws_jump_fail(int r, const int* __restrict__ in,
                                                               const int* __restrict__ cnt, long long hw,
                                                               int* __restrict__ status, int stride) {
  const int n = cnt[r];
  for (int i = blockIdx.x * kJumpThreads + threadIdx.x; i < n; i += gridDim.x * kJumpThreads)
    status[(in[i] / hw) * stride] = -1;
}

// per FOV: the relax rounds converged when the last one left no border change / capped tile;
// status = 100 * (relax rounds used) + (jump rounds the batch needed); k_ws_jump_fail then
// overrides FOVs whose labels are still unresolved
__global__ void k_ws_status(const unsigned char* __restrict__ Fr, int per, const int* __restrict__ last,
                            const int* __restrict__ cnt, int jump_rounds, int* __restrict__ status,
                            int stride) {
  const int fov = blockIdx.x;
  int bad = 0;
  for (int i = threadIdx.x; i < per; i += blockDim.x)
    bad |= Fr[fov * per + i] & (kUp | kLeft | kRight | kDown | kSelf);
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    int used = jump_rounds;
    for (int r = 0; r <= jump_rounds; ++r)
      if (cnt[r] == 0) {
        used = r;
        break;
      }
    status[(long long)fov * stride] = bad ? -1 : (last[fov * 2] + 1) * 100 + used;
  }
}

}  // namespace

extern "C" int cpx_watershed_cells(cpx_ctx* ctx, const int32_t* nuclei_dev, const float* corr_dev,
                                   int B, int C, int cell_channel, int H, int W, int distance,
                                   int relax_rounds, int label_rounds, int32_t* cells_dev,
                                   int32_t* cyto_dev, int32_t* status_dev, int status_stride) {
  CPX_REQUIRE(ctx && nuclei_dev && corr_dev && cells_dev && cyto_dev && status_dev, CPX_ERR_ARG,
              "cpx_watershed_cells: null argument");
  CPX_REQUIRE(relax_rounds <= 64 && label_rounds <= 64 && B > 0 && B <= 65535 && C > 0 && cell_channel >= 0 && cell_channel < C && H > 0 &&
                  W > 0 && (long long)H * W <= (1ll << kKeyShift) && relax_rounds > 0 &&
                  label_rounds > 0 && status_stride > 0,
              CPX_ERR_ARG, "cpx_watershed_cells: bad sizes (H*W <= 2^23, 0 <= cell_channel < C, rounds 1..64)");
  const int ntx = cpx_div_up(W, kT), nty = cpx_div_up(H, kT), per = ntx * nty, total = B * per;
  const size_t nB = sizeof(unsigned long long) * (size_t)B * H * W;
  const size_t nF = (size_t)total;
  const size_t nI = (sizeof(unsigned short) * (size_t)B * H * W + 255) / 256 * 256;
  const size_t nP = (sizeof(int) * (size_t)B * H * W + 255) / 256 * 256;  // ptr, two lists
  CPX_REQUIRE((long long)B * H * W < (1ll << 31), CPX_ERR_ARG, "cpx_watershed_cells: batch too large");
  const size_t nR = sizeof(unsigned long long) * kRing * (size_t)total;
  char* ws = (char*)cpx_ws(ctx, WS_WATERSHED, nB + nI + 3 * nP + nR + 5 * nF + sizeof(int) * (2 * B + 80) + 2048);
  if (!ws) return CPX_ERR_OOM;
  // the footprint (mask), the Cytoplasm of every pixel the flood does not relabel, and every
  // tile's initial border ring
  unsigned long long* ring = (unsigned long long*)(ws + nB + nI + 3 * nP);
  int rc = cpx_expand_labels_ring(ctx, nuclei_dev, B, H, W, distance, cells_dev, cyto_dev,
                                  corr_dev + (size_t)cell_channel * H * W, (long long)C * H * W, ring);
  if (rc != CPX_OK) return rc;
  WsArgs a;
  a.nuc = nuclei_dev;
  a.foot = cells_dev;
  a.corr = corr_dev;
  a.C = C;
  a.ch = cell_channel;
  a.H = H;
  a.W = W;
  a.ntx = ntx;
  a.nty = nty;
  a.total = total;
  a.Bg = (unsigned long long*)ws;
  a.inv = (unsigned short*)(ws + nB);
  int* ptr = (int*)(ws + nB + nI);
  int* lists[2] = {(int*)(ws + nB + nI + nP), (int*)(ws + nB + nI + 2 * nP)};
  a.ring = ring;
  unsigned char* F = (unsigned char*)(ws + nB + nI + 3 * nP + nR);  // relax ping-pong, tile-free
  unsigned char* Fr[2] = {F, F + nF};
  a.tfree = F + 4 * nF;
  a.last = (int*)(((uintptr_t)(F + 5 * nF) + 255) & ~(uintptr_t)255);
  int* cnt = a.last + 2 * B;  // jump list counts, one per round
  const bool debug = getenv("CPX_WS_DEBUG") != nullptr;
  a.dbg = nullptr;
  if (debug) {
    CPX_CHECK_HIP(hipMallocAsync((void**)&a.dbg, sizeof(unsigned long long) * 2 * 64 * 4, ctx->stream));
    CPX_CHECK_HIP(hipMemsetAsync(a.dbg, 0, sizeof(unsigned long long) * 2 * 64 * 4, ctx->stream));
  }
  CPX_CHECK_HIP(hipMemsetAsync(a.last, 0xff, sizeof(int) * 2 * B, ctx->stream));
  CPX_CHECK_HIP(hipMemsetAsync(cnt, 0, sizeof(int) * (label_rounds + 1), ctx->stream));
  // eight one-wave blocks per CU fit the LDS; each block takes a share of kShare0 (round 0) or
  // kShare tiles of its XCD's range
  const int grid0 = cpx_div_up(total, kShare0), grid = cpx_div_up(total, kShare);
  // The expand footprint is read in every relax round; the label rounds then overwrite the
  // free pixels of cells / cyto (the footprint is no longer needed: blocked <=> B == kBlocked).
  for (int r = 0; r < relax_rounds; ++r)
    hipLaunchKernelGGL(r == 0 ? k_ws_relax<true> : k_ws_relax<false>, dim3(r == 0 ? grid0 : grid), dim3(kThreads), 0,
                       ctx->stream, a, r, (const unsigned char*)Fr[(r + 1) & 1], Fr[r & 1]);
  const int jgrid = ctx->n_cu * 8;
  hipLaunchKernelGGL(k_ws_ptr_init, dim3(total), dim3(kJumpThreads), 0, ctx->stream, a, cells_dev, cyto_dev,
                     ptr, lists[0], cnt);
  for (int r = 0; r < label_rounds; ++r)
    hipLaunchKernelGGL(k_ws_jump, dim3(jgrid), dim3(kJumpThreads), 0, ctx->stream, r, cells_dev, cyto_dev,
                       ptr, (const int*)lists[r & 1], lists[(r + 1) & 1], cnt);
  hipLaunchKernelGGL(k_ws_status, dim3(B), dim3(256), 0, ctx->stream,
                     (const unsigned char*)Fr[(relax_rounds - 1) & 1], per, (const int*)a.last,
                     (const int*)cnt, label_rounds, status_dev, status_stride);
  hipLaunchKernelGGL(k_ws_jump_fail, dim3(64), dim3(kJumpThreads), 0, ctx->stream, label_rounds,
                     (const int*)lists[label_rounds & 1], (const int*)cnt, (long long)H * W, status_dev,
                     status_stride);
  CPX_CHECK_LAUNCH("cpx_watershed_cells");
  if (debug) {  // profiling aid: per round tiles / drain steps / items / overflows
    unsigned long long h[2 * 64 * 4];
    CPX_CHECK_HIP(hipMemcpyAsync(h, a.dbg, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
    CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    for (int k = 0; k < 1; ++k)
      for (int r = 0; r < relax_rounds; ++r) {
        const unsigned long long* c = h + (k * 64 + r) * 4;
        if (c[0]) fprintf(stderr, "ws %s round %d: tiles %llu steps %llu items %llu overflow %llu\n",
                          k ? "label" : "relax", r, c[0], c[1], c[2], c[3]);
      }
    CPX_CHECK_HIP(hipFreeAsync(a.dbg, ctx->stream));
    int hc[65];
    CPX_CHECK_HIP(hipMemcpy(hc, cnt, sizeof(int) * (label_rounds + 1), hipMemcpyDeviceToHost));
    fprintf(stderr, "ws jump list sizes:");
    for (int r = 0; r <= label_rounds; ++r) fprintf(stderr, " %d", hc[r]);
    fprintf(stderr, "\n");
  }
  return CPX_OK;
}
