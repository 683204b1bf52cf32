// Flood-level encoding of the Cells watershed (k_watershed.hip), shared with the expand_labels
// pass (k_expand.hip) that writes every tile's initial border ring.  See k_watershed.hip's header
// for the algorithm; DESIGN.md §7 for the stated inputs.
#pragma once
#include "cpx_internal.h"

namespace wsl {

constexpr int kT = 32;                                   // tile edge
constexpr int kRing = 4 * kT;                            // ring values per tile: top, bottom, left, right
constexpr unsigned long long kBlocked = ~0ull;           // outside the mask / the image
constexpr unsigned long long kUnreached = ~0ull - 1ull;  // free pixel the flood has not reached
constexpr unsigned kMark = 1u << 16, kBlk = 1u << 17;
constexpr int kKeyShift = 23;

__device__ __forceinline__ unsigned q16(float v) {
  if (!(v < 65535.0f)) return 65535u;  // NaN, inf, >= 65535
  return v > 0.0f ? (unsigned)v : 0u;  // truncation
}

__device__ __forceinline__ unsigned long long key_of(unsigned inf, long long pix) {
  return ((unsigned long long)(inf & 0xffffu) << kKeyShift) | (unsigned long long)pix;
}

__device__ __forceinline__ unsigned long long init_level(unsigned inf, long long pix) {
  if (inf & kBlk) return kBlocked;
  if (inf & kMark) return key_of(inf, pix);
  return kUnreached;
}

// info word from the three inputs (nuclei label, footprint label, cell channel): (65535 - q) |
// marker | blocked
__device__ __forceinline__ unsigned info_of(int n, int f, float v) {
  if (n != 0) return (65535u - q16(v)) | kMark;
  if (f == 0) return kBlk;
  return 65535u - q16(v);
}

// Ring layout: ring[(tile * 4 + side) * kT + k], side 0 = top row (y 0, x k), 1 = bottom row
// (y kT - 1, x k), 2 = left column (y k, x 0), 3 = right column (y k, x kT - 1); tile = fov *
// nty * ntx + ty * ntx + tx.  The ring holds levels (markers: their key), so a tile's halo is four
// contiguous 256-byte reads of its neighbours' rings instead of 2 x kT column lines.
__device__ __forceinline__ void ring_store(unsigned long long* ring, long long tile, int y, int x,
                                          unsigned long long v) {
  unsigned long long* r = ring + tile * kRing;
  if (y == 0) r[x] = v;
  if (y == kT - 1) r[kT + x] = v;
  if (x == 0) r[2 * kT + y] = v;
  if (x == kT - 1) r[3 * kT + y] = v;
}

}  // namespace wsl

// expand_labels (k_expand.hip) that also writes the watershed tiles' initial rings (ring may be
// null: plain cpx_expand_labels); corr_cell = the cell channel of FOV 0, corr_stride = elements
// between consecutive FOVs' cell channels
int cpx_expand_labels_ring(cpx_ctx* ctx, const int32_t* nuclei_dev, int B, int H, int W, int distance,
                           int32_t* cells_dev, int32_t* cyto_dev, const float* corr_cell,
                           long long corr_stride, unsigned long long* ring);
