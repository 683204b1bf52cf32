// Internal helpers shared by the libcpx HIP translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>
#include <algorithm>
#include "../../include/cpx.h"

constexpr int kWsSlots = 16;

struct cpx_fov_state;  // per-FOV session state (capi_fov.hip)

struct cpx_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // no side streams: every extra stream of a process competes for the GPU_MAX_HW_QUEUES (4)
  // hardware queues, and two pipelines' streams sharing one queue serialise (measured: a
  // per-context fork/join side stream cost 14 % of the two-pipeline bench)
  // generic growable device workspaces (never shrunk; see cpx_reserve)
  void* ws[kWsSlots] = {nullptr};
  size_t ws_bytes[kWsSlots] = {0};
  // allocation generation per slot: a cache of uploaded tables is valid only for the generation
  // it was uploaded into (a regrown slot can come back at the same address, with fresh contents)
  unsigned int ws_gen[kWsSlots] = {0};
  int n_cu = 256;
  // QC FFT twiddle tables currently uploaded (WS_QC_MISC)
  int qc_H = 0, qc_W = 0;
  unsigned int qc_gen = 0;
  // segmentation coefficient tables currently uploaded (WS_SEG_TAB)
  int seg_key[6] = {0, 0, 0, 0, 0, 0};
  unsigned int seg_gen = 0;
  cpx_fov_state* fov = nullptr;
  // re-binning coefficient tables currently uploaded (WS_REBIN): W, out_w, H, out_h
  int rebin_key[4] = {0, 0, 0, 0};
  unsigned int rebin_gen = 0;
  // embedding preprocessing coefficient table currently uploaded (WS_EMBED): S, D
  int embed_key[2] = {0, 0};
  unsigned int embed_gen = 0;
  // k_tex_glcm launch timing (cpx_debug_glcm_timing, bench.py's GLCM roofline): event pairs
  // recorded around each launch while enabled, summed by cpx_debug_glcm_ms
  static constexpr int kGlcmEv = 64;
  int glcm_timing = 0, glcm_nev = 0;
  hipEvent_t glcm_ev[kGlcmEv][2] = {};
  // segmentation post-processing timing (cpx_debug_seg_timing, bench.py's flow-following and
  // flow-error rooflines): per cpx_seg_masks call, events around the follow rounds and around
  // the register flow-error kernels, the per-round item counts (pinned host copy) and steps
  static constexpr int kSegEv = 16;
  int seg_timing = 0, seg_nev = 0;
  hipEvent_t seg_ev[kSegEv][4] = {};
  int* seg_cnt[kSegEv] = {};          // pinned: [B] n_moving, then [rounds][B] items of rounds >= 1
  int seg_cnt_cap[kSegEv] = {};
  int seg_B[kSegEv] = {}, seg_rounds[kSegEv] = {};
  int seg_K[kSegEv][64] = {};         // steps per round
};

void cpx_fov_free(cpx_ctx* ctx);

// workspace slots
enum {
  WS_PARTIALS = 0,   // illum per-block partials
  WS_QC_ROWS = 1,    // row-pass spectrum [plane][H][R+1] complex f64
  WS_QC_RINGS = 2,   // per-column ring partials
  WS_QC_MISC = 3,    // FFT twiddles / plans
  WS_MISC = 4,
  WS_FEAT = 5,
  WS_SEG_PCT = 6,    // percentile histograms + state
  WS_SEG_TAB = 7,    // resize / nearest coefficient tables
  WS_SEG_DYN = 8,    // dPs, p, h, M, M0, seeds, counts
  WS_SEG_OBJ = 9,    // label stats / objects for flow error + fill holes
  WS_SEG_FILL = 10,  // fill-hole owner map
  WS_REBIN = 11,     // LANCZOS re-binning bounds + weights (both axes)
  WS_REBIN_TMP = 12, // re-binning horizontal-pass intermediate (16-bit)
  WS_EMBED = 13,     // embedding preprocessing coefficients + horizontal-pass intermediate
  WS_WATERSHED = 14, // Cells watershed flood levels + tile flags
  WS_MISC2 = 15,     // the second object set's feature workspace (cpx_features_pair)
};

void cpx_set_error(const char* fmt, ...);
int cpx_hip_fail(hipError_t e, const char* what);
// Ensure workspace slot has >= bytes; returns nullptr on failure (error already set).
void* cpx_ws(cpx_ctx* ctx, int slot, size_t bytes);

#define CPX_CHECK_HIP(expr)                                  \
  do {                                                       \
    hipError_t _e = (expr);                                  \
    if (_e != hipSuccess) return cpx_hip_fail(_e, #expr);    \
  } while (0)

#define CPX_CHECK_LAUNCH(what)                                       \
  do {                                                               \
    hipError_t _e = hipGetLastError();                               \
    if (_e != hipSuccess) return cpx_hip_fail(_e, what);             \
  } while (0)

#define CPX_REQUIRE(cond, code, ...)      \
  do {                                    \
    if (!(cond)) {                        \
      cpx_set_error(__VA_ARGS__);         \
      return (code);                      \
    }                                     \
  } while (0)

static inline int cpx_div_up(long long a, long long b) { return (int)((a + b - 1) / b); }

// Wave-64 reductions (gfx950 wavefront = 64 lanes).
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    T o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    T o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

// Work-claim bound of the flow-error kernels: a block claims at most total + 1 items from a
// queue counter that only grows, so a loop past that is broken (e.g. a shared item re-read
// instead of re-claimed, as once happened in a one-wave block) — it ORs kClaimBroken into its
// counter (which also drains the other blocks) and exits; cpx_seg_masks reports it as
// CPX_SEG_ERR_INTERNAL in every FOV's stats instead of a kernel that never ends.
constexpr int kClaimBroken = 1 << 30;

// Flow-error register classes (k_flowerr_reg.hip fe_reg_class): every such mask's bbox is within
// kFeRegMaxLong x kFeRegMaxShort in one orientation or the other (k_seg.hip checks that the fp32
// screening's largest LDS class holds all of them)
constexpr int kFeRegMaxLong = 128, kFeRegMaxShort = 120;

// Objects handled by the LDS fast paths in k_texture.hip; the rest go to the k_features.hip
// fallback kernels (the two predicates must agree between the translation units).
constexpr int kFastShapeWords = 4096;  // 32 KiB of LDS for both masks: 5 blocks per CU (watershed
                                       // Cells reach ~320 x 320 bboxes)
__host__ __device__ inline bool cpx_shape_fits(int bh, int bw) {
  return (bh + 4) * ((bw + 4 + 31) >> 5) <= kFastShapeWords;
}
// Objects the fast paths skip, listed per FOV by k_crop_offsets so the fallback kernels visit
// only them: shape[fov * max_label + i] (i < n_shape[fov]) and tex[...] (i < n_tex[fov]).
struct cpx_fallback_lists {
  int* shape;
  int* tex;
  int* n_shape;
  int* n_tex;
};
// Fallback launcher cpx_features_fast calls on its stream once the lists exist.
typedef int (*cpx_fallback_fn)(cpx_ctx* ctx, hipStream_t stream, const cpx_fallback_lists& fb,
                               void* arg);
// register-resident fp32 flow-error screening (k_flowerr_reg.hip): flags the masks it decides in
// bad[] (and lists the undecided ones in und) before the LDS screening kernels of cpx_seg_masks;
// uses the queue counters ctr[0 .. 2] (zeroed by the caller)
int cpx_flow_error_reg_launch(int n_cu, hipStream_t stream, const int* m0, const float2* dpf, int Dy, int Dx,
                              int B, int ML, const cpx_object* obj, const int* off, int* ctr, double thr,
                              unsigned char* bad, int* und);
int cpx_features_fast(cpx_ctx* ctx, const int32_t* labels_dev, const float* corr_dev, int B, int C,
                      int H, int W, int max_label, int F, const cpx_object* objects_dev,
                      const cpx_fov_objects* hdr_dev, double* feats_dev, cpx_fallback_lists* fb,
                      cpx_fallback_fn fallback, void* fallback_arg);
// Two object sets whose second set's objects lie inside the first's with the same labels (Cells,
// Cytoplasm): the LDS fast paths of both (k_texture.hip); the caller launches both fallbacks.
int cpx_features_pair_fast(cpx_ctx* ctx, const int32_t* labels_dev, const int32_t* tlabels_dev,
                           const float* corr_dev, int B, int C, int H, int W, int max_label, int F,
                           const cpx_object* objects_dev, const cpx_fov_objects* hdr_dev, double* feats_dev,
                           const cpx_object* tobjects_dev, const cpx_fov_objects* thdr_dev, double* tfeats_dev,
                           cpx_fallback_lists* fb, cpx_fallback_lists* tfb);
