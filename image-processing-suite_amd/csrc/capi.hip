// Context management and error plumbing for libcpx (the C ABI declared in include/cpx.h).
#include "cpx_internal.h"
#include <stdarg.h>
#include <stdio.h>
#include <new>

static thread_local char g_err[1024] = {0};

void cpx_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int cpx_hip_fail(hipError_t e, const char* what) {
  cpx_set_error("HIP error %d (%s) in %s", (int)e, hipGetErrorString(e), what);
  // consume the runtime's sticky last-error so the next launch check does not report it again
  (void)hipGetLastError();
  return e == hipErrorOutOfMemory ? CPX_ERR_OOM : CPX_ERR_HIP;
}

void* cpx_ws(cpx_ctx* ctx, int slot, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (ctx->ws_bytes[slot] >= bytes) return ctx->ws[slot];
  if (ctx->ws[slot]) {
    // the old buffer may still be in use by enqueued work
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->ws[slot]);
    ctx->ws[slot] = nullptr;
    ctx->ws_bytes[slot] = 0;
  }
  size_t want = bytes + bytes / 4;  // headroom so small growth does not re-allocate
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, want);
  if (e != hipSuccess) {
    cpx_hip_fail(e, "workspace hipMalloc");
    return nullptr;
  }
  ctx->ws[slot] = p;
  ctx->ws_bytes[slot] = want;
  ++ctx->ws_gen[slot];  // never 0 after the first allocation: caches start at generation 0
  return p;
}

extern "C" {

int cpx_abi_version(void) { return CPX_ABI_VERSION; }

const char* cpx_last_error(void) { return g_err; }

int cpx_init(int device, cpx_ctx** out) {
  CPX_REQUIRE(out != nullptr, CPX_ERR_ARG, "cpx_init: out is NULL");
  g_err[0] = 0;
  int n = 0;
  CPX_CHECK_HIP(hipGetDeviceCount(&n));
  CPX_REQUIRE(device >= 0 && device < n, CPX_ERR_ARG, "cpx_init: device %d of %d", device, n);
  CPX_CHECK_HIP(hipSetDevice(device));
  cpx_ctx* c = new (std::nothrow) cpx_ctx();
  CPX_REQUIRE(c != nullptr, CPX_ERR_OOM, "cpx_init: host allocation failed");
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return cpx_hip_fail(e, "hipStreamCreate");
  }
  c->stream = c->own_stream;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
  *out = c;
  return CPX_OK;
}

void cpx_destroy(cpx_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  cpx_fov_free(ctx);
  for (int i = 0; i < kWsSlots; ++i)
    if (ctx->ws[i]) (void)hipFree(ctx->ws[i]);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  for (int i = 0; i < cpx_ctx::kGlcmEv; ++i)
    for (int k = 0; k < 2; ++k)
      if (ctx->glcm_ev[i][k]) (void)hipEventDestroy(ctx->glcm_ev[i][k]);
  for (int i = 0; i < cpx_ctx::kSegEv; ++i) {
    for (int k = 0; k < 4; ++k)
      if (ctx->seg_ev[i][k]) (void)hipEventDestroy(ctx->seg_ev[i][k]);
    if (ctx->seg_cnt[i]) (void)hipHostFree(ctx->seg_cnt[i]);
  }
  delete ctx;
}

int cpx_debug_glcm_timing(cpx_ctx* ctx, int enable) {
  CPX_REQUIRE(ctx != nullptr, CPX_ERR_ARG, "cpx_debug_glcm_timing: ctx is NULL");
  if (enable && !ctx->glcm_ev[0][0])
    for (int i = 0; i < cpx_ctx::kGlcmEv; ++i)
      for (int k = 0; k < 2; ++k) CPX_CHECK_HIP(hipEventCreate(&ctx->glcm_ev[i][k]));
  ctx->glcm_timing = enable ? 1 : 0;
  ctx->glcm_nev = 0;
  return CPX_OK;
}

int cpx_debug_glcm_ms(cpx_ctx* ctx, double* ms_out, int* launches_out) {
  CPX_REQUIRE(ctx && ms_out, CPX_ERR_ARG, "cpx_debug_glcm_ms: null argument");
  double ms = 0.0;
  for (int i = 0; i < ctx->glcm_nev; ++i) {
    CPX_CHECK_HIP(hipEventSynchronize(ctx->glcm_ev[i][1]));
    float t = 0.0f;
    CPX_CHECK_HIP(hipEventElapsedTime(&t, ctx->glcm_ev[i][0], ctx->glcm_ev[i][1]));
    ms += t;
  }
  *ms_out = ms;
  if (launches_out) *launches_out = ctx->glcm_nev;
  ctx->glcm_nev = 0;
  return CPX_OK;
}

int cpx_debug_seg_timing(cpx_ctx* ctx, int enable) {
  CPX_REQUIRE(ctx != nullptr, CPX_ERR_ARG, "cpx_debug_seg_timing: ctx is NULL");
  if (enable && !ctx->seg_ev[0][0])
    for (int i = 0; i < cpx_ctx::kSegEv; ++i)
      for (int k = 0; k < 4; ++k) CPX_CHECK_HIP(hipEventCreate(&ctx->seg_ev[i][k]));
  ctx->seg_timing = enable ? 1 : 0;
  ctx->seg_nev = 0;
  return CPX_OK;
}

int cpx_debug_seg_stats(cpx_ctx* ctx, double* follow_ms, double* item_steps, double* fe_reg_ms, int* calls) {
  CPX_REQUIRE(ctx && follow_ms && item_steps && fe_reg_ms, CPX_ERR_ARG, "cpx_debug_seg_stats: null argument");
  double fm = 0.0, st = 0.0, fe = 0.0;
  for (int i = 0; i < ctx->seg_nev; ++i) {
    CPX_CHECK_HIP(hipEventSynchronize(ctx->seg_ev[i][3]));
    float t = 0.0f;
    CPX_CHECK_HIP(hipEventElapsedTime(&t, ctx->seg_ev[i][0], ctx->seg_ev[i][1]));
    fm += t;
    CPX_CHECK_HIP(hipEventElapsedTime(&t, ctx->seg_ev[i][2], ctx->seg_ev[i][3]));
    fe += t;
    const int B = ctx->seg_B[i];
    const int* c = ctx->seg_cnt[i];
    for (int r = 0; r < ctx->seg_rounds[i]; ++r)
      for (int b = 0; b < B; ++b) st += (double)c[r * B + b] * ctx->seg_K[i][r];
  }
  *follow_ms = fm;
  *item_steps = st;
  *fe_reg_ms = fe;
  if (calls) *calls = ctx->seg_nev;
  ctx->seg_nev = 0;
  return CPX_OK;
}

int cpx_set_stream(cpx_ctx* ctx, void* hip_stream) {
  CPX_REQUIRE(ctx != nullptr, CPX_ERR_ARG, "cpx_set_stream: ctx is NULL");
  // NULL selects the legacy default stream (torch's default stream handle is 0)
  ctx->stream = (hipStream_t)hip_stream;
  // the context's own stream is released once the caller supplies one: idle streams still hold
  // one of the process's GPU_MAX_HW_QUEUES hardware-queue slots, and streams beyond that share
  // queues (and serialise)
  if (ctx->own_stream && ctx->stream != ctx->own_stream) {
    (void)hipStreamSynchronize(ctx->own_stream);
    (void)hipStreamDestroy(ctx->own_stream);
    ctx->own_stream = nullptr;
  }
  return CPX_OK;
}

int cpx_sync(cpx_ctx* ctx) {
  CPX_REQUIRE(ctx != nullptr, CPX_ERR_ARG, "cpx_sync: ctx is NULL");
  CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return CPX_OK;
}

int cpx_stream_create_cu_mask(int device, const uint32_t* cu_mask, int n_words, void** out) {
  CPX_REQUIRE(cu_mask && out && n_words > 0, CPX_ERR_ARG, "cpx_stream_create_cu_mask: bad argument");
  int n = 0;
  CPX_CHECK_HIP(hipGetDeviceCount(&n));
  CPX_REQUIRE(device >= 0 && device < n, CPX_ERR_ARG, "cpx_stream_create_cu_mask: device %d of %d", device, n);
  int prev = 0;
  CPX_CHECK_HIP(hipGetDevice(&prev));
  CPX_CHECK_HIP(hipSetDevice(device));
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, cu_mask);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return cpx_hip_fail(e, "hipExtStreamCreateWithCUMask");
  *out = (void*)s;
  return CPX_OK;
}

int cpx_stream_destroy(void* stream) {
  CPX_REQUIRE(stream != nullptr, CPX_ERR_ARG, "cpx_stream_destroy: stream is NULL");
  CPX_CHECK_HIP(hipStreamSynchronize((hipStream_t)stream));
  CPX_CHECK_HIP(hipStreamDestroy((hipStream_t)stream));
  return CPX_OK;
}

}  // extern "C"

extern "C" int cpx_reserve(cpx_ctx* ctx, int max_planes, int H, int W, int max_fovs,
                           int max_label) {
  CPX_REQUIRE(ctx != nullptr, CPX_ERR_ARG, "cpx_reserve: ctx is NULL");
  CPX_REQUIRE(max_planes > 0 && H > 0 && W > 0 && max_fovs >= 0 && max_label >= 0, CPX_ERR_ARG,
              "cpx_reserve: bad sizes");
  // keep in sync with k_illum.hip (64 blocks/plane x 48-B partials) and k_qc.hip
  if (!cpx_ws(ctx, WS_PARTIALS, (size_t)48 * 64 * max_planes)) return CPX_ERR_OOM;
  const int K = std::max(std::min(H, W) / 8, 1);
  const int nr = std::max(K - 2, 1);
  if (!cpx_ws(ctx, WS_QC_ROWS, (size_t)16 * max_planes * H * K)) return CPX_ERR_OOM;
  size_t ring = (size_t)8 * max_planes * K * nr;
  ring = ((ring + 255) / 256) * 256 + (size_t)8 * max_planes + 256;
  if (!cpx_ws(ctx, WS_QC_RINGS, ring)) return CPX_ERR_OOM;
  if (!cpx_ws(ctx, WS_QC_MISC, (size_t)16 * (H + W) + 256)) return CPX_ERR_OOM;
  return CPX_OK;
}
