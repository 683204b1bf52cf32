// Per-FOV session API (include/cpx.h "per-FOV drop-in boundary"): host planes in, host tables out,
// one context per GPU, mirroring the reference's per-site workers
//   Illumination_QC_mult.process_site (:131-162) with its illum_cache (:180-199),
//   MaxProjection.max_projection (:33-52),
//   Cellpose_GPU_s3fs producer/consumer (:47-232) around the PyTorch CPnet forward.
// Built on the batch kernels of the other translation units (B = 1); every call is enqueued on
// the context's stream, and only the *_qc / *_objects / *_features / read calls synchronise.
#include "cpx_internal.h"
#include <new>
#include <vector>

struct cpx_fov_state {
  // illum cache, one entry per channel (dtype NONE = no correction)
  std::vector<void*> illum;
  std::vector<int> illum_dtype, illum_H, illum_W;
  // current FOV
  int C = 0, Z = 0, H = 0, W = 0;
  int64_t site_id = -1;
  bool have = false;
  uint16_t* raw = nullptr;    // [C][Z][H][W] staging
  uint16_t* zplane = nullptr;  // [C][H][W] z max-projection (owned, allocated for Z > 1)
  uint16_t* plane = nullptr;   // view of the current planes: zplane (Z > 1) or raw (Z == 1)
  float* corr = nullptr;      // [C][H][W]
  cpx_plane_stats* stats = nullptr;
  cpx_qc_result* qc = nullptr;
  size_t raw_cap = 0, zplane_cap = 0, corr_cap = 0;
  int chan_cap = 0;
  // object tables
  int max_label = 0;
  cpx_label_stats* lstats = nullptr;
  cpx_object* objects = nullptr;
  cpx_fov_objects* hdr = nullptr;
  double* feats = nullptr;
  int feat_C = 0;
  float* yf = nullptr;
  size_t yf_cap = 0;
};

void cpx_fov_free(cpx_ctx* ctx) {
  cpx_fov_state* f = ctx->fov;
  if (!f) return;
  for (void* p : f->illum)
    if (p) (void)hipFree(p);
  void* bufs[] = {f->raw, f->zplane, f->corr, f->stats, f->qc,
                  f->lstats, f->objects, f->hdr, f->feats, f->yf};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  delete f;
  ctx->fov = nullptr;
}

namespace {

cpx_fov_state* state(cpx_ctx* ctx) {
  if (!ctx->fov) ctx->fov = new (std::nothrow) cpx_fov_state();
  return ctx->fov;
}

int grow(cpx_ctx* ctx, void** p, size_t* cap, size_t bytes, const char* what) {
  if (*cap >= bytes && *p) return CPX_OK;
  if (*p) {
    CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    CPX_CHECK_HIP(hipFree(*p));
    *p = nullptr;
    *cap = 0;
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return cpx_hip_fail(e, what);
  *cap = bytes;
  return CPX_OK;
}

int ensure_tables(cpx_ctx* ctx, cpx_fov_state* f, int max_label, int C) {
  if (f->max_label >= max_label && f->feat_C >= C && f->objects) return CPX_OK;
  CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  void* old[] = {f->lstats, f->objects, f->hdr, f->feats};
  for (void* p : old)
    if (p) CPX_CHECK_HIP(hipFree(p));
  f->lstats = nullptr;
  f->objects = nullptr;
  f->hdr = nullptr;
  f->feats = nullptr;
  const int ml = std::max(max_label, f->max_label);
  const int fc = std::max(C, f->feat_C);
  const size_t F = (size_t)CPX_N_SHAPE + (size_t)fc * CPX_FEATURES_PER_CHANNEL;
  CPX_CHECK_HIP(hipMalloc((void**)&f->lstats, sizeof(cpx_label_stats) * (ml + 1)));
  CPX_CHECK_HIP(hipMalloc((void**)&f->objects, sizeof(cpx_object) * ml));
  CPX_CHECK_HIP(hipMalloc((void**)&f->hdr, sizeof(cpx_fov_objects)));
  CPX_CHECK_HIP(hipMalloc((void**)&f->feats, sizeof(double) * ml * F));
  f->max_label = ml;
  f->feat_C = fc;
  return CPX_OK;
}

const void* illum_for(cpx_fov_state* f, int c, int* dtype) {
  *dtype = CPX_DTYPE_NONE;
  if (c >= (int)f->illum.size() || !f->illum[c]) return nullptr;
  // Illumination_QC_mult.py:148-153: a shape mismatch falls back to the raw plane
  if (f->illum_H[c] != f->H || f->illum_W[c] != f->W) return nullptr;
  *dtype = f->illum_dtype[c];
  return f->illum[c];
}

}  // namespace

extern "C" {

int cpx_set_illum(cpx_ctx* ctx, int ch, const void* host, int dtype, int H, int W) {
  CPX_REQUIRE(ctx && ch >= 0 && ch < 64, CPX_ERR_ARG, "cpx_set_illum: bad channel");
  cpx_fov_state* f = state(ctx);
  CPX_REQUIRE(f, CPX_ERR_OOM, "cpx_set_illum: host allocation failed");
  if ((int)f->illum.size() <= ch) {
    f->illum.resize(ch + 1, nullptr);
    f->illum_dtype.resize(ch + 1, CPX_DTYPE_NONE);
    f->illum_H.resize(ch + 1, 0);
    f->illum_W.resize(ch + 1, 0);
  }
  if (f->illum[ch]) {
    CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    CPX_CHECK_HIP(hipFree(f->illum[ch]));
    f->illum[ch] = nullptr;
  }
  f->illum_dtype[ch] = CPX_DTYPE_NONE;
  if (!host) return CPX_OK;  // no illumination file for this channel (:195-197)
  CPX_REQUIRE(dtype == CPX_DTYPE_F32 || dtype == CPX_DTYPE_F64, CPX_ERR_ARG,
              "cpx_set_illum: dtype must be CPX_DTYPE_F32 or CPX_DTYPE_F64");
  CPX_REQUIRE(H > 0 && W > 0, CPX_ERR_ARG, "cpx_set_illum: bad shape");
  const size_t bytes = (size_t)H * W * (dtype == CPX_DTYPE_F32 ? 4 : 8);
  CPX_CHECK_HIP(hipMalloc(&f->illum[ch], bytes));
  CPX_CHECK_HIP(hipMemcpy(f->illum[ch], host, bytes, hipMemcpyHostToDevice));
  f->illum_dtype[ch] = dtype;
  f->illum_H[ch] = H;
  f->illum_W[ch] = W;
  return CPX_OK;
}

int cpx_fov_submit(cpx_ctx* ctx, int64_t site_id, const uint16_t* const* planes, int C, int Z,
                   int H, int W) {
  CPX_REQUIRE(ctx && planes, CPX_ERR_ARG, "cpx_fov_submit: null argument");
  CPX_REQUIRE(C > 0 && C <= 64 && Z > 0 && Z <= 256 && H > 0 && W > 0, CPX_ERR_ARG,
              "cpx_fov_submit: bad sizes");
  for (int k = 0; k < C * Z; ++k)
    CPX_REQUIRE(planes[k] != nullptr, CPX_ERR_ARG, "cpx_fov_submit: plane %d is NULL", k);
  cpx_fov_state* f = state(ctx);
  CPX_REQUIRE(f, CPX_ERR_OOM, "cpx_fov_submit: host allocation failed");
  const size_t N = (size_t)H * W;
  int rc;
  if ((rc = grow(ctx, (void**)&f->raw, &f->raw_cap, (size_t)C * Z * N * 2, "fov raw")) != CPX_OK) return rc;
  if (Z > 1) {
    if ((rc = grow(ctx, (void**)&f->zplane, &f->zplane_cap, (size_t)C * N * 2, "fov plane")) != CPX_OK) return rc;
    f->plane = f->zplane;
  } else {
    f->plane = f->raw;  // non-owning view: a single Z plane needs no projection buffer
  }
  if ((rc = grow(ctx, (void**)&f->corr, &f->corr_cap, (size_t)C * N * 4, "fov corr")) != CPX_OK) return rc;
  if (f->chan_cap < C) {
    CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    if (f->stats) CPX_CHECK_HIP(hipFree(f->stats));
    if (f->qc) CPX_CHECK_HIP(hipFree(f->qc));
    CPX_CHECK_HIP(hipMalloc((void**)&f->stats, sizeof(cpx_plane_stats) * C));
    CPX_CHECK_HIP(hipMalloc((void**)&f->qc, sizeof(cpx_qc_result) * C));
    f->chan_cap = C;
  }
  f->C = C;
  f->Z = Z;
  f->H = H;
  f->W = W;
  f->site_id = site_id;
  // planes are plane-major like the reference's chunk order (MaxProjection.py:81-86:
  // chunk.iloc[j + p*C] is channel j of z-plane p); device layout [c][z][N]
  for (int z = 0; z < Z; ++z)
    for (int c = 0; c < C; ++c)
      CPX_CHECK_HIP(hipMemcpyAsync(f->raw + ((size_t)c * Z + z) * N, planes[(size_t)z * C + c],
                                   N * 2, hipMemcpyHostToDevice, ctx->stream));
  if (Z > 1 && (rc = cpx_zmax_u16(ctx, f->raw, C, Z, (int64_t)N, f->plane)) != CPX_OK) return rc;
  for (int c = 0; c < C; ++c) {
    int dt;
    const void* ill = illum_for(f, c, &dt);
    if ((rc = cpx_illum_correct(ctx, f->plane + c * N, ill, dt, 1, 1, H, W, f->corr + c * N,
                                f->stats + c)) != CPX_OK)
      return rc;
  }
  f->have = true;
  return CPX_OK;
}

int cpx_fov_qc(cpx_ctx* ctx, double* slope_out, double* pctmax_out, int* status) {
  CPX_REQUIRE(ctx && ctx->fov && ctx->fov->have, CPX_ERR_STATE, "cpx_fov_qc: no FOV submitted");
  cpx_fov_state* f = ctx->fov;
  const size_t N = (size_t)f->H * f->W;
  int rc;
  for (int c = 0; c < f->C; ++c) {
    int dt;
    const void* ill = illum_for(f, c, &dt);
    if ((rc = cpx_qc_rps(ctx, f->plane + c * N, ill, dt, 1, 1, f->H, f->W, f->stats + c, nullptr,
                         f->qc + c)) != CPX_OK)
      return rc;
  }
  std::vector<cpx_qc_result> q(f->C);
  CPX_CHECK_HIP(hipMemcpyAsync(q.data(), f->qc, sizeof(cpx_qc_result) * f->C,
                               hipMemcpyDeviceToHost, ctx->stream));
  CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  for (int c = 0; c < f->C; ++c) {
    if (slope_out) slope_out[c] = q[c].slope;
    if (pctmax_out) pctmax_out[c] = q[c].pct_max;
    if (status) status[c] = q[c].slope != q[c].slope ? CPX_QC_NAN
                            : (q[c].n_valid <= 2 ? CPX_QC_FLAT : CPX_QC_OK);
  }
  return CPX_OK;
}

int cpx_fov_planes(cpx_ctx* ctx, const float** corr_dev, const uint16_t** plane_dev) {
  CPX_REQUIRE(ctx && ctx->fov && ctx->fov->have, CPX_ERR_STATE, "cpx_fov_planes: no FOV submitted");
  if (corr_dev) *corr_dev = ctx->fov->corr;
  if (plane_dev) *plane_dev = ctx->fov->plane;
  return CPX_OK;
}

int cpx_fov_read_plane(cpx_ctx* ctx, int ch, uint16_t* host) {
  CPX_REQUIRE(ctx && host && ctx->fov && ctx->fov->have, CPX_ERR_STATE,
              "cpx_fov_read_plane: no FOV submitted");
  cpx_fov_state* f = ctx->fov;
  CPX_REQUIRE(ch >= 0 && ch < f->C, CPX_ERR_ARG, "cpx_fov_read_plane: bad channel");
  const size_t N = (size_t)f->H * f->W;
  CPX_CHECK_HIP(hipMemcpyAsync(host, f->plane + ch * N, N * 2, hipMemcpyDeviceToHost, ctx->stream));
  CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return CPX_OK;
}

int cpx_fov_segment_post(cpx_ctx* ctx, const void* net_dev, int layout, const cpx_seg_geom* geom,
                         const float* taper_dev, int niter, double flow_threshold, int min_size,
                         int max_objects, int resample, int32_t* labels_dev,
                         cpx_seg_stats* stats_dev) {
  CPX_REQUIRE(ctx && net_dev && geom && taper_dev && labels_dev && stats_dev, CPX_ERR_ARG,
              "cpx_fov_segment_post: null argument");
  CPX_REQUIRE(ctx->fov && ctx->fov->have, CPX_ERR_STATE, "cpx_fov_segment_post: no FOV submitted");
  cpx_fov_state* f = ctx->fov;
  int rc;
  const size_t need = sizeof(float) * 3 * (size_t)geom->Ly * geom->Lx;
  if ((rc = grow(ctx, (void**)&f->yf, &f->yf_cap, need, "fov flows")) != CPX_OK) return rc;
  if ((rc = cpx_seg_average(ctx, net_dev, layout, 1, 3, geom, taper_dev, f->yf)) != CPX_OK) return rc;
  return cpx_seg_masks(ctx, f->yf, 1, geom, f->H, f->W, niter, flow_threshold, min_size,
                       max_objects, resample, labels_dev, stats_dev);
}

int cpx_fov_object_table(cpx_ctx* ctx, const int32_t* labels_dev, int box, int max_objects,
                    cpx_object* host_out, int* n_out) {
  CPX_REQUIRE(ctx && labels_dev && n_out && max_objects > 0, CPX_ERR_ARG,
              "cpx_fov_object_table: bad argument");
  CPX_REQUIRE(ctx->fov && ctx->fov->have, CPX_ERR_STATE, "cpx_fov_object_table: no FOV submitted");
  cpx_fov_state* f = ctx->fov;
  int rc;
  if ((rc = ensure_tables(ctx, f, max_objects, f->C)) != CPX_OK) return rc;
  if ((rc = cpx_objects(ctx, labels_dev, 1, f->H, f->W, max_objects, box, f->lstats, f->objects,
                        f->hdr)) != CPX_OK)
    return rc;
  cpx_fov_objects h;
  CPX_CHECK_HIP(hipMemcpyAsync(&h, f->hdr, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  *n_out = h.n_objects;
  if (h.overflow) {
    cpx_set_error("cpx_fov_object_table: label %d exceeds max_objects %d", h.max_label, max_objects);
    return CPX_ERR_SHAPE;
  }
  if (host_out && h.n_objects > 0) {
    CPX_CHECK_HIP(hipMemcpy(host_out, f->objects, sizeof(cpx_object) * h.n_objects,
                            hipMemcpyDeviceToHost));
  }
  return CPX_OK;
}

int cpx_fov_features(cpx_ctx* ctx, const int32_t* labels_dev, int max_objects, double* host_out,
                     int* n_out) {
  CPX_REQUIRE(ctx && labels_dev && n_out && max_objects > 0, CPX_ERR_ARG,
              "cpx_fov_features: bad argument");
  CPX_REQUIRE(ctx->fov && ctx->fov->have, CPX_ERR_STATE, "cpx_fov_features: no FOV submitted");
  cpx_fov_state* f = ctx->fov;
  int rc;
  if ((rc = cpx_fov_object_table(ctx, labels_dev, 0, max_objects, nullptr, n_out)) != CPX_OK) return rc;
  if ((rc = cpx_features(ctx, labels_dev, f->corr, 1, f->C, f->H, f->W, max_objects, f->objects,
                         f->hdr, f->feats)) != CPX_OK)
    return rc;
  const size_t F = (size_t)CPX_N_SHAPE + (size_t)f->C * CPX_FEATURES_PER_CHANNEL;
  if (host_out && *n_out > 0) {
    // device rows have the stride of max_objects' table; copy the first n rows (contiguous)
    CPX_CHECK_HIP(hipMemcpyAsync(host_out, f->feats, sizeof(double) * F * (*n_out),
                                 hipMemcpyDeviceToHost, ctx->stream));
  }
  CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return CPX_OK;
}

int cpx_fov_wait(cpx_ctx* ctx) {
  CPX_REQUIRE(ctx, CPX_ERR_ARG, "cpx_fov_wait: null context");
  CPX_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return CPX_OK;
}

}  // extern "C"
