/*
 * cpx.h — C ABI of the MI355X-native per-field-of-view (FOV) cell-painting hot path.
 *
 * This is the drop-in boundary: a plain C ABI (pointers, sizes, int error codes; no torch or
 * HIP types in any signature) over the hand-written gfx950 HIP kernels in libcpx.so.  The
 * reference (Saguaro-Biosciences/image-processing-suite) has no FFI of its own — its per-FOV
 * workers are Python functions — so each entry point below names the reference function whose
 * per-FOV arithmetic it replaces (file:line in the reference checkout).  The Python host package
 * (`image-processing-suite_amd/cpx`) mirrors those Python signatures on top of this ABI; see
 * INTEGRATION.md for the ctypes binding a maintainer of the reference would add.
 *
 * Conventions
 *   - Every compute entry point only ENQUEUES work on the context's HIP stream (cpx_set_stream)
 *     and returns; device pointers ("dev") must stay valid until cpx_sync() or a later sync on
 *     that stream.  Host pointers ("host") are read/written synchronously.
 *   - Return value 0 = CPX_OK; otherwise a CPX_ERR_* code and a message from cpx_last_error()
 *     (thread-local).  Nothing aborts the process.
 *   - Images are planar: a plane is H*W contiguous pixels, row-major.  A batch of FOVs is
 *     [fov][channel][H][W].  Label images are int32 [fov][H][W], 0 = background.
 *   - One context per GPU per host process (single-threaded use).
 */
#ifndef CPX_H
#define CPX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPX_ABI_VERSION 1

#define CPX_OK 0
#define CPX_ERR_ARG 1     /* bad argument (null pointer, bad size)                    */
#define CPX_ERR_HIP 2     /* HIP runtime error                                        */
#define CPX_ERR_SHAPE 3   /* unsupported shape (e.g. FFT length with a prime > 13)    */
#define CPX_ERR_OOM 4     /* device allocation failed                                 */
#define CPX_ERR_STATE 5   /* context misuse                                           */

#define CPX_DTYPE_NONE 0  /* no flat-field: raw planes are used uncorrected           */
#define CPX_DTYPE_F32 1
#define CPX_DTYPE_F64 2
#define CPX_DTYPE_IMAGE_F64 3 /* the "illum" buffer is the float64 plane itself (raw ignored): QC of
                                 an image corrected on the host, calculate_qc_metrics(image, ch) */

typedef struct cpx_ctx cpx_ctx;

/* Per-plane statistics of the flat-field-corrected plane, all computed on the fp64 quotient
 * raw/illum exactly as Illumination_QC_mult.py:145-150 does (uint16 -> float64 / illum).   */
typedef struct cpx_plane_stats {
  double max_q;       /* np.max of the quotient (NaN if any NaN)                          */
  double min_q;       /* np.min of the quotient                                           */
  double sum_q;       /* fp64 sum (fixed-order), used for the FFT mean removal            */
  double pct_max;     /* ImageQuality_PercentMaximal = 100*count_max/n (:73-95)           */
  int64_t count_max;  /* # pixels equal to max_q                                          */
  int64_t n;          /* pixel count                                                      */
  int32_t has_nan;    /* any NaN                                                          */
  int32_t has_inf;    /* any +-inf                                                        */
  int64_t _pad;
} cpx_plane_stats;    /* 64 bytes */

/* Per-plane QC result (Illumination_QC_mult.py:98-125). */
typedef struct cpx_qc_result {
  double slope;       /* ImageQuality_PowerLogLogSlope (0.0 when <= 2 valid rings)        */
  double pct_max;     /* ImageQuality_PercentMaximal                                      */
  int32_t n_valid;    /* rings with powersum > 0                                          */
  int32_t n_rings;    /* len(labels) = max(0, floor(min(H,W)/8) - 2)                      */
} cpx_qc_result;      /* 24 bytes */

/* Raw per-label accumulators (device), index = label value, 0..max_label.  Exact integers. */
typedef struct cpx_label_stats {
  int64_t area, sum_r, sum_c, sum_rr, sum_cc, sum_rc;
  int32_t rmin, rmax, cmin, cmax; /* inclusive; rmin = INT32_MAX when the label is absent    */
} cpx_label_stats;    /* 64 bytes */

/* One object in ascending-label order (skimage regionprops order; Cellpose_GPU_s3fs.py:149-170). */
typedef struct cpx_object {
  int32_t label;      /* label value                                                      */
  int32_t area;       /* pixel count                                                      */
  int32_t bbox[4];    /* min_row, min_col, max_row (excl), max_col (excl) = regionprops.bbox */
  double centroid_r;  /* regionprops.centroid (float64 mean of pixel coords)              */
  double centroid_c;
  int32_t yc, xc;     /* map(int, centroid): truncation (:160)                            */
  int32_t kept;       /* 1 if the box x box crop lies inside the image (:162)             */
  int32_t cell_idx;   /* 0-based rank among kept objects (Cell_ID suffix, :391-393), else -1 */
} cpx_object;         /* 56 bytes */

/* Per-FOV object-table header (device). */
typedef struct cpx_fov_objects {
  int32_t n_objects;  /* present labels                                                   */
  int32_t n_kept;     /* objects whose crop box is inside the image                       */
  int32_t max_label;  /* largest label value seen                                         */
  int32_t overflow;   /* 1 if a label exceeded the table capacity (objects dropped)       */
} cpx_fov_objects;

/* ---- feature table layout (per object, float64) ---------------------------------------- */
/* Shape block (AreaShape_*, skimage 0.18.3 regionprops definitions). */
#define CPX_SHAPE_AREA 0
#define CPX_SHAPE_PERIMETER 1
#define CPX_SHAPE_CENTER_Y 2
#define CPX_SHAPE_CENTER_X 3
#define CPX_SHAPE_BBOX_AREA 4
#define CPX_SHAPE_EXTENT 5
#define CPX_SHAPE_EQUIV_DIAMETER 6
#define CPX_SHAPE_MAJOR_AXIS 7
#define CPX_SHAPE_MINOR_AXIS 8
#define CPX_SHAPE_ECCENTRICITY 9
#define CPX_SHAPE_ORIENTATION 10
#define CPX_SHAPE_BBOX_MIN_Y 11
#define CPX_SHAPE_BBOX_MIN_X 12
#define CPX_SHAPE_BBOX_MAX_Y 13
#define CPX_SHAPE_BBOX_MAX_X 14
#define CPX_N_SHAPE 15
/* Intensity block, per channel (Intensity_*_<ch>). */
#define CPX_INT_INTEGRATED 0
#define CPX_INT_MEAN 1
#define CPX_INT_STD 2
#define CPX_INT_MIN 3
#define CPX_INT_MAX 4
#define CPX_N_INT 5
/* Texture block, per channel, per angle a in {0, 45, 90, 135} deg, distance 3, 256 levels
 * (skimage greycomatrix/greycoprops on the masked 8-bit bbox crop); index = a*6 + prop.   */
#define CPX_TEX_CONTRAST 0
#define CPX_TEX_DISSIMILARITY 1
#define CPX_TEX_HOMOGENEITY 2
#define CPX_TEX_ASM 3
#define CPX_TEX_ENERGY 4
#define CPX_TEX_CORRELATION 5
#define CPX_N_TEX_PROPS 6
#define CPX_N_ANGLES 4
#define CPX_N_TEX (CPX_N_TEX_PROPS * CPX_N_ANGLES)
#define CPX_TEX_DISTANCE 3
/* Row layout: [shape(15)] + C * [intensity(5) + texture(24)]. */
#define CPX_FEATURES_PER_CHANNEL (CPX_N_INT + CPX_N_TEX)

/* ---- context ------------------------------------------------------------------------ */
int cpx_abi_version(void);
/* Select HIP device `device`, create the context (workspace grows on demand). */
int cpx_init(int device, cpx_ctx** out);
void cpx_destroy(cpx_ctx* ctx);
/* Message of the last error on this thread ("" if none). */
const char* cpx_last_error(void);
/* Enqueue all further work on `hip_stream` (a hipStream_t; NULL = the legacy default stream).
 * Until the first call the context uses a private non-blocking stream, which the first call
 * releases.  The Python host passes torch's current stream so allocations and kernels stay
 * ordered.                                                                                  */
int cpx_set_stream(cpx_ctx* ctx, void* hip_stream);
int cpx_sync(cpx_ctx* ctx);
/* A HIP stream on `device` restricted to the CUs set in cu_mask (n_words 32-bit words, bit i =
 * CU i; hipExtStreamCreateWithCUMask), created by libcpx's own HIP runtime — the one the
 * context's launches use — so the handle is valid for cpx_set_stream.  One pipeline per stream
 * (the host's per-GPU batches in flight; no reference counterpart: the reference
 * runs one consumer per GPU, Cellpose_GPU_s3fs.py:97).  The caller owns the stream and releases
 * it with cpx_stream_destroy (which waits for its work first).                                */
int cpx_stream_create_cu_mask(int device, const uint32_t* cu_mask, int n_words, void** out);
int cpx_stream_destroy(void* stream);
/* Pre-size internal workspaces (so a later hipGraph capture performs no allocation). */
int cpx_reserve(cpx_ctx* ctx, int max_planes, int H, int W, int max_fovs, int max_label);

/* ---- a1 + a4: flat-field correction fused with PercentMaximal --------------------------- *
 * Replaces Illumination_QC_mult.py:145-153 (read, astype(float), img/illum) + :73-95
 * (calculate_saturation_cp_exact) and Cellpose_GPU_s3fs.py:72 (tifffile.imread(p)/illum[n]).
 * raw_dev   : uint16 [n_planes][H][W]; plane p is channel (p % C).
 * illum_dev : [C][H][W] of illum_dtype (CPX_DTYPE_F32/F64), or NULL with CPX_DTYPE_NONE.
 * corr_dev  : float32 [n_planes][H][W] out, the producer-path value raw/illum rounded to fp32
 *             (bit-exact to numpy's uint16/float32 division); may be NULL.
 * stats_dev : cpx_plane_stats [n_planes] out (fp64 quotient statistics, the QC-path values). */
int cpx_illum_correct(cpx_ctx* ctx, const uint16_t* raw_dev, const void* illum_dev,
                      int illum_dtype, int C, int n_planes, int H, int W, float* corr_dev,
                      cpx_plane_stats* stats_dev);

/* ---- a2 + a3: radial power spectrum slope (rps + linregress) ------------------------- *
 * Replaces Illumination_QC_mult.py:31-70 (rps) and :104-116 (linregress of log powersum).
 * Recomputes the fp64 quotient from raw/illum (same inputs as cpx_illum_correct, whose stats
 * must already be enqueued), runs a pruned fp64 2-D DFT (only rings 2..floor(min(H,W)/8)-1 are
 * needed) and bins power by the reference's folded radii.  H and W must factor into
 * {2,3,4,5,7,8,11,13} and be <= 4096.
 * powersum_dev : float64 [n_planes][n_rings] out (may be NULL); qc_dev: cpx_qc_result [n_planes]. */
int cpx_qc_rps(cpx_ctx* ctx, const uint16_t* raw_dev, const void* illum_dev, int illum_dtype,
               int C, int n_planes, int H, int W, const cpx_plane_stats* stats_dev,
               double* powersum_dev, cpx_qc_result* qc_dev);

/* ---- a5: z max-projection ---------------------------------------------------------------- *
 * Replaces MaxProjection.py:45 (np.maximum.reduce over the Z planes of one channel group).
 * src_dev: uint16 [G][Z][N] ; out_dev: uint16 [G][N].                                        */
int cpx_zmax_u16(cpx_ctx* ctx, const uint16_t* src_dev, int G, int Z, int64_t N,
                 uint16_t* out_dev);

/* ---- 8(f) rank 4: image re-binning ------------------------------------------------------- *
 * Replaces Image_re-binning.py:12-22 (PIL Image.resize(target, LANCZOS) of a 16-bit TIFF plane)
 * for G planes: src_dev uint16 [G][H][W] -> dst_dev uint16 [G][out_h][out_w], bit-identical to
 * Pillow's separable LANCZOS-3 resampler (fp64 weights and sums, 16-bit intermediate).       */
int cpx_rebin_u16(cpx_ctx* ctx, const uint16_t* src_dev, int G, int H, int W, int out_h,
                  int out_w, uint16_t* dst_dev);

/* ---- 8(f) rank 1: per-time profiles (Pycyto_pertime.py:29-172) --------------------------- *
 * Per-well aggregation, normalisation, feature-selection statistics and cosine similarities,
 * each bit-identical to the library call the reference makes (oracle/profiles_oracle.py).   */

/* pandas `groupby(keys).mean()` (Pycyto_pertime.py:69-72; pandas group_mean: Kahan sum per
 * group and column in row order, NaN skipped).  values_dev: fp64 rows [n_rows][ld] (first K
 * columns used); order_dev: int32 row indices grouped by group, original order within a group;
 * offs_dev: int32 [G+1] group starts in order_dev.  Optional site scaling
 * (Normalize_CP_ami.py:95-111): where col_scaled_dev[j] != 0, value * row_scale_dev[row] is
 * summed (both NULL: no scaling).  sum/comp/nobs [G][K] carry the state (zero them first), so
 * a table may be streamed in row order over several calls.                                   */
int cpx_group_kahan_accumulate(cpx_ctx* ctx, const double* values_dev, int n_rows, int K,
                               long long ld, const int32_t* order_dev, const int32_t* offs_dev,
                               int G, const double* row_scale_dev, const uint8_t* col_scaled_dev,
                               double* sum_dev, double* comp_dev, int64_t* nobs_dev);
/* pandas `groupby(...).median()` (Normalize_CP_ami.py:113, well_agg_func="median"): same row
 * layout and optional site scaling as cpx_group_kahan_accumulate, out_dev [G][K]; groups of at
 * most 16384 rows (max_group_rows = the largest group).                                       */
int cpx_group_median(cpx_ctx* ctx, const double* values_dev, int n_rows, int K, long long ld,
                     const int32_t* order_dev, const int32_t* offs_dev, int G, int max_group_rows,
                     const double* row_scale_dev, const uint8_t* col_scaled_dev, double* out_dev);
/* out_dev [G][K] = sum / nobs (NaN where nobs == 0).                                          */
int cpx_group_mean_finalize(cpx_ctx* ctx, const double* sum_dev, const int64_t* nobs_dev, int G,
                            int K, double* out_dev);

/* pandas DataFrame.corr(method="pearson") (pycytominer correlation_threshold,
 * Pycyto_pertime.py:93-104): mat_dev column-major [K][N] (N <= 8192), out_dev [K][K].         */
int cpx_nancorr(cpx_ctx* ctx, const double* mat_dev, int N, int K, double* out_dev);

/* pycytominer RobustMAD.fit (normalize(method="mad_robustize"), Pycyto_pertime.py:83-88):
 * per column of mat_dev (column-major [K][N]) over the rows fit_rows_dev[n_fit] (n_fit <= 4096):
 * med = median of the non-NaN values, mad = median(|x - med|) / scale (scale = 1/1.4826).     */
int cpx_robust_mad(cpx_ctx* ctx, const double* mat_dev, int N, int K, const int32_t* fit_rows_dev,
                   int n_fit, double scale, double* med_dev, double* mad_dev);

/* RobustMAD.transform (Normalize_CP_ami.py:119-124, Pycyto_pertime.py:83-88), column-major:
 * z = (x - med[j]) / (mad[j] + eps); with double_sigmoid != 0 also Pycyto_pertime.py:13-16,
 * 89-91: out = |(z/alpha)^3 / sqrt(1 + (z/alpha)^6)|, powers correctly rounded.              */
int cpx_mad_transform(cpx_ctx* ctx, const double* mat_dev, int N, int K, const double* med_dev,
                      const double* mad_dev, double eps, int double_sigmoid, double alpha,
                      double* out_dev);

/* feature_select statistics (variance_threshold, drop_na_columns, drop_outliers) per column of
 * mat_dev (column-major [K][N], N <= 4096).                                                  */
typedef struct cpx_column_stat {
  int64_t na_count;      /* NaN rows */
  int64_t nunique;       /* distinct non-NaN values */
  int64_t top_count;     /* largest value count */
  int64_t second_count;  /* second largest value count (0 if one distinct value) */
  double max, min;       /* over non-NaN values (NaN if none) */
} cpx_column_stat;
int cpx_column_stats(cpx_ctx* ctx, const double* mat_dev, int N, int K, cpx_column_stat* stats_dev);

/* sklearn cosine_similarity within groups of consecutive rows, upper triangle only
 * (Pycyto_pertime.py:115-140; NaN read as 0 = fillna(0)).  x_dev row-major [N][F]; offs_dev
 * int32 [G+1] row starts; pair_offs_dev int64 [G+1] output starts (group g has n(n-1)/2 pairs in
 * np.triu_indices(n, 1) order); norms_dev [N] scratch; out_dev [n_pairs].                     */
int cpx_cosine_groups(cpx_ctx* ctx, const double* x_dev, int N, int F, const int32_t* offs_dev,
                      const int64_t* pair_offs_dev, int G, long long n_pairs, double* norms_dev,
                      double* out_dev);

/* ---- a7: object table (regionprops order, int centroids, edge filter, kept index) ------- *
 * Replaces Cellpose_GPU_s3fs.py:149-163 (regionprops(masks), map(int, centroid), box test).
 * labels_dev : int32 [B][H][W].  max_label: capacity per FOV (labels above it are flagged in
 * overflow and ignored).  stats_dev: cpx_label_stats [B][max_label+1] (workspace, out).
 * objects_dev: cpx_object [B][max_label] out (first n_objects rows valid per FOV).
 * hdr_dev    : cpx_fov_objects [B] out.                                                    */
int cpx_objects(cpx_ctx* ctx, const int32_t* labels_dev, int B, int H, int W, int max_label,
                int box, cpx_label_stats* stats_dev, cpx_object* objects_dev,
                cpx_fov_objects* hdr_dev);

/* ---- a7 crops + a9 scale_to_8bit ------------------------------------------------------------ *
 * Replaces Cellpose_GPU_s3fs.py:164-170 (img[y1:y2,x1:x2,:] * (mask==label)) and :34-43 /
 * :178-181 (scale_to_8bit per crop-channel).  For every kept object of every FOV, writes
 * crops_dev [B][max_crops][box][box][C] float32 (HWC, as the reference's crop) and
 * crops8_dev [B][max_crops][C][box][box] uint8; either may be NULL (not both).  Slot = cell_idx; cell_idx >= max_crops is
 * skipped.  corr_dev is planar [B][C][H][W].                                                    */
int cpx_crops(cpx_ctx* ctx, const int32_t* labels_dev, const float* corr_dev, int B, int C,
              int H, int W, int max_label, const cpx_object* objects_dev,
              const cpx_fov_objects* hdr_dev, int box, int max_crops, float* crops_dev,
              uint8_t* crops8_dev);

/* ---- a8: per-object features (AreaShape / Intensity / Texture) --------------------------- *
 * Replaces the CellProfiler measurement step launched by Feature_extraction_opt.py:164-167
 * (pipeline not in the reference; definitions pinned to skimage 0.18.3).
 * feats_dev: float64 [B][max_label][CPX_N_SHAPE + C*CPX_FEATURES_PER_CHANNEL]; row k is the
 * k-th object of the FOV's table (rows >= n_objects untouched).                               */
int cpx_features(cpx_ctx* ctx, const int32_t* labels_dev, const float* corr_dev, int B, int C,
                 int H, int W, int max_label, const cpx_object* objects_dev,
                 const cpx_fov_objects* hdr_dev, double* feats_dev);
/* cpx_features of the Cells and the Cytoplasm object sets in one call (same outputs as two
 * cpx_features calls): a Cytoplasm object with the same label and bbox as its Cells object is
 * measured from the same reads of the channel planes.  cyto_dev must be the Cytoplasm of
 * cells_dev (every Cytoplasm pixel carries its cell's label, as cpx_watershed_cells /
 * cpx_expand_labels produce it).                                                              */
int cpx_features_pair(cpx_ctx* ctx, const int32_t* cells_dev, const int32_t* cyto_dev,
                      const float* corr_dev, int B, int C, int H, int W, int max_label,
                      const cpx_object* cells_objects_dev, const cpx_fov_objects* cells_hdr_dev,
                      double* cells_feats_dev, const cpx_object* cyto_objects_dev,
                      const cpx_fov_objects* cyto_hdr_dev, double* cyto_feats_dev);

/* ---- secondary objects for the Cells / Cytoplasm tables (Pycyto_pertime.py:46-49) -------- *
 * cells = skimage.segmentation.expand_labels(nuclei, distance) (0.18.3: nearest label pixel by
 * scipy's exact Euclidean feature transform, kept where the distance <= `distance`);
 * cyto = cells where nuclei == 0 (Cytoplasm shares the Cells/Nuclei ObjectNumber).  Either
 * output may be NULL.  All int32 [B][H][W]; label values below 2^23.                        */
int cpx_expand_labels(cpx_ctx* ctx, const int32_t* nuclei_dev, int B, int H, int W, int distance,
                      int32_t* cells_dev, int32_t* cyto_dev);

/* Cells by marker watershed (skimage 0.18.3 segmentation.watershed,
 * skimage/segmentation/_watershed.py:94, connectivity 1) from the Nuclei, bit-identical to
 *   watershed(key, markers=nuclei, mask=expand_labels(nuclei, distance) > 0)
 * with the stated elevation key(p) = (65535 - q16(corr[cell_channel](p))) * 2^23 + (y*W + x),
 * q16(v) = 65535 if !(v < 65535) else max(0, trunc(v))  (inverted 16-bit cell channel, raster
 * index tie-break).  cyto = cells where nuclei == 0.  corr_dev: fp32 [B][C][H][W].
 * The flood levels converge in up to `relax_rounds` tile rounds and the labels in up to
 * `label_rounds` pointer-jumping rounds, without host synchronisation; status_dev[b *
 * status_stride] (int32) receives 100 * (relax rounds used) + (jump rounds used), or -1 when the
 * rounds enqueued did not reach the fixed point (labels then invalid; the host must raise).
 * H * W <= 2^23.                                                                               */
int cpx_watershed_cells(cpx_ctx* ctx, const int32_t* nuclei_dev, const float* corr_dev, int B, int C,
                        int cell_channel, int H, int W, int distance, int relax_rounds,
                        int label_rounds, int32_t* cells_dev, int32_t* cyto_dev, int32_t* status_dev,
                        int status_stride);

/* ---- a6: segmentation (Cellpose <= v3 evaluation, restated) -- *
 * Replaces the work inside cell_model.eval(image_4ch, diameter=100) (Cellpose_GPU_s3fs.py:143)
 * except the CPnet U-Net forward itself, which runs in PyTorch-ROCm between cpx_seg_tiles and
 * cpx_seg_average.                                                                           */
#define CPX_SEG_MAX_TILES_AXIS 16
typedef struct cpx_seg_geom {
  int32_t Ly, Lx;     /* network-resolution image (int(H * diam_mean / diameter))             */
  int32_t py0, px0;   /* zero padding before the image (transforms.pad_image_ND)              */
  int32_t Lyp, Lxp;   /* padded size                                                         */
  int32_t by, bx;     /* tile size (224)                                                     */
  int32_t ny, nx;     /* tiles per axis (transforms.make_tiles, overlap 0.1)                  */
  int32_t ys[CPX_SEG_MAX_TILES_AXIS], xs[CPX_SEG_MAX_TILES_AXIS]; /* tile origins             */
} cpx_seg_geom;

typedef struct cpx_seg_stats {
  int32_t n_moving;   /* pixels that follow the flow (|dY/5| > 1e-3 inside cellprob > 0)       */
  int32_t n_seeds;    /* histogram maxima (h > 10)                                            */
  int32_t n_masks;    /* labels after get_masks (big masks removed, renumbered)               */
  int32_t n_bad_flow; /* masks removed by the flow-error test                                 */
  int32_t n_final;    /* labels after fill_holes_and_remove_small_masks                       */
  int32_t overflow;   /* CPX_SEG_OVF_* bits; 0 = the labels are complete                       */
  int32_t cells_status; /* written by cpx_watershed_cells when pointed here (else untouched)     */
  int32_t n_seeds_found; /* histogram maxima found (n_seeds is min(found, max_objects))          */
  int32_t n_fill_partial; /* masks partly inside earlier holes (CPX_SEG_OVF_FILL_PARTIAL, below)   */
  int32_t _reserved[3];
} cpx_seg_stats;      /* 48 bytes */

/* cpx_seg_stats.overflow bits.  The reference (Cellpose get_masks / fill_holes, regionprops,
 * Cellpose_GPU_s3fs.py:143-170) has no capacity limit; libcpx's per-FOV tables hold max_objects:
 *   CPX_SEG_OVF_SEEDS  more seeds than max_objects were found: only the first max_objects (raster
 *                      order) were expanded, so masks are missing; re-run the FOV with
 *                      max_objects >= n_seeds_found (masks <= seeds: that run cannot overflow).
 *   CPX_SEG_OVF_FILL_PARTIAL informational, the labels are complete: a mask lay partly (not
 *                      wholly) inside an earlier mask's filled holes (disconnected or diagonal-
 *                      touching masks), where the parallel fill is not the reference's
 *                      order-dependent loop, so this FOV's fill ran as that sequential loop on
 *                      the GPU (n_fill_partial = such masks).
 *   CPX_SEG_ERR_INTERNAL a flow-error work loop reached its claim bound (cannot happen in a correct
 *                      build; the labels are invalid and the host must raise).
 * Fill-holes has no size limit (masks whose bbox exceeds the LDS bitmasks use global memory). */
#define CPX_SEG_OVF_SEEDS 1
#define CPX_SEG_OVF_FILL_PARTIAL 2
#define CPX_SEG_ERR_INTERNAL 8

#define CPX_TILE_F32_NCHW 0  /* tiles/net output as float32 [n][c][by][bx]                   */
#define CPX_TILE_BF16_NHWC 1 /* tiles/net output as bfloat16 [n][by][bx][c] (channels_last)  */
#define CPX_TILE_F32_NHWC 2  /* tiles/net output as float32 [n][by][bx][c] (channels_last)    */

/* normalize99 statistics: pct_dev float64 [B][nchan][2] = (p1, p99) of channels 0..nchan-1 of
 * each FOV (exact order statistics of the fp32 corrected planes, linear interpolation).       */
int cpx_seg_percentiles(cpx_ctx* ctx, const float* corr_dev, int B, int C, int H, int W,
                        int nchan, double* pct_dev);
/* Normalise, bilinearly resize to (Ly, Lx), zero-pad and cut the network tiles:
 * tiles_dev: [B * ny * nx] tiles of nchan channels in `layout`.                               */
int cpx_seg_tiles(cpx_ctx* ctx, const float* corr_dev, int B, int C, int H, int W, int nchan,
                  const double* pct_dev, const cpx_seg_geom* geom, int layout, void* tiles_dev);
/* Taper-weighted average of the network outputs (transforms.average_tiles), pad cropped:
 * taper_dev float32 [by][bx] (transforms._taper_mask, computed by the host with numpy);
 * yf_dev float32 [B][nout][Ly][Lx] (dy, dx, cellprob).                                       */
int cpx_seg_average(cpx_ctx* ctx, const void* net_dev, int layout, int B, int nout,
                    const cpx_seg_geom* geom, const float* taper_dev, float* yf_dev);
/* dynamics.compute_masks on the averaged network output yf_dev (Ly x Lx): follow_flows
 * (niter Euler steps, CPU map_coordinates arithmetic), get_masks, flow-error filter,
 * fill_holes_and_remove_small_masks.  resample = 1 (CellposeModel.eval's default, the
 * reference call Cellpose_GPU_s3fs.py:143): the flows are first resized to H x W
 * (transforms.resize_image, cv2 INTER_LINEAR) and everything runs at full resolution, with
 * niter = uint32(200 / rescale) (1176 for nuclei at diameter 100; the host passes it).
 * resample = 0: dynamics at Ly x Lx, masks nearest-resized to H x W (Cellpose's resize=).
 * labels_dev int32 [B][H][W]; stats_dev cpx_seg_stats [B].  max_objects bounds the seeds and
 * hence the labels per FOV (CPX_SEG_OVF_SEEDS when a FOV has more: re-run it with more).        */
int cpx_seg_masks(cpx_ctx* ctx, const float* yf_dev, int B, const cpx_seg_geom* geom, int H,
                  int W, int niter, double flow_threshold, int min_size, int max_objects,
                  int resample, int32_t* labels_dev, cpx_seg_stats* stats_dev);

/* ---- f3: embedding preprocessing ------------------------------------ *
 * Replaces Cellpose_GPU_s3fs.py:177-187 between scale_to_8bit and the EfficientNetV2-L forward:
 * PIL L -> RGB, TimmWrapperImageProcessor (Image.resize(D, BICUBIC) with Pillow's 8-bit fixed
 * point resampler, CenterCrop, ToTensor /255, Normalize (x - mean) / std), fp16 autocast.
 * crops8_dev: uint8 S x S images; image i of the batch is crops8_dev + index_dev[i] * S * S
 * (index_dev int64 [N], device).  out_dev: fp16 [N][3][D][D] (R = G = B).                  */
int cpx_embed_preprocess(cpx_ctx* ctx, const uint8_t* crops8_dev, const int64_t* index_dev, int N,
                         int S, int D, float mean, float stdv, void* out_dev);

/* ---- f3: the EfficientNetV2-L forward (Cellpose_GPU_s3fs.py:109-110,184-194: timm
 * tf_efficientnetv2_l, fp16 autocast, pooler_output) -------------------------------------- *
 * NHWC fp16 activations, fp16 MFMA products with fp32 accumulation; BatchNorm folded to fp32
 * scale/shift [C]; TF 'same' padding (output ceil(i / stride), pad_lo = total / 2).
 * cpx_effnet_stem: x = cpx_embed_preprocess output fp16 [N][3][H][W]; w fp32 [32][3][3][3];
 *   out fp16 [N][ceil(H/2)][ceil(W/2)][32] = silu(scale conv + shift).
 * cpx_effnet_conv: ks 1 or 3, stride 1 or 2, cin % 32 == 0; w fp16 [cout][ks*ks][cin];
 *   out [N][Ho][Wo][cout] = (act ? silu : id)(scale conv(in, w * gate) + shift) + res, with the
 *   optional squeeze-excite gate fp32 [N][cin] and residual fp16 [N][Ho][Wo][cout] (stride 1).
 * cpx_effnet_dw: depthwise 3x3, C % 64 == 0, w fp32 [C][9]; out = silu(scale dw + shift);
 *   partial fp32 [N][cpx_effnet_dw_blocks(H, W, stride)][C] = per-block channel sums of out.
 * cpx_effnet_se: gate fp32 [N][C] = sigmoid(be + we [C][rd] . silu(br + wr [rd][C] . mean)),
 *   mean = sum of partial / HW.
 * cpx_effnet_pool: out fp32 [N][C] = mean over HW of in fp16 [N][HW][C] (pooler_output).   */
int cpx_effnet_stem(cpx_ctx* ctx, const void* x, int N, int H, int W, const float* w,
                    const float* scale, const float* shift, void* out);
int cpx_effnet_conv(cpx_ctx* ctx, const void* in, int N, int H, int W, int cin, int cout, int ks,
                    int stride, const void* w, const float* scale, const float* shift, int act,
                    const void* res, const float* gate, void* out);
int cpx_effnet_dw(cpx_ctx* ctx, const void* in, int N, int H, int W, int C, int stride,
                  const float* w, const float* scale, const float* shift, void* out, float* partial);
int cpx_effnet_dw_blocks(int H, int W, int stride);
int cpx_effnet_se(cpx_ctx* ctx, const float* partial, int N, int pblks, int HW, int C, int rd,
                  const float* wr, const float* br, const float* we, const float* be, float* gate);
int cpx_effnet_pool(cpx_ctx* ctx, const void* in, int N, int HW, int C, float* out);

/* ---- a4 CPnet glue (bf16 NHWC activations around MIOpen convolutions) ----------------------
 * Cellpose resnet_torch.CPnet forward (used at Cellpose_GPU_s3fs.py:108-110 through
 * models.CellposeModel.eval): every batchconv is BatchNorm -> ReLU -> Conv2d, blocks add
 * residuals and (up path) a per-image style bias before the BatchNorm.  cpx_cpnet_epilogue
 * fuses everything between two convolutions into one pass over [N, Hh, Ww, Cn] bf16:
 *   t = conv + bias[c] + res          (conv, bias, res optional; res_up: res is [N,Hh/2,Ww/2,Cn]
 *                                      read nearest-upsampled)            -> y_out (optional)
 *   z = relu?(scale[c] * (t + style[n*Cn+c]) + shift[c])  (style, scale/shift optional)
 *                                                                        -> z_out (optional;
 *                                      z_up: written 2x nearest-upsampled, [N,2Hh,2Ww,Cn])
 * cpx_cpnet_pool: 2x2/2 max-pool of [N,2Hh,2Ww,Cn] -> x_out [N,Hh,Ww,Cn] and
 *   z_out = relu?(scale[c] * x + shift[c]).  fp32 arithmetic, bf16 (RNE) stores.            */
int cpx_cpnet_epilogue(cpx_ctx* ctx, const void* conv, const float* bias, const void* res,
                       int res_up, const float* style, const float* scale, const float* shift,
                       int relu, int N, int Hh, int Ww, int Cn, void* y_out, void* z_out,
                       int z_up);
int cpx_cpnet_pool(cpx_ctx* ctx, const void* in, const float* scale, const float* shift,
                   int relu, int N, int Hh, int Ww, int Cn, void* x_out, void* z_out);
/* 3x3 / pad 1 convolution of in [N,H,W,cin] bf16 (MFMA implicit GEMM) with the epilogue of
 * cpx_cpnet_epilogue fused (the raw convolution is never stored).  cin, cout in {32, 64, 128,
 * 256} (pairs used by CPnet).  wpk = weights packed by cpx_cpnet_conv_cfg's (bn, ck):
 * [cout/bn][cin/ck][ky][kx][bn][ck] bf16.                                                    */
int cpx_cpnet_conv_cfg(int cin, int cout, int* bn, int* ck);
int cpx_cpnet_conv3x3(cpx_ctx* ctx, const void* in, int N, int H, int W, int cin, int cout,
                      const void* wpk, const float* bias, const void* res, int res_up,
                      const float* style, const float* scale, const float* shift, int relu,
                      void* y_out, void* z_out, int z_up);
/* cpx_cpnet_conv3x3 (cout = 32) whose BatchNorm+ReLU output z feeds the CPnet output 1x1
 * convolution directly (Cellpose resnet_torch.CPnet.output; z is never stored):
 *   head_out [N,H,W,n_head] bf16 = head_b[j] + sum_c head_w[j][c] * bf16(z[c]),  n_head <= 4. */
int cpx_cpnet_conv3x3_head(cpx_ctx* ctx, const void* in, int N, int H, int W, int cin, int cout,
                           const void* wpk, const float* bias, const void* res, int res_up,
                           const float* style, const float* scale, const float* shift, int relu,
                           void* y_out, const float* head_w, const float* head_b, int n_head,
                           void* head_out);
/* CPnet stem (first down block's entry) on x [N,H,W,2] bf16, one pass:
 *   z0 = bf16(relu(scale0 * x + shift0))        (input BatchNorm + ReLU, zero-padded conv input)
 *   z_out [N,H,W,32] = relu(scale1 * (conv3x3(z0, w0) + bias0) + shift1)
 *   p_out [N,H,W,32] = conv1x1(x, wp)           (block projection, BatchNorm folded into wp)
 * w0 fp32 [32][2][3][3], wp fp32 [32][2]; fp32 arithmetic, bf16 (RNE) stores.                */
int cpx_cpnet_stem(cpx_ctx* ctx, const void* x, int N, int H, int W, const float* scale0,
                   const float* shift0, const float* w0, const float* bias0, const float* scale1,
                   const float* shift1, const float* wp, void* p_out, void* z_out);

/* ---- a6 CPnet at the reference's precision (split fp16, "f16x3") ---------------------------
 * The fp32 U-Net the reference runs (Cellpose_GPU_s3fs.py:108,143: CellposeModel without half
 * precision) on the fp16 matrix cores.  Activations are "split" tensors: NHWC, channels in slabs
 * of 16, per pixel and slab 16 f16 hi halves then 16 f16 lo halves (4 bytes per channel), value
 * = hi + lo * 2^-11 (hi = f16(a), lo = f16((a - hi) * 2^11)); weights are packed split by the
 * host as [cout/bm][cin/16][ky][kx][bm][hi|lo][16] f16 (bm from cpx_cpnet_x3_cfg).  Every
 * product is formed as wh*xh + (wh*xl + wl*xh) * 2^-11 in fp32 (three v_mfma_f32_32x32x16_f16
 * per 16 channels), ~2^-22 relative per operand: the fp32 network to its rounding noise.
 * ovf (device int [N], optional): ovf[n] is OR-ed with 1 when an activation of image n that is
 * not below 65504 in magnitude would be stored (the caller re-runs those images in fp32).
 * cpx_cpnet_x3_conv: ks = 3 (pad 1) or 1 (the block projections); the epilogue of
 * cpx_cpnet_conv3x3 (bias, res [split, res_up], y_out, style [N][style_stride], scale/shift,
 * relu, z_out [z_up]) or, for the last 3x3 convolution (cout 32), the output head:
 * head_out fp32 [N][H][W][n_head] = head_b + head_w [n_head][32] . z (z in fp32).  N, H, W are
 * the output sizes; in_up = 1 reads `in` as the [N][H/2][W/2][cin] tensor, 2x nearest-upsampled
 * on the fly (the up path's nn.Upsample(scale_factor=2) is never materialised).              */
int cpx_cpnet_x3_cfg(int ks, int cin, int cout, int variant, int* bm);
int cpx_cpnet_x3_conv(cpx_ctx* ctx, int ks, int variant, const void* in, int in_up, int N, int H,
                      int W, int cin, int cout, const void* wpk, const float* bias, const void* res,
                      int res_up, const float* style, int style_stride, const float* scale,
                      const float* shift, int relu, void* y_out, void* z_out, int z_up,
                      const float* head_w, const float* head_b, int n_head, float* head_out,
                      int* ovf);
/* 3x3 convolution (pad 1) with its block's residual projection folded in: the sums are
 * conv3x3(in, wpk) + conv1x1(in2, wpk2) with in2 [N][H][W][cin2] split (the block input the
 * 1x1 projection reads; wpk2 packed like a 1x1 conv with the 3x3's bm), then the epilogue of
 * cpx_cpnet_x3_conv without a residual tensor (bias = conv bias + projection bias).  Replaces a
 * cpx_cpnet_x3_conv(ks = 1) pass + the residual read of the 3x3 convolution.                 */
int cpx_cpnet_x3_conv_proj(cpx_ctx* ctx, int variant, const void* in, int N, int H, int W, int cin,
                           int cout, const void* wpk, const void* in2, int cin2, const void* wpk2,
                           const float* bias, const float* style, int style_stride, const float* scale,
                           const float* shift, int relu, void* y_out, void* z_out, int z_up, int* ovf);
/* 3x3 convolution with residual whose y tile is also 2x2/2 max-pooled in the epilogue (a down
 * block's last convolution, fused with the next block's entry): y_out = conv(in) + bias + res,
 * pool_x [N][H/2][W/2][cout] = max_pool2d(y) (the maximum's own hi/lo pair, first maximum) and
 * pool_z = split(relu(pool_scale pool_x + pool_shift)) — cpx_cpnet_x3_conv followed by
 * cpx_cpnet_x3_pool, bit for bit, without reading y back.  H and W even.                      */
int cpx_cpnet_x3_conv_pool(cpx_ctx* ctx, int variant, const void* in, int N, int H, int W, int cin,
                           int cout, const void* wpk, const float* bias, const void* res, void* y_out,
                           void* pool_x, void* pool_z, const float* pool_scale, const float* pool_shift,
                           int* ovf);
/* stem on the fp32 network input x [N][H][W][2] (CPX_TILE_F32_NHWC tiles): z0 = relu(scale0 x
 * + shift0), z_out = relu(scale1 (conv3x3(z0, w0) + bias0) + shift1), p_out = conv1x1(x, wp),
 * fp32 arithmetic, split stores (32 channels).                                               */
int cpx_cpnet_x3_stem(cpx_ctx* ctx, const float* x, int N, int H, int W, const float* scale0,
                      const float* shift0, const float* w0, const float* bias0, const float* scale1,
                      const float* shift1, const float* wp, void* p_out, void* z_out, int* ovf);
/* 2x2/2 max-pool of split [N][2Hh][2Ww][Cn] -> x_out (exact) and z_out = relu?(scale x + shift). */
int cpx_cpnet_x3_pool(cpx_ctx* ctx, const void* in, const float* scale, const float* shift,
                      int relu, int N, int Hh, int Ww, int Cn, void* x_out, void* z_out, int* ovf);
/* head_out [N][H][W][nout] fp32 of every image n with ovf[n] != 0 := flows 0, last channel
 * (cell probability) -1: an image whose activations overflowed yields no masks (its FOV is
 * re-run in fp32 by the host) instead of post-processing saturated values.                    */
int cpx_cpnet_x3_mask_overflow(cpx_ctx* ctx, float* out, int N, int H, int W, int nout, const int* ovf);
/* style vector of split x [N][H][W][C] (mean over pixels, L2-normalised; CPnet.forward) and the
 * up path's Linear layers: out [N][J] = lin_b + lin_w [J][C] . style.                          */
int cpx_cpnet_x3_style(cpx_ctx* ctx, const void* x, int N, int H, int W, int C, const float* lin_w,
                       const float* lin_b, int J, float* out);

/* ==== per-FOV drop-in boundary ============================================
 * Host planes in, host tables out, one context per GPU and one FOV at a time — the shape of the
 * reference's per-site workers, for callers that are not PyTorch programs.  Everything is
 * enqueued on the context's stream; cpx_fov_qc / _object_table / _features / _read_plane return
 * results (they synchronise), cpx_fov_wait drains the stream.                                */
#define CPX_QC_OK 0    /* slope from linregress                                               */
#define CPX_QC_FLAT 1  /* <= 2 rings with power > 0: slope reported as 0.0 (:109-114)         */
#define CPX_QC_NAN 2   /* the reference's exception path: slope NaN (:115-116)                */

/* Illumination cache entry for channel `ch` (Illumination_QC_mult.py:180-199 illum_cache /
 * Cellpose_GPU_s3fs.py:56-60): host [H][W] of dtype CPX_DTYPE_F32 / _F64, copied to the device.
 * host == NULL: no file for this channel, raw planes are used (:195-197).  An illum whose shape
 * differs from a FOV's planes is skipped for that FOV (:148-153).                            */
int cpx_set_illum(cpx_ctx* ctx, int ch, const void* host, int dtype, int H, int W);
/* Submit one FOV: planes[z*C + c] are host uint16 [H][W] (the plane-major chunk order of
 * MaxProjection.py:81-86; Z = 1 for a plain site).  H2D, z max-projection (Z > 1,
 * MaxProjection.py:45), flat-field division + PercentMaximal statistics per channel
 * (Illumination_QC_mult.py:145-153 / Cellpose_GPU_s3fs.py:72).  The host planes must stay
 * valid until the next synchronising call.                                                  */
int cpx_fov_submit(cpx_ctx* ctx, int64_t site_id, const uint16_t* const* planes, int C, int Z,
                   int H, int W);
/* a2-a4 for the submitted FOV (calculate_qc_metrics, Illumination_QC_mult.py:98-125):
 * slope_out / pctmax_out / status: [C] (any may be NULL).                                    */
int cpx_fov_qc(cpx_ctx* ctx, double* slope_out, double* pctmax_out, int* status);
/* Device views of the submitted FOV: corrected float32 [C][H][W] and the (z-max'd) uint16
 * planes [C][H][W] (valid until the next cpx_fov_submit).                                     */
int cpx_fov_planes(cpx_ctx* ctx, const float** corr_dev, const uint16_t** plane_dev);
/* Copy channel `ch` of the (z-max'd) uint16 planes to host [H][W] (MaxProjection output).   */
int cpx_fov_read_plane(cpx_ctx* ctx, int ch, uint16_t* host);
/* a6 post-processing of one FOV from the CPnet output tiles (net_dev in `layout`, geom as for
 * cpx_seg_average): tile average, then cpx_seg_masks (resample as there)
 * (Cellpose_GPU_s3fs.py:108,143-147, models.CellposeModel.eval).  labels_dev int32 [H][W].  */
int cpx_fov_segment_post(cpx_ctx* ctx, const void* net_dev, int layout, const cpx_seg_geom* geom,
                         const float* taper_dev, int niter, double flow_threshold, int min_size,
                         int max_objects, int resample, int32_t* labels_dev,
                         cpx_seg_stats* stats_dev);
/* a7 object table of a label image (int32 [H][W], device) for the submitted FOV's shape:
 * regionprops order, int centroids, `box` edge filter, kept index (Cellpose_GPU_s3fs.py:
 * 149-163).  host_out: cpx_object [max_objects] (may be NULL, then only *n_out is set).
 * A label above max_objects is an error (CPX_ERR_SHAPE) — size max_objects >= max label.   */
int cpx_fov_object_table(cpx_ctx* ctx, const int32_t* labels_dev, int box, int max_objects,
                    cpx_object* host_out, int* n_out);
/* a8 feature rows of every object of labels_dev over the submitted FOV's corrected planes:
 * host_out float64 [n][CPX_N_SHAPE + C*CPX_FEATURES_PER_CHANNEL] (row k = k-th object in
 * ascending label order; the CellProfiler step of Feature_extraction_opt.py:164-167).       */
int cpx_fov_features(cpx_ctx* ctx, const int32_t* labels_dev, int max_objects, double* host_out,
                     int* n_out);
int cpx_fov_wait(cpx_ctx* ctx);

/* ---- profiling: device time of the k_tex_glcm launches (bench.py's GLCM LDS roofline) ----- *
 * While enabled, every cpx_features / cpx_features_pair call records a HIP event pair around
 * its GLCM launch (up to 64 between reads); cpx_debug_glcm_ms waits for them and returns the
 * summed milliseconds and the launch count, then forgets them.  Not for timed regions.       */
int cpx_debug_glcm_timing(cpx_ctx* ctx, int enable);
int cpx_debug_glcm_ms(cpx_ctx* ctx, double* ms_out, int* launches_out);
/* Segmentation post-processing instrumentation (bench.py's flow-following and flow-error
 * rooflines): while enabled, each cpx_seg_masks call (up to 16 between reads) records events
 * around its flow-following rounds and around its register flow-error kernels, and copies the
 * per-round item counts to pinned host memory (a synchronous copy on the context's stream: not
 * for captured or production runs).  cpx_debug_seg_stats waits for them and returns the summed
 * milliseconds and the item-steps of the rounds (items per round x steps per round: an upper
 * bound, an item at an exact fixed point stops early), then resets.                           */
int cpx_debug_seg_timing(cpx_ctx* ctx, int enable);
int cpx_debug_seg_stats(cpx_ctx* ctx, double* follow_ms, double* item_steps, double* fe_reg_ms, int* calls);

/* ---- host: CSV rows of the measurement tables (Pycyto_pertime.py:46-49 reads them) ------- *
 * Rows [row0, row1) of a table of n_cols columns, column c at cols[c] with element stride
 * strides[c] (in elements), types[c] 0 = int64 (decimal) or 1 = float64 (Python repr, the text
 * pandas.DataFrame.to_csv writes; NaN -> empty field): comma-separated, '\n'-terminated, into
 * out (cap bytes, at least 33 * n_cols per row).  Returns the bytes written, or -1 (bad
 * arguments / cap too small).  Pure host code, thread-safe: cpx.csvout formats row ranges on
 * several threads.  Replaces the to_csv text of the reference's CSV outputs.                 */
int64_t cpx_csv_format(int64_t row0, int64_t row1, int n_cols, const void* const* cols, const int* types,
                       const int64_t* strides, char* out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* CPX_H */
