/*
 * fmpnp.h -- C ABI of libfmpnp.so, the MI355X (gfx950) feature-metric PnP refiner.
 *
 * Drop-in boundary for the reference's hot path (aunagar/FeatureMetric-PnP):
 *
 *   fmpnp_refine_batch / fmpnp_refine_batch_async
 *       replace sparseFeaturePnP.forward          featurePnP/model.py:245-494
 *       (and, with FMPNP_MODE_COMPUTE_COST,
 *        sparseFeaturePnP.compute_cost            featurePnP/model.py:216-243)
 *       -- the LM loop, the losses of          featurePnP/helpers/utils.py:15-78,
 *          optimizer_step                       featurePnP/model.py:37-72,
 *          indexing_ / points_within_image      featurePnP/model.py:74-117,
 *          ratio_threshold_feature_errors       featurePnP/model.py:120-129,
 *          so3exp_map                           featurePnP/helpers/utils.py:209-221.
 *   fmpnp_pack_features / fmpnp_pack_features_batch / fmpnp_pack_features_f
 *       replaces sobel_filter + the fp64 cast   featurePnP/helpers/utils.py:81-104,
 *                                               optimize_feature_pnp.py:57,61
 *       (fused Sobel + channels-last [H][W][3][C] packing).
 *   fmpnp_gather_reference
 *   fmpnp_gather_reference_async / fmpnp_gather_reference_batch
 *       replaces the per-point fref gather       optimize_feature_pnp.py:51-56.
 *   fmpnp_point_costs
 *       replaces find_inliers' per-point costs   featurePnP/model.py:132-146
 *       (projection, support mask, indexing_, 0.5||e||^2; the loss and ratio mask,
 *        model.py:147-152, stay in the façade).
 *
 * Conventions: plain pointers and sizes, no torch types.  Feature / point
 * buffers are caller-owned DEVICE memory; results and traces of the
 * synchronous entry points are host memory.  Every entry point returns 0 on
 * success, a negative FMPNP_E* code for invalid arguments, or a positive
 * hipError_t; nothing throws.
 *
 * Threads: the asynchronous entry points touch only caller-owned memory.  The synchronous ones
 * (fmpnp_refine_batch, fmpnp_feature_pnp) keep their scratch per (entry point, device, stream), each
 * behind its own mutex, and drain their stream before returning an error once work is queued: calls
 * on distinct streams or devices run concurrently, calls on one stream from several threads
 * serialise.  Multi-GPU = one host thread (or process) per device.
 */
#ifndef FMPNP_H
#define FMPNP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FMPNP_ABI_VERSION 4  /* 3: fmpnp_problem.window (windowed f-only packs); 4: fmpnp_feature_pnp */

/* robust losses, featurePnP/helpers/utils.py:15-78 */
typedef enum {
    FMPNP_SQUARED = 0,        /* squared_loss          :16-17 */
    FMPNP_HUBER = 1,          /* huber_loss            :20-29 */
    FMPNP_CAUCHY = 2,         /* cauchy_loss = barron(alpha=0)   :32-34 */
    FMPNP_GEMAN_MCCLURE = 3,  /* geman_mcclure = barron(alpha=-2) :37-38 */
    FMPNP_BARRON = 4          /* barron_loss(x, alpha) :40-78 */
} fmpnp_loss;

typedef enum {
    FMPNP_NEAREST = 0,   /* the reference: round(K P / z) - 1, floor rescale (model.py:88-89,306-308) */
    FMPNP_BILINEAR = 1   /* extension: 2x2 bilinear taps of f, gx, gy; the map must have
                            Hf < 32768 and Wf < 65535 (FMPNP_ETOOBIG otherwise) */
} fmpnp_sampling;

typedef enum { FMPNP_F32 = 0, FMPNP_F64 = 1 } fmpnp_dtype;

typedef enum {
    FMPNP_LAYOUT_FGRAD = 0, /* feat = [Hf][Wf][3][cstride]: f, gx, gy (fmpnp_pack_features) */
    FMPNP_LAYOUT_F = 1      /* feat = [Hf][Wf][cstride]: f only (fmpnp_pack_features_f); the LM kernel
                               forms a texel's Sobel gradients from its 3x3 neighbourhood, in fp64,
                               when it gathers the texel.  fp32 storage, nearest sampling. */
} fmpnp_layout;

typedef enum {
    FMPNP_MODE_FORWARD = 0,       /* sparseFeaturePnP.forward */
    FMPNP_MODE_COMPUTE_COST = 1   /* sparseFeaturePnP.compute_cost at (R0, t0) */
} fmpnp_mode;

/* per-problem status bits (fmpnp_result.status) */
#define FMPNP_STATUS_OK 0
#define FMPNP_STATUS_NO_SUPPORT 1        /* no point inside the image at (R0,t0): model.py:316-320 */
#define FMPNP_STATUS_NAN 2               /* NaN step: model.py:411-413 (reference: NameError) */
#define FMPNP_STATUS_NO_SUPPORT_TRIAL 4  /* no point inside at a trial pose: model.py:441-445 */
#define FMPNP_STATUS_SYNC_TIMEOUT 8      /* internal: a cross-workgroup exchange timed out */
#define FMPNP_STATUS_HELPER_WAIT 16      /* informational: a first-evaluation helper workgroup did not
                                            publish in time and the main workgroup gathered that block
                                            itself (results unaffected: same gather code) */
#define FMPNP_STATUS_WINDOW 32           /* a point reached a texel whose 3x3 neighbourhood lies outside
                                            the problem's packed window (fmpnp_problem.window): the
                                            problem stopped early and its result is invalid -- pack its
                                            map in full and refine it again (fmpnp.pipeline does) */

/* argument errors (negative return codes) */
#define FMPNP_EINVAL -1
#define FMPNP_EALIGN -2
#define FMPNP_ENOMEM -3
#define FMPNP_ETOOBIG -4
#define FMPNP_ENODEV -5
#define FMPNP_ERANGE -6  /* fmpnp_feature_pnp: a reference inlier maps outside the reference map
                            (the reference raises IndexError, optimize_feature_pnp.py:56) */

typedef struct {
    int mode;               /* fmpnp_mode */
    int n_iters;            /* sparseFeaturePnP(n_iters) */
    double lambda0;         /* sparseFeaturePnP(lambda_), default 0.01 */
    int use_ratio;          /* ratio_threshold is not None */
    double ratio_threshold; /* keep |rho| < max|rho| * thr */
    int loss;               /* fmpnp_loss */
    double barron_alpha;    /* FMPNP_BARRON only */
    int sampling;           /* fmpnp_sampling */
    int dtype;              /* fmpnp_dtype of the packed features and fref */
    int wgs_per_problem;    /* workgroups cooperating on one problem; 0 = auto */
    int max_teams;          /* cap on concurrently resident problem teams; 0 = auto */
    int no_memo;            /* 1: re-gather every point's texel at every evaluation (the
                               reference's data movement); 0 (default): re-gather only points
                               whose texel changed and, where the planner enables it, also gather
                               the texels points are predicted to move to next beside the LM tail
                               (speculation: on by default; -DFMPNP_SPEC=0 compiles it out);
                               2: memoised without speculation -- all bit-identical results.
                               FMPNP_BILINEAR: 0/2 keep each point's cell memo (the six sums as
                               quadratics over its 2x2 cell, rebuilt when the cell changes; same
                               sums up to fp64 rounding), 1 samples every point every evaluation */
    int layout;             /* fmpnp_layout of every problem's feat */
    int sobel_flags;        /* FMPNP_LAYOUT_F: bit 0 normalized (/8), bit 1 replicate padding
                               (the flags fmpnp_pack_features would have been given) */
    int helpers;            /* first-evaluation helper workgroups per problem (small batches with
                               idle CUs): 0 = the planner's choice, < 0 = none (e.g. when other
                               kernels share the device and could keep helpers from being
                               resident: the main workgroups would wait up to 0.2 s for them),
                               > 0 = at most this many.  Results do not depend on it. */
} fmpnp_options;

typedef struct {
    const void *feat;       /* device, [Hf][Wf][3][cstride] of dtype: planes f, gx, gy
                               (FMPNP_LAYOUT_F: [Hf][Wf][cstride], f only) */
    const void *fref;       /* device, [N][ld_ref] of dtype; columns [c_begin, c_end) used */
    const double *pts3d;    /* device, [N][3] fp64 */
    int Hf, Wf, cstride, c_begin, c_end, ld_ref, N;
    int im_width, im_height;        /* image size in pixels (forward's im_width/im_height) */
    double K[9], R0[9], t0[3];      /* row-major */
    const unsigned char *window;    /* NULL: feat holds every texel.  Else (FMPNP_LAYOUT_F, one workgroup
                                       per problem) device [2][Hf][Wf] bytes written by
                                       fmpnp_pack_features_f_window_batch: plane 0 = texel packed, plane 1 =
                                       texel whose whole 3x3 neighbourhood is packed.  The LM kernel checks
                                       plane 1 at every gather and stops the problem with
                                       FMPNP_STATUS_WINDOW on a miss, so a result without that bit equals the
                                       fully packed map's bit for bit.  FMPNP_LAYOUT_FGRAD (nearest
                                       sampling; fmpnp_feature_pnp's windowed packs): plane 0 is checked,
                                       and a miss only sets FMPNP_STATUS_WINDOW (the problem finishes). */
} fmpnp_problem;

typedef struct {
    double R[9], t[3];      /* returned pose (R_best/t_best, or the current pose on early exit) */
    double initial_cost;    /* mean rho at (R0,t0) (forward i==0 / compute_cost); NaN if none */
    double best_cost;       /* best_cost_ (NaN when never set) */
    double final_lambda, final_lr;
    int best_num_inliers;   /* best_num_inliers_ (-1 when never set) */
    int n_evals;            /* tracked evaluations: 1 + trials */
    int n_steps;            /* optimizer steps taken */
    int n_accepted;
    int status;             /* FMPNP_STATUS_* bits */
    int has_best;           /* best_cost_ was set */
    long long texel_gathers; /* point-texel gathers actually read from memory by the problem's
                                first workgroup (a texel is re-read only when a point's pixel
                                changes: the channel sums of an unchanged texel are reused) */
} fmpnp_result;

typedef struct {            /* one tracked evaluation (model.track_, model.py:170-176) */
    double R[9], t[3];
    double cost;            /* mean rho at this pose */
    double lambda_after, lr_after;
    int n_supported, n_kept, accepted;
} fmpnp_trace_entry;

/* library identity / device check */
int fmpnp_abi_version(void);
const char *fmpnp_build_info(void);
int fmpnp_device_check(int device); /* 0 if `device` is a gfx950 the library can run on */

/* Fused Sobel (3x3, unnormalised unless sobel_normalized -> /8; zero or replicate
 * padding) + channels-last pack: chw [C][H][W] (dtype_in) -> out [H][W][3][cstride]
 * (dtype_out).  When gx_chw/gy_chw are non-NULL they are packed as given instead of
 * computing the Sobel (forward() receives its gradients from the caller). */
int fmpnp_pack_features(const void *chw, const void *gx_chw, const void *gy_chw, int dtype_in, int C, int H,
                        int W, void *out, int dtype_out, int cstride, int sobel_normalized,
                        int sobel_replicate_pad, void *hip_stream);

/* Channels-last copy of f only, [H][W][cstride] fp32 (dtype_out = FMPNP_F32, cstride a
 * multiple of 4, out 16-byte aligned; channels [C, cstride) zero-filled): the
 * FMPNP_LAYOUT_F input of the LM kernel, a third of fmpnp_pack_features' output bytes. */
int fmpnp_pack_features_f(const void *chw, int dtype_in, int C, int H, int W, void *out, int dtype_out,
                          int cstride, void *hip_stream);

/* fref gather of optimize_feature_pnp.py:51-56: for each of the N reference
 * inliers (x, y) (device [N][2] fp64), row = trunc(y * W_ref / img1),
 * col = trunc(x * H_ref / img0) of ref_chw [C][H_ref][W_ref] -> out [N][ld_out]. */
int fmpnp_gather_reference(const void *ref_chw, int dtype_in, int C, int H_ref, int W_ref,
                           const double *ref_inliers, int N, int img0, int img1, void *out, int dtype_out,
                           int ld_out, void *hip_stream);

/* Asynchronous form of fmpnp_gather_reference: nothing is synchronised; an inlier
 * outside the reference map ORs 1 into *err_flag (a device int the caller zeroes
 * beforehand and reads after the stream reached this point) and zeroes its row.
 * The batch pipeline (fmpnp.pipeline) uses it so preparing one batch never waits
 * for the device. */
int fmpnp_gather_reference_async(const void *ref_chw, int dtype_in, int C, int H_ref, int W_ref,
                                 const double *ref_inliers, int N, int img0, int img1, void *out, int dtype_out,
                                 int ld_out, int *err_flag, void *hip_stream);

/* Batched forms for a caller preparing many queries at once (fmpnp.pipeline): one host
 * call, one launch per item on hip_stream, nothing synchronised.  Host arrays of n entries;
 * shape[4*i..] = (C, H, W, cstride) of map i, ref_shape[3*i..] = (C, H_ref, W_ref) of
 * reference map i; err_flags is a DEVICE int[n] the caller zeroes (set as in
 * fmpnp_gather_reference_async).  Every item is validated before anything is launched. */
int fmpnp_pack_features_batch(int n, const void *const *chw, void *const *out, const int *shape, int dtype_in,
                              int dtype_out, int sobel_normalized, int sobel_replicate_pad, int layout,
                              void *hip_stream);
/* Windowed f-only pack (FMPNP_LAYOUT_F) of n problems: only the texels within `radius` texels
 * (Chebyshev distance, radius >= 2) of a point's texel at the problem's initial pose (R0, t0) are
 * written to feat ([Hf][Wf][cstride] fp32, channels [c_end, cstride) zero), and window ([2][Hf][Wf]
 * bytes, see fmpnp_problem.window) records which: plane 1 marks the texels within radius - 1.
 * The reference's refinement reads only the 3x3 neighbourhoods of the texels its points visit
 * (optimize_feature_pnp.py:57-61 packs all of them), so a radius a little above the points' motion
 * in texels leaves most of the map unwritten and mostly unread.  probs_dev / probs_host: the same
 * descriptors in device / host memory (feat and window set, c_begin = 0, C = c_end channels);
 * chw[i]: map i, [c_end][Hf][Wf] of dtype_in.  Asynchronous on hip_stream. */
int fmpnp_pack_features_f_window_batch(const fmpnp_problem *probs_dev, const fmpnp_problem *probs_host, int n,
                                       const void *const *chw, int dtype_in, int radius, void *hip_stream);
int fmpnp_gather_reference_batch(int n, const void *const *ref_chw, const int *ref_shape,
                                 const double *const *ref_inliers, const int *n_inliers, int img0, int img1,
                                 void *const *out, const int *ld_out, int dtype_in, int dtype_out, int *err_flags,
                                 void *hip_stream);

/* Per-point residual costs at the descriptor's pose (R0, t0): the projection,
 * points_within_image and indexing_ of find_inliers (featurePnP/model.py:132-146).
 * supported[i] = 1 when point i's rounded pixel lies in the image, and then
 * cost[i] = 0.5 * sum over [c_begin, c_end) of (f(p_i) - fref_i)^2 (fp64), else 0.
 * cost ([N] fp64) and supported ([N] int32) are DEVICE arrays; the descriptor is host
 * memory; asynchronous on hip_stream.  layout / dtype as in fmpnp_options (FMPNP_LAYOUT_F
 * is fp32 only).  The façade's find_inliers applies the loss and the ratio mask. */
int fmpnp_point_costs(const fmpnp_problem *prob, int layout, int dtype, double *cost, int *supported,
                      void *hip_stream);

/* compute_cost (featurePnP/model.py:216-243) at the descriptor's pose (R0, t0): the mean over the
 * supported points -- after the ratio test when use_ratio (model.py:230-236) -- of
 * 0.5 ||f(p_i) - fref_i||^2 over [c_begin, c_end).  fmpnp_point_costs (one wave per point) into
 * cost / supported (DEVICE [N] fp64 / int32 scratch), then one fixed-order reduction into *result
 * (DEVICE): initial_cost (NaN when the ratio test keeps nothing), status FMPNP_STATUS_NO_SUPPORT when
 * no point is supported (the reference returns None), R / t = (R0, t0).  The descriptor is host
 * memory; asynchronous on hip_stream.  One evaluation: it is not an LM launch. */
int fmpnp_compute_cost_async(const fmpnp_problem *prob, int layout, int dtype, int use_ratio, double ratio_threshold,
                             double *cost, int *supported, fmpnp_result *result, void *hip_stream);

/* Device workspace needed by fmpnp_refine_batch_async for n problems (team exchange slots and,
 * for small batches, the first-evaluation helpers' records; no initialisation needed, reusable
 * by later launches on the same stream). */
size_t fmpnp_workspace_size(const fmpnp_problem *probs_host, int n, const fmpnp_options *opt);

/* Asynchronous batched refinement: descriptors, results and trace in DEVICE
 * memory; nothing is synchronised.  probs_host: the same descriptors in host memory
 * (required: the launch plan reads every problem's sizes and channel slice); max_N is
 * unused (kept for ABI stability). */
int fmpnp_refine_batch_async(const fmpnp_problem *probs_dev, const fmpnp_problem *probs_host, int n, int max_N,
                             const fmpnp_options *opt, fmpnp_result *results_dev, fmpnp_trace_entry *trace_dev,
                             int trace_stride, void *workspace, size_t workspace_bytes, void *hip_stream);

/* Synchronous convenience: host descriptors in, host results (and optional
 * trace, [n][trace_stride] entries) out.  Uploads descriptors, launches on
 * hip_stream and waits for that stream.  Its device workspace and pinned staging are this
 * (device, stream)'s own (see Threads above). */
int fmpnp_refine_batch(const fmpnp_problem *probs_host, int n, const fmpnp_options *opt, fmpnp_result *results,
                       fmpnp_trace_entry *trace, int trace_stride, void *hip_stream);

/* CPU twin of fmpnp_refine_batch: the same descriptors, options, results and trace
 * with HOST pointers -- feat (the packed [Hf][Wf][3][cstride] of fmpnp_pack_features, or the f-only
 * [Hf][Wf][cstride] of FMPNP_LAYOUT_F), fref and pts3d in host memory.  The LM loop of
 * sparseFeaturePnP.forward (featurePnP/model.py:245-494; compute_cost :216-243 with
 * FMPNP_MODE_COMPUTE_COST) on n_threads host threads (0: every core), one problem per thread at a
 * time.  Nearest sampling only (FMPNP_BILINEAR: FMPNP_EINVAL); no windows.  An explicit CPU entry
 * point -- the timed CPU baseline and a parity bridge -- never a fallback of the HIP entry points.
 * Returns 0 or FMPNP_EINVAL. */
int fmpnp_refine_batch_cpu(const fmpnp_problem *probs_host, int n, const fmpnp_options *opt, fmpnp_result *results,
                           fmpnp_trace_entry *trace, int trace_stride, int n_threads);

/* One channel level of multilevel_optimization's pyramid (featurePnP/model.py:193-210): the
 * channel range [c_begin, c_end) of the query map (input_configs/default_robotcar.gin:75). */
typedef struct {
    int c_begin, c_end;
} fmpnp_level;

/* One query of feature_pnp (s2dhm/pose_prediction/optimize_feature_pnp.py:50-71) in one call,
 * with one host wait: pack the query map (opt->layout; opt->sobel_flags are the Sobel's flags),
 * gather the reference descriptors of the N reference inliers (x, y) with the adapter's
 * truncation, then
 *   n_levels == 0: forward over channels [0, C)                     (model.py:245-494)
 *                  -> results[0];
 *   n_levels >  0: multilevel_optimization over the channel levels  (model.py:178-213):
 *                  compute_cost at (R0, t0) over [0, C) -> results[0] (status NO_SUPPORT: the
 *                  reference returns (R0, t0) without refining -- the caller applies that), then
 *                  forward per level, each from the previous level's result pose -> results[1 + l].
 * query_chw [C][H][W] and ref_chw [C_ref][H_ref][W_ref] (C_ref == C) are DEVICE maps; ref_inliers
 * [N][2], pts3d [N][3], K, R0, t0 (row-major) and results / trace ([max(n_levels, 1)][trace_stride]
 * entries, or NULL) are HOST memory.  opt->mode must be FMPNP_MODE_FORWARD; opt->dtype is the
 * packed storage.  Returns 0, FMPNP_ERANGE when an inlier maps outside the reference map (results
 * are still written), another FMPNP_E* code or a hipError_t.  The library keeps, per (device,
 * hip_stream), the device buffers, a pinned staging buffer and a second stream with two events
 * between calls (see Threads above): with levels, the first level's channels are packed first and the
 * other channels' pack and compute_cost run on that second stream under the first level's launch. */
int fmpnp_feature_pnp(const void *query_chw, int dtype_query, int C, int H, int W, const void *ref_chw,
                      int dtype_ref, int C_ref, int H_ref, int W_ref, const double *ref_inliers,
                      const double *pts3d, int N, const double K[9], const double R0[9], const double t0[3],
                      int img0, int img1, const fmpnp_level *levels, int n_levels, const fmpnp_options *opt,
                      int window_radius, fmpnp_result *results, fmpnp_trace_entry *trace, int trace_stride,
                      void *hip_stream);
/* window_radius > 0 (FMPNP_LAYOUT_FGRAD, nearest sampling): pack only the texels within that many texels
 * (Chebyshev) of a point's texel at (R0, t0) -- the refinement reads the texels its points visit, a
 * few from where they start.  An LM gather outside the window marks the attempt invalid and the call
 * runs again fully packed, so the results are the full pack's bit for bit either way.  0: full pack.
 * fmpnp_feature_pnp_reruns(): how many calls of this process ran again after a window miss. */
long long fmpnp_feature_pnp_reruns(void);

/* Debug: when device_buf != NULL, later LM launches write per-workgroup phase cycle
 * totals (s_memtime) to device_buf[grid][8 waves][12] (8 phases, then the first evaluation's
 * projection, gather, loss and contribution phases separately; phases 3-7 are wave 0's LM tail);
 * NULL switches it off. */
int fmpnp_debug_stamps(unsigned long long *device_buf);

/* Last launch geometry of this thread (for benches / tests). */
int fmpnp_last_launch(int *teams, int *wgs_per_problem, int *grid, int *lds_bytes);

/* LM kernel builds (fmpnp_launch_info.build) */
#define FMPNP_BUILD_WIDE 1        /* 256-thread workgroups, one wave per SIMD (bilinear cell memo) */
#define FMPNP_BUILD_LATENCY 2     /* 512-thread workgroups, one per CU */
#define FMPNP_BUILD_THROUGHPUT 4  /* 256-thread workgroups, two per CU (batches >= 2 per CU) */

/* LM kernel variants (fmpnp_launch_info.variant): which code paths are compiled into the
 * kernel that ran -- the loss / sampling / layout specialisation, the speculative next-texel
 * gathers (_SPEC) and the first-evaluation helpers' hand-off (_H) */
#define FMPNP_VAR_NEAREST 0        /* any loss, nearest sampling, packed f/gx/gy (and compute_cost) */
#define FMPNP_VAR_GM 1             /* Geman-McClure forward, nearest, packed */
#define FMPNP_VAR_BILINEAR 2       /* bilinear cell memo */
#define FMPNP_VAR_F_NEAREST 3      /* FMPNP_LAYOUT_F, any loss */
#define FMPNP_VAR_F_GM 4           /* FMPNP_LAYOUT_F, Geman-McClure */
#define FMPNP_VAR_BIL_DIRECT 5     /* bilinear, every point sampled every evaluation */
#define FMPNP_VAR_GM_SPEC 6
#define FMPNP_VAR_NEAREST_SPEC 7
#define FMPNP_VAR_GM_SPEC_H 8
#define FMPNP_VAR_NEAREST_SPEC_H 9
#define FMPNP_VAR_GM_H 10
#define FMPNP_VAR_NEAREST_H 11
#define FMPNP_VAR_GM_SPEC_512 12    /* GM_SPEC / GM_SPEC_H compiled for a 512-point workgroup (the LDS carve at */
#define FMPNP_VAR_GM_SPEC_H_512 13  /* compile-time offsets: configs[1]/[2]'s N = 512, fp32); otherwise as those */
#define FMPNP_VAR_GM_W 14          /* GM / NEAREST / GM_H / NEAREST_H with the packed-window check compiled */
#define FMPNP_VAR_NEAREST_W 15     /* in (fmpnp_problem.window on the packed f/gx/gy planes: fmpnp_feature_pnp's */
#define FMPNP_VAR_GM_H_W 16        /* windowed packs); the other packed variants carry no check */
#define FMPNP_VAR_NEAREST_H_W 17

typedef struct {
    int teams, wgs_per_problem, grid, lds_bytes;
    int build;              /* FMPNP_BUILD_* */
    int variant;            /* FMPNP_VAR_* */
    int team;               /* 1: wgs_per_problem > 1 (cross-workgroup exchange compiled in) */
    int ratio;              /* 1: the ratio-test specialisation */
    int dtype;              /* fmpnp_dtype of the texels */
    int helpers;            /* first-evaluation helper workgroups per problem */
    int speculate;          /* speculative next-texel gathers enabled */
} fmpnp_launch_info;

/* The LM launch plan for these problems and options, without launching anything (needs
 * the current device: CU count and occupancy).  Returns 0 or the launch's error code. */
int fmpnp_plan(const fmpnp_problem *probs_host, int n, const fmpnp_options *opt, fmpnp_launch_info *out);

/* Plan of the last LM launch of this thread. */
int fmpnp_last_launch_info(fmpnp_launch_info *out);

#ifdef __cplusplus
}
#endif
#endif /* FMPNP_H */
