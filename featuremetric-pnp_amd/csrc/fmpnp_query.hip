// fmpnp_query.hip -- fmpnp_feature_pnp: one query of the reference adapter in ONE host call.
//
// feature_pnp (s2dhm/pose_prediction/optimize_feature_pnp.py:50-71) prepares a query on the
// host -- fref gather, fp64 cast, Sobel -- and then runs forward or multilevel_optimization
// (featurePnP/model.py:178-213, 245-494).  Here the whole call is one stream of device work
// with a single host wait at the end:
//
//   H2D   reference inliers, 3D points and the launch descriptors, one copy from a pinned
//         staging buffer the library owns (no pageable copies, no allocation per call);
//   pack  the query map (fused Sobel + channels-last, or the f-only copy) into a cached buffer;
//   fref  gather of the reference descriptors (out-of-map inliers set a device flag -- the
//         reference's IndexError -- read with the results, no wait here);
//   LM    forward over the whole map, or compute_cost + one forward per channel level, each
//         level's initial pose copied from the previous level's result on the device;
//   D2H   results (+ trace) and the flag, one copy, one stream synchronisation.
//
// The kernels are the ones the separate entry points launch, with the same descriptors, so the
// results equal pack + gather + refine called one by one, bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>

#include "fmpnp.h"
#include "fmpnp_internal.h"

using namespace fmpnp;

namespace {

inline size_t al(size_t x) { return (x + 255) / 256 * 256; }

std::atomic<long long> g_window_reruns{0};  // fmpnp_feature_pnp calls re-run fully packed after a window miss

}  // namespace

extern "C" int fmpnp_compute_cost_async(const fmpnp_problem *prob, int layout, int dtype, int use_ratio,
                                        double ratio_threshold, double *cost, int *supported, fmpnp_result *result,
                                        void *hip_stream) {
    if (!prob || !result || (prob->N > 0 && (!cost || !supported))) return FMPNP_EINVAL;
    const fmpnp_problem &p = *prob;
    if (layout != FMPNP_LAYOUT_FGRAD && layout != FMPNP_LAYOUT_F) return FMPNP_EINVAL;
    if (dtype != FMPNP_F32 && dtype != FMPNP_F64) return FMPNP_EINVAL;
    if (layout == FMPNP_LAYOUT_F && dtype != FMPNP_F32) return FMPNP_EINVAL;
    if (p.N < 0 || p.c_end <= p.c_begin) return FMPNP_EINVAL;
    if (p.N > 0) {
        const int rc = fmpnp_point_costs(prob, layout, dtype, cost, supported, hip_stream);  // (validates the rest)
        if (rc) return rc;
    }
    return (int)launch_cost_mean(p, use_ratio, ratio_threshold, cost, supported, result, (hipStream_t)hip_stream);
}

extern "C" int fmpnp_feature_pnp(const void *query_chw, int dtype_query, int C, int H, int W, const void *ref_chw,
                                 int dtype_ref, int C_ref, int H_ref, int W_ref, const double *ref_inliers,
                                 const double *pts3d, int N, const double K[9], const double R0[9], const double t0[3],
                                 int img0, int img1, const fmpnp_level *levels, int n_levels,
                                 const fmpnp_options *opt, int window_radius, fmpnp_result *results,
                                 fmpnp_trace_entry *trace, int trace_stride, void *hip_stream) {
    if (!query_chw || !ref_chw || !opt || !results || !K || !R0 || !t0 || N < 0 || C <= 0 || H <= 0 || W <= 0 ||
        C_ref != C || H_ref <= 0 || W_ref <= 0 || img0 <= 0 || img1 <= 0 || n_levels < 0 || (n_levels > 0 && !levels))
        return FMPNP_EINVAL;
    if (N > 0 && (!ref_inliers || !pts3d)) return FMPNP_EINVAL;
    if ((dtype_query != FMPNP_F32 && dtype_query != FMPNP_F64) || (dtype_ref != FMPNP_F32 && dtype_ref != FMPNP_F64))
        return FMPNP_EINVAL;
    if (opt->mode != FMPNP_MODE_FORWARD || (trace && trace_stride < 1)) return FMPNP_EINVAL;
    // packed windows: the fused Sobel pack of the packed f, gx, gy planes, nearest sampling
    if (window_radius < 0 || window_radius > 4096 ||
        (window_radius > 0 && (opt->layout != FMPNP_LAYOUT_FGRAD || opt->sampling != FMPNP_NEAREST)))
        return FMPNP_EINVAL;
    for (int l = 0; l < n_levels; ++l)
        if (levels[l].c_begin < 0 || levels[l].c_end <= levels[l].c_begin || levels[l].c_end > C) return FMPNP_EINVAL;
    const bool lay_f = opt->layout == FMPNP_LAYOUT_F;
    const int es = opt->dtype == FMPNP_F64 ? 8 : 4;
    const int cs = (C + 3) / 4 * 4;
    const int planes = lay_f ? 1 : 3;
    const int n_fwd = n_levels > 0 ? n_levels : 1;
    const int n_res = n_levels > 0 ? n_levels + 1 : 1;  // [compute_cost,] forward per level
    const int stride = trace ? trace_stride : 0;

    // host-side descriptors: [0] compute_cost over the whole map (levels only), then the forwards
    fmpnp_problem hd[1 + 64];
    if (n_res > 65) return FMPNP_EINVAL;
    for (int r = 0; r < n_res; ++r) {
        fmpnp_problem &p = hd[r];
        memset(&p, 0, sizeof(p));
        p.Hf = H;
        p.Wf = W;
        p.cstride = cs;
        p.ld_ref = cs;
        p.N = N;
        p.im_width = img0;
        p.im_height = img1;
        memcpy(p.K, K, sizeof(p.K));
        memcpy(p.R0, R0, sizeof(p.R0));
        memcpy(p.t0, t0, sizeof(p.t0));
        const int l = n_levels > 0 ? r - 1 : 0;
        p.c_begin = (n_levels > 0 && r > 0) ? levels[l].c_begin : 0;
        p.c_end = (n_levels > 0 && r > 0) ? levels[l].c_end : C;
        // (pointers are set below, once the device buffer is placed; the plans need only sizes)
        p.feat = p.fref = (const void *)(uintptr_t)256;
        p.pts3d = (const double *)(uintptr_t)256;
    }
    // the LM workspace of the largest plan (the launches run one after another on the stream)
    // (with and without the window: a window miss re-runs the call fully packed)
    size_t ws = 0;
    for (int wi = 0; wi < (window_radius > 0 ? 2 : 1); ++wi)
        for (int r = n_levels > 0 ? 1 : 0; r < n_res; ++r) {  // (compute_cost: point costs + one reduction)
            fmpnp_problem pw = hd[r];
            pw.window = wi ? (const unsigned char *)(uintptr_t)256 : nullptr;
            const size_t w = fmpnp_workspace_size(&pw, 1, opt);
            if (w == 0) return FMPNP_EINVAL;  // (fmpnp_workspace_size: invalid problem / options)
            ws = std::max(ws, w);
        }
    // device carve: [inl | pts | descs] (the one upload), [results | err | trace] (the one
    // download), the packed map, fref, the LM workspace
    const size_t b_inl = al((size_t)N * 16), b_pts = al((size_t)N * 24), b_desc = al(sizeof(fmpnp_problem) * n_res);
    const size_t b_res = al(sizeof(fmpnp_result) * n_res), b_err = 256;
    const size_t b_tr = trace ? al(sizeof(fmpnp_trace_entry) * (size_t)n_fwd * stride) : 0;
    const size_t b_feat = al((size_t)H * W * planes * cs * es), b_fref = al((size_t)std::max(N, 1) * cs * es);
    const size_t b_cost = n_levels > 0 ? al((size_t)std::max(N, 1) * 12) : 0;  // compute_cost's per-point costs
    const size_t up = b_inl + b_pts + b_desc, down = b_res + b_err + b_tr;
    const size_t b_win = window_radius > 0 ? al((size_t)2 * H * W) : 0;  // [2][H][W] window map
    const size_t need = up + down + b_feat + b_fref + al(ws) + b_cost + b_win;

    hipStream_t s = (hipStream_t)hip_stream;
    // this stream's scratch (fmpnp_internal.h StreamScratch): the device carve and a pinned staging
    // buffer, grown on demand and reused; calls on other streams or devices use their own
    StreamScratch *sc = stream_scratch(SCRATCH_QUERY, s, nullptr);
    if (!sc) return FMPNP_ENODEV;
    std::lock_guard<std::mutex> lock(sc->mu);  // (held until this call's stream has drained)
    int rc = scratch_grow(*sc, need, up + down, (size_t)64 << 20, s);
    if (rc) return rc;
    hipError_t e = hipSuccess;
    unsigned char *d = sc->dev, *h = sc->host;
    double *d_inl = (double *)d, *d_pts = (double *)(d + b_inl);
    fmpnp_problem *d_desc = (fmpnp_problem *)(d + b_inl + b_pts);
    fmpnp_result *d_res = (fmpnp_result *)(d + up);
    int *d_err = (int *)(d + up + b_res);
    fmpnp_trace_entry *d_tr = trace ? (fmpnp_trace_entry *)(d + up + b_res + b_err) : nullptr;
    unsigned char *d_feat = d + up + down, *d_fref = d_feat + b_feat, *d_ws = d_fref + b_fref;
    double *d_cost = (double *)(d_ws + al(ws));
    int *d_sup = (int *)(d_cost + std::max(N, 1));
    unsigned char *d_win = (unsigned char *)d_cost + b_cost;
    for (int r = 0; r < n_res; ++r) {
        hd[r].feat = d_feat;
        hd[r].fref = d_fref;
        hd[r].pts3d = d_pts;
    }
    // an error once work is queued: wait for the stream before returning, so the pinned staging buffer
    // and the device carve are never reused (by the next call) while an earlier copy still reads them
    auto drain = [s, sc](int code) {
        (void)hipStreamSynchronize(s);
        if (sc->side) (void)hipStreamSynchronize(sc->side);
        return code;
    };
    // the first level's channels [sb, se) packed on the main stream and the other channels on the side
    // stream, under the first level's LM launch (one workgroup and its helpers: the rest of the device is
    // idle).  Only with channel boundaries on 128-byte lines (sb, se multiples of 32), so no cache line
    // holds channels of both streams' packs; FMPNP_QUERY_SPLIT=0 switches it off (A/B knob)
    static const bool split_on = [] { const char *v = getenv("FMPNP_QUERY_SPLIT"); return !(v && *v == '0'); }();
    const int sb = n_levels >= 2 ? levels[0].c_begin : 0, se = n_levels >= 2 ? levels[0].c_end : C;
    const bool split = split_on && n_levels >= 2 && !lay_f && (sb > 0 || se < C) && sb % 32 == 0 &&
                       (se % 32 == 0 || se == C);
    if (split) {
        const int rc2 = scratch_side(*sc);
        if (rc2) return rc2;
    }
    // Sobel pack of channels [c0, c1) (fmpnp_pack.hip: a channel's gradients read only its own plane, so a
    // channel range is the whole-map pack's bytes for those channels) on stream st
    bool win = false;
    auto pack_range = [&](int c0, int c1, hipStream_t st) -> hipError_t {
        const void *src = (const unsigned char *)query_chw + (size_t)c0 * H * W * (dtype_query == FMPNP_F64 ? 8 : 4);
        void *dst = d_feat + (size_t)c0 * es;
        if (win)
            return launch_pack_win(src, dtype_query, c1 - c0, H, W, dst, opt->dtype, cs, opt->sobel_flags & 1,
                                   (opt->sobel_flags >> 1) & 1, d_win, st);
        return launch_pack(src, nullptr, nullptr, dtype_query, c1 - c0, H, W, dst, opt->dtype, cs,
                           opt->sobel_flags & 1, (opt->sobel_flags >> 1) & 1, st, planes);
    };
  for (int attempt = 0; attempt < 2; ++attempt) {
    // attempt 0: windowed when asked; attempt 1 (only after a window miss): the full pack
    win = attempt == 0 && window_radius > 0;
    if (attempt == 1 && window_radius == 0) break;
    for (int r = 0; r < n_res; ++r) hd[r].window = win ? d_win : nullptr;
    // the one upload
    if (N > 0) {
        memcpy(h, ref_inliers, (size_t)N * 16);
        memcpy(h + b_inl, pts3d, (size_t)N * 24);
    }
    memcpy(h + b_inl + b_pts, hd, sizeof(fmpnp_problem) * n_res);
    e = hipMemcpyAsync(d, h, up, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return drain((int)e);
    e = hipMemsetAsync(d_err, 0, sizeof(int), s);
    if (e != hipSuccess) return drain((int)e);
    if (trace) {
        e = hipMemsetAsync(d_tr, 0, b_tr, s);
        if (e != hipSuccess) return drain((int)e);
    }
    // pack (optimize_feature_pnp.py:57,61): the Sobel pack writes channels < C, so a padded
    // stride is zeroed first; the f-only copy fills the padding itself.  Not for a windowed attempt:
    // its unmarked texels are never trusted anyway (a miss re-runs the call), and no kernel reads a
    // channel >= C (every level's [c_begin, c_end) lies below C), so zeroing the whole map there would
    // only add the full-map write the window exists to avoid
    if (!lay_f && cs != C && !win) {
        e = hipMemsetAsync(d_feat, 0, b_feat, s);
        if (e != hipSuccess) return drain((int)e);
    }
    if (win) {
        // only the texels within window_radius of a point's texel at (R0, t0) (its square in plane 0 of
        // the window map): the refinement reads the texels its points visit, a few from where they
        // start; the LM flags a gather outside the window (FMPNP_STATUS_WINDOW) and the call re-runs
        e = launch_win_mark(d_desc, 1, window_radius, N, (long)H * W, s);
        if (e != hipSuccess) return drain((int)e);
    }
    // with a split, only the first level's channels here; the rest on the side stream below
    e = split ? pack_range(sb, se, s) : pack_range(0, C, s);
    if (e != hipSuccess) return drain((int)e);
    // fref (optimize_feature_pnp.py:51-56): the reference map's first C channels
    if (N > 0) {
        if (cs != C) {
            e = hipMemsetAsync(d_fref, 0, b_fref, s);
            if (e != hipSuccess) return drain((int)e);
        }
        e = launch_gather_ref(ref_chw, dtype_ref, C_ref, H_ref, W_ref, d_inl, N, img0, img1, d_fref, opt->dtype, cs,
                              d_err, s);
        if (e != hipSuccess) return drain((int)e);
    }
    if (split) {
        // the side stream: after the first level's pack and the fref gather, the other channels' pack and
        // compute_cost (which reads every channel); the main stream meets it before the second level
        e = hipEventRecord(sc->ev[0], s);
        if (e == hipSuccess) e = hipStreamWaitEvent(sc->side, sc->ev[0], 0);
        if (e == hipSuccess && sb > 0) e = pack_range(0, sb, sc->side);
        if (e == hipSuccess && se < C) e = pack_range(se, C, sc->side);
        if (e != hipSuccess) return drain((int)e);
        e = launch_compute_cost(hd[0], opt->layout, opt->dtype, opt->use_ratio, opt->ratio_threshold, d_cost, d_sup,
                                d_res, sc->side);
        if (e == hipSuccess) e = hipEventRecord(sc->ev[1], sc->side);
        if (e != hipSuccess) return drain((int)e);
    }
    // the LM launches
    for (int r = 0; r < n_res; ++r) {
        const bool cost = n_levels > 0 && r == 0;
        if (cost) {
            // compute_cost (model.py:216-243): every point's cost at once (one wave each), one
            // fixed-order reduction -- one evaluation, so not an LM launch (a latency chain there)
            // (with a split it runs on the side stream, above)
            if (!split)
                e = launch_compute_cost(hd[0], opt->layout, opt->dtype, opt->use_ratio, opt->ratio_threshold, d_cost,
                                        d_sup, d_res, s);
            if (e != hipSuccess) return drain((int)e);
            continue;
        }
        if (split && r == 2) {
            e = hipStreamWaitEvent(s, sc->ev[1], 0);
            if (e != hipSuccess) return drain((int)e);
        }
        if (n_levels > 0 && r >= 2) {
            // level r - 1 starts from level r - 2's result: R[9], t[3] -> R0[9], t0[3] (contiguous)
            static_assert(offsetof(fmpnp_problem, t0) == offsetof(fmpnp_problem, R0) + 72, "R0, t0 contiguous");
            static_assert(offsetof(fmpnp_result, t) == offsetof(fmpnp_result, R) + 72, "R, t contiguous");
            e = hipMemcpyAsync((unsigned char *)(d_desc + r) + offsetof(fmpnp_problem, R0),
                               (const unsigned char *)(d_res + r - 1) + offsetof(fmpnp_result, R), 96,
                               hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return drain((int)e);
        }
        fmpnp_trace_entry *tr = (trace && !cost) ? d_tr + (size_t)(n_levels > 0 ? r - 1 : 0) * stride : nullptr;
        rc = fmpnp_refine_batch_async(d_desc + r, &hd[r], 1, N, opt, d_res + r, tr, stride, d_ws, ws, hip_stream);
        if (rc) return drain(rc);
    }
    // the one download
    e = hipMemcpyAsync(h, d_res, down, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return drain((int)e);
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return drain((int)e);
    bool miss = false;
    for (int r = 0; r < n_res; ++r) miss = miss || (((const fmpnp_result *)h)[r].status & FMPNP_STATUS_WINDOW);
    if (win && miss) {
        g_window_reruns.fetch_add(1);
        continue;  // a point left its window: every result of this attempt is invalid
    }
    memcpy(results, h, sizeof(fmpnp_result) * n_res);
    if (trace) memcpy(trace, h + b_res + b_err, sizeof(fmpnp_trace_entry) * (size_t)n_fwd * stride);
    const int err = *(const int *)(h + b_res);
    return err ? FMPNP_ERANGE : 0;
  }
    return FMPNP_EINVAL;  // (not reached)
}

extern "C" long long fmpnp_feature_pnp_reruns(void) { return g_window_reruns.load(); }
