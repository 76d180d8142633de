// fmpnp_api.hip -- the C ABI of libfmpnp.so (declared in include/fmpnp.h).
//
// Host-side launch planning for the LM kernel: how many workgroups cooperate on a
// problem (G), how many problem teams are resident at once, the dynamic LDS carve
// and the per-team exchange workspace.  No compute happens here; there is no CPU
// fallback of any kernel.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>

#include "fmpnp.h"
#include "fmpnp_internal.h"

using namespace fmpnp;

namespace {

struct Plan {
    int G = 1, teams = 1, teams_pad = 8, gw = 8, grid = 8, nc_max = 1, max_n = 0;
    int mmax = 0, lds = 0, wps = WPS_LATENCY, spec = 0, helpers = 0, grid_main = 8;
    int var = 0, ratio = 0, dtype = 0;  // the kernel variant the launch runs
    size_t ws_counters = 0, ws_partials = 0, ws_max = 0, ws_hrec = 0, ws_hflag = 0, ws_total = 0;
};

thread_local Plan g_last;
unsigned long long *g_stamps = nullptr;  // debug phase stamps for the next launches

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int elem_size(int dtype) { return dtype == FMPNP_F64 ? 8 : 4; }

// Per-problem bounds shared by the LM launch and fmpnp_point_costs: every projected pixel
// maps to a texel < Hf*Wf through 32-bit unsigned products, and the map size is bounded.
int validate_problem(const fmpnp_problem &p, int layout, int sampling) {
    if (p.N < 0 || p.Hf <= 0 || p.Wf <= 0 || p.im_width <= 0 || p.im_height <= 0) return FMPNP_EINVAL;
    if (p.c_begin < 0 || p.c_end < p.c_begin || p.c_end > p.cstride || p.c_end > p.ld_ref) return FMPNP_EINVAL;
    if (p.N > 0 && (!p.feat || !p.fref || !p.pts3d)) return FMPNP_EINVAL;
    if (layout == FMPNP_LAYOUT_F && (p.Hf >= 65536 || p.Wf >= 65536)) return FMPNP_ETOOBIG;
    // a packed window (fmpnp_pack_features_f_window_batch, fmpnp_feature_pnp) is read by nearest
    // sampling's gathers only
    if (p.window && sampling != FMPNP_NEAREST) return FMPNP_EINVAL;
    // bilinear cell keys pack (row + 1, column + 1) into 15 + 16 bits
    if (sampling == FMPNP_BILINEAR && (p.Hf >= 32768 || p.Wf >= 65535)) return FMPNP_ETOOBIG;
    // the packed map must hold 3*cstride per texel
    if ((long long)p.Hf * p.Wf * 3 * (long long)p.cstride > (1LL << 40)) return FMPNP_ETOOBIG;
    // pixel -> texel rescale in 32-bit unsigned arithmetic: y * Hf < 2^32, x * Wf < 2^32
    if ((long long)p.im_height * p.Hf >= (1LL << 32) || (long long)p.im_width * p.Wf >= (1LL << 32))
        return FMPNP_ETOOBIG;
    return 0;
}

int validate(const fmpnp_problem *probs, int n, const fmpnp_options *opt) {
    if (!opt || n < 0 || (n > 0 && !probs)) return FMPNP_EINVAL;
    if (opt->dtype != FMPNP_F32 && opt->dtype != FMPNP_F64) return FMPNP_EINVAL;
    if (opt->loss < FMPNP_SQUARED || opt->loss > FMPNP_BARRON) return FMPNP_EINVAL;
    if (opt->mode != FMPNP_MODE_FORWARD && opt->mode != FMPNP_MODE_COMPUTE_COST) return FMPNP_EINVAL;
    if (opt->sampling != FMPNP_NEAREST && opt->sampling != FMPNP_BILINEAR) return FMPNP_EINVAL;
    if (opt->layout != FMPNP_LAYOUT_FGRAD && opt->layout != FMPNP_LAYOUT_F) return FMPNP_EINVAL;
    // the f-only layout: fp32 texels, nearest sampling (the LM kernel's in-gather Sobel)
    if (opt->layout == FMPNP_LAYOUT_F && (opt->dtype != FMPNP_F32 || opt->sampling != FMPNP_NEAREST))
        return FMPNP_EINVAL;
    if (opt->sobel_flags & ~3) return FMPNP_EINVAL;
    if (opt->no_memo < 0 || opt->no_memo > 2) return FMPNP_EINVAL;
    for (int i = 0; i < n; ++i) {
        const int rc = validate_problem(probs[i], opt->layout, opt->sampling);
        if (rc) return rc;
    }
    return 0;
}

int device_cus(int *ncu) {
    // FMPNP_PLAN_CUS: plan for that many CUs without a device (host-side planner tests, the
    // sanitizer run of tools/sanitize.sh); the occupancy query then falls back to one block per CU
    // (a test knob: on a host with a device it is ignored, with a note, so a stray value never
    // changes a real launch's plan -- workgroups per problem, helpers -- or breaks the planner's
    // all-resident assumption)
    if (const char *fc = getenv("FMPNP_PLAN_CUS")) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
            (void)hipGetLastError();
            *ncu = std::max(1, atoi(fc));
            return 0;
        }
        static std::once_flag note;
        std::call_once(note, [] { fprintf(stderr, "fmpnp: FMPNP_PLAN_CUS ignored (a device is present)\n"); });
    }
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    e = hipDeviceGetAttribute(ncu, hipDeviceAttributeMultiprocessorCount, dev);
    return (int)e;
}

int make_plan(const fmpnp_problem *probs, int n, const fmpnp_options *opt, Plan *pl) {
    int rc = validate(probs, n, opt);
    if (rc) return rc;
    Plan P;
    P.max_n = 0;
    for (int i = 0; i < n; ++i) P.max_n = std::max(P.max_n, probs[i].N);
    P.nc_max = std::max(1, (P.max_n + CH - 1) / CH);
    int ncu = 256;
    rc = device_cus(&ncu);
    if (rc) return rc;
    const int lds_cu = 160 * 1024;  // LDS per CU
    // speculative next-texel gathers (fmpnp_lm_impl.h spec_pass): memoised nearest sampling of
    // a forward run; no_memo = 2 keeps the memo without them (a measurement knob)
    // (the f-only layout's nine-texel gathers are too heavy to hide: B=128 0.68 -> 0.75 ms with it)
    // Only where it pays (measured): every problem's channel slice within one 16-byte round per
    // half-wave lane (C <= 64 V: 256 fp32 channels; at C = 512 the gathers outgrow wave 0's
    // tail, 0.437 vs 0.415 ms on the pyramid's coarse level) and, below, one workgroup per
    // problem on the latency build (a team's waves 4-7 own no block at these sizes).
    int max_span = 0;
    for (int i = 0; i < n; ++i) max_span = std::max(max_span, probs[i].c_end - probs[i].c_begin);
    static const int spec_maxc = [] { const char *e = getenv("FMPNP_SPEC_MAXC"); return e ? atoi(e) : 0; }();
    const int maxc = spec_maxc > 0 ? spec_maxc : 64 * (16 / elem_size(opt->dtype));  // (measurement knob)
    // packed windows (fmpnp_feature_pnp, the windowed f-only packs): the speculative gathers would read
    // predicted texels outside the window, so they are off (variants that withdraw such predictions were
    // measured slower on the RobotCar call, 1.290 -> 1.311 ms: profiles/r06_spec_window_ab.txt)
    bool windows = false;
    for (int i = 0; i < n; ++i) windows = windows || probs[i].window != nullptr;
    P.spec = (FMPNP_SPEC && !windows && opt->no_memo == 0 && opt->sampling == FMPNP_NEAREST &&
              opt->mode == FMPNP_MODE_FORWARD && opt->layout == FMPNP_LAYOUT_FGRAD && max_span <= maxc) ? 1 : 0;
    // bilinear sampling keeps each point's cell memo in LDS (at most BIL_MAX_M points per
    // workgroup) unless no_memo asks for every point sampled every evaluation
    const bool bil_memo = opt->sampling == FMPNP_BILINEAR && opt->no_memo != 1;
    auto m_for = [&](int G) { return ((P.nc_max + G - 1) / G) * CH; };
    auto lds_for = [&](int G) {
        return lds_fixed_bytes() + (int)lm_dyn_lds_bytes(m_for(G), P.nc_max, P.spec != 0, bil_memo);
    };
    auto fits = [&](int G) { return lds_for(G) <= lds_cu && (!bil_memo || m_for(G) <= BIL_MAX_M); };
    // resident workgroups per CU (VGPR and LDS limits).  Hardware admission of 256-thread
    // blocks is also bounded by SGPRs: floor(800 / (ceil(sgpr/16)*16 + 16)) >= 6 for any
    // kernel (<= 112 SGPRs incl. VCC), and the API over-reports only above that
    // (MI355X_MICROARCH.md, Residency) -> min(api, 6).
    auto occupancy = [&](int lds) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb,
                                                         lm_kernel_ptr(opt->dtype, P.wps, P.G > 1,
                                                                       opt->use_ratio != 0,
                                                                       P.spec ? spec_variant(lm_variant(*opt))
                                                                              : lm_variant(*opt)),
                                                         P.wps == WPS_LATENCY ? NT : NT_THROUGHPUT, lds) !=
            hipSuccess)
            return 1;
        return std::max(1, std::min(nb, 6));
    };
    // workgroups per problem: one while the batch covers at least half of the CUs (a
    // team member saves less per evaluation than its cross-workgroup exchange costs:
    // measured B=128 on 256 CUs, G=1 0.367 ms vs G=2 0.386 ms; per evaluation a lone wave's
    // point phase is 6.7k cycles either way and the exchange ~3.6k); smaller batches spread
    // each problem so that the teams cover every CU.  Bounded by the chunks of the
    // largest problem and by what fits in LDS at the resulting density.
    int G;
    if (opt->wgs_per_problem > 0) {
        G = std::min(opt->wgs_per_problem, P.nc_max);
    } else {
        // (no_memo re-reads every texel each evaluation: bandwidth-bound, so every CU gets a
        // workgroup; bilinear without the memo at B=128: G=2 7.32 ms vs G=1 7.75 ms)
        const bool streaming = opt->no_memo == 1;
        G = (n <= 0 || (2L * n >= ncu && !streaming)) ? 1 : (ncu + n - 1) / n;
        // memoised packed-gradient loop on problems of <= 512 points: the evaluation is a
        // latency chain and a member's exchange costs about what the split saves, so one
        // workgroup per problem however small the batch (cfg2, ms per launch, G=1 vs the
        // spread-out G=8: B=8 0.307 vs 0.326, B=16 0.311 vs 0.328, B=32 0.315 vs 0.332,
        // B=1 0.305 vs 0.313).  Larger problems keep spreading (cfg5, 2048 points at
        // C=512: G=4 0.64 ms vs G=32 0.58 ms at B=1)
        // (not bilinear: its memo builds are VALU work that more CUs share)
        // (compute_cost is ONE evaluation in which every point gathers: bandwidth, not a latency
        // chain, so it keeps the spread -- RobotCar C = 1664, 295 points: one workgroup 184 us)
        if (!streaming && !bil_memo && opt->layout == FMPNP_LAYOUT_FGRAD && P.nc_max <= 8 &&
            opt->mode == FMPNP_MODE_FORWARD)
            G = 1;
        G = std::max(1, std::min(G, P.nc_max));
    }
    G = std::min(G, MAX_G);
    // packed windows: one workgroup per problem (a window miss stops the problem inside its
    // workgroup, fmpnp_lm_impl.h eval_pass; a team would wait on the stopped member)
    // (packed f, gx, gy planes: the miss is only flagged and the problem finishes, so teams stay)
    if (windows && opt->layout == FMPNP_LAYOUT_F) G = 1;
    while (!(windows && opt->layout == FMPNP_LAYOUT_F) && G < std::min(P.nc_max, MAX_G) && !fits(G)) ++G;
    if (!fits(G)) return FMPNP_ETOOBIG;
    P.G = G;
    P.mmax = ((P.nc_max + G - 1) / G) * CH;
    P.lds = lds_for(G);
    // build: with more problems than CUs the throughput build (256-thread workgroups,
    // two per CU: one problem's LM tail overlaps the other's point work) -- one workgroup per
    // problem, no speculation (its LDS would not leave room for two workgroups, and with every
    // CU busy there is no idle memory time to hide it in).  FMPNP_LM_WPS=2|4 forces a build.
    const char *wps_env = getenv("FMPNP_LM_WPS");
    const int want = wps_env ? atoi(wps_env) : 0;
    const bool tp_ok = !bil_memo && !windows && opt->layout == FMPNP_LAYOUT_FGRAD && G == 1 && (long)n >= ncu &&
                       2 * (lds_fixed_bytes() + (int)lm_dyn_lds_bytes(P.mmax, P.nc_max, false, bil_memo)) <= lds_cu;
    // (from more problems than CUs on: a second round of one-per-CU latency workgroups costs more than
    // two throughput workgroups per CU -- ms per launch at B = 288 / 384 / 448 on 256 CUs: 0.684 / 0.700 /
    // 0.721 latency against 0.580 / 0.606 / 0.632 throughput, profiles/r05_wps_mid_batch.txt)
    const bool tp = tp_ok && (want == WPS_THROUGHPUT || (want == 0 && (long)n > ncu));
    P.wps = tp ? WPS_THROUGHPUT : WPS_LATENCY;
    if (bil_memo) P.wps = WPS_WIDE;  // the memo build's registers: one wave per SIMD
    if (tp || G > 1) {
        P.spec = 0;
        P.lds = lds_for(G);
    }
    const int per_cu = occupancy(P.lds);
    long cap = (long)ncu * per_cu;
    if (G == 1) cap = std::max(cap, (long)n);  // no cross-workgroup waits: any grid is safe
    long max_teams = cap / G;
    if (opt->max_teams > 0) max_teams = std::min<long>(max_teams, opt->max_teams);
    // teams are padded to a multiple of the mapping group (8, the XCD count, or fewer
    // teams) for the XCD-aware blockIdx mapping; the padded grid stays within the
    // resident capacity whenever team members wait on each other (G > 1)
    long teams = std::min<long>(std::max(n, 1), max_teams);
    auto padded = [](long t) { long gw = t >= 8 ? 8 : t; return ((t + gw - 1) / gw) * gw; };
    while (teams > 1 && G > 1 && padded(teams) * G > cap) --teams;
    if (teams < 1 || (G > 1 && padded(teams) * G > cap)) return FMPNP_ETOOBIG;
    P.teams = (int)teams;
    P.gw = teams >= 8 ? 8 : (int)teams;
    P.teams_pad = (int)padded(teams);
    P.grid = P.teams_pad * G;
    P.ws_counters = align_up((size_t)P.teams_pad * 16 * sizeof(unsigned), 256);
    P.ws_partials = align_up((size_t)P.teams * 2 * P.nc_max * NV * sizeof(double), 256);
    P.ws_max = align_up((size_t)P.teams * 2 * G * sizeof(double), 256);
    // first-evaluation helpers: with every problem on one resident workgroup and idle CUs left
    // (grid + n * H <= CUs), H more workgroups per problem gather the initial pose's texels of
    // its 64-point blocks, so the first evaluation (all N points dirty) is spread over 1 + H
    // CUs (ms per launch without / with them: B = 1 0.298 / 0.279, B = 8 0.305 / 0.289,
    // B = 32 0.310 / 0.302, B = 64 0.341 / 0.333); FMPNP_HELPERS=0 switches them off
    P.grid_main = P.grid;
    {
        // opt->helpers < 0 switches them off (callers sharing the device with other kernels),
        // > 0 caps them; FMPNP_HELPERS=0 (environment) switches them off too
        const char *eh = getenv("FMPNP_HELPERS");
        const bool on = (!eh || atoi(eh) != 0) && opt->helpers >= 0;
        // (helpers beside the padded main grid, all resident at once: the mains wait on them)
        long spare = ((long)ncu - P.grid) / std::max(n, 1);
        // (packed nearest memoised forward runs; a single helper per problem -- B > CUs/3 -- measured
        // slower at B = 128: 0.380 vs 0.360 ms, the first evaluation being HBM-bound there)
        if (on && G == 1 && P.wps == WPS_LATENCY && !bil_memo && opt->sampling == FMPNP_NEAREST &&
            opt->no_memo != 1 && opt->mode == FMPNP_MODE_FORWARD && opt->layout == FMPNP_LAYOUT_FGRAD &&
            P.teams == n && P.nc_max >= 2 && spare >= 2)
            P.helpers = (int)std::min<long>(std::min<long>(std::min<long>(spare, P.nc_max), 8),
                                            opt->helpers > 0 ? opt->helpers : 8);
    }
    P.grid = P.grid_main + n * P.helpers;
    P.ws_hrec = P.helpers ? align_up((size_t)n * P.nc_max * CH * HREC * sizeof(double), 256) : 0;
    P.ws_hflag = P.helpers ? align_up((size_t)n * P.nc_max * sizeof(unsigned long long), 256) : 0;
    P.ws_total = P.ws_counters + P.ws_partials + P.ws_max + P.ws_hrec + P.ws_hflag;
    P.var = P.spec ? spec_variant(lm_variant(*opt)) : lm_variant(*opt);
    if (P.helpers) P.var = help_variant(P.var);
    // one 512-point workgroup per problem (N in 449..512, fp32): the compile-time carve (B = 128: 0.3222 ->
    // 0.3174 ms, single query 0.2513 -> 0.2424 ms, interleaved x3, profiles/r06_ab_m512.txt)
    if (P.mmax == MMAX_512 && G == 1 && P.wps == WPS_LATENCY && opt->dtype == FMPNP_F32) P.var = m512_variant(P.var);
    // (packed windows: the variant with the window check; the f-only variants always carry theirs)
    if (windows && opt->layout == FMPNP_LAYOUT_FGRAD) P.var = win_variant(P.var);
    P.ratio = opt->use_ratio != 0;
    P.dtype = opt->dtype;
    *pl = P;
    return 0;
}

}  // namespace

namespace fmpnp {

StreamScratch *stream_scratch(int pool, hipStream_t s, int *dev_out) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    if (dev_out) *dev_out = dev;
    static std::mutex mu;
    static std::map<std::tuple<int, int, uintptr_t>, std::unique_ptr<StreamScratch>> pools;
    std::lock_guard<std::mutex> lock(mu);  // (the lookup only: each entry has its own mutex)
    std::unique_ptr<StreamScratch> &e = pools[std::make_tuple(pool, dev, (uintptr_t)s)];
    if (!e) e.reset(new StreamScratch());
    return e.get();
}

int scratch_grow(StreamScratch &c, size_t dbytes, size_t hbytes, size_t dmin, hipStream_t s) {
    if (c.dev_bytes < dbytes) {
        // (the entry's earlier calls drained this stream before returning: nothing still reads it)
        if (c.dev) (void)hipFreeAsync(c.dev, s);
        c.dev = nullptr;
        c.dev_bytes = 0;
        const size_t b = std::max(dbytes, dmin);
        if (hipMallocAsync((void **)&c.dev, b, s) != hipSuccess) {
            c.dev = nullptr;
            return FMPNP_ENOMEM;
        }
        c.dev_bytes = b;
    }
    if (c.host_bytes < hbytes) {
        if (c.host) (void)hipHostFree(c.host);
        c.host = nullptr;
        c.host_bytes = 0;
        const size_t b = std::max(hbytes, (size_t)1 << 20);
        if (hipHostMalloc((void **)&c.host, b, hipHostMallocDefault) != hipSuccess) {
            c.host = nullptr;
            return FMPNP_ENOMEM;
        }
        c.host_bytes = b;
    }
    return 0;
}

int scratch_side(StreamScratch &c) {
    hipError_t e = hipSuccess;
    if (!c.side) e = hipStreamCreateWithFlags(&c.side, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; ++i)
        if (!c.ev[i]) e = hipEventCreateWithFlags(&c.ev[i], hipEventDisableTiming);
    return (int)e;
}

}  // namespace fmpnp

extern "C" {

int fmpnp_abi_version(void) { return FMPNP_ABI_VERSION; }

#define FMPNP_STR2(x) #x
#define FMPNP_STR(x) FMPNP_STR2(x)
#ifndef FMPNP_SOURCE_DIGEST
#define FMPNP_SOURCE_DIGEST "unknown"  // (builds outside the Makefile, e.g. tools/build_ab.sh)
#endif
const char *fmpnp_build_info(void) {
    return "fmpnp gfx950: lm_kernel(NT=512 wave-owned blocks, CH=64, NV=32, fp64 accumulation, bilinear cell memo), "
           "pack_kernel(Sobel+HWC3), gather_ref_kernel; speculative_gathers=" FMPNP_STR(FMPNP_SPEC)
           "; source_digest=" FMPNP_SOURCE_DIGEST;
}

int fmpnp_device_check(int device) {
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return (int)e;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return FMPNP_ENODEV;
    return 0;
}

int fmpnp_pack_features(const void *chw, const void *gx_chw, const void *gy_chw, int dtype_in, int C, int H, int W,
                        void *out, int dtype_out, int cstride, int sobel_normalized, int sobel_replicate_pad,
                        void *hip_stream) {
    if (!chw || !out || C <= 0 || H <= 0 || W <= 0 || cstride < C) return FMPNP_EINVAL;
    if ((gx_chw == nullptr) != (gy_chw == nullptr)) return FMPNP_EINVAL;
    if ((dtype_in != FMPNP_F32 && dtype_in != FMPNP_F64) || (dtype_out != FMPNP_F32 && dtype_out != FMPNP_F64))
        return FMPNP_EINVAL;
    return (int)launch_pack(chw, gx_chw, gy_chw, dtype_in, C, H, W, out, dtype_out, cstride, sobel_normalized,
                            sobel_replicate_pad, (hipStream_t)hip_stream);
}

static bool gather_args_ok(const void *ref_chw, int C, int H_ref, int W_ref, const double *ref_inliers, int N,
                           int img0, int img1, const void *out, int ld_out) {
    return ref_chw && ref_inliers && out && C > 0 && H_ref > 0 && W_ref > 0 && N > 0 && ld_out >= C && img0 > 0 &&
           img1 > 0;
}

int fmpnp_gather_reference_async(const void *ref_chw, int dtype_in, int C, int H_ref, int W_ref,
                                 const double *ref_inliers, int N, int img0, int img1, void *out, int dtype_out,
                                 int ld_out, int *err_flag, void *hip_stream) {
    if (N == 0) return 0;
    if (!err_flag || !gather_args_ok(ref_chw, C, H_ref, W_ref, ref_inliers, N, img0, img1, out, ld_out))
        return FMPNP_EINVAL;
    return (int)launch_gather_ref(ref_chw, dtype_in, C, H_ref, W_ref, ref_inliers, N, img0, img1, out, dtype_out,
                                  ld_out, err_flag, (hipStream_t)hip_stream);
}

int fmpnp_gather_reference(const void *ref_chw, int dtype_in, int C, int H_ref, int W_ref, const double *ref_inliers,
                           int N, int img0, int img1, void *out, int dtype_out, int ld_out, void *hip_stream) {
    if (N == 0) return 0;
    if (!gather_args_ok(ref_chw, C, H_ref, W_ref, ref_inliers, N, img0, img1, out, ld_out)) return FMPNP_EINVAL;
    hipStream_t s = (hipStream_t)hip_stream;
    int *err = nullptr;
    hipError_t e = hipMallocAsync((void **)&err, sizeof(int), s);
    if (e != hipSuccess) return (int)e;
    (void)hipMemsetAsync(err, 0, sizeof(int), s);
    e = launch_gather_ref(ref_chw, dtype_in, C, H_ref, W_ref, ref_inliers, N, img0, img1, out, dtype_out, ld_out, err,
                          s);
    int herr = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&herr, err, sizeof(int), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFreeAsync(err, s);
    if (e != hipSuccess) return (int)e;
    return herr ? FMPNP_EINVAL : 0;  // an inlier outside the reference map (reference: IndexError)
}

int fmpnp_point_costs(const fmpnp_problem *prob, int layout, int dtype, double *cost, int *supported,
                      void *hip_stream) {
    if (!prob || !cost || !supported) return FMPNP_EINVAL;
    const fmpnp_problem &p = *prob;
    if (p.N == 0) return 0;
    if (layout != FMPNP_LAYOUT_FGRAD && layout != FMPNP_LAYOUT_F) return FMPNP_EINVAL;
    if (p.c_end <= p.c_begin) return FMPNP_EINVAL;
    const int rc = validate_problem(p, layout, FMPNP_NEAREST);  // the LM path's bounds (32-bit texel rescale)
    if (rc) return rc;
    if (dtype != FMPNP_F32 && dtype != FMPNP_F64) return FMPNP_EINVAL;
    if (layout == FMPNP_LAYOUT_F && dtype != FMPNP_F32) return FMPNP_EINVAL;
    return (int)launch_point_costs(p, layout, dtype, cost, supported, (hipStream_t)hip_stream);
}

int fmpnp_pack_features_f(const void *chw, int dtype_in, int C, int H, int W, void *out, int dtype_out,
                          int cstride, void *hip_stream) {
    if (!chw || !out || C <= 0 || H <= 0 || W <= 0 || cstride < C || cstride % 4) return FMPNP_EINVAL;
    if ((dtype_in != FMPNP_F32 && dtype_in != FMPNP_F64) || dtype_out != FMPNP_F32) return FMPNP_EINVAL;
    if ((uintptr_t)out % 16) return FMPNP_EALIGN;
    return (int)launch_pack(chw, nullptr, nullptr, dtype_in, C, H, W, out, dtype_out, cstride, 0, 0,
                            (hipStream_t)hip_stream, 1);
}

int fmpnp_pack_features_batch(int n, const void *const *chw, void *const *out, const int *shape, int dtype_in,
                              int dtype_out, int sobel_normalized, int sobel_replicate_pad, int layout,
                              void *hip_stream) {
    if (n < 0 || (n > 0 && (!chw || !out || !shape))) return FMPNP_EINVAL;
    if (layout != FMPNP_LAYOUT_FGRAD && layout != FMPNP_LAYOUT_F) return FMPNP_EINVAL;
    if ((dtype_in != FMPNP_F32 && dtype_in != FMPNP_F64) || (dtype_out != FMPNP_F32 && dtype_out != FMPNP_F64))
        return FMPNP_EINVAL;
    if (layout == FMPNP_LAYOUT_F && dtype_out != FMPNP_F32) return FMPNP_EINVAL;
    for (int i = 0; i < n; ++i) {  // every item checked before anything is launched
        const int *sh = shape + 4 * i;
        if (!chw[i] || !out[i] || sh[0] <= 0 || sh[1] <= 0 || sh[2] <= 0 || sh[3] < sh[0]) return FMPNP_EINVAL;
        if (layout == FMPNP_LAYOUT_F && (sh[3] % 4 || (uintptr_t)out[i] % 16)) return FMPNP_EINVAL;
    }
    if (layout == FMPNP_LAYOUT_F) {  // one launch per 32 maps
        static const int via_sobel = [] { const char *e = getenv("FMPNP_PACK_F_SOBEL"); return e && *e == '1'; }();
        if (!via_sobel) return (int)launch_pack_f_batch(n, chw, out, shape, dtype_in, (hipStream_t)hip_stream);
    }
    for (int i = 0; i < n; ++i) {
        const int *sh = shape + 4 * i;
        const hipError_t e = launch_pack(chw[i], nullptr, nullptr, dtype_in, sh[0], sh[1], sh[2], out[i], dtype_out,
                                         sh[3], sobel_normalized, sobel_replicate_pad, (hipStream_t)hip_stream,
                                         layout == FMPNP_LAYOUT_F ? 1 : 3);
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

int fmpnp_pack_features_f_window_batch(const fmpnp_problem *probs_dev, const fmpnp_problem *probs_host, int n,
                                       const void *const *chw, int dtype_in, int radius, void *hip_stream) {
    if (n < 0 || (n > 0 && (!probs_dev || !probs_host || !chw))) return FMPNP_EINVAL;
    if ((dtype_in != FMPNP_F32 && dtype_in != FMPNP_F64) || radius < 2 || radius > 4096) return FMPNP_EINVAL;
    int max_n = 0;
    long max_hw = 0;
    for (int i = 0; i < n; ++i) {  // every item checked before anything is launched
        const fmpnp_problem &p = probs_host[i];
        const int rc = validate_problem(p, FMPNP_LAYOUT_F, FMPNP_NEAREST);
        if (rc) return rc;
        if (!chw[i] || !p.feat || !p.window || p.c_begin != 0 || p.c_end <= 0 || p.cstride % 4 ||
            (uintptr_t)p.feat % 16 || (p.N > 0 && !p.pts3d))
            return FMPNP_EINVAL;
        max_n = std::max(max_n, p.N);
        max_hw = std::max(max_hw, (long)p.Hf * p.Wf);
    }
    if (n == 0) return 0;
    return (int)launch_pack_f_window(probs_dev, probs_host, n, chw, dtype_in, radius, max_n, max_hw,
                                     (hipStream_t)hip_stream);
}

int fmpnp_gather_reference_batch(int n, const void *const *ref_chw, const int *ref_shape,
                                 const double *const *ref_inliers, const int *n_inliers, int img0, int img1,
                                 void *const *out, const int *ld_out, int dtype_in, int dtype_out, int *err_flags,
                                 void *hip_stream) {
    if (n < 0 || (n > 0 && (!ref_chw || !ref_shape || !ref_inliers || !n_inliers || !out || !ld_out || !err_flags)))
        return FMPNP_EINVAL;
    for (int i = 0; i < n; ++i) {
        const int *sh = ref_shape + 3 * i;
        if (n_inliers[i] < 0) return FMPNP_EINVAL;
        if (n_inliers[i] > 0 &&
            !gather_args_ok(ref_chw[i], sh[0], sh[1], sh[2], ref_inliers[i], n_inliers[i], img0, img1, out[i], ld_out[i]))
            return FMPNP_EINVAL;
    }
    {
        const hipError_t e = launch_gather_ref_batch(n, ref_chw, ref_shape, ref_inliers, n_inliers, img0, img1, out,
                                                     ld_out, dtype_in, dtype_out, err_flags, (hipStream_t)hip_stream);
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

size_t fmpnp_workspace_size(const fmpnp_problem *probs_host, int n, const fmpnp_options *opt) {
    Plan P;
    if (make_plan(probs_host, n, opt, &P)) return 0;
    return P.ws_total;
}

int fmpnp_refine_batch_async(const fmpnp_problem *probs_dev, const fmpnp_problem *probs_host, int n, int max_N,
                             const fmpnp_options *opt, fmpnp_result *results_dev, fmpnp_trace_entry *trace_dev,
                             int trace_stride, void *workspace, size_t workspace_bytes, void *hip_stream) {
    (void)max_N;
    if (n == 0) return 0;
    if (!probs_dev || !probs_host || !results_dev) return FMPNP_EINVAL;
    Plan P;
    int rc = make_plan(probs_host, n, opt, &P);
    if (rc) return rc;
    if (workspace_bytes < P.ws_total || (!workspace && P.ws_total)) return FMPNP_ENOMEM;
    hipStream_t s = (hipStream_t)hip_stream;
    LaunchArgs a;
    a.probs = probs_dev;
    a.n = n;
    a.opt = *opt;
    a.results = results_dev;
    a.trace = trace_dev;
    a.trace_stride = trace_dev ? trace_stride : 0;
    a.G = P.G;
    a.teams = P.teams;
    a.nc_max = P.nc_max;
    a.gw = P.gw;
    unsigned char *ws = (unsigned char *)workspace;
    a.counters = (unsigned *)ws;
    a.partials = (double *)(ws + P.ws_counters);
    a.maxslots = (double *)(ws + P.ws_counters + P.ws_partials);
    a.helpers = P.helpers;
    a.grid_main = P.grid_main;
    a.hrec = (double *)(ws + P.ws_counters + P.ws_partials + P.ws_max);
    a.hflag = (unsigned long long *)(ws + P.ws_counters + P.ws_partials + P.ws_max + P.ws_hrec);
    {
        // flags from earlier launches carry smaller sequence numbers; the magic high bits keep
        // any other bytes the workspace held from matching
        static std::atomic<unsigned long long> seq{0};
        const unsigned long long sq = ++seq;
        a.htag = 0xF3A9000000000000ull | (sq & 0xFFFFFFFFFFFFull);
    }
    a.mmax = P.mmax;
    a.stamps = g_stamps;
    a.wps = P.wps;
    a.spec = P.spec;
    {
        // speculative gathers per wave per evaluation (waves >= 1 gather during wave 0's LM tail:
        // more than fit in it would delay the evaluation's closing barrier)
        // (read per launch: measurement and test knobs, FMPNP_SPEC_CAP / FMPNP_SPEC_W0)
        const char *ec = getenv("FMPNP_SPEC_CAP"), *ew = getenv("FMPNP_SPEC_W0");
        a.spec_cap = ec ? std::max(0, atoi(ec)) : 2;
        a.spec_w0 = ew ? std::max(0, atoi(ew)) : 3;  // round 3: wave 3 (no tail role) speculates too
    }
    {
        const char *e = getenv("FMPNP_DBG");  // debug knob, read per launch (fmpnp_internal.h LaunchArgs::dbg)
        a.dbg = e ? atoi(e) : 0;
    }
    // teams of G > 1 workgroups count their arrivals and add their texel gathers into zeroed
    // memory; with G = 1 the kernel writes every result field itself and nothing is zeroed
    hipError_t e = hipSuccess;
    if (P.G > 1) {
        e = hipMemsetAsync(a.counters, 0, P.ws_counters, s);
        if (e != hipSuccess) return (int)e;
        e = hipMemsetAsync(results_dev, 0, sizeof(fmpnp_result) * (size_t)n, s);  // texel_gathers accumulate
        if (e != hipSuccess) return (int)e;
    }
    e = launch_lm(a, opt->dtype, P.var, P.grid, (size_t)P.lds, s);
    g_last = P;
    return (int)e;
}

int fmpnp_refine_batch(const fmpnp_problem *probs_host, int n, const fmpnp_options *opt, fmpnp_result *results,
                       fmpnp_trace_entry *trace, int trace_stride, void *hip_stream) {
    if (n == 0) return 0;
    if (!probs_host || !results) return FMPNP_EINVAL;
    Plan P;
    int rc = make_plan(probs_host, n, opt, &P);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)hip_stream;
    const size_t b_probs = align_up(sizeof(fmpnp_problem) * n, 256);
    const size_t b_res = align_up(sizeof(fmpnp_result) * n, 256);
    const size_t b_tr = trace ? align_up(sizeof(fmpnp_trace_entry) * (size_t)n * trace_stride, 256) : 0;
    const size_t need = b_probs + b_res + b_tr + P.ws_total;
    StreamScratch *sc = stream_scratch(SCRATCH_REFINE, s, nullptr);
    if (!sc) return FMPNP_ENODEV;
    std::lock_guard<std::mutex> lock(sc->mu);  // (one call at a time on this stream)
    if (scratch_grow(*sc, need, 0, (size_t)1 << 20, s)) return FMPNP_ENOMEM;
    unsigned char *base = sc->dev;
    fmpnp_problem *d_probs = (fmpnp_problem *)base;
    fmpnp_result *d_res = (fmpnp_result *)(base + b_probs);
    fmpnp_trace_entry *d_tr = trace ? (fmpnp_trace_entry *)(base + b_probs + b_res) : nullptr;
    void *d_ws = base + b_probs + b_res + b_tr;
    // an error once work is queued: wait for the stream before returning, so that the scratch is never
    // reused by the next call on this stream while a copy or launch of this one is still in flight
    auto drain = [s](int code) {
        (void)hipStreamSynchronize(s);
        return code;
    };
    hipError_t e = hipMemcpyAsync(d_probs, probs_host, sizeof(fmpnp_problem) * n, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return drain((int)e);
    if (d_tr) {
        e = hipMemsetAsync(d_tr, 0, b_tr, s);
        if (e != hipSuccess) return drain((int)e);
    }
    rc = fmpnp_refine_batch_async(d_probs, probs_host, n, P.max_n, opt, d_res, d_tr, trace_stride, d_ws, P.ws_total,
                                  hip_stream);
    if (rc) return drain(rc);
    e = hipMemcpyAsync(results, d_res, sizeof(fmpnp_result) * n, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return drain((int)e);
    if (trace) {
        e = hipMemcpyAsync(trace, d_tr, sizeof(fmpnp_trace_entry) * (size_t)n * trace_stride, hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return drain((int)e);
    }
    e = hipStreamSynchronize(s);
    return (int)e;
}

int fmpnp_debug_stamps(unsigned long long *device_buf) {
    g_stamps = device_buf;
    return 0;
}

int fmpnp_last_launch(int *teams, int *wgs_per_problem, int *grid, int *lds_bytes) {
    if (teams) *teams = g_last.teams;
    if (wgs_per_problem) *wgs_per_problem = g_last.G;
    if (grid) *grid = g_last.grid;
    if (lds_bytes) *lds_bytes = g_last.lds;
    return 0;
}

static void plan_info(const Plan &P, fmpnp_launch_info *o) {
    o->teams = P.teams;
    o->wgs_per_problem = P.G;
    o->grid = P.grid;
    o->lds_bytes = P.lds;
    o->build = P.wps;
    o->variant = P.var;
    o->team = P.G > 1;
    o->ratio = P.ratio;
    o->dtype = P.dtype;
    o->helpers = P.helpers;
    o->speculate = P.spec;
}

int fmpnp_plan(const fmpnp_problem *probs_host, int n, const fmpnp_options *opt, fmpnp_launch_info *out) {
    if (!out || n <= 0 || !probs_host) return FMPNP_EINVAL;
    Plan P;
    const int rc = make_plan(probs_host, n, opt, &P);
    if (rc) return rc;
    plan_info(P, out);
    return 0;
}

int fmpnp_last_launch_info(fmpnp_launch_info *out) {
    if (!out) return FMPNP_EINVAL;
    plan_info(g_last, out);
    return 0;
}

}  // extern "C"
