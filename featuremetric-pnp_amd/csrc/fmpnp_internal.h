// fmpnp_internal.h -- launch-side definitions shared by the fmpnp HIP sources.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include <mutex>

#include "fmpnp.h"

// Speculative next-texel gathers (fmpnp_lm_impl.h spec_pass; variants VAR_*_SPEC), on the waves
// without an LM-tail role (waves >= spec_w0 = 3: the later wave of each SIMD, which finishes its
// point phase after its SIMD partner, and wave 3, idle in the tail) and at most spec_cap = 2 per
// wave per evaluation, which fit in wave 0's LM tail (round 3, B=128: spec_w0 3 / 4 / 5 / 6
// 0.331 / 0.333 / 0.337 / 0.342 ms; cap 2 0.332 ms, cap 1 / 3 / 4 0.341 / 0.344 / 0.340; every
// wave speculating, the tail waves' blocks adopted by waves 3, 5, 6: 0.385 -- DESIGN.md §4.1.1).
// Build with -DFMPNP_SPEC=0 to compile them out.
#ifndef FMPNP_SPEC
#define FMPNP_SPEC 1
#endif

namespace fmpnp {

constexpr int NT = 512;         // threads per workgroup of the LM kernel (8 waves)
constexpr int CH = 64;          // points per reduction chunk = one wave block (fixed: results do not depend on G)
constexpr int NV = 32;          // reduced vector: 21 H + 6 g + rho + kept + supported + 2 pad
constexpr int NSTAMP = 13;      // debug phase-stamp slots: 8 phases + eval-0 proj/gather/loss/contrib + wave 0 speculation
constexpr int RECW = 8;         // per-point record: 6 channel sums + rho + rho'
constexpr int MAX_G = 64;       // workgroups per problem
// LM kernel builds: WPS_LATENCY = one 512-thread workgroup (8 waves) per problem and per CU;
// WPS_THROUGHPUT = 256-thread workgroups (4 waves, two 64-point blocks per wave at N=512),
// two resident per CU, so one problem's serial LM tail overlaps the other's point work
// (batches of >= 2 problems per CU).  Both keep 2 waves per SIMD: up to 256 VGPRs.
constexpr int WPS_LATENCY = FMPNP_BUILD_LATENCY, WPS_THROUGHPUT = FMPNP_BUILD_THROUGHPUT;
constexpr int NT_THROUGHPUT = 256;
// WPS_WIDE = 256-thread workgroups, one wave per SIMD: up to 512 registers per lane (VGPRs +
// AGPRs), for the bilinear cell memo (its LDS allows one workgroup per CU anyway)
constexpr int WPS_WIDE = FMPNP_BUILD_WIDE;

// Kernel arguments (by value).
struct LaunchArgs {
    const fmpnp_problem *probs;   // device descriptors
    int n;
    fmpnp_options opt;
    fmpnp_result *results;        // device
    fmpnp_trace_entry *trace;     // device or null
    int trace_stride;
    int G, teams, nc_max, gw;     // gw: teams per XCD-mapping group (8, or fewer teams)
    unsigned *counters;           // [teams_pad][16], zeroed every launch
    double *partials;             // [teams][2][nc_max][NV]
    double *maxslots;             // [teams][2][G]
    int mmax;                     // max points per workgroup (multiple of CH): dynamic LDS carve
    unsigned long long *stamps;   // debug: [grid][8 waves][NSTAMP] phase cycle totals, or null
    int wps;                      // occupancy variant (WPS_LATENCY / WPS_THROUGHPUT)
    int spec;                     // speculative next-texel gathers (memoised nearest modes)
    int spec_cap;                 // at most this many speculative gathers per wave per evaluation
    int spec_w0;                  // waves >= spec_w0 speculate (the later wave of each SIMD: 4)
    int dbg;                      // debug knob (FMPNP_DBG): bit 2 per-evaluation stamps, bit 3 helpers
                                  // never publish (exercises the main workgroups' bounded wait)
    // first-evaluation helpers (small batches, one workgroup per problem): workgroups
    // grid_main .. grid_main + n * helpers - 1 gather the initial pose's records of their
    // problem's blocks into hrec and publish each block with a tagged flag (lm_kernel)
    int helpers, grid_main;
    unsigned long long htag;      // this launch's flag value (a process-wide sequence + a magic)
    double *hrec;                 // [n][nc_max * CH][HREC] (six sums, then the texel offset)
    unsigned long long *hflag;    // [n][nc_max]
};
constexpr int HREC = 7;

// Fixed LDS head: the LM state + per-problem context (sized generously, 16-B aligned).
// Debug instrumentation (phase stamps, per-evaluation stamps, the evaluation timeline) exists only
// in a diagnostics build (-DFMPNP_STAMPS=1 on every unit, tools/build_ab.sh); its LDS arrays then
// enlarge the head below, so every unit must see the same value.
#ifndef FMPNP_STAMPS
#define FMPNP_STAMPS 0
#endif
// LDS head of the LM kernel (LMState, fmpnp_lm_impl.h): 2 KB in the product build
__host__ __device__ constexpr int lds_fixed_bytes() { return FMPNP_STAMPS ? 4608 : 2304; }
// row stride (doubles) of the LM kernel's structure-of-arrays LDS records: odd, so the
// writers of one point's fields fall in distinct banks (fmpnp_lm_impl.h lds_X / lds_rec)
__host__ __device__ constexpr int lds_rs(int mmax) { return mmax + 1; }
// speculative next-texel records (fmpnp_lm_impl.h lds_rec2 ...): rec2[6][rs] doubles, and
// 32-bit words for tex, tex2, spec, slot, qp[2] per point (16-B padded); without speculation
// only tex
__host__ __device__ constexpr int lds_spec_doubles(int mmax, bool spec) { return spec ? 6 * lds_rs(mmax) : 0; }
__host__ __device__ constexpr int lds_words(int mmax, bool spec) { return ((spec ? 6 : 1) * mmax + 3) / 4 * 4; }
// bilinear cell memo (fmpnp_lm_impl.h eval_pass_bil): per point the Bernstein coefficients of
// the six channel sums as functions of the position inside the point's 2x2 cell, memo[BIL_NB][rs]
// doubles after the partials.  It bounds a workgroup to BIL_MAX_M points (four 64-point blocks).
constexpr int BIL_NB = 54;
constexpr int BIL_MAX_M = 256;
size_t lm_dyn_lds_bytes(int mmax, int nc_max, bool spec, bool bil_memo = false);

// var: the plan's variant (spec_variant / help_variant already applied)
hipError_t launch_lm(const LaunchArgs &a, int dtype, int var, int grid, size_t lds, hipStream_t stream);
// LM kernel variants (fmpnp_lm_impl.h): Geman-McClure forward with nearest sampling (the
// hot path), any loss / mode with nearest sampling, bilinear sampling
// (the values are the public FMPNP_VAR_* codes of fmpnp_launch_info)
constexpr int VAR_NEAREST = FMPNP_VAR_NEAREST, VAR_GM = FMPNP_VAR_GM, VAR_BILINEAR = FMPNP_VAR_BILINEAR;
// ... and the same two nearest variants on FMPNP_LAYOUT_F maps (fp32 only); bilinear sampling
// without the cell memo (no_memo = 1: every supported point sampled at every evaluation)
constexpr int VAR_F_NEAREST = FMPNP_VAR_F_NEAREST, VAR_F_GM = FMPNP_VAR_F_GM, VAR_BIL_DIRECT = FMPNP_VAR_BIL_DIRECT;
// ... and the two packed nearest variants with the speculative next-texel gathers compiled in
// (the latency build, one workgroup per problem: the planner's P.spec); the other variants are
// built without them, so their code does not pay for speculation they do not run
constexpr int VAR_GM_SPEC = FMPNP_VAR_GM_SPEC, VAR_NEAREST_SPEC = FMPNP_VAR_NEAREST_SPEC;
inline int spec_variant(int var) {
    return var == VAR_GM ? VAR_GM_SPEC : var == VAR_NEAREST ? VAR_NEAREST_SPEC : var;
}
// ... and those two with the first-evaluation helpers' hand-off compiled in (small batches:
// LaunchArgs::helpers; the headline-size batches run without it and without its code)
constexpr int VAR_GM_SPEC_H = FMPNP_VAR_GM_SPEC_H, VAR_NEAREST_SPEC_H = FMPNP_VAR_NEAREST_SPEC_H,
              VAR_GM_H = FMPNP_VAR_GM_H, VAR_NEAREST_H = FMPNP_VAR_NEAREST_H;
// ... and those two compiled for one 512-point workgroup (mmax = 512 at compile time: the LDS carve's
// offsets are immediates, ~25 fewer scalar registers spilled; fp32 texels, the latency build)
constexpr int VAR_GM_SPEC_512 = FMPNP_VAR_GM_SPEC_512, VAR_GM_SPEC_H_512 = FMPNP_VAR_GM_SPEC_H_512;
constexpr int MMAX_512 = 512;
inline int m512_variant(int var) {
    return var == VAR_GM_SPEC ? VAR_GM_SPEC_512 : var == VAR_GM_SPEC_H ? VAR_GM_SPEC_H_512 : var;
}
inline int help_variant(int var) {
    return var == VAR_GM_SPEC ? VAR_GM_SPEC_H : var == VAR_NEAREST_SPEC ? VAR_NEAREST_SPEC_H
         : var == VAR_GM ? VAR_GM_H : var == VAR_NEAREST ? VAR_NEAREST_H : var;
}
// ... and the packed non-speculating ones with the packed-window check compiled in (a window on the
// f, gx, gy planes: fmpnp_feature_pnp's windowed packs); without a window the check's code alone cost
// the non-speculating variants up to 6 %, so the other variants do not carry it
constexpr int VAR_GM_W = FMPNP_VAR_GM_W, VAR_NEAREST_W = FMPNP_VAR_NEAREST_W, VAR_GM_H_W = FMPNP_VAR_GM_H_W,
              VAR_NEAREST_H_W = FMPNP_VAR_NEAREST_H_W;
inline int win_variant(int var) {
    return var == VAR_GM ? VAR_GM_W : var == VAR_NEAREST ? VAR_NEAREST_W : var == VAR_GM_H ? VAR_GM_H_W
         : var == VAR_NEAREST_H ? VAR_NEAREST_H_W : var;
}
// Scratch of the synchronous entry points (fmpnp_refine_batch, fmpnp_feature_pnp), one per (entry
// point, device, stream): SURVEY.md 8b asks for calls that are thread-safe across distinct streams and
// devices, so calls on different streams (or devices) use different buffers and run concurrently, and
// calls on one stream serialise on its mutex (held until the call's stream has drained, so no copy of an
// earlier call still reads the buffers).  Growing frees only the entry's own buffer, stream-ordered on
// its own stream (no device-wide synchronisation, never another device's memory).
struct StreamScratch {
    std::mutex mu;
    unsigned char *dev = nullptr;   // device memory of the entry's device
    size_t dev_bytes = 0;
    unsigned char *host = nullptr;  // pinned staging (fmpnp_feature_pnp)
    size_t host_bytes = 0;
    // fmpnp_feature_pnp's second stream on the entry's device (the channels the first level does not read
    // are packed there, under the first level's LM launch) and its two fences; created on first use
    hipStream_t side = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
};
enum { SCRATCH_REFINE = 0, SCRATCH_QUERY = 1 };
// the entry of (pool, current device, stream); *dev_out: the current device.  nullptr on a HIP error.
StreamScratch *stream_scratch(int pool, hipStream_t s, int *dev_out);
// at least dbytes of device memory and hbytes of pinned host memory (call with c.mu held); 0 or FMPNP_ENOMEM
int scratch_grow(StreamScratch &c, size_t dbytes, size_t hbytes, size_t dmin, hipStream_t s);
// the entry's side stream and events (call with c.mu held, on the entry's device); 0 or a hipError_t
int scratch_side(StreamScratch &c);
int lm_variant(const fmpnp_options &o);
const void *lm_kernel_ptr(int dtype, int wps, bool team, bool ratio, int var);

hipError_t launch_pack(const void *chw, const void *gx, const void *gy, int dtype_in, int C, int H, int W, void *out,
                       int dtype_out, int cs, int normalized, int replicate, hipStream_t stream, int planes = 3);
hipError_t launch_gather_ref(const void *ref, int dtype_in, int C, int H, int W, const double *inl, int N, int img0,
                             int img1, void *out, int dtype_out, int ld_out, int *err, hipStream_t stream);
// the window map of n problems ([2][Hf][Wf] bytes at fmpnp_problem.window): cleared, then every point's
// square of `radius` texels around its texel at (R0, t0) marked in plane 0 (radius - 1 in plane 1)
hipError_t launch_win_mark(const fmpnp_problem *probs_dev, int n, int radius, int max_n, long max_hw, hipStream_t stream);
// fused Sobel + channels-last pack of the texels marked in win ([H][W] bytes, plane 0) only
hipError_t launch_pack_win(const void *chw, int dtype_in, int C, int H, int W, void *out, int dtype_out, int cs,
                           int normalized, int replicate, const unsigned char *win, hipStream_t stream);
// n f-only packs (FMPNP_LAYOUT_F, fp32 out) in ceil(n / 32) launches; shape[4i..] = C, H, W, cstride
hipError_t launch_pack_f_batch(int n, const void *const *chw, void *const *out, const int *shape, int dtype_in,
                               hipStream_t stream);
// windowed f-only packs of n problems (fmpnp_pack_features_f_window_batch): clear the window maps,
// mark each point's initial texel neighbourhood, pack the marked texels
hipError_t launch_pack_f_window(const fmpnp_problem *probs_dev, const fmpnp_problem *probs_host, int n,
                                const void *const *chw, int dtype_in, int radius, int max_n, long max_hw,
                                hipStream_t stream);
// n gathers in ceil(n / 32) launches (item table in the kernel arguments); err: [n] device flags
hipError_t launch_gather_ref_batch(int n, const void *const *ref, const int *ref_shape, const double *const *inl,
                                   const int *n_inl, int img0, int img1, void *const *out, const int *ld_out,
                                   int dtype_in, int dtype_out, int *err, hipStream_t stream);

// per-point 0.5 ||f(p_i) - fref_i||^2 and support at the descriptor's pose (fmpnp_point_costs)
hipError_t launch_point_costs(const fmpnp_problem &p, int layout, int dtype, double *cost, int *supported,
                              hipStream_t stream);
// compute_cost (model.py:216-243) at the descriptor's pose: point costs into cost / supported (device,
// [N] each), then one fixed-order reduction into *out (device): initial_cost, NO_SUPPORT status
hipError_t launch_compute_cost(const fmpnp_problem &p, int layout, int dtype, int use_ratio, double thr,
                               double *cost, int *supported, fmpnp_result *out, hipStream_t stream);
hipError_t launch_cost_mean(const fmpnp_problem &p, int use_ratio, double thr, const double *cost,
                            const int *supported, fmpnp_result *out, hipStream_t stream);

}  // namespace fmpnp
