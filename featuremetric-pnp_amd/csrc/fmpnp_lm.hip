// fmpnp_lm.hip -- the feature-metric LM refiner on gfx950 (MI355X).
//
// One launch runs the WHOLE Levenberg-Marquardt loop of every problem of a batch
// (sparseFeaturePnP.forward, featurePnP/model.py:245-494) on the device.
//
// Work decomposition
//   * A "team" of G workgroups (512 threads = 8 waves each) owns one problem at a time;
//     teams walk the batch persistently (problem = team, team + T, ...).
//   * Points are cut into chunks of CH = 16; workgroup s of a team owns a contiguous
//     range of chunks, and wave w of the workgroup owns the 64-point blocks w, w+8, ...
//     of that range.  Per evaluation a wave carries each of its blocks from projection
//     to chunk partials with NO workgroup barrier:
//       project  (lane per point, fp64, exact pixel rounding) -> texel offset, P;
//       gather   the points whose texel changed (ballot), two per wave: each half-wave
//                issues 16-byte loads of the channels-last [H][W][3][C] texel and fref
//                and reduces the six channel sums  sum e^2, sum gx e, sum gy e, sum gx^2,
//                sum gx gy, sum gy^2  in fp64 (the C x 6 Jacobian is never materialised:
//                J = G A with the 2x6 pose chain A, so J^T e = A^T (G^T e),
//                J^T J = A^T (G^T G) A); unchanged texels keep their sums (memoisation);
//       loss + normal equations (lane per point) -> 21 + 6 entries, rho and counters,
//                reduced per 16-point chunk by a fixed transposed DPP tree.
//   * The chunk partials are summed by wave 0 with a fixed tree over CHUNK INDICES.  Results
//     are therefore deterministic and independent of G: the LM accept test `new > prev`
//     (model.py:469-472) compares costs that tie exactly whenever the pixel sets are
//     equal, and a scheduling-dependent sum would break those ties.
//   * G > 1: chunk partials go to a per-team slot with write-through (sc1) stores,
//     every storing wave drains, one lane bumps the team's arrival counter, one lane
//     polls it (bounded spin), one agent-scope acquire; then wave 0 of every member
//     reads all partials and runs the identical 6x6 solve + LM update (no second exchange).
//   * One evaluation per iteration: the trial evaluation at (R', t') also produces that
//     pose's normal equations.  On acceptance they are the next linearisation; on
//     rejection the cached ones are reused -- bit-identical to the reference's
//     recomputation at the unchanged pose (model.py:472-476).
//   * The ratio test (model.py:324-336) needs max|rho| over the team before any point's
//     weight is known: with it, loss values are parked in LDS, the maximum is exchanged,
//     and a second pass over the blocks forms the normal equations.
#include <hip/hip_runtime.h>

#include "fmpnp.h"
#include "fmpnp_internal.h"

namespace fmpnp {

// per-storage-type variant tables (fmpnp_lm_f32.hip, fmpnp_lm_f64.hip)
const void *lm_kernel_ptr_f32(int wps, bool team, bool ratio, int var);
const void *lm_kernel_ptr_f64(int wps, bool team, bool ratio, int var);

const void *lm_kernel_ptr(int dtype, int wps, bool team, bool ratio, int var) {
    return dtype == FMPNP_F32 ? lm_kernel_ptr_f32(wps, team, ratio, var) : lm_kernel_ptr_f64(wps, team, ratio, var);
}

int lm_variant(const fmpnp_options &o) {
    if (o.sampling == FMPNP_BILINEAR) return o.no_memo == 1 ? VAR_BIL_DIRECT : VAR_BILINEAR;
    const bool gm = o.loss == FMPNP_GEMAN_MCCLURE && o.mode == FMPNP_MODE_FORWARD;
    if (o.layout == FMPNP_LAYOUT_F) return gm ? VAR_F_GM : VAR_F_NEAREST;
    return gm ? VAR_GM : VAR_NEAREST;
}

hipError_t launch_lm(const LaunchArgs &a, int dtype, int var, int grid, size_t lds, hipStream_t stream) {
    typedef void (*LmFn)(LaunchArgs);
    const LmFn f = (LmFn)lm_kernel_ptr(dtype, a.wps, a.G > 1, a.opt.use_ratio != 0, var);
    if (!f) return hipErrorInvalidDeviceFunction;
    hipLaunchKernelGGL(f, dim3(grid), dim3(a.wps == WPS_LATENCY ? NT : NT_THROUGHPUT), lds, stream, a);
    return hipGetLastError();
}

size_t lm_dyn_lds_bytes(int mmax, int nc_max, bool spec, bool bil_memo) {
    // X[3][rs] + rec[RECW][rs] (+ rec2[6][rs]) doubles (rs = mmax + 1), 32-bit per-point words
    // (tex; + tex2, spec, qp[2] with speculation; 16-B padded), part[nc_max][NV] doubles
    // (+ the bilinear cell memo[BIL_NB][rs] doubles)
    return ((size_t)(3 + RECW) * lds_rs(mmax) + lds_spec_doubles(mmax, spec)) * 8 + (size_t)lds_words(mmax, spec) * 4 +
           (size_t)nc_max * NV * 8 + (bil_memo ? (size_t)BIL_NB * lds_rs(mmax) * 8 : 0);
}

}  // namespace fmpnp
