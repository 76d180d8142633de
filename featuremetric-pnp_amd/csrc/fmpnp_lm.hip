// fmpnp_lm.hip -- the feature-metric LM refiner on gfx950 (MI355X).
//
// One launch runs the WHOLE Levenberg-Marquardt loop of every problem of a batch
// (sparseFeaturePnP.forward, featurePnP/model.py:245-494) on the device.
//
// The kernel template and its work decomposition: fmpnp_lm_impl.h.  This unit holds the
// variant choice (lm_variant), the launch and the LDS sizing.
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
