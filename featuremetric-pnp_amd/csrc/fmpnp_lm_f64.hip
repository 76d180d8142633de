// fmpnp_lm_f64.hip -- LM kernel variants for double texels (see fmpnp_lm_impl.h).  One
// translation unit per storage type, so the variants compile in parallel.
#include "fmpnp_lm_impl.h"

namespace fmpnp {

typedef void (*LmFn)(LaunchArgs);
template <int WPS, bool TEAM, bool RATIO>
static LmFn pick_var(int var) {
    if (var == VAR_F_NEAREST || var == VAR_F_GM) return nullptr;  // FMPNP_LAYOUT_F is fp32-only (validated)
    if (var == VAR_GM) return lm_kernel<double, WPS, TEAM, RATIO, VAR_GM>;
    if (var == VAR_GM_SPEC || var == VAR_NEAREST_SPEC || var == VAR_GM_SPEC_H || var == VAR_NEAREST_SPEC_H) {
        if constexpr (WPS == WPS_LATENCY && !TEAM) {  // speculation (+ helpers): latency build, G = 1
            if (var == VAR_GM_SPEC) return lm_kernel<double, WPS, TEAM, RATIO, VAR_GM_SPEC>;
            if (var == VAR_NEAREST_SPEC) return lm_kernel<double, WPS, TEAM, RATIO, VAR_NEAREST_SPEC>;
            if (var == VAR_GM_SPEC_H) return lm_kernel<double, WPS, TEAM, RATIO, VAR_GM_SPEC_H>;
            return lm_kernel<double, WPS, TEAM, RATIO, VAR_NEAREST_SPEC_H>;
        }
        return nullptr;
    }
    if (var == VAR_GM_SPEC_512 || var == VAR_GM_SPEC_H_512) return nullptr;  // (fp32 texels only)
    if (var == VAR_GM_H || var == VAR_NEAREST_H) {  // first-evaluation helpers without speculation
        if constexpr (WPS == WPS_LATENCY && !TEAM) {
            if (var == VAR_GM_H) return lm_kernel<double, WPS, TEAM, RATIO, VAR_GM_H>;
            return lm_kernel<double, WPS, TEAM, RATIO, VAR_NEAREST_H>;
        }
        return nullptr;
    }
    if (var == VAR_GM_W || var == VAR_NEAREST_W) {  // packed windows (fmpnp_feature_pnp): latency build
        if constexpr (WPS == WPS_LATENCY) {
            if (var == VAR_GM_W) return lm_kernel<double, WPS, TEAM, RATIO, VAR_GM_W>;
            return lm_kernel<double, WPS, TEAM, RATIO, VAR_NEAREST_W>;
        }
        return nullptr;
    }
    if (var == VAR_GM_H_W || var == VAR_NEAREST_H_W) {  // ... with the first-evaluation helpers
        if constexpr (WPS == WPS_LATENCY && !TEAM) {
            if (var == VAR_GM_H_W) return lm_kernel<double, WPS, TEAM, RATIO, VAR_GM_H_W>;
            return lm_kernel<double, WPS, TEAM, RATIO, VAR_NEAREST_H_W>;
        }
        return nullptr;
    }
    if (var == VAR_BILINEAR) return nullptr;  // the cell memo runs on the WPS_WIDE build only
    if (var == VAR_BIL_DIRECT) return lm_kernel<double, WPS, TEAM, RATIO, VAR_BIL_DIRECT>;
    return lm_kernel<double, WPS, TEAM, RATIO, VAR_NEAREST>;
}
template <int WPS>
static LmFn pick(bool team, bool ratio, int var) {
    if (team) return ratio ? pick_var<WPS, true, true>(var) : pick_var<WPS, true, false>(var);
    return ratio ? pick_var<WPS, false, true>(var) : pick_var<WPS, false, false>(var);
}

const void *lm_kernel_ptr_f64(int wps, bool team, bool ratio, int var) {
    // the 128-VGPR throughput build is only planned with G == 1
    if (wps == WPS_WIDE) {  // the bilinear cell memo only
        if (var != VAR_BILINEAR) return nullptr;
        if (team) return ratio ? (const void *)lm_kernel<double, WPS_WIDE, true, true, VAR_BILINEAR>
                               : (const void *)lm_kernel<double, WPS_WIDE, true, false, VAR_BILINEAR>;
        return ratio ? (const void *)lm_kernel<double, WPS_WIDE, false, true, VAR_BILINEAR>
                     : (const void *)lm_kernel<double, WPS_WIDE, false, false, VAR_BILINEAR>;
    }
    if (wps == WPS_THROUGHPUT) return (const void *)(ratio ? pick_var<WPS_THROUGHPUT, false, true>(var)
                                                           : pick_var<WPS_THROUGHPUT, false, false>(var));
    return (const void *)pick<WPS_LATENCY>(team, ratio, var);
}

}  // namespace fmpnp
