// fmpnp_device.h -- device helpers shared by the fmpnp HIP kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "fmpnp.h"

namespace fmpnp {

// 16-byte vector of the storage type: one dwordx4 load per lane.
template <typename T> struct V16;
template <> struct V16<float> { typedef float4 type; static constexpr int n = 4; };
template <> struct V16<double> { typedef double2 type; static constexpr int n = 2; };

// torch.finfo(torch.float).eps as the reference uses it (helpers/utils.py:25,58)
constexpr double kEpsF32 = 1.1920928955078125e-07;

// Robust losses, featurePnP/helpers/utils.py:15-78.  rho and rho' (the reference's
// second derivative output is always zero and unused by the LM loop).
__device__ __forceinline__ void loss_eval(int loss, double alpha, double x, double &rho, double &d1) {
    if (loss == FMPNP_SQUARED) { rho = x; d1 = 1.0; return; }           // :16-17
    if (loss == FMPNP_HUBER) {                                          // :20-29 (rho = 1)
        double sx = sqrt(x);
        double inv = 1.0 / sx;
        double isx = (inv > kEpsF32 || isnan(inv)) ? inv : kEpsF32;
        if (x <= 1.0) { rho = x; d1 = 1.0; } else { rho = 2.0 * sx - 1.0; d1 = isx; }
        return;
    }
    if (loss == FMPNP_CAUCHY) alpha = 0.0;                              // :32-34
    else if (loss == FMPNP_GEMAN_MCCLURE) alpha = -2.0;                 // :37-38
    if (alpha == 0.0) {                                                 // :54-55
        double h = 0.5 * x;
        if (!(h <= 33e37)) h = isnan(h) ? h : 33e37;
        rho = 2.0 * log1p(h);
        d1 = 2.0 / (x + 2.0);
    } else if (alpha == 2.0) {                                          // :51-52
        rho = x;
        d1 = 1.0;
    } else if (alpha == -2.0) {
        // Geman-McClure: beta_safe = 4, alpha_safe = -2 -> rho = -4 (b^-1 - 1), rho' = b^-2 with
        // b = x/4 + 1.  b^-1 is the correctly rounded 1/b (what a correctly rounded pow returns);
        // b^-2 as (1/b)^2 is within 2 ulp of pow -- only the weights see it.
        const double b = x / 4.0 + 1.0;
        const double r = 1.0 / b;
        rho = -4.0 * (r - 1.0);
        d1 = r * r;
    } else {                                                            // :58-68
        double beta_safe = fabs(alpha - 2.0);
        beta_safe = beta_safe < kEpsF32 ? kEpsF32 : beta_safe;
        double aa = fabs(alpha);
        aa = aa < kEpsF32 ? kEpsF32 : aa;
        double alpha_safe = (alpha >= 0.0 ? 1.0 : -1.0) * aa;
        double b = x / beta_safe + 1.0;
        rho = 2.0 * (beta_safe / alpha_safe) * (pow(b, 0.5 * alpha) - 1.0);
        d1 = pow(b, 0.5 * alpha - 1.0);
    }
}

// P = R X + t exactly as torch.mm computes it for these shapes (sequential, no FMA):
// the pixel rounding below must see the same bits as the reference (model.py:303).
__device__ __forceinline__ void transform_pt(const double *R, const double *t, double X0, double X1, double X2,
                                             double P[3]) {
#pragma clang fp contract(off)
    for (int i = 0; i < 3; ++i) {
        double s = R[3 * i + 0] * X0;
        s = s + R[3 * i + 1] * X1;
        s = s + R[3 * i + 2] * X2;
        P[i] = s + t[i];
    }
}

// Pixel of a camera-frame point: round_half_even(K P / P_z) - 1 and the image mask
// (model.py:306-311, points_within_image :99-117; z<0 is NOT masked).
__device__ __forceinline__ bool project_px(const double *K, const double P[3], int W, int H, int &x, int &y) {
#pragma clang fp contract(off)
    double u[3];
    for (int i = 0; i < 3; ++i) {
        double s = K[3 * i + 0] * P[0];
        s = s + K[3 * i + 1] * P[1];
        s = s + K[3 * i + 2] * P[2];
        u[i] = s;
    }
    double px = rint(u[0] / u[2]) - 1.0;
    double py = rint(u[1] / u[2]) - 1.0;
    if (!(px >= 0.0 && px < (double)W && py >= 0.0 && py < (double)H)) return false;
    x = (int)px;
    y = (int)py;
    return true;
}

}  // namespace fmpnp
