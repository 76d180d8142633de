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

// ---------------------------------------------------------------------------
// Cross-lane exchange of doubles without the LDS path (ds_bpermute): DPP inside a row
// of 16 lanes, v_permlane{16,32}_swap across rows (gfx950).  Partners used by the
// reductions: xor 1, xor 2 (quad_perm), i^7 within 8 (row_half_mirror), i^15 within 16
// (row_mirror); each flips the bit being split and keeps every higher bit.
// ---------------------------------------------------------------------------
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_MIRROR8 = 0x141, DPP_MIRROR16 = 0x140;

template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double join64(unsigned lo, unsigned hi) {
    return __longlong_as_double(((long long)hi << 32) | lo);
}

// Rows (0,1) and (2,3) exchange: odd rows of a swap with even rows of b.  Returns
// (a', b') -- even rows: (own a, partner's a); odd rows: (partner's b, own b).
__device__ __forceinline__ void swap16(double &a, double &b) {
    const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
    const auto l = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)y, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
    a = join64(l[0], h[0]);
    b = join64(l[1], h[1]);
}
// Same across the two 32-lane halves of the wave.
__device__ __forceinline__ void swap32(double &a, double &b) {
    const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
    const auto l = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)y, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
    a = join64(l[0], h[0]);
    b = join64(l[1], h[1]);
}

// One halving step of a transposed reduction with an in-row DPP partner: the lane keeps
// `hi` when its split bit is set, else `lo`, and adds the partner's copy of the same.
template <int CTRL>
__device__ __forceinline__ double tstep(double lo, double hi, bool bit) {
    const double send = bit ? lo : hi, keep = bit ? hi : lo;
    return keep + dpp64<CTRL>(send);
}

// NaN-propagating max (the reference's torch.max over |rho| propagates NaN)
__device__ __forceinline__ double nanmax(double a, double b) {
    return (isnan(b) || b > a) ? (isnan(a) ? a : b) : a;
}
// max over the 64 lanes of a wave (order-free: exact)
// wave maximum / minimum of non-NaN values (v_max_f64 / v_min_f64 semantics)
__device__ __forceinline__ double wave_fmax(double v) {
    v = fmax(v, dpp64<DPP_XOR1>(v));
    v = fmax(v, dpp64<DPP_XOR2>(v));
    v = fmax(v, dpp64<DPP_MIRROR8>(v));
    v = fmax(v, dpp64<DPP_MIRROR16>(v));
    double a = v, b = v;
    swap16(a, b);
    v = fmax(a, b);
    a = v, b = v;
    swap32(a, b);
    return fmax(a, b);
}
__device__ __forceinline__ double wave_fmin(double v) {
    v = fmin(v, dpp64<DPP_XOR1>(v));
    v = fmin(v, dpp64<DPP_XOR2>(v));
    v = fmin(v, dpp64<DPP_MIRROR8>(v));
    v = fmin(v, dpp64<DPP_MIRROR16>(v));
    double a = v, b = v;
    swap16(a, b);
    v = fmin(a, b);
    a = v, b = v;
    swap32(a, b);
    return fmin(a, b);
}
__device__ __forceinline__ double wave_nanmax(double v) {
    v = nanmax(v, dpp64<DPP_XOR1>(v));
    v = nanmax(v, dpp64<DPP_XOR2>(v));
    v = nanmax(v, dpp64<DPP_MIRROR8>(v));
    v = nanmax(v, dpp64<DPP_MIRROR16>(v));
    double a = v, b = v;
    swap16(a, b);
    v = nanmax(a, b);
    a = v, b = v;
    swap32(a, b);
    return nanmax(a, b);
}

// 1/x by v_rcp_f64 and two Newton steps (about 0.5 ulp; not always the correctly rounded
// quotient): used where the reference's division only feeds weights, Jacobians or the
// mean cost -- and by project_pc (fmpnp_lm_impl.h) for the nearest path's rounded pixel, behind
// a guard: a quotient within 2^-49 relative of a half-integer (rint's boundary), a z outside
// [2^-1000, 2^1000] or a non-finite quotient takes the exact IEEE division instead.  A change to
// this function's precision must re-check that guard's bound.
__device__ __forceinline__ double recip(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    return fma(fma(-x, r, 1.0), r, r);
}

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
        // b = x/4 + 1.  b^-1 by a Newton-refined reciprocal (within an ulp of pow's correctly
        // rounded value; rho only enters the mean cost), b^-2 as (1/b)^2.
        const double b = x / 4.0 + 1.0;
#if FMPNP_GM_POW  // the reference's pow form (A/B only: profiles/r06_gm_pow_ab.txt)
        rho = -4.0 * (pow(b, -1.0) - 1.0);
        d1 = pow(b, -2.0);
#else
        const double r = recip(b);
        rho = -4.0 * (r - 1.0);
        d1 = r * r;
#endif
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

// Exact floor(a / d) for 0 <= a < 2^32, 1 <= d < 2^31 by an invariant multiplier
// (Granlund & Montgomery 1994; "round-up" method with a 33-bit multiplier):
// l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1, t = mulhi(m, a),
// q = (t + ((a - t) >> 1)) >> (l - 1)   (l = 0: q = a).
struct UDiv {
    unsigned m;
    int s1, s2;
};
__host__ __device__ inline UDiv udiv_make(unsigned d) {
    int l = 0;
    while ((1ull << l) < d) ++l;
    const unsigned long long m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
    return UDiv{(unsigned)m, l ? 1 : 0, l ? l - 1 : 0};
}
__device__ __forceinline__ unsigned udiv(unsigned a, UDiv u) {
    const unsigned t = __umulhi(u.m, a);
    return (t + ((a - t) >> u.s1)) >> u.s2;
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
// (model.py:306-311, points_within_image :99-117; z<0 is NOT masked).  qx, qy: the
// unrounded K P / P_z (bilinear sampling).
__device__ __forceinline__ bool project_px(const double *K, const double P[3], int W, int H, int &x, int &y,
                                          double &qx, double &qy) {
#pragma clang fp contract(off)
    double u[3];
    for (int i = 0; i < 3; ++i) {
        double s = K[3 * i + 0] * P[0];
        s = s + K[3 * i + 1] * P[1];
        s = s + K[3 * i + 2] * P[2];
        u[i] = s;
    }
    qx = u[0] / u[2];
    qy = u[1] / u[2];
    double px = rint(qx) - 1.0;
    double py = rint(qy) - 1.0;
    if (!(px >= 0.0 && px < (double)W && py >= 0.0 && py < (double)H)) return false;
    x = (int)px;
    y = (int)py;
    return true;
}

// Bilinear sampling (FMPNP_BILINEAR, an extension: the reference's indexing_ is
// nearest-texel).  The definition is shared bit-for-bit with the oracle
// (oracle/fmpnp_oracle.c bilinear_taps): sx = ((qx - 0.5) Wf) / W - 0.5 (image pixel
// index i = round(q) - 1 is centred at q = i + 1, texel c at sx = c), taps at
// floor(sx), floor(sx) + 1 (rows likewise) clamped to the map, weights
// w00 = (1-ax)(1-ay), w01 = ax(1-ay), w10 = (1-ax)ay, w11 = ax ay.
struct Taps {
    int off[4];       // texel offsets (row * Wf + col): [y0x0, y0x1, y1x0, y1x1]
    double w[4];
    double ax, ay;    // the point's position inside its cell
    int key;          // the cell: ((y0 + 1) << 16) | (x0 + 1) of the unclamped floors (bil_cell_taps)
};
__device__ __forceinline__ void bilinear_taps(double qx, double qy, int Hf, int Wf, int W, int H, Taps &t) {
#pragma clang fp contract(off)
    const double sx = ((qx - 0.5) * (double)Wf) / (double)W - 0.5;
    const double sy = ((qy - 0.5) * (double)Hf) / (double)H - 0.5;
    const double fx0 = floor(sx), fy0 = floor(sy);
    const double ax = sx - fx0, ay = sy - fy0;
    int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
    // a supported pixel has -1 <= floor <= size - 1; clamping the key's floors into that range
    // changes no tap (every tap is clamped to the map below)
    t.key = ((min(max(y0, -1), Hf - 1) + 1) << 16) | (min(max(x0, -1), Wf - 1) + 1);
    t.ax = ax;
    t.ay = ay;
    x0 = min(max(x0, 0), Wf - 1);
    x1 = min(max(x1, 0), Wf - 1);
    y0 = min(max(y0, 0), Hf - 1);
    y1 = min(max(y1, 0), Hf - 1);
    t.off[0] = y0 * Wf + x0;
    t.off[1] = y0 * Wf + x1;
    t.off[2] = y1 * Wf + x0;
    t.off[3] = y1 * Wf + x1;
    t.w[0] = (1.0 - ax) * (1.0 - ay);
    t.w[1] = ax * (1.0 - ay);
    t.w[2] = (1.0 - ax) * ay;
    t.w[3] = ax * ay;
}
// The four tap offsets of a cell key (bilinear_taps' clamping, the same offsets).
__device__ __forceinline__ void bil_cell_taps(int key, int Hf, int Wf, int o[4]) {
    const int fy = (key >> 16) - 1, fx = (key & 0xffff) - 1;
    const int x0 = max(fx, 0), x1 = min(fx + 1, Wf - 1), y0 = max(fy, 0), y1 = min(fy + 1, Hf - 1);
    o[0] = y0 * Wf + x0;
    o[1] = y0 * Wf + x1;
    o[2] = y1 * Wf + x0;
    o[3] = y1 * Wf + x1;
}
// one sampled value: fma(w11, v11, fma(w10, v10, fma(w01, v01, w00 v00)))
__device__ __forceinline__ double sample4(const double w[4], double v0, double v1, double v2, double v3) {
    return fma(w[3], v3, fma(w[2], v2, fma(w[1], v1, w[0] * v0)));
}

__device__ __forceinline__ double rlane64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// An fp64 literal materialised where it is used: without this the compiler hoists the
// 64-bit constants of the tail out of the problem loop into ~30 VGPRs that stay live (and
// get spilled) through the point phase.  The volatile no-op pins the value to its use site
// in an SGPR pair (two s_mov on the scalar unit).
__host__ __device__ __forceinline__ double kc(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(v));
#endif
    return v;
}
// The same constant materialised by two s_mov_b32 of its halves inside volatile asm, so it can
// be neither hoisted out of the loop nor kept live (and spilled to VGPR lanes) between uses:
// kc() pins the use site, but the compiler may still hoist the constant's s_mov pair out of the
// problem loop and spill the SGPR pair, which costs v_readlane reloads on the LM tail.
template <unsigned long long B>
__host__ __device__ __forceinline__ double kcb() {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned lo, hi;
    asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((int)(unsigned)(B & 0xffffffffull)));
    asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((int)(unsigned)(B >> 32)));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
#else
    return __builtin_bit_cast(double, B);
#endif
}
#ifndef FMPNP_KC_ASM
#define FMPNP_KC_ASM 1
#endif
#if FMPNP_KC_ASM
#define KC(x) ::fmpnp::kcb<__builtin_bit_cast(unsigned long long, (double)(x))>()
#else
#define KC(x) ::fmpnp::kc(x)
#endif

// sin, cos of 0 <= x <= pi/4 by Horner-form Taylor series to x^17 / x^18 (truncation
// below 1e-19 relative; a few ulp of rounding): ~20 register-resident fp64 operations
// instead of the library's range-reduced sincos on the LM tail's critical path.
__host__ __device__ __forceinline__ void sincos_small(double x, double &s, double &c) {
    const double z = x * x;
    double ps = KC(1.0 / 355687428096000.0);
    ps = fma(ps, z, KC(-1.0 / 1307674368000.0));
    ps = fma(ps, z, KC(1.0 / 6227020800.0));
    ps = fma(ps, z, KC(-1.0 / 39916800.0));
    ps = fma(ps, z, KC(1.0 / 362880.0));
    ps = fma(ps, z, KC(-1.0 / 5040.0));
    ps = fma(ps, z, KC(1.0 / 120.0));
    ps = fma(ps, z, KC(-1.0 / 6.0));
    s = fma(x * z, ps, x);
    double pc = KC(-1.0 / 6402373705728000.0);
    pc = fma(pc, z, KC(1.0 / 20922789888000.0));
    pc = fma(pc, z, KC(-1.0 / 87178291200.0));
    pc = fma(pc, z, KC(1.0 / 479001600.0));
    pc = fma(pc, z, KC(-1.0 / 3628800.0));
    pc = fma(pc, z, KC(1.0 / 40320.0));
    pc = fma(pc, z, KC(-1.0 / 720.0));
    pc = fma(pc, z, KC(1.0 / 24.0));
    pc = fma(pc, z, -0.5);
    c = fma(z, pc, 1.0);
}

// The three even functions of a rotation angle theta that so3exp_map needs, as polynomials in
// z = theta^2 (no square root, no division) for 0 <= z <= (pi/4)^2: cos theta, sin(theta)/theta and
// (1 - cos theta)/theta^2 (Horner-form Taylor series, truncation below 1e-19 relative).  With
// W = [w]x of the unnormalised axis-angle w (|w| = theta), W^2 = w w^T - theta^2 I, so
// helpers/utils.py:209-221's I + sin(theta) [w/theta]x + (1 - cos theta) [w/theta]x^2 is
// cos(theta) I + (sin(theta)/theta) W + ((1 - cos theta)/theta^2) w w^T.
#ifndef FMPNP_SO3_SHORT
#define FMPNP_SO3_SHORT 1
#endif
__host__ __device__ __forceinline__ void so3_coeffs_small(double z, double &c, double &a, double &b) {
#if FMPNP_SO3_SHORT
    if (z <= 2.5e-5) {
        // theta <= 0.005 (an LM step near convergence): the series to z^4 -- the next terms are
        // below z^5 / 11! = 2.5e-31 relative, far under the last bit -- with a third of the operations
        double pb = fma(KC(1.0 / 3628800.0), -z, KC(1.0 / 40320.0));  // 1/10!, 1/8!
        pb = fma(pb, -z, KC(1.0 / 720.0));
        pb = fma(pb, -z, KC(1.0 / 24.0));
        pb = fma(pb, -z, 0.5);
        b = pb;
        c = fma(pb, -z, 1.0);
        double pa = fma(KC(1.0 / 362880.0), -z, KC(1.0 / 5040.0));  // 1/9!, 1/7!
        pa = fma(pa, -z, KC(1.0 / 120.0));
        pa = fma(pa, -z, KC(1.0 / 6.0));
        a = fma(pa, -z, 1.0);
        return;
    }
#endif
    double pc = KC(1.0 / 6402373705728000.0);       // 1/18!
    pc = fma(pc, -z, KC(1.0 / 20922789888000.0));  // 1/16!
    pc = fma(pc, -z, KC(1.0 / 87178291200.0));
    pc = fma(pc, -z, KC(1.0 / 479001600.0));
    pc = fma(pc, -z, KC(1.0 / 3628800.0));
    pc = fma(pc, -z, KC(1.0 / 40320.0));
    pc = fma(pc, -z, KC(1.0 / 720.0));
    pc = fma(pc, -z, KC(1.0 / 24.0));
    pc = fma(pc, -z, 0.5);                           // b = sum (-z)^k / (2k+2)!, k = 0..8
    b = pc;
    c = fma(pc, -z, 1.0);                            // cos = 1 - z b
    double pa = KC(1.0 / 121645100408832000.0);     // 1/19!
    pa = fma(pa, -z, KC(1.0 / 355687428096000.0));  // 1/17!
    pa = fma(pa, -z, KC(1.0 / 1307674368000.0));
    pa = fma(pa, -z, KC(1.0 / 6227020800.0));
    pa = fma(pa, -z, KC(1.0 / 39916800.0));
    pa = fma(pa, -z, KC(1.0 / 362880.0));
    pa = fma(pa, -z, KC(1.0 / 5040.0));
    pa = fma(pa, -z, KC(1.0 / 120.0));
    pa = fma(pa, -z, KC(1.0 / 6.0));
    a = fma(pa, -z, 1.0);                            // sin(theta)/theta
}

// The library sincos for the huge-angle branch below, out of line: its constant tables stay
// inside the call and never occupy registers of the caller's hot loop.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __attribute__((noinline)) double2 sincos_lib(double x) {
    double s, c;
    sincos(x, &s, &c);
    return make_double2(s, c);
}
#else
inline double2 sincos_lib(double x) {
    double2 r;
    r.x = sin(x);
    r.y = cos(x);
    return r;
}
#endif

// sin, cos of a finite x > pi/4 (a rotation step of more than 45 degrees: rare): Cody-Waite
// reduction by pi/2 (fdlibm's two-part constant, exact products for |n| < 2^20), then the
// polynomial above on |r| <= pi/4 and the quadrant swap.  Replaces the library sincos,
// whose table of 64-bit constants the compiler would otherwise hoist into registers that
// stay live through the point phase.  Beyond 2^19 pi/2 (|n| >= 2^19: the two-part
// reduction loses accuracy) the out-of-line library routine (Payne-Hanek) takes over, so
// every finite step gives the reference's torch.sin / torch.cos (helpers/utils.py:209-221).
// Non-finite x gives NaN (as the library does).
__host__ __device__ __forceinline__ void sincos_rr(double x, double &s, double &c) {
    if (!(x < 1e300)) {
        s = c = __builtin_nan("");
        return;
    }
    if (x > 823549.6654402911) {  // 2^19 * pi / 2
        const double2 r = sincos_lib(x);
        s = r.x;
        c = r.y;
        return;
    }
    const double n = rint(x * KC(6.36619772367581382433e-01));  // 2 / pi
    double r = fma(-n, KC(1.57079632673412561417e+00), x);      // pio2_1 (33 bits)
    r = fma(-n, KC(6.07710050650619224932e-11), r);             // pio2_1t
    double sr, cr;
    sincos_small(fabs(r), sr, cr);
    if (r < 0.0) sr = -sr;
    const int q = (int)(n - 4.0 * floor(n * 0.25));             // n mod 4, exact
    s = q == 0 ? sr : (q == 1 ? cr : (q == 2 ? -sr : -cr));
    c = q == 0 ? cr : (q == 1 ? -sr : (q == 2 ? -cr : sr));
}

}  // namespace fmpnp
