// Host check of the LM tail's sin/cos (fmpnp_device.h: sincos_small, sincos_rr) against
// libm over the rotation-step range: prints the largest error in ulp-scaled units and exits
// non-zero above the bound.  Built by the Makefile, run by tests/test_abi.py (CPU).
#include <math.h>
#include <stdio.h>

#include "fmpnp_device.h"

int main() {
    double worst = 0.0, worst_x = 0.0;
    const int n = 2000000;
    for (int i = 0; i <= n; ++i) {
        const double x = 200.0 * i / n;  // [0, 200] rad: 0..32 turns
        double s, c;
        if (x <= 0.78539816339744828) fmpnp::sincos_small(x, s, c);
        else fmpnp::sincos_rr(x, s, c);
        const double es = fabs(s - sin(x)), ec = fabs(c - cos(x));
        const double e = fmax(es, ec) / 2.220446049250313e-16;  // in units of eps (|sin|, |cos| <= 1)
        if (e > worst) { worst = e; worst_x = x; }
    }
    // larger steps, log-spaced: the two-part Cody-Waite reduction up to 2^19 pi/2, the
    // out-of-line library routine beyond (a near-singular step; the reference's torch.sin/cos)
    for (int i = 0; i <= 200000; ++i) {
        const double x = 200.0 * pow(1e10, i / 200000.0);  // 200 .. 2e12 rad
        double s, c;
        fmpnp::sincos_rr(x, s, c);
        const double e = fmax(fabs(s - sin(x)), fabs(c - cos(x))) / 2.220446049250313e-16;
        if (e > worst) { worst = e; worst_x = x; }
    }
    // so3exp_map's coefficients as polynomials in z = theta^2 (fmpnp_device.h so3_coeffs_small)
    // against libm: cos, sin/theta, (1 - cos)/theta^2 (the last from the half-angle form
    // 2 sin^2(theta/2)/theta^2, accurate where 1 - cos cancels), relative to their size
    double worst3 = 0.0, worst3_x = 0.0;
    for (int i = 1; i <= 1000000; ++i) {
        const double x = 0.78539816339744828 * i / 1000000;
        double cz, az, bz;
        fmpnp::so3_coeffs_small(x * x, cz, az, bz);
        const double sh = sin(0.5 * x);
        const double e = fmax(fabs(cz - cos(x)), fmax(fabs(az - sin(x) / x), fabs(bz - 2.0 * sh * sh / (x * x)) / 0.5)) /
                         2.220446049250313e-16;
        if (e > worst3) { worst3 = e; worst3_x = x; }
    }
    printf("so3 coefficients: max error %.3f eps at theta = %.17g\n", worst3, worst3_x);
    double s, c;
    fmpnp::sincos_rr(INFINITY, s, c);
    const bool nan_ok = isnan(s) && isnan(c);
    printf("max error %.3f eps at x = %.17g; inf -> nan: %d\n", worst, worst_x, (int)nan_ok);
    return (worst <= 8.0 && worst3 <= 8.0 && nan_ok) ? 0 : 1;
}
