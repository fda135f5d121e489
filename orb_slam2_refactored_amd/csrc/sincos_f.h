// (float)sin((double)x) and (float)cos((double)x) for float x in [0, 8), as ComputeOrbDescriptor
// computes a = (float)cos(angle), b = (float)sin(angle) with ::cos / ::sin (double)
// (ORBextractor.cc:105-107).  A short double-precision path replaces the general library sincos:
// Cody-Waite reduction by pi/2 in two parts (x is a float and n <= 5, so x - n*pio2_1 is exact and
// the reduced argument keeps ~2^-60 relative accuracy) and the classic minimax kernels for
// |r| <= pi/4 (fdlibm __kernel_sin / __kernel_cos coefficients, < 1 ulp).  Like any < 1 ulp double
// result, the float rounding equals glibc's except when cos / sin lies within 1 double ulp of a
// float rounding boundary; tests/native/sincos_check.cpp compares every float in [0, 6.2832].
// Plain IEEE double ops (the library is built with -ffp-contract=off), so host and device agree
// bit for bit.
#pragma once

#if defined(__HIPCC__)
#define ORB_HD __host__ __device__ __forceinline__
#else
#define ORB_HD inline
#endif

namespace orbamd {

ORB_HD void sincos_f2d(float xf, float* s_out, float* c_out) {
    const double x = (double)xf;
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;    // first 33 bits of pi/2
    const double pio2_1t = 6.07710050650619224932e-11;   // pi/2 - pio2_1
    const double n_d = __builtin_rint(x * invpio2);
    const int n = (int)n_d;
    const double r0 = x - n_d * pio2_1;                  // exact
    const double w = n_d * pio2_1t;
    const double r = r0 - w;
    const double y = (r0 - r) - w;                       // tail of the reduced argument
    const double z = r * r;
    // __kernel_sin(r, y, 1)
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double v = z * r;
    const double rs = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double sn = r - ((z * (0.5 * y - v * rs) - y) - v * S1);
    // __kernel_cos(r, y)
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double cs;
    const double ar = r < 0 ? -r : r;
    if (ar < 0.3) {
        cs = 1.0 - (0.5 * z - (z * rc - r * y));
    } else {
        double qx;
        if (ar > 0.78125) {
            qx = 0.28125;
        } else {   // |r| / 4 with the low word cleared
            const unsigned long long bits = __builtin_bit_cast(unsigned long long, ar);
            qx = __builtin_bit_cast(double, (bits - (0x00200000ull << 32)) & 0xffffffff00000000ull);
        }
        const double hz = 0.5 * z - qx;
        const double a = 1.0 - qx;
        cs = a - (hz - (z * rc - r * y));
    }
    double s, c;
    switch (n & 3) {
        case 0: s = sn; c = cs; break;
        case 1: s = cs; c = -sn; break;
        case 2: s = -sn; c = -cs; break;
        default: s = -cs; c = sn; break;
    }
    *s_out = (float)s;
    *c_out = (float)c;
}

}  // namespace orbamd
