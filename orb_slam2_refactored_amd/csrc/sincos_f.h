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

#include "sincos_tab.inc"

namespace orbamd {

// The fdlibm form's double constants.  sincos_f2d_k reads them through K: from a constexpr table they
// fold to literals (the host checks and sincos_f2d), from a __constant__ copy they arrive by scalar
// loads (describe_kernel, round 6: a literal double costs two s_mov_b32 of a wave's SALU issue, and
// describe was bound by SALU issue).  The operations and their order are the same either way.
struct SincosK {
    double invpio2, pio2_1, pio2_1t;
    double S1, S2, S3, S4, S5, S6;
    double C1, C2, C3, C4, C5, C6;
    double t_030, t_078125, t_028125;
};
static constexpr SincosK kSincosK = {
    6.36619772367581382433e-01,   // 2 / pi
    1.57079632673412561417e+00,   // first 33 bits of pi/2
    6.07710050650619224932e-11,   // pi/2 - pio2_1
    -1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04,
    2.75573137070700676789e-06, -2.50507602534068634195e-08, 1.58969099521155010221e-10,
    4.16666666666666019037e-02, -1.38888888888741095749e-03, 2.48015872894767294178e-05,
    -2.75573143513906633035e-07, 2.08757232129817482790e-09, -1.13596475577881948265e-11,
    0.3, 0.78125, 0.28125};

// sincos_f2d: the fdlibm form, the one describe_kernel evaluates (rounds 1-6).
template <class KT>
ORB_HD void sincos_f2d_k(float xf, float* s_out, float* c_out, const KT& K) {
#ifdef SINCOS_FMA_DIAG   // diagnostic A/B only (round 4's fused sincos; DESIGN §4 describe round 4)
#pragma clang fp contract(fast)
#endif
    const double x = (double)xf;
    const double n_d = __builtin_rint(x * K.invpio2);
    const int n = (int)n_d;
    const double r0 = x - n_d * K.pio2_1;                // exact
    const double w = n_d * K.pio2_1t;
    const double r = r0 - w;
    const double y = (r0 - r) - w;                       // tail of the reduced argument
    const double z = r * r;
    // __kernel_sin(r, y, 1)
    const double v = z * r;
    const double rs = K.S2 + z * (K.S3 + z * (K.S4 + z * (K.S5 + z * K.S6)));
    const double sn = r - ((z * (0.5 * y - v * rs) - y) - v * K.S1);
    // __kernel_cos(r, y)
    const double rc = z * (K.C1 + z * (K.C2 + z * (K.C3 + z * (K.C4 + z * (K.C5 + z * K.C6)))));
    double cs;
    const double ar = r < 0 ? -r : r;
    if (ar < K.t_030) {
        cs = 1.0 - (0.5 * z - (z * rc - r * y));
    } else {
        double qx;
        if (ar > K.t_078125) {
            qx = K.t_028125;
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
ORB_HD void sincos_f2d(float xf, float* s_out, float* c_out) { sincos_f2d_k(xf, s_out, c_out, kSincosK); }

// sincos_f2d_tab (round 5): the same function by a table reduction, about half the double operations of
// the fdlibm form above.  Measured slower in describe (its table entry arrives by a scalar load on the
// wave's one dependent chain; DESIGN §4 describe round 5), so describe keeps sincos_f2d; this form is
// kept, tested, for callers without that chain.  Domain: [0, 2 pi] (the angle ComputeOrbDescriptor
// takes); the table index is clamped to the table, so any other input reads inside it (inexactly).
// theta = k C + d with k = rint(theta / C), C = 2 pi / 256 in two parts (k C_HI exact), |d| <= pi / 256;
// sin theta = S_k cos d + C_k sin d, cos theta = C_k cos d - S_k sin d with S_k, C_k = sin / cos (k C)
// from a 257-entry table of doubles (tools/gen_sincos_tab.cpp, x87 long double rounded to double) and
// sin d = d + d^3 (-1/6 + d^2 / 120), cos d = 1 + d^2 (-1/2 + d^2 (1/24 - d^2 / 720)) (truncation
// < 1e-17).  Its float results equal glibc's (float)sin / cos((double)x) on EVERY float in [0, 6.2832]
// (tests/native/sincos_check.cpp, mode t: 1,086,918,649 values, 0 mismatches) -- the domain is finite, so
// that is the proof; a sine or cosine polynomial one term shorter gives 3 mismatches.  In describe the
// table index is wave-uniform: the two table entries come by scalar loads.
struct SincosTabEntry {
    double s, c;
};
static constexpr SincosTabEntry kSincosTab[ORB_SINCOS_TAB_N + 1] = {ORB_SINCOS_TAB_VALUES};

// UNIFORM (device): the caller guarantees xf is the same on every lane of the wavefront (describe: one
// keypoint per wavefront), so the table index is read from lane 0 and the entry comes by scalar loads.
template <bool UNIFORM>
ORB_HD void sincos_f2d_tab_t(float xf, float* s_out, float* c_out) {
    const double x = (double)xf;
    const double kd = __builtin_rint(x * (ORB_SINCOS_TAB_N / 6.283185307179586476925286766559));
    int k = (int)kd;
    k = k < 0 ? 0 : (k > ORB_SINCOS_TAB_N ? ORB_SINCOS_TAB_N : k);   // [0, 2 pi] maps to 0..N; outside: clamped
#if defined(__HIP_DEVICE_COMPILE__)
    if (UNIFORM) k = __builtin_amdgcn_readfirstlane(k);
#endif
    const double d = (x - kd * ORB_SINCOS_C_HI) - kd * ORB_SINCOS_C_LO;
    const double z = d * d;
    const double sd = d + d * z * (-1.0 / 6 + z * (1.0 / 120));
    const double cd = 1.0 + z * (-0.5 + z * (1.0 / 24 + z * (-1.0 / 720)));
    const SincosTabEntry t = kSincosTab[k];
    *s_out = (float)(t.s * cd + t.c * sd);
    *c_out = (float)(t.c * cd - t.s * sd);
}
ORB_HD void sincos_f2d_tab(float xf, float* s_out, float* c_out) { sincos_f2d_tab_t<false>(xf, s_out, c_out); }

// sinf / cosf of glibc >= 2.28 (the generic sysdeps/ieee754/flt-32 s_sinf.c / s_cosf.c, from ARM's
// optimized-routines, and their FMA ifunc variants): what `cos(angle)` / `sin(angle)` compute when the
// float overloads std::cos(float) / std::sin(float) are visible at ORBextractor.cc:107 (a `using
// namespace std` or a libstdc++ <math.h> wrapper included anywhere before it).  For 0 <= x < 120:
// n = round(x * 2/pi) via the 2^24-scaled integer path, r = x - n * pi/2 in double, then the
// quadrant's double polynomial (sin: x + x^3 s1 + x^7 (s2 + x^2 s3); cos: c0 + x^2 c1 + x^4 c2 +
// x^6 (c3 + x^2 c4)), negated cosine coefficients in quadrants 2 / 3.  Plain double ops: with or
// without contraction the float results equal glibc's sinf / cosf on every float in [0, 6.2832]
// (tests/native/sincos_check.cpp, mode f: 1,086,918,649 values, 0 mismatches either way).
struct SincosfTab { double c0, c1, c2, c3, c4; };
ORB_HD float sincosf_poly(double x, double x2, const SincosfTab& p, int n) {
    const double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double t1 = s2 + x2 * s3;
        const double x7 = x3 * x2;
        const double s = x + x3 * s1;
        return (float)(s + x7 * t1);
    }
    const double x4 = x2 * x2;
    const double t2 = p.c3 + x2 * p.c4;
    const double t1 = p.c0 + x2 * p.c1;
    const double x6 = x4 * x2;
    const double c = t1 + x4 * p.c2;
    return (float)(c + x6 * t2);
}

ORB_HD void sincosf_glibc(float y, float* s_out, float* c_out) {
    const SincosfTab pos = {0x1p0, -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10,
                            0x1.99343027bf8c3p-16};
    const SincosfTab neg = {-0x1p0, 0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10,
                            -0x1.99343027bf8c3p-16};
    double x = (double)y;
    const unsigned top = (__builtin_bit_cast(unsigned, y) >> 20) & 0x7ffu;   // abstop12
    if (top < 0x3f4u) {   // |y| < pi/4 (abstop12(0x1.921fb6p-1f))
        if (top < 0x398u) {   // |y| < 2^-12
            *s_out = y;
            *c_out = 1.0f;
            return;
        }
        const double x2 = x * x;
        *s_out = sincosf_poly(x, x2, pos, 0);
        *c_out = sincosf_poly(x, x2, pos, 1);
        return;
    }
    // reduce_fast (!TOINT_INTRINSICS): r = x * (2/pi * 2^24), n = ((int)r + 2^23) >> 24
    const double r = x * 0x1.45F306DC9C883p+23;
    const int n = ((int)r + 0x800000) >> 24;
    x = x - (double)n * 0x1.921FB54442D18p0;
    const double sg = ((n + 1) & 2) ? -1.0 : 1.0;   // sign[n & 3] = {1, -1, -1, 1}
    const SincosfTab& p = (n & 2) ? neg : pos;
    const double xs = x * sg, x2 = x * x;
    *s_out = sincosf_poly(xs, x2, p, n);
    *c_out = sincosf_poly(xs, x2, p, n ^ 1);
}

}  // namespace orbamd
