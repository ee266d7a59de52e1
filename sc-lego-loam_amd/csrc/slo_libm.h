// slo_libm.h — glibc-2.35-exact single-precision elementary functions, usable
// from host C++ and from HIP device code (gfx950).
//
// Why this exists: the reference's discrete decisions (range-image row/column,
// ground marks, the 60-degree segmentation edge test, deskew halves, Scan
// Context sector bins) are taken on values produced by glibc's float atan2f /
// sinf / cosf, because `using namespace std` in utility.h:49 makes
// `atan2(float,float)` resolve to the float overload (e.g. imageProjection.cpp
// :229, :235, :284, :421; featureAssociation.cpp:504, :871).  ROCm's ocml
// implementations differ from glibc in the last ulp, which flips those
// decisions on a handful of points per scan.  Restating glibc's published
// algorithms here (fdlibm-derived atanf/atan2f, the 2018 double-evaluated
// sinf/cosf, fdlibm-derived asinf) gives the device exactly the host's bits.
// tests/test_libm.py checks every function against the host glibc on tens of
// millions of inputs (libm_selftest in the oracle library).
//
// Build rule: every translation unit that includes this header must be
// compiled with -ffp-contract=off (the Makefiles do); where glibc's x86-64
// multiarch build contracts a*b+c into an FMA (the -mfma ifunc variants of
// sinf/cosf) the fusion is written explicitly with fma().
#pragma once

#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SLO_HD __host__ __device__ inline
#else
#define SLO_HD inline
#endif

namespace slo_libm {

SLO_HD uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
SLO_HD float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
SLO_HD uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

// ---------------------------------------------------------------- atanf
// glibc sysdeps/ieee754/flt-32/s_atanf.c (fdlibm float port).
SLO_HD float atanf_(float x) {
    const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f,
                atanhi2 = 9.8279368877e-01f, atanhi3 = 1.5707962513e+00f;
    const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f,
                atanlo2 = 3.4473217170e-08f, atanlo3 = 7.5497894159e-08f;
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f,
                aT2 = 1.4285714924e-01f, aT3 = -1.1111110449e-01f,
                aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f,
                aT8 = 4.9768779427e-02f, aT9 = -3.6531571299e-02f,
                aT10 = 1.6285819933e-02f;
    int32_t hx = (int32_t)f2u(x);
    int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {              // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;  // NaN
        if (hx > 0) return atanhi3 + atanlo3;
        return -atanhi3 - atanlo3;
    }
    if (ix < 0x3ee00000) {               // |x| < 0.4375
        if (ix < 0x31000000) return x;   // |x| < 2^-29
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {           // |x| < 1.1875
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    float z = x * x;
    float w = z * z;
    float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
    float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
    z = hi - ((x * (s1 + s2) - lo) - x);
    return (hx < 0) ? -z : z;
}

// ---------------------------------------------------------------- atan2f
// glibc sysdeps/ieee754/flt-32/e_atan2f.c (fdlibm float port).
SLO_HD float atan2f_(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f,
                pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                pi_lo = -8.7422776573e-08f;
    int32_t hx = (int32_t)f2u(x), hy = (int32_t)f2u(y);
    int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;   // NaN
    if (hx == 0x3f800000) return atanf_(y);                 // x == 1.0
    int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
            case 0: case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        } else {
            switch (m) {
                case 0: return 0.0f;
                case 1: return -0.0f;
                case 2: return pi + tiny;
                default: return -pi - tiny;
            }
        }
    }
    if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    float z;
    int32_t k = (iy - ix) >> 23;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = atanf_(fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return u2f(f2u(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// ---------------------------------------------------------------- sinf/cosf
// glibc sysdeps/ieee754/flt-32/s_sinf.c / s_cosf.c / sincosf.h (2018
// double-evaluated implementation).  On x86-64 with FMA+AVX2, glibc's ifunc
// selects the -mfma build of the same source, where GCC fuses each a + b*c:
// SLO_SINCOS_FMA=1 (default) writes those fusions out with fma().
#ifndef SLO_SINCOS_FMA
#define SLO_SINCOS_FMA 1
#endif

struct sincos_tab {
    double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};

SLO_HD double madd_(double a, double b, double c) {  // a*b + c as glibc-fma built it
#if SLO_SINCOS_FMA
    return fma(a, b, c);
#else
    return a * b + c;
#endif
}

SLO_HD sincos_tab sincos_table(int which) {
    sincos_tab t;
    t.hpi_inv = 0x1.45F306DC9C883p+23;
    t.hpi = 0x1.921FB54442D18p0;
    const double sg = which ? -1.0 : 1.0;
    t.c0 = sg * 0x1p0;
    t.c1 = sg * -0x1.ffffffd0c621cp-2;
    t.c2 = sg * 0x1.55553e1068f19p-5;
    t.c3 = sg * -0x1.6c087e89a359dp-10;
    t.c4 = sg * 0x1.99343027bf8c3p-16;
    t.s1 = -0x1.555545995a603p-3;
    t.s2 = 0x1.1107605230bc4p-7;
    t.s3 = -0x1.994eb3774cf24p-13;
    return t;
}

SLO_HD float sincosf_poly_(double x, double x2, const sincos_tab& p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = madd_(x2, p.s3, p.s2);
        double x7 = x3 * x2;
        double s = madd_(x3, p.s1, x);
        return (float)madd_(x7, s1, s);
    } else {
        double x4 = x2 * x2;
        double c2 = madd_(x2, p.c4, p.c3);
        double c1 = madd_(x2, p.c1, p.c0);
        double x6 = x4 * x2;
        double c = madd_(x4, p.c2, c1);
        return (float)madd_(x6, c2, c);
    }
}

SLO_HD uint32_t abstop12_(float x) { return (f2u(x) >> 20) & 0x7ff; }

SLO_HD double reduce_fast_(double x, const sincos_tab& p, int* np) {
    double r = x * p.hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
#if SLO_SINCOS_FMA
    return fma(-(double)n, p.hpi, x);
#else
    return x - n * p.hpi;
#endif
}

SLO_HD double reduce_large_(uint32_t xi, int* np) {
    const uint32_t inv_pio4[24] = {
        0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415,
        0x4e441529, 0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5,
        0x57d1f534, 0xd1f534dd, 0xf534ddc0, 0x34ddc0db, 0xddc0db62, 0xc0db6295,
        0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};
    const uint32_t* arr = &inv_pio4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = (uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * 0x1.921FB54442D18p-62;
}

SLO_HD float sinf_(float y) {
    const float pio4 = 0x1.921FB6p-1f;
    double x = y;
    int n;
    if (abstop12_(y) < abstop12_(pio4)) {
        double s = x * x;
        if (abstop12_(y) < abstop12_(0x1p-12f)) return y;
        return sincosf_poly_(x, s, sincos_table(0), 0);
    } else if (abstop12_(y) < abstop12_(120.0f)) {
        x = reduce_fast_(x, sincos_table(0), &n);
        double s = ((n & 3) == 0 || (n & 3) == 3) ? 1.0 : -1.0;
        const sincos_tab p = sincos_table((n & 2) ? 1 : 0);
        return sincosf_poly_(x * s, x * x, p, n);
    } else if (abstop12_(y) < abstop12_(__builtin_inff())) {
        uint32_t xi = f2u(y);
        int sign = xi >> 31;
        x = reduce_large_(xi, &n);
        int q = (n + sign) & 3;
        double s = (q == 0 || q == 3) ? 1.0 : -1.0;
        const sincos_tab p = sincos_table(((n + sign) & 2) ? 1 : 0);
        return sincosf_poly_(x * s, x * x, p, n);
    }
    return (y - y) / (y - y);
}

SLO_HD float cosf_(float y) {
    const float pio4 = 0x1.921FB6p-1f;
    double x = y;
    int n;
    if (abstop12_(y) < abstop12_(pio4)) {
        double x2 = x * x;
        if (abstop12_(y) < abstop12_(0x1p-12f)) return 1.0f;
        return sincosf_poly_(x, x2, sincos_table(0), 1);
    } else if (abstop12_(y) < abstop12_(120.0f)) {
        x = reduce_fast_(x, sincos_table(0), &n);
        double s = ((n & 3) == 0 || (n & 3) == 3) ? 1.0 : -1.0;
        const sincos_tab p = sincos_table((n & 2) ? 1 : 0);
        return sincosf_poly_(x * s, x * x, p, n ^ 1);
    } else if (abstop12_(y) < abstop12_(__builtin_inff())) {
        uint32_t xi = f2u(y);
        int sign = xi >> 31;
        x = reduce_large_(xi, &n);
        int q = (n + sign) & 3;
        double s = (q == 0 || q == 3) ? 1.0 : -1.0;
        const sincos_tab p = sincos_table(((n + sign) & 2) ? 1 : 0);
        return sincosf_poly_(x * s, x * x, p, n ^ 1);
    }
    return (y - y) / (y - y);
}

// sinf_ and cosf_ of one argument with one range reduction (the same
// expressions as the two functions above, so the same bits)
SLO_HD void sincosf_(float y, float* sp, float* cp) {
    const float pio4 = 0x1.921FB6p-1f;
    double x = y;
    int n;
    if (abstop12_(y) < abstop12_(pio4)) {
        double s = x * x;
        if (abstop12_(y) < abstop12_(0x1p-12f)) { *sp = y; *cp = 1.0f; return; }
        *sp = sincosf_poly_(x, s, sincos_table(0), 0);
        *cp = sincosf_poly_(x, s, sincos_table(0), 1);
        return;
    } else if (abstop12_(y) < abstop12_(120.0f)) {
        x = reduce_fast_(x, sincos_table(0), &n);
        double s = ((n & 3) == 0 || (n & 3) == 3) ? 1.0 : -1.0;
        const sincos_tab p = sincos_table((n & 2) ? 1 : 0);
        *sp = sincosf_poly_(x * s, x * x, p, n);
        *cp = sincosf_poly_(x * s, x * x, p, n ^ 1);
        return;
    } else if (abstop12_(y) < abstop12_(__builtin_inff())) {
        uint32_t xi = f2u(y);
        int sign = xi >> 31;
        x = reduce_large_(xi, &n);
        int q = (n + sign) & 3;
        double s = (q == 0 || q == 3) ? 1.0 : -1.0;
        const sincos_tab p = sincos_table(((n + sign) & 2) ? 1 : 0);
        *sp = sincosf_poly_(x * s, x * x, p, n);
        *cp = sincosf_poly_(x * s, x * x, p, n ^ 1);
        return;
    }
    *sp = *cp = (y - y) / (y - y);
}

// ---------------------------------------------------------------- asinf
// glibc sysdeps/ieee754/flt-32/e_asinf.c (fdlibm float port with the
// single-precision polynomial R(x^2)).
SLO_HD float asinf_(float x) {
    const float one = 1.0f, huge = 1.000e+30f,
                pio2_hi = 1.57079637050628662109375f,
                pio2_lo = -4.37113900018624283e-8f,
                pio4_hi = 0.785398185253143310546875f,
                p0 = 1.666675248e-01f, p1 = 7.495297643e-02f, p2 = 4.547037598e-02f,
                p3 = 2.417951451e-02f, p4 = 4.216630880e-02f;
    float t, w, p, q, c, r, s;
    int32_t hx = (int32_t)f2u(x);
    int32_t ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;
    else if (ix > 0x3f800000) return (x - x) / (x - x);
    else if (ix < 0x3f000000) {
        if (ix < 0x32000000) {
            if (huge + x > one) return x;
        } else {
            t = x * x;
            w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
            return x + x * w;
        }
    }
    w = one - fabsf(x);
    t = w * 0.5f;
    p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    s = sqrtf(t);
    if (ix >= 0x3F79999A) {
        t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
    } else {
        w = s;
        w = u2f(f2u(w) & 0xfffff000u);
        c = (t - w * w) / (s + w);
        r = p;
        p = 2.0f * s * r - (pio2_lo - 2.0f * c);
        q = pio4_hi - 2.0f * w;
        t = pio4_hi - (p - q);
    }
    return (hx > 0) ? t : -t;
}

// ---------------------------------------------------------------- hypotf
// glibc sysdeps/ieee754/flt-32/e_hypotf.c: evaluated in double.
SLO_HD float hypotf_(float x, float y) {
    uint32_t ha = f2u(x) & 0x7fffffffu, hb = f2u(y) & 0x7fffffffu;
    if (ha == 0x7f800000u) return fabsf(x);
    if (hb == 0x7f800000u) return fabsf(y);
    if (ha > 0x7f800000u || hb > 0x7f800000u) return fabsf(x) * fabsf(y);
    if (ha == 0) return fabsf(y);
    if (hb == 0) return fabsf(x);
    double dx = x, dy = y;
    return (float)sqrt(dx * dx + dy * dy);
}

}  // namespace slo_libm
