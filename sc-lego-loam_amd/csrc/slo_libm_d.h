// slo_libm_d.h — double sin / cos / atan / atan2 / asin that give the same
// bits on the host and on the device (gfx950).
//
// Used only by the mapping node's f64 angle round trips (slo_pose.h
// odom_handoff / keyframe_estimate and their restatement in
// oracle/oracle_tf.h).  Those round trips end in a float cast,
// but for small angles the cast does not hide the last double bit, and the
// device's ocml and the host's glibc disagree in that bit now and then — so
// both builds evaluate the one implementation below.  The algorithms are
// fdlibm's (Sun's freely distributable libm: k_sin.c, k_cos.c, e_rem_pio2.c
// medium-argument path, s_atan.c, e_atan2.c, e_asin.c) with the integer
// word tests written on the bit pattern.  Against glibc's (correctly rounded
// in practice) results they are within 1 ulp; tests/test_libm.py measures
// that.  Arguments here are pose angles (|x| < 2^20 pi/2, the range of the
// medium reduction); no large-argument reduction.
//
// Build rule: -ffp-contract=off, like slo_libm.h.
#pragma once

#include "slo_libm.h"

namespace slo_libm {

SLO_HD double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
SLO_HD int32_t hi32(double d) { return (int32_t)(d2u(d) >> 32); }
SLO_HD double with_lo0(double d) { return u2d(d2u(d) & 0xffffffff00000000ull); }

// __kernel_sin(x, y, iy) on [-pi/4, pi/4], y the tail of x
SLO_HD double ksin_d(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    if ((hi32(x) & 0x7fffffff) < 0x3e400000) return x;   // |x| < 2^-27
    const double z = x * x, v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

// __kernel_cos(x, y) on [-pi/4, pi/4]
SLO_HD double kcos_d(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const int32_t ix = hi32(x) & 0x7fffffff;
    if (ix < 0x3e400000) return 1.0;   // |x| < 2^-27
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ix < 0x3fd33333) return 1.0 - (0.5 * z - (z * r - x * y));   // |x| < 0.3
    const double qx = ix > 0x3fe90000 ? 0.28125 : u2d((uint64_t)(uint32_t)(ix - 0x00200000) << 32);   // x/4
    const double hz = 0.5 * z - qx, a = 1.0 - qx;
    return a - (hz - (z * r - x * y));
}

// x = n pi/2 + (y0 + y1), medium arguments (e_rem_pio2.c, |x| < 2^20 pi/2)
SLO_HD int rem_pio2_d(double x, double& y0, double& y1) {
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const double pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21;
    const double pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
    const int32_t hx = hi32(x), ix = hx & 0x7fffffff;
    const double t = fabs(x);
    const int n = (int)(t * invpio2 + 0.5);
    const double fn = (double)n;
    double r = t - fn * pio2_1, w = fn * pio2_1t;
    y0 = r - w;
    const int j = ix >> 20;
    if (j - ((hi32(y0) >> 20) & 0x7ff) > 16) {   // cancellation: second round (118 bits)
        double u = r;
        w = fn * pio2_2;
        r = u - w;
        w = fn * pio2_2t - ((u - r) - w);
        y0 = r - w;
        if (j - ((hi32(y0) >> 20) & 0x7ff) > 49) {   // third round (151 bits)
            u = r;
            w = fn * pio2_3;
            r = u - w;
            w = fn * pio2_3t - ((u - r) - w);
            y0 = r - w;
        }
    }
    y1 = (r - y0) - w;
    if (hx < 0) { y0 = -y0; y1 = -y1; return -n; }
    return n;
}

SLO_HD double sin_d(double x) {
    if ((hi32(x) & 0x7fffffff) <= 0x3fe921fb) return ksin_d(x, 0.0, 0);   // |x| <= pi/4
    double y0, y1;
    const int n = rem_pio2_d(x, y0, y1);
    switch (n & 3) {
        case 0: return ksin_d(y0, y1, 1);
        case 1: return kcos_d(y0, y1);
        case 2: return -ksin_d(y0, y1, 1);
        default: return -kcos_d(y0, y1);
    }
}

SLO_HD double cos_d(double x) {
    if ((hi32(x) & 0x7fffffff) <= 0x3fe921fb) return kcos_d(x, 0.0);
    double y0, y1;
    const int n = rem_pio2_d(x, y0, y1);
    switch (n & 3) {
        case 0: return kcos_d(y0, y1);
        case 1: return -ksin_d(y0, y1, 1);
        case 2: return -kcos_d(y0, y1);
        default: return ksin_d(y0, y1, 1);
    }
}

// s_atan.c
SLO_HD double atan_d(double x) {
    const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                              1.57079632679489655800e+00};
    const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                              6.12323399573676603587e-17};
    const double aT[11] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                           -1.11111104054623557880e-01, 9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                           6.66107313738753120669e-02,  -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                           -3.65315727442169155270e-02, 1.62858201153657823623e-02};
    const int32_t hx = hi32(x), ix = hx & 0x7fffffff;
    if (ix >= 0x44100000) {   // |x| >= 2^66
        if (x != x) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    int id;
    if (ix < 0x3fdc0000) {   // |x| < 0.4375
        if (ix < 0x3e200000) return x;   // |x| < 2^-29
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000) {   // |x| < 1.1875
            if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
            else { id = 1; x = (x - 1.0) / (x + 1.0); }
        } else {
            if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }
            else { id = 3; x = -1.0 / x; }
        }
    }
    const double z = x * x, w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

// e_atan2.c (finite arguments)
SLO_HD double atan2_d(double y, double x) {
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16,
                 pi_o_2 = 1.5707963267948965580e+00;
    if (x != x || y != y) return x + y;
    if (x == 1.0) return atan_d(y);
    const int32_t hx = hi32(x), hy = hi32(y), ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);   // 2 sign(x) + sign(y)
    if (y == 0.0) {
        switch (m) {
            case 0: case 1: return y;
            case 2: return pi;
            default: return -pi;
        }
    }
    if (x == 0.0) return hy < 0 ? -pi_o_2 : pi_o_2;
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0;
    else z = atan_d(fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// e_asin.c
SLO_HD double asin_d(double x) {
    const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17,
                 pio4_hi = 7.85398163397448278999e-01;
    const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
                 qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    const int32_t hx = hi32(x), ix = hx & 0x7fffffff;
    if (ix >= 0x3ff00000) {   // |x| >= 1
        if (x == 1.0 || x == -1.0) return x * pio2_hi + x * pio2_lo;
        return (x - x) / (x - x);
    }
    if (ix < 0x3fe00000) {   // |x| < 0.5
        if (ix < 0x3e400000) return x;
        const double t = x * x;
        const double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
        const double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
        return x + x * (p / q);
    }
    const double w0 = 1.0 - fabs(x);
    double t = w0 * 0.5;
    double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
    double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
    const double s = sqrt(t);
    if (ix >= 0x3fef3333) {   // |x| > 0.975
        const double w = p / q;
        t = pio2_hi - (2.0 * (s + s * w) - pio2_lo);
    } else {
        const double w = with_lo0(s);
        const double c = (t - w * w) / (s + w);
        const double r = p / q;
        p = 2.0 * s * r - (pio2_lo - 2.0 * c);
        q = pio4_hi - 2.0 * w;
        t = pio4_hi - (p - q);
    }
    return hx > 0 ? t : -t;
}

}  // namespace slo_libm
