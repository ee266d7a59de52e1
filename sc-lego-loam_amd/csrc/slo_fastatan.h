// slo_fastatan.h — a cheap bracket around slo_libm::atan2f_ (glibc's atan2f).
//
// The image projection decides integer bins and predicates from atan2f
// values: the row / column of a point (IP:229-240), the ground test of a
// row pair (IP:286-293) and the segment edge test (IP:411-423).  Each of
// those decisions is a monotone function of the atan2f value (the float
// pipelines after it — x 180, / pi, + ang_bottom, / ang_res, truncation or
// round(), comparisons — never reverse order).  So a polynomial atan2 with a
// proven error bound E gives lo <= atan2f_(y, x) <= hi, and when the decision
// is the same at lo and at hi it is the decision at the exact value; only
// points within ~1e-5 rad of a bin boundary (well under 1 %) pay for the
// exact glibc-faithful atan2f_.
//
// E: the degree-13 odd polynomial below, evaluated in float without FMA
// (-ffp-contract=off), differs from atan2 by < 6e-7 rad over the float plane
// (measured over 4e7 random and 8e7 grid points); glibc's atan2f is within
// 1 ulp (< 2.4e-7 at |angle| <= pi).  E = 2.5e-6 keeps a 3x margin, and the
// bracket property itself is checked against atan2f_ by
// tests/cpp/atan_bracket_check.cpp.
#pragma once

#include "slo_libm.h"

namespace slo_fast {

#define SLO_FAST_ATAN_E 2.5e-6f

// false for inputs the polynomial does not cover (both zero, inf, NaN)
SLO_HD bool atan2_bracket(float y, float x, float& lo, float& hi) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    if (!(mx > 0.0f) || !(mx <= 3.402823466e38f)) return false;
    const float a = mn / mx;
    const float s = a * a;
    float p = 0.0068117305636405945f;
    p = p * s + -0.03360404819250107f;
    p = p * s + 0.0796234980225563f;
    p = p * s + -0.13233335316181183f;
    p = p * s + 0.19807815551757812f;
    p = p * s + -0.3331736922264099f;
    p = p * s + 0.9999961256980896f;
    float r = p * a;
    if (ay > ax) r = 1.5707963267948966f - r;
    if (x < 0.0f) r = 3.141592653589793f - r;
    r = copysignf(r, y);
    lo = r - SLO_FAST_ATAN_E;
    hi = r + SLO_FAST_ATAN_E;
    return true;
}

}  // namespace slo_fast
