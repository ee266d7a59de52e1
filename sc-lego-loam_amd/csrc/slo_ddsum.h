// slo_ddsum.h — order-independent normal-equation sums (host + device).
//
// The reference forms AtA / AtB with OpenCV's GEMM on float Mats
// (featureAssociation.cpp:1324-1326, 1425-1427; mapOptmization.cpp:1445-1447);
// its internal accumulation order is not pinned.  Every
// term here is a product of two floats, which is exact in double, so the only
// rounding is in the summation.  The batched kernels sum in a tree, the CPU
// restatement sequentially; to make both give the same float they accumulate
// in double-double (Knuth TwoSum, ~106-bit significand) and round the result
// once, correctly, to float.  That is the correctly rounded float of the exact
// sum whenever the accumulated error (~n * 2^-104 * sum|x|) stays below the
// distance to a float rounding boundary — i.e. always, except for sums that
// land within ~2^-80 relative of a float midpoint.  Needs -ffp-contract=off
// (no FMA contraction inside TwoSum), which both builds use.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SLO_DD_HD __host__ __device__ inline
#else
#include <cmath>
#define SLO_DD_HD inline
#endif

namespace slo_dd {

struct DD {
    double hi, lo;
};

SLO_DD_HD DD zero() { return DD{0.0, 0.0}; }

// x += v (v exact, e.g. a product of two floats)
SLO_DD_HD void add(DD& x, double v) {
    const double s = x.hi + v;
    const double bb = s - x.hi;
    const double e = (x.hi - (s - bb)) + (v - bb) + x.lo;
    x.hi = s + e;
    x.lo = e - (x.hi - s);
}

// x += y
SLO_DD_HD void merge(DD& x, const DD& y) {
    const double s = x.hi + y.hi;
    const double bb = s - x.hi;
    const double e = (x.hi - (s - bb)) + (y.hi - bb) + (x.lo + y.lo);
    x.hi = s + e;
    x.lo = e - (x.hi - s);
}

// correctly rounded (to nearest, ties to even) float of hi + lo
SLO_DD_HD float to_float(const DD& x) {
    const float f = (float)x.hi;
    if (!(f - f == 0.0f)) return f;   // inf / nan
    const double d = ((double)x.hi - (double)f) + x.lo;   // residual, hi - f exact
    if (d == 0.0) return f;
    const float g = nextafterf(f, d > 0 ? __builtin_huge_valf() : -__builtin_huge_valf());
    const double h = ((double)g - (double)f) * 0.5;        // signed half gap toward d
    if (d > 0 ? d > h : d < h) return g;
    if (d == h) {                                          // exact tie: even significand
        unsigned int uf;
        __builtin_memcpy(&uf, &f, 4);
        return (uf & 1u) ? g : f;
    }
    return f;
}

}  // namespace slo_dd
