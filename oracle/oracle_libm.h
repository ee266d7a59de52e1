// oracle_libm.h — TEST INFRASTRUCTURE: the oracle's elementary functions are
// the host glibc's own, called directly.
//
// The reference calls glibc: `using namespace std` (utility.h:49) resolves
// atan2(float, float) / sin(float) / cos(float) / asin(float) to atan2f /
// sinf / cosf / asinf (imageProjection.cpp:229, :235, :284, :421;
// featureAssociation.cpp:504, :871, ...), and tf's double quaternion / getRPY
// conversions (mapOptmization.cpp:1601-1611, transformFusion.cpp) and the IMU
// gravity terms (featureAssociation.cpp:391-393) to the double sin / cos /
// atan2 / asin.  The oracle therefore calls those same functions, and shares no
// arithmetic with the product's device restatements (csrc/slo_libm.h,
// csrc/slo_libm_d.h): GPU parity pins those restatements to glibc.  The
// restatements are also checked against glibc directly on the CPU
// (tests/cpp/libm_check.cpp, tests/test_oracle_cpu.py).
//
// The names keep the restatements' spelling (atan2f_, sin_d, ...) so that the
// oracle's line-by-line transcriptions read the same as the product's.
#pragma once

#include <math.h>
#include <stdint.h>
#include <string.h>

namespace oracle_libm {

inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

inline float atan2f_(float y, float x) { return ::atan2f(y, x); }
inline float atanf_(float x) { return ::atanf(x); }
inline float sinf_(float x) { return ::sinf(x); }
inline float cosf_(float x) { return ::cosf(x); }
inline float asinf_(float x) { return ::asinf(x); }

inline double sin_d(double x) { return ::sin(x); }
inline double cos_d(double x) { return ::cos(x); }
inline double atan2_d(double y, double x) { return ::atan2(y, x); }
inline double asin_d(double x) { return ::asin(x); }

}  // namespace oracle_libm
