// libm_check.cpp — the product's host/device libm restatements
// (csrc/slo_libm.h float, csrc/slo_libm_d.h double) against the host glibc.
// Built as a small shared library by tests/test_oracle_cpu.py (g++
// -ffp-contract=off, the product's build rule).  The oracle itself calls glibc
// directly (oracle/oracle_libm.h), so these checks are the CPU-side half of
// pinning the restatements; GPU parity is the other half.
#include <cmath>
#include <cstdint>
#include "../../sc-lego-loam_amd/csrc/slo_libm.h"
#include "../../sc-lego-loam_amd/csrc/slo_libm_d.h"

extern "C" {

// atan2f, sinf, cosf, atanf, asinf of n pseudo-random inputs (raw bit
// patterns and scaled integers alternately): how many differ from glibc
long libm_selftest(long n, unsigned long seed) {
    uint64_t st = seed * 0x9E3779B97F4A7C15ULL + 1;
    auto nx = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    auto same = [](float a, float b) { return slo_libm::f2u(a) == slo_libm::f2u(b) || (std::isnan(a) && std::isnan(b)); };
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        const uint64_t r = nx();
        float y = slo_libm::u2f((uint32_t)r), x = slo_libm::u2f((uint32_t)(r >> 32));
        if (i & 1) {
            y = (float)((int32_t)(r & 0xffffff) - 0x800000) * 1e-5f;
            x = (float)((int32_t)((r >> 24) & 0xffffff) - 0x800000) * 1e-5f;
        }
        bad += !same(slo_libm::atan2f_(y, x), atan2f(y, x));
        bad += !same(slo_libm::sinf_(y), sinf(y));
        bad += !same(slo_libm::cosf_(y), cosf(y));
        bad += !same(slo_libm::atanf_(y), atanf(y));
        const float u = fmodf(y, 1.0f);
        bad += !same(slo_libm::asinf_(u), asinf(u));
    }
    return bad;
}

// slo_libm_d.h elementwise: which = 0 sin, 1 cos, 2 atan2(a, b), 3 asin
void libm_d(int which, const double* a, const double* b, double* out, int n) {
    for (int i = 0; i < n; ++i)
        out[i] = which == 0 ? slo_libm::sin_d(a[i]) : which == 1 ? slo_libm::cos_d(a[i])
               : which == 2 ? slo_libm::atan2_d(a[i], b[i]) : slo_libm::asin_d(a[i]);
}

}  // extern "C"
