// atan_bracket_check.cpp — slo_fast::atan2_bracket (the image projection's
// fast path, sc-lego-loam_amd/csrc/slo_fastatan.h) must bracket
// slo_libm::atan2f_ (glibc atan2f, bit-exact) for every input it accepts.
// Random float pairs over many magnitudes, LiDAR-like coordinates, axes and
// signed zeros.  Built and run by tests/test_oracle_cpu.py; prints
// "<violations> <cases> <max |r - atan2f_|>".
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include "../../sc-lego-loam_amd/csrc/slo_fastatan.h"

int main() {
    uint64_t st = 0x9E3779B97F4A7C15ULL;
    auto nx = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    auto uni = [&]() { return (double)(nx() >> 11) * (1.0 / 9007199254740992.0); };
    long bad = 0, cases = 0;
    double worst = 0;
    auto check = [&](float y, float x) {
        float lo, hi;
        if (!slo_fast::atan2_bracket(y, x, lo, hi)) return;
        const float e = slo_libm::atan2f_(y, x);
        ++cases;
        if (!(lo <= e && e <= hi)) ++bad;
        worst = std::fmax(worst, std::fabs(0.5 * ((double)lo + (double)hi) - (double)e));
    };
    for (int i = 0; i < 20000000; ++i) {   // LiDAR-like: coordinates in +-200 m
        const float a = (float)(uni() * 400.0 - 200.0), b = (float)(uni() * 400.0 - 200.0);
        check(a, b);
        check(a * 1e-3f, b);
    }
    for (int i = 0; i < 4000000; ++i) {    // random bit patterns (finite)
        uint32_t u = (uint32_t)nx(), w = (uint32_t)(nx() >> 32);
        float y, x;
        std::memcpy(&y, &u, 4);
        std::memcpy(&x, &w, 4);
        if (!std::isfinite(y) || !std::isfinite(x)) continue;
        check(y, x);
    }
    const float edge[] = {0.0f, -0.0f, 1.0f, -1.0f, 1e-30f, -1e-30f, 1e30f, -1e30f, 3.0e38f, -3.0e38f};
    for (float y : edge)
        for (float x : edge) check(y, x);
    std::printf("%ld %ld %.3e\n", bad, cases, worst);
    return 0;
}
