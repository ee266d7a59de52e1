// sincos_check.cpp — slo_libm::sincosf_ (one range reduction, used by the
// GPU pose transforms) against slo_libm::sinf_ / cosf_ bit for bit, and both
// against the host glibc sinf / cosf.  Built and run by
// tests/test_oracle_cpu.py.  Prints the mismatch count and the case count.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include "../../sc-lego-loam_amd/csrc/slo_libm.h"

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

int main() {
    uint64_t st = 0x243F6A8885A308D3ULL;
    auto nx = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    long bad = 0, cases = 0;
    auto check = [&](float y) {
        float s, c;
        slo_libm::sincosf_(y, &s, &c);
        const float s1 = slo_libm::sinf_(y), c1 = slo_libm::cosf_(y);
        bad += bits(s) != bits(s1) || bits(c) != bits(c1);
        if (std::isfinite(y)) bad += bits(s1) != bits(sinf(y)) || bits(c1) != bits(cosf(y));
        ++cases;
    };
    for (int i = 0; i < 400000; ++i) {
        const uint32_t u = (uint32_t)nx();
        float y;
        std::memcpy(&y, &u, 4);
        if (std::isnan(y)) continue;
        check(y);
    }
    for (int i = 0; i < 400000; ++i) check((float)((double)(nx() % 2000001) / 1000.0 - 1000.0) * 0.01f);
    const float edge[] = {0.0f, -0.0f, 0x1p-12f, 0x1.921FB6p-1f, 120.0f, -120.0f, 1e30f, -1e30f};
    for (float y : edge) check(y);
    std::printf("%ld %ld\n", bad, cases);
    return 0;
}
