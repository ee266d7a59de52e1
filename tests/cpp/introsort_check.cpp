// introsort_check.cpp — compares slo_sort::std_sort and std_sort_small (the restatements the GPU
// feature extraction runs per lane) with the host libstdc++ std::sort on
// cloudSmoothness-like arrays full of ties (FA:699 sorts by value only, so the
// permutation of equal keys is implementation-defined and must match).
// Built and run by tests/test_oracle_cpu.py.  Prints the mismatch count.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
#include "../../sc-lego-loam_amd/csrc/slo_introsort.h"

struct Smooth { float value; int ind; };

int main() {
    uint64_t st = 0x9E3779B97F4A7C15ULL;
    auto nx = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    long bad = 0, cases = 0;
    const int sizes[] = {0, 1, 2, 3, 15, 16, 17, 31, 32, 33, 64, 100, 256, 300, 1000, 4096};
    for (int n : sizes)
        for (int rep = 0; rep < 60; ++rep) {
            const int levels = 1 + (int)(nx() % 8) * (rep % 3 == 0 ? 1 : 37);   // heavy and light ties
            std::vector<Smooth> a(n);
            for (int i = 0; i < n; ++i) a[i] = {(float)(nx() % levels) * 0.25f, i};
            if (rep % 7 == 1) std::sort(a.begin(), a.end(), [](const Smooth& x, const Smooth& y) { return x.ind > y.ind; });
            if (rep % 11 == 2)   // sorted / reverse-sorted inputs drive the depth limit
                std::sort(a.begin(), a.end(), [](const Smooth& x, const Smooth& y) { return x.value > y.value; });
            std::vector<Smooth> b = a, c = a;
            auto less = [](const Smooth& x, const Smooth& y) { return x.value < y.value; };
            std::sort(a.begin(), a.end(), less);
            slo_sort::std_sort(b.data(), n, less);
            slo_sort::std_sort_small(c.data(), n, less);   // the packed-stack form the GPU lanes run
            ++cases;
            for (int i = 0; i < n; ++i)
                if (a[i].ind != b[i].ind || a[i].value != b[i].value || a[i].ind != c[i].ind) { ++bad; break; }
        }
    // introsort_range_small against introsort_range (the PCL-sort lane tasks:
    // a sub-range with `depth` levels of budget left, depth 0 included)
    for (int rep = 0; rep < 3000; ++rep) {
        const int n = (int)(nx() % 300), depth = (int)(nx() % 27), levels = 1 + (int)(nx() % 12);
        std::vector<Smooth> a(n);
        for (int i = 0; i < n; ++i) a[i] = {(float)(nx() % levels), i};
        if (rep % 5 == 1) std::sort(a.begin(), a.end(), [](const Smooth& x, const Smooth& y) { return x.value > y.value; });
        std::vector<Smooth> b = a;
        auto less = [](const Smooth& x, const Smooth& y) { return x.value < y.value; };
        slo_sort::introsort_range(a.data(), n, depth, less);
        slo_sort::introsort_range_small(b.data(), n, depth, less);
        ++cases;
        for (int i = 0; i < n; ++i)
            if (a[i].ind != b[i].ind) { ++bad; break; }
    }
    printf("%ld %ld\n", bad, cases);
    return 0;
}
