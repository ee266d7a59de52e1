// pcl_sort_model.cpp — TEST INFRASTRUCTURE.  The data-parallel formulation
// of libstdc++'s std::sort that the GPU VoxelGrid uses for PCL's in-voxel
// order (csrc/slo_vgpcl.hip), checked against the host's std::sort on the
// (voxel index, point index) pairs PCL sorts (VoxelGrid::applyFilter,
// featureAssociation.cpp:779-780, mapOptmization.cpp:1224-1262).
//
// One partition step of [f, l) (size > 16, depth > 0): the median of
// a[f+1], a[f+(l-f)/2], a[l-1] is swapped to f (pivot p); over [f+1, l) a
// "left stopper" is an element with !(a < p), a "right stopper" one with
// !(p < a).  The unguarded Hoare loop swaps the k-th left stopper from the
// left (i_k) with the k-th right stopper from the right (j_k) for k = 1..m,
// m = max k with i_k < j_k = max over boundaries x of
// min(#left stoppers before x, #right stoppers at or after x), and returns
// cut = min(i_{m+1}, j_m) (absent terms are +inf).  Both children keep
// depth - 1; depth 0 is heapsort; leaves (size <= 16) end up stably sorted by
// the final insertion sort.  All of this depends only on the flags of the
// segment as it was before the step, so a step is a few scans.
//
//   pcl_sort_model <points.f32 file> <leaf> [T]   -> stats + "OK" / "MISMATCH"
//   pcl_sort_model --random <seed> <n> <nkeys>   -> same, random keys
//   pcl_sort_model --killer <n> <out.u32> [div] -> writes n keys that drive
//       libstdc++'s introsort into its depth limit (heapsort), by McIlroy's
//       "killer adversary" run against the host std::sort, then checks them;
//       with div, every key divided by div (ties inside the heapsort)
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <math.h>
#include <float.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include <random>
#include "../../sc-lego-loam_amd/csrc/slo_introsort.h"

struct It { unsigned int idx, pt; };
static bool lt(const It& a, const It& b) { return a.idx < b.idx; }

struct Stats { int max_level = 0, heapsorts = 0, leaves = 0; long long pairs = 0, items_levels = 0; int big_levels = 0; };

// the formulation: flags on the segment as it stands, then the pair swaps
static int partition_step(std::vector<It>& a, int f, int l, long long& pairs) {
    const int mid = f + (l - f) / 2;
    slo_sort::move_median_to_first_(&a[f], &a[f + 1], &a[mid], &a[l - 1], lt);
    const unsigned int p = a[f].idx;
    std::vector<int> L, R;
    for (int x = f + 1; x < l; ++x) if (!(a[x].idx < p)) L.push_back(x);
    for (int x = l - 1; x > f; --x) if (!(p < a[x].idx)) R.push_back(x);
    // m = max over x of min(#L < x, #R >= x)
    int m = 0;
    {
        int cl = 0, cr = (int)R.size();
        for (int x = f + 1; x <= l; ++x) {   // boundary before position x
            m = std::max(m, std::min(cl, cr));
            if (x < l) { if (!(a[x].idx < p)) ++cl; if (!(p < a[x].idx)) --cr; }
        }
    }
    for (int k = 0; k < m; ++k) std::swap(a[L[k]], a[R[k]]);
    pairs += m;
    const long long INF = 1ll << 40;
    const long long i_next = m < (int)L.size() ? L[m] : INF;
    const long long j_m = m > 0 ? R[m - 1] : INF;
    return (int)std::min(i_next, j_m);
}

static void model_sort(std::vector<It>& a, int T, Stats& st) {
    const int n = (int)a.size();
    if (n <= 1) return;
    struct Seg { int f, l, d, level; };
    std::vector<Seg> work{{0, n, 2 * slo_sort::lg_(n), 0}};
    std::vector<Seg> leaves;
    while (!work.empty()) {
        Seg s = work.back();
        work.pop_back();
        if (s.l - s.f <= 16) { leaves.push_back(s); continue; }
        if (s.l - s.f > T) st.big_levels = std::max(st.big_levels, s.level + 1);
        if (s.d == 0) {
            slo_sort::heap_sort_(&a[s.f], s.l - s.f, lt);
            ++st.heapsorts;
            continue;
        }
        st.max_level = std::max(st.max_level, s.level + 1);
        st.items_levels += s.l - s.f;
        const int cut = partition_step(a, s.f, s.l, st.pairs);
        work.push_back({s.f, cut, s.d - 1, s.level + 1});
        work.push_back({cut, s.l, s.d - 1, s.level + 1});
    }
    for (const Seg& s : leaves) {   // final insertion sort == stable sort of each leaf
        std::stable_sort(a.begin() + s.f, a.begin() + s.l, lt);
        ++st.leaves;
    }
}

static int check(std::vector<It> items, int T, const char* what) {
    std::vector<It> ref = items;
    std::sort(ref.begin(), ref.end(), lt);
    Stats st;
    model_sort(items, T, st);
    bool same = true;
    for (size_t i = 0; i < ref.size(); ++i)
        if (ref[i].idx != items[i].idx || ref[i].pt != items[i].pt) { same = false; break; }
    printf("%s n=%zu levels=%d levels_above_T=%d heapsorts=%d leaves=%d pairs/n=%.3f items*levels/n=%.2f %s\n", what,
           ref.size(), st.max_level, st.big_levels, st.heapsorts, st.leaves, (double)st.pairs / std::max<size_t>(1, ref.size()),
           (double)st.items_levels / std::max<size_t>(1, ref.size()), same ? "OK" : "MISMATCH");
    return same ? 0 : 1;
}

// McIlroy, "A killer adversary for quicksort" (1999): values are fixed
// lazily as the sort compares them ("gas" until one of a pair must be
// decided), which steers any quicksort to its worst case.
static std::vector<unsigned int> killer(int n) {
    std::vector<int> val(n, n - 1), ptr(n);
    int nsolid = 0, candidate = 0;
    const int gas = n - 1;
    for (int i = 0; i < n; ++i) ptr[i] = i;
    auto cmp = [&](int x, int y) -> int {
        if (val[x] == gas && val[y] == gas) {
            if (x == candidate) val[x] = nsolid++;
            else val[y] = nsolid++;
        }
        if (val[x] == gas) candidate = x;
        else if (val[y] == gas) candidate = y;
        return val[x] - val[y];
    };
    std::sort(ptr.begin(), ptr.end(), [&](int a, int b) { return cmp(a, b) < 0; });
    return std::vector<unsigned int>(val.begin(), val.end());
}

int main(int argc, char** argv) {
    if (argc >= 4 && !strcmp(argv[1], "--killer")) {
        const int n = atoi(argv[2]);
        std::vector<unsigned int> k = killer(n);
        if (argc >= 5)
            for (auto& x : k) x /= (unsigned)std::max(1, atoi(argv[4]));
        FILE* fo = fopen(argv[3], "wb");
        if (!fo) return 2;
        fwrite(k.data(), 4, k.size(), fo);
        fclose(fo);
        std::vector<It> v(n);
        for (int i = 0; i < n; ++i) v[i] = {k[i], (unsigned)i};
        return check(v, 4096, "killer");
    }
    if (argc >= 5 && !strcmp(argv[1], "--random")) {
        std::mt19937 rng((unsigned)atoi(argv[2]));
        const int n = atoi(argv[3]), nk = atoi(argv[4]);
        const int T = argc > 5 ? atoi(argv[5]) : 4096;
        int bad = 0;
        for (int mode = 0; mode < 5; ++mode) {
            std::vector<It> v(n);
            for (int i = 0; i < n; ++i) {
                unsigned int k = rng() % (unsigned)std::max(1, nk);
                if (mode == 1) k = (unsigned)(i / std::max(1, n / std::max(1, nk)));        // sorted runs
                if (mode == 2) k = (unsigned)((n - i) / std::max(1, n / std::max(1, nk)));  // reversed
                if (mode == 3) k = 7;                                                         // all equal
                if (mode == 4) k = (unsigned)((i * 2654435761u) >> 7) % (unsigned)std::max(1, nk) + (i & 1);
                v[i] = {k, (unsigned)i};
            }
            char what[64];
            snprintf(what, sizeof what, "random mode %d", mode);
            bad |= check(v, T, what);
        }
        return bad;
    }
    if (argc < 3) { fprintf(stderr, "usage\n"); return 2; }
    FILE* fp = fopen(argv[1], "rb");
    if (!fp) return 2;
    std::vector<float> buf;
    float tmp[4096];
    size_t r;
    while ((r = fread(tmp, 4, 4096, fp)) > 0) buf.insert(buf.end(), tmp, tmp + r);
    fclose(fp);
    const float leaf = (float)atof(argv[2]);
    const int T = argc > 3 ? atoi(argv[3]) : 4096;
    const size_t n = buf.size() / 4;
    const float inv = 1.0f / leaf;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) mn[k] = std::min(mn[k], buf[4 * i + k]);
    float mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) mx[k] = std::max(mx[k], buf[4 * i + k]);
    int minb[3], maxb[3];
    for (int k = 0; k < 3; ++k) { minb[k] = (int)floorf(mn[k] * inv); maxb[k] = (int)floorf(mx[k] * inv); }
    const int divx = maxb[0] - minb[0] + 1, divy = maxb[1] - minb[1] + 1;
    std::vector<It> items(n);
    for (size_t i = 0; i < n; ++i) {
        int a = (int)(floorf(buf[4 * i] * inv) - (float)minb[0]);
        int b = (int)(floorf(buf[4 * i + 1] * inv) - (float)minb[1]);
        int c = (int)(floorf(buf[4 * i + 2] * inv) - (float)minb[2]);
        items[i] = {(unsigned)(a + b * divx + c * divx * divy), (unsigned)i};
    }
    return check(items, T, argv[1]);
}
