// slo_pclsort.h — PCL's VoxelGrid order, computed in parallel.
//
// VoxelGrid<PointXYZI>::applyFilter (PCL 1.8; the reference calls it at
// featureAssociation.cpp:779-780 and mapOptmization.cpp:1224-1262) sorts the
// (voxel index, point index) pairs of the cloud with std::sort, comparing the
// voxel index only, and sums each voxel's points in the order that leaves.
// std::sort is not stable, so that order — and with it every centroid's
// float sum — is whatever libstdc++'s introsort makes of the input order.
// This header computes exactly that order for a range of up to 4097 items
// with one wave (wave_sort) or a few (block_sort).
//
// The formulation (checked against the host std::sort by
// tests/cpp/pcl_sort_model.cpp).  One introsort step on [f, l), size > 16,
// depth > 0: the median of a[f+1], a[f+(l-f)/2], a[l-1] is swapped to f
// (pivot p); over [f+1, l) a "left stopper" is an element with !(a < p) and a
// "right stopper" one with !(p < a).  The unguarded Hoare loop swaps the k-th
// left stopper from the left (i_k) with the k-th right stopper from the right
// (j_k), k = 1..m, where
//     m = max over boundaries x of min(#left stoppers before x,
//                                      #right stoppers at or after x),
// and returns cut = min(i_{m+1}, j_m) (absent terms +inf).  Both halves keep
// depth - 1; depth 0 is heapsort; a range of <= 16 ends up stably sorted by
// the final insertion sort.  Every quantity depends only on the flags of the
// range as it stood before the step: a step is two scans and one swap pass.
//
// wave_sort: the items of the range sit in LDS as 64-bit words (voxel index
// << 32 | point index).  The wave walks the introsort recursion depth first
// (an explicit stack of right halves; disjoint ranges are independent, so the
// order of the walk does not change the result) and takes each step with all
// 64 lanes:
//   * a range of more than 129 items: stream_step — rows of 64 positions are
//     streamed from LDS three times (stopper counts per row, kept one per lane
//     of a register; the right stoppers that swap, by rank, into a table; the
//     left stoppers' swaps), about 30 instructions per row and step;
//   * 17..129 items (when TLANE is below that): wave_step, the rows held in
//     registers across the step;
//   * at most TLANE (<= 64) items: wave_small_sort — one item per lane in
//     registers, every segment of the range stepped at once (lane masks,
//     lane permutes), the leaves ranked by (key, lane);
//   * a spent depth budget: a lane task.  Tasks queue up and 64 of them run
//     at once, one per lane, through the sequential libstdc++ restatement
//     (slo_sort::introsort_range: heapsort, then the final insertion sort
//     restricted to the range, which is all the global final insertion sort
//     does to it).  Adversarial inputs only.
// A full stack hands the range to a lane task (exact), a step whose cut falls
// outside (f, l) — impossible for a correct step — as well (then sorted but not
// necessarily in std::sort's order, instead of a hang); both count in *err,
// which the callers report and the tests require to stay 0.
#pragma once

#include "slo_introsort.h"

namespace slo_pcl {

typedef unsigned long long u64;

// Items: 64-bit (voxel index << 32 | point index), or 32-bit within one LDS
// range whose keys span less than 2^20 ((key - min) << 12 | position in the
// range, k_pc_finish32).  Only keys are ever compared.
constexpr int kPosBits = 12;
__host__ __device__ inline unsigned int vkey(u64 it) { return (unsigned int)(it >> 32); }
__host__ __device__ inline unsigned int vkey(unsigned int it) { return it >> kPosBits; }
struct Less {
    __host__ __device__ bool operator()(const u64& a, const u64& b) const { return (a >> 32) < (b >> 32); }
};
template <class It>
struct LessT {
    __host__ __device__ bool operator()(const It& a, const It& b) const { return vkey(a) < vkey(b); }
};
// the key at position x, read as a 32-bit word
__device__ __forceinline__ unsigned int key_at(const u64* a, int x) {
    return reinterpret_cast<const unsigned int*>(a)[2 * x + 1];
}
__device__ __forceinline__ unsigned int key_at(const unsigned int* a, int x) { return a[x] >> kPosBits; }

__host__ __device__ inline int lg2(int n) {
    int r = 0;
    while (n > 1) { n >>= 1; ++r; }
    return r;
}

constexpr int kQ = 64;        // lane tasks per flush
constexpr int kStack = 64;    // wave stack entries (the depth budget, <= 62, bounds the stack)

// per-wave LDS besides the items: the stack and the lane-task queue
struct WaveSmem {
    unsigned int stk[kStack];
    unsigned int q[kQ];
    unsigned char tw[128];   // wave_small_sort's partner tables
};

__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ int lane_prefix(unsigned long long b) {   // set bits of b below this lane
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned int)(b >> 32), __builtin_amdgcn_mbcnt_lo((unsigned int)b, 0u));
}

// libstdc++ __move_median_to_first on the keys at f + 1, mid, l - 1: which of
// them (0, 1, 2) is swapped to f
__host__ __device__ inline int median3(unsigned int a, unsigned int b, unsigned int c) {
    if (a < b) {
        if (b < c) return 1;
        if (a < c) return 2;
        return 0;
    }
    if (a < c) return 0;
    if (b < c) return 2;
    return 1;
}

// range encoding of the stack and the queue: first | end << 13 | depth << 26
__device__ __forceinline__ unsigned int renc(int f, int l, int d) {
    return (unsigned int)f | ((unsigned int)l << 13) | ((unsigned int)d << 26);
}

// one introsort step of [f, l) (l - f - 1 <= 64 R) with the range's positions
// f + 1 + 64 r + lane held in R rows of registers.  The median swap is taken
// virtually while the rows are read (one LDS round trip), m comes from the
// ballot of the crossing and two lane reads, and the LDS sees the median
// swap, the right-stopper table (tbl[f / 2 + rank]), its reads, the partner reads and
// the swaps.  Returns the cut.
template <int R, class It>
__device__ __forceinline__ int wave_step(It* items, unsigned short* tbl, int f, int l) {
    const int lane = threadIdx.x & 63;
    constexpr int INF = 0x7fffffff;
    const int mid = f + (l - f) / 2;
    const It a0 = items[f], a1 = items[f + 1], a2 = items[mid], a3 = items[l - 1];
    It it[R];
#pragma unroll
    for (int r = 0; r < R; ++r) it[r] = items[min(f + 1 + 64 * r + lane, l - 1)];
    const int w = median3(vkey(a1), vkey(a2), vkey(a3));
    const int med = w == 0 ? f + 1 : (w == 1 ? mid : l - 1);
    const It pit = w == 0 ? a1 : (w == 1 ? a2 : a3);
    const unsigned int p = vkey(pit);
    bool iL[R], iR[R];
    int pl[R], pr[R];
    int cl = 0, cr = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int x = f + 1 + 64 * r + lane;
        if (x == med) it[r] = a0;   // the item the median swap leaves there
        const bool act = x < l;
        const unsigned int k = vkey(it[r]);
        iL[r] = act && !(k < p);
        iR[r] = act && !(p < k);
        const unsigned long long bl = __ballot(iL[r]), br = __ballot(iR[r]);
        pl[r] = cl + lane_prefix(bl);
        pr[r] = cr + lane_prefix(br);
        cl += __popcll(bl);
        cr += __popcll(br);
    }
    const int TR = cr;
    // m = max over boundaries b of min(Lb, Rb) (left stoppers before b, right
    // ones at or after it): Lb grows and Rb falls with b, so the maximum sits
    // at the first boundary X with Lb >= Rb (there Rb) or just before it (there
    // Lb); the boundary at l always qualifies (Rb = 0)
    int X = l;
#pragma unroll
    for (int r = R - 1; r >= 0; --r) {
        const unsigned long long fx = __ballot(f + 1 + 64 * r + lane < l && pl[r] >= TR - pr[r]);
        if (fx) X = f + 1 + 64 * r + __builtin_ctzll(fx);
    }
    int m = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int base = f + 1 + 64 * r;
        if (X < l && X >= base && X < base + 64) m = max(m, TR - __builtin_amdgcn_readlane(pr[r], X - base));
        if (X - 1 >= f + 1 && X - 1 >= base && X - 1 < base + 64)
            m = max(m, __builtin_amdgcn_readlane(pl[r], X - 1 - base));
    }
    int cutA = INF, cutB = INF;
#pragma unroll
    for (int r = R - 1; r >= 0; --r) {   // i_{m+1}: the left stopper of rank m; j_m: the right one of rank m - 1
        const unsigned long long ba = __ballot(iL[r] && pl[r] == m);
        const unsigned long long bb = __ballot(iR[r] && TR - 1 - pr[r] == m - 1);
        if (ba) cutA = f + 1 + 64 * r + __builtin_ctzll(ba);
        if (bb) cutB = f + 1 + 64 * r + __builtin_ctzll(bb);
    }
    if (lane == 0) {   // the median swap, made real
        items[f] = pit;
        items[med] = a0;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int kr = TR - 1 - pr[r];
        if (iR[r] && kr < m) tbl[(f >> 1) + kr] = (unsigned short)(f + 1 + 64 * r + lane);
    }
    wave_fence();
    int y[R];
    It py[R];
#pragma unroll
    for (int r = 0; r < R; ++r) y[r] = (iL[r] && pl[r] < m) ? (int)tbl[(f >> 1) + pl[r]] : -1;
#pragma unroll
    for (int r = 0; r < R; ++r) py[r] = items[y[r] >= 0 ? y[r] : f];
    wave_fence();
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (y[r] >= 0) {
            items[f + 1 + 64 * r + lane] = py[r];
            items[y[r]] = it[r];
        }
    wave_fence();
    return min(cutA, m > 0 ? cutB : INF);
}

// one introsort step of [f, l), l - f - 1 <= 64 * 64, rows streamed from LDS.
// rowL / rowR hold, in lane r, the left / right stoppers before row r, so a
// row's exclusive prefixes are one lane read and a lane count away in every
// later pass; keys are the high words of the items.
template <class It>
__device__ __forceinline__ int stream_step(It* items, unsigned short* tbl, int f, int l) {
    const int lane = threadIdx.x & 63;
    constexpr int INF = 0x7fffffff;
    constexpr int U = 4;   // rows in flight
    const int mid = f + (l - f) / 2;
    const It a0 = items[f], a1 = items[f + 1], a2 = items[mid], a3 = items[l - 1];
    const int w = median3(vkey(a1), vkey(a2), vkey(a3));
    const int med = w == 0 ? f + 1 : (w == 1 ? mid : l - 1);
    const It pit = w == 0 ? a1 : (w == 1 ? a2 : a3);
    const unsigned int p = vkey(pit), k0 = vkey(a0);
    const int b0 = f + 1, R = (l - b0 + 63) >> 6;   // rows of [f + 1, l)
    // (1) stopper counts per row (the median swap taken virtually)
    int rowL = 0, rowR = 0, cl = 0, cr = 0;
    for (int r0 = 0; r0 < R; r0 += U) {
        unsigned int kk[U];
#pragma unroll
        for (int u = 0; u < U; ++u) kk[u] = key_at(items, min(b0 + 64 * (r0 + u) + lane, l - 1));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = r0 + u;
            if (r < R) {
                const int x = b0 + 64 * r + lane;
                const unsigned int k = x == med ? k0 : kk[u];
                const bool act = x < l;
                const unsigned long long bl = __ballot(act && !(k < p)), br = __ballot(act && !(p < k));
                rowL = lane == r ? cl : rowL;
                rowR = lane == r ? cr : rowR;
                cl += __popcll(bl);
                cr += __popcll(br);
            }
        }
    }
    const int TL = cl, TR = cr;
    // (2) m: the crossing (the first boundary X with Lb >= Rb) lies in the
    // first row c whose end boundary qualifies — its start boundary (row c - 1's
    // end) does not, so X is past row c's first position unless c = 0 and
    // X = f + 1.  The last row's end (Lb = TL, Rb = 0) always qualifies.
    int eL = __shfl_down(rowL, 1, 64), eR = __shfl_down(rowR, 1, 64);
    if (lane == R - 1) { eL = TL; eR = TR; }
    const int c = __builtin_ctzll(__ballot(lane < R && eL >= TR - eR));
    // a row's stoppers with their exclusive prefixes (the median swap virtual)
    auto row_flags = [&](int r, bool& iL, bool& iR, int& pl, int& pr) {
        const int x = b0 + 64 * r + lane;
        unsigned int k = key_at(items, min(x, l - 1));
        k = x == med ? k0 : k;
        const bool act = x < l;
        iL = act && !(k < p);
        iR = act && !(p < k);
        pl = __builtin_amdgcn_readlane(rowL, r) + lane_prefix(__ballot(iL));
        pr = __builtin_amdgcn_readlane(rowR, r) + lane_prefix(__ballot(iR));
    };
    int m;
    {
        bool iL, iR;
        int pl, pr;
        row_flags(c, iL, iR, pl, pr);
        const int bc = b0 + 64 * c;
        const unsigned long long fx = __ballot(bc + lane < l && pl >= TR - pr);
        if (fx) {
            const int xl = __builtin_ctzll(fx);
            m = TR - __builtin_amdgcn_readlane(pr, xl);                 // Rb(X)
            if (xl > 0) m = max(m, __builtin_amdgcn_readlane(pl, xl - 1));   // Lb(X - 1)
        } else {   // X = the row's end boundary
            const int last = min(63, l - 1 - bc);
            m = max(TR - __builtin_amdgcn_readlane(eR, c), __builtin_amdgcn_readlane(pl, last));
        }
    }
    // (3) the cuts: i_{m+1} (left stopper of rank m), j_m (right stopper with
    // TR - m right stoppers before it), each from its row
    int cutA = INF, cutB = INF, rA = R - 1, rB = 0;
    if (m < TL) {
        rA = __builtin_ctzll(__ballot(lane < R && rowL <= m && m < eL));
        bool iL, iR;
        int pl, pr;
        row_flags(rA, iL, iR, pl, pr);
        cutA = b0 + 64 * rA + __builtin_ctzll(__ballot(iL && pl == m));
    }
    if (m > 0) {
        const int t = TR - m;
        rB = __builtin_ctzll(__ballot(lane < R && rowR <= t && t < eR));
        bool iL, iR;
        int pl, pr;
        row_flags(rB, iL, iR, pl, pr);
        cutB = b0 + 64 * rB + __builtin_ctzll(__ballot(iR && pr == t));
    }
    if (lane == 0) {   // the median swap, made real
        items[f] = pit;
        items[med] = a0;
    }
    wave_fence();
    if (m > 0) {
        // (4) the m last right stoppers (rows rB ..), by rank from the right
        for (int r0 = rB; r0 < R; r0 += U) {
            unsigned int kk[U];
#pragma unroll
            for (int u = 0; u < U; ++u) kk[u] = key_at(items, min(b0 + 64 * (r0 + u) + lane, l - 1));
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = r0 + u;
                if (r < R) {
                    const int x = b0 + 64 * r + lane;
                    const bool iR = x < l && !(p < kk[u]);
                    const int kr = TR - 1 - (__builtin_amdgcn_readlane(rowR, r) + lane_prefix(__ballot(iR)));
                    if (iR && kr < m) tbl[(f >> 1) + kr] = (unsigned short)x;
                }
            }
        }
        wave_fence();
        // (5) the m first left stoppers (rows .. rA) swap with their partners;
        // every swapped left stopper lies before the crossing and every
        // partner at or after it, so a batch's loads see no earlier write
        const int rEnd = m < TL ? rA : R - 1;
        for (int r0 = 0; r0 <= rEnd; r0 += U) {
            It it[U], py[U];
            int y[U];
#pragma unroll
            for (int u = 0; u < U; ++u) it[u] = items[min(b0 + 64 * (r0 + u) + lane, l - 1)];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = r0 + u;
                y[u] = -1;
                if (r <= rEnd) {
                    const int x = b0 + 64 * r + lane;
                    const bool iL = x < l && !(vkey(it[u]) < p);
                    const int pl = __builtin_amdgcn_readlane(rowL, r) + lane_prefix(__ballot(iL));
                    if (iL && pl < m) y[u] = pl;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) y[u] = y[u] >= 0 ? (int)tbl[(f >> 1) + y[u]] : -1;
#pragma unroll
            for (int u = 0; u < U; ++u) py[u] = items[y[u] >= 0 ? y[u] : f];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (y[u] >= 0) {
                    items[b0 + 64 * (r0 + u) + lane] = py[u];
                    items[y[u]] = it[u];
                }
        }
        wave_fence();
    }
    return min(cutA, m > 0 ? cutB : INF);
}

// ---- ranges of at most 64 items: one item per lane, in registers.  Every
// segment still over 16 items with depth left takes its introsort step at
// once (the wave holds several segments side by side: lane masks), the
// median swap and the pair swaps are lane permutes, the partner of each
// stopper comes from a 64-entry LDS table; a segment of <= 16 items (a leaf)
// ends stably sorted — each lane's place is its rank in the leaf by (key,
// lane).  A segment over 16 items with its depth spent (only adversarial
// inputs) is left in place and returned for a lane task (heapsort).
__device__ __forceinline__ unsigned long long lanes_below(int k) {   // bits [0, k), 0 <= k <= 64
    return k >= 64 ? ~0ull : ((1ull << k) - 1ull);
}
__device__ __forceinline__ u64 shfl64(u64 v, int src) {
    const unsigned int lo = (unsigned int)__shfl((int)(unsigned int)v, src, 64);
    const unsigned int hi = (unsigned int)__shfl((int)(unsigned int)(v >> 32), src, 64);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 ishfl(u64 v, int src) { return shfl64(v, src); }
__device__ __forceinline__ unsigned int ishfl(unsigned int v, int src) {
    return (unsigned int)__shfl((int)v, src, 64);
}

// items[f, f + n), n <= 64, as one or more adjacent ranges: lane i's range is
// [lo0, hi0) (relative to f) with depth dd0 — several small ranges sorted in
// one call (wave_sort_range merges the adjacent ones off its stack); tw: 128
// bytes of this wave's LDS.  Returns the lanes that start a spent-depth
// segment (bit lo), the segment's end in *hend (per lane) for the caller's
// lane tasks.
template <class It>
__device__ __forceinline__ unsigned long long wave_small_sort(It* items, int f, int n, int lo0, int hi0, int dd0,
                                                              unsigned char* tw, int* hend) {
    const int i = threadIdx.x & 63;
    const bool live = i < n;
    It it = items[f + min(i, n - 1)];
    int lo = lo0, hi = hi0, dd = dd0;
    for (;;) {
        const bool act = live && hi - lo > 16 && dd > 0;
        if (__ballot(act) == 0) break;
        const int mid = lo + (hi - lo) / 2;
        const unsigned int key0 = vkey(it);
        const unsigned int ka = (unsigned int)__shfl((int)key0, act ? lo + 1 : i, 64);
        const unsigned int kb = (unsigned int)__shfl((int)key0, act ? mid : i, 64);
        const unsigned int kc = (unsigned int)__shfl((int)key0, act ? hi - 1 : i, 64);
        const int w = median3(ka, kb, kc);
        const int med = w == 0 ? lo + 1 : (w == 1 ? mid : hi - 1);
        const unsigned int p = w == 0 ? ka : (w == 1 ? kb : kc);
        it = ishfl(it, act ? (i == lo ? med : (i == med ? lo : i)) : i);   // the median swap
        const unsigned int k = vkey(it);
        const bool inr = act && i > lo;
        const bool iL = inr && !(k < p), iR = inr && !(p < k);
        const unsigned long long BL = __ballot(iL), BR = __ballot(iR);
        const unsigned long long seg = lanes_below(hi) & ~lanes_below(lo + 1), below = lanes_below(i) & seg;
        const int pl = __popcll(BL & below), pr = __popcll(BR & below);
        const int TL = __popcll(BL & seg), TR = __popcll(BR & seg);
        const unsigned long long Q = __ballot(inr && pl >= TR - pr) & seg;
        const int X = Q ? __builtin_ctzll(Q) : hi;   // the first boundary with Lb >= Rb
        const int prX = __shfl(pr, act && X < hi ? X : i, 64), plX1 = __shfl(pl, act && X - 1 > lo ? X - 1 : i, 64);
        const int m = max(X < hi ? TR - prX : 0, X - 1 > lo ? plX1 : 0);
        const unsigned long long A = __ballot(iL && pl == m) & seg, B = __ballot(iR && TR - 1 - pr == m - 1) & seg;
        const int cut = min(m < TL && A ? __builtin_ctzll(A) : 64, m > 0 && B ? __builtin_ctzll(B) : 64);
        // partners: left stopper of rank k <-> right stopper of rank k from the right
        const bool sL = iL && pl < m, sR = iR && TR - 1 - pr < m;
        if (sL) tw[lo + pl] = (unsigned char)i;
        if (sR) tw[64 + lo + (TR - 1 - pr)] = (unsigned char)i;
        wave_fence();
        int src = i;
        if (sL) src = tw[64 + lo + pl];
        if (sR) src = tw[lo + (TR - 1 - pr)];
        wave_fence();
        it = ishfl(it, src);
        if (act) {
            if (i < cut) hi = cut;
            else lo = cut;
            --dd;
        }
    }
    // leaves: an item's place is its rank in the leaf by (key, lane)
    const unsigned int k = vkey(it);
    const bool heap = live && hi - lo > 16;   // dd == 0
    int rank = 0;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const int j = lo + t;
        const unsigned int kj = (unsigned int)__shfl((int)k, min(j, 63), 64);
        rank += (j < hi) & ((kj < k) | ((kj == k) & (j < i)));
    }
    wave_fence();
    if (live) items[f + (heap ? i : lo + rank)] = it;
    wave_fence();
    *hend = hi;
    return __ballot(heap && i == lo);
}

// ---- std::sort's heapsort of a whole range (a spent depth budget; libstdc++
// __partial_sort(first, last, last): make_heap, then sort_heap — the
// restatement is slo_sort::heap_sort_), by one wave, exactly:
//   * make_heap adjusts the parents from the last to the first; parents of
//     one tree level own disjoint subtrees and every deeper parent comes
//     first, so the wave takes a level at a time, one parent per lane;
//   * each pop (__pop_heap, __adjust_heap, __push_heap) moves the hole from
//     the root to a leaf along the larger children (ties: the right one) —
//     a path that does not depend on the value being placed — and the value
//     then rises while its parent is less.  Along a root-to-leaf path of a
//     heap the keys do not increase, so it settles below the m path nodes
//     not less than it: path node i < m takes node i + 1's item, node m the
//     value.  The wave holds the top six levels (63 nodes) in registers, one
//     per lane, and loads the deeper part of the path five levels (62 nodes)
//     at a time: one LDS round trip per pop for ranges under 2048 items,
//     against two dependent loads per level for one lane.
// The final insertion sort std::sort runs over a heapsorted range moves
// nothing (slo_sort::introsort_range), so it is not run.
__device__ __forceinline__ u64 rl64(u64 x, int i) {
    i = __builtin_amdgcn_readfirstlane(i);
    const unsigned int lo = (unsigned int)__builtin_amdgcn_readlane((int)(unsigned int)x, i);
    const unsigned int hi = (unsigned int)__builtin_amdgcn_readlane((int)(unsigned int)(x >> 32), i);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 irl(u64 x, int i) { return rl64(x, i); }
__device__ __forceinline__ unsigned int irl(unsigned int x, int i) {
    return (unsigned int)__builtin_amdgcn_readlane((int)x, __builtin_amdgcn_readfirstlane(i));
}
// Global: `a` in global memory (pc_fallback_entry's scratch): the lanes' stores
// are ordered before the next reads by a workgroup-scope fence instead of the
// LDS wave fence.
template <bool Global>
__device__ __forceinline__ void heap_fence() {
    if (Global) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
    } else {
        wave_fence();
    }
}
template <class It, bool Global = false>
__device__ inline void wave_heap_sort(It* a, int n) {
    const int lane = threadIdx.x & 63;
    if (n < 2) return;
    const int P = (n - 2) / 2;   // the last parent
    for (int L = lg2(P + 1); L >= 0; --L) {
        const int lo = (1 << L) - 1, hi = min((1 << (L + 1)) - 2, P);
        for (int x = lo + lane; x <= hi; x += 64) slo_sort::adjust_heap_(a, x, n, a[x], LessT<It>());
        heap_fence<Global>();
    }
    constexpr int TOPN = 63;
    It top = lane < min(n, TOPN) ? a[lane] : (It)0;
    const int tlev = 31 - __builtin_clz(lane + 1);        // tree level of node `lane`
    const int cj = 31 - __builtin_clz(lane + 2), cq = lane + 2 - (1 << cj);   // chunk slot: level cj, position cq
    for (int len = n - 1; len >= 1; --len) {
        // __pop_heap(first, first + len, first + len)
        const It mx = irl(top, 0);
        It v;
        if (len < TOPN) {
            v = irl(top, len);
            if (lane == len) top = mx;
        } else {
            v = a[len];
            if (lane == 0) a[len] = mx;
        }
        const int lim = (len - 1) / 2;   // nodes below lim have two children
        int h = 0, k = 0, ph = 0;
        It pv = 0;
        while (h < lim && 2 * h + 2 < TOPN) {   // the path through the register levels
            const int r = 2 * h + 2;
            const It R = irl(top, r), Lf = irl(top, r - 1);
            const bool left = vkey(R) < vkey(Lf);
            h = left ? r - 1 : r;
            ++k;
            if (lane == k) { ph = h; pv = left ? Lf : R; }
        }
        while (h < lim) {   // deeper: the five levels below h in one load
            const int node = (h + 1) * (1 << cj) - 1 + cq;
            const It sub = (lane < 62 && node < len) ? a[node] : (It)0;
            int rel = 0;
            for (int j = 1; j <= 5 && h < lim; ++j) {
                const int tr = (1 << j) - 1 + 2 * rel;   // the right child's slot
                const It R = irl(sub, tr), Lf = irl(sub, tr - 1);
                const bool left = vkey(R) < vkey(Lf);
                rel = 2 * rel + (left ? 0 : 1);
                h = 2 * h + (left ? 1 : 2);
                ++k;
                if (lane == k) { ph = h; pv = left ? Lf : R; }
            }
        }
        if ((len & 1) == 0 && h == (len - 2) / 2) {   // the last parent's only child
            const int c = 2 * h + 1;
            const It cv = c < TOPN ? irl(top, c) : a[c];
            ++k;
            if (lane == k) { ph = c; pv = cv; }
        }
        const unsigned int kv = vkey(v);
        const int m = __popcll(__ballot(lane >= 1 && lane <= k && !(vkey(pv) < kv)));
        const It up = ishfl(pv, min(lane + 1, 63));   // (every lane takes part: a permute reads no inactive lane)
        const It w = lane < m ? up : v;
        const int phl = __shfl(ph, min(tlev, 63), 64);
        const It wl = ishfl(w, min(tlev, 63));
        if (lane <= m && ph >= TOPN) a[ph] = w;
        if (lane < TOPN && tlev <= m && phl == lane) top = wl;
        heap_fence<Global>();
    }
    if (lane < min(n, TOPN)) a[lane] = top;
    heap_fence<Global>();
}

// wave_heap_sort with the heap in global memory (pc_fallback_entry: spent-depth
// ranges over 4 Ki items) and its levels 6 .. 10 (nodes 63 .. 2046) cached in
// LDS for the sort_heap phase: a pop's path then costs one LDS round trip for
// those five levels and one L2 round trip for the five below (up to 2^16
// items), against two L2 round trips with the whole path in global memory.
// mid: this wave's LDS array of kMidN items (nodes [0, kMidN); the first 63
// are held in registers as in wave_heap_sort).  Same moves, same result.
constexpr int kMidN = 2047;
template <class It>
__device__ inline void wave_heap_sort_cached(It* a, int n, It* mid) {
    const int lane = threadIdx.x & 63;
    if (n < 2) return;
    const int P = (n - 2) / 2;   // the last parent
    for (int L = lg2(P + 1); L >= 0; --L) {   // make_heap in global memory, a tree level at a time
        const int lo = (1 << L) - 1, hi = min((1 << (L + 1)) - 2, P);
        for (int x = lo + lane; x <= hi; x += 64) slo_sort::adjust_heap_(a, x, n, a[x], LessT<It>());
        heap_fence<true>();
    }
    constexpr int TOPN = 63;
    const int nm = min(n, kMidN);
    for (int x = TOPN + lane; x < nm; x += 64) mid[x] = a[x];
    It top = lane < min(n, TOPN) ? a[lane] : (It)0;
    wave_fence();
    const int tlev = 31 - __builtin_clz(lane + 1);        // tree level of node `lane`
    const int cj = 31 - __builtin_clz(lane + 2), cq = lane + 2 - (1 << cj);   // chunk slot: level cj, position cq
    // node x's item: registers (x < 63), LDS (x < kMidN), else global
    auto at = [&](int x) -> It { return x < kMidN ? mid[x] : a[x]; };
    for (int len = n - 1; len >= 1; --len) {
        const It mx = irl(top, 0);
        It v;
        if (len < TOPN) {
            v = irl(top, len);
            if (lane == len) top = mx;
        } else {
            v = at(len);
            if (lane == 0) {
                if (len < kMidN) mid[len] = mx;
                else a[len] = mx;
            }
        }
        const int lim = (len - 1) / 2;   // nodes below lim have two children
        int h = 0, k = 0, ph = 0;
        It pv = 0;
        // The path takes the larger child at every level (ties: the right
        // one).  Every node's choice is computed at once — lane t compares
        // its node's two children — and the walk reads them from a ballot:
        // scalar bit steps instead of a chain of lane reads and compares.
        {
            const It cl = ishfl(top, min(2 * lane + 1, 63)), cr = ishfl(top, min(2 * lane + 2, 63));
            const unsigned long long BR = __ballot(lane < 31 && !(vkey(cr) < vkey(cl)));
            while (h < lim && 2 * h + 2 < TOPN) {   // the register levels
                h = 2 * h + 1 + (int)((BR >> h) & 1ull);
                ++k;
                if (lane == k) ph = h;
            }
            const It tv = ishfl(top, min(ph, 63));
            if (lane >= 1 && lane <= k) pv = tv;
        }
        while (h < lim) {   // deeper: the five levels below h in one load (LDS for levels 6 .. 10)
            const int node = (h + 1) * (1 << cj) - 1 + cq;
            const It sub = (lane < 62 && node < len) ? at(node) : (It)0;
            // chunk slot (level j, position q) = 2^j - 2 + q; its children: slots 2^(j+1) - 2 + 2q, + 1
            const int cs = (1 << (cj + 1)) - 2 + 2 * cq;
            const It sl = ishfl(sub, min(cs, 63)), sr = ishfl(sub, min(cs + 1, 63));
            const unsigned long long BC = __ballot(lane < 30 && !(vkey(sr) < vkey(sl)));
            const bool r0 = !(vkey(irl(sub, 1)) < vkey(irl(sub, 0)));   // h's own children: slots 0, 1
            const int k0 = k;
            int rel = r0 ? 1 : 0, pslot = 0;
            h = 2 * h + 1 + rel;
            ++k;
            if (lane == k) { ph = h; pslot = rel; }
            for (int j = 2; j <= 5 && h < lim; ++j) {
                const int b = (int)((BC >> ((1 << (j - 1)) - 2 + rel)) & 1ull);
                rel = 2 * rel + b;
                h = 2 * h + 1 + b;
                ++k;
                if (lane == k) { ph = h; pslot = (1 << j) - 2 + rel; }
            }
            const It sv = ishfl(sub, min(pslot, 63));
            if (lane > k0 && lane <= k) pv = sv;
        }
        if ((len & 1) == 0 && h == (len - 2) / 2) {   // the last parent's only child
            const int c = 2 * h + 1;
            const It cv = c < TOPN ? irl(top, c) : at(c);
            ++k;
            if (lane == k) { ph = c; pv = cv; }
        }
        const unsigned int kv = vkey(v);
        const int m = __popcll(__ballot(lane >= 1 && lane <= k && !(vkey(pv) < kv)));
        const It up = ishfl(pv, min(lane + 1, 63));
        const It w = lane < m ? up : v;
        const int phl = __shfl(ph, min(tlev, 63), 64);
        const It wl = ishfl(w, min(tlev, 63));
        if (lane <= m && ph >= TOPN) {
            if (ph < kMidN) mid[ph] = w;
            else a[ph] = w;
        }
        if (lane < TOPN && tlev <= m && phl == lane) top = wl;
        heap_fence<true>();   // the global stores (and the LDS ones) before the next pop's loads
    }
    if (lane < min(n, TOPN)) a[lane] = top;
    for (int x = TOPN + lane; x < nm; x += 64) a[x] = mid[x];
    heap_fence<true>();
}

// the queued lane tasks, one per lane, through the sequential restatement
template <class It>
__device__ __forceinline__ void lane_flush(It* items, const unsigned int* q, int nq) {
    const int lane = threadIdx.x & 63;
    wave_fence();
    if (lane < nq) {
        const unsigned int e = q[lane];
        const int f = (int)(e & 0x1fffu), l = (int)((e >> 13) & 0x1fffu), d = (int)(e >> 26);
        slo_sort::introsort_range_small(items + f, l - f, d, LessT<It>());
    }
    wave_fence();
}

// The workgroup's pool of ranges (block_sort, W > 1): waves that finish
// their range take the next one, and a wave stepping a range of more than
// kPushT items hands its right half to the pool instead of its own stack, so
// one deep range no longer keeps one wave busy while the others wait.  Slots
// are claimed with an LDS counter and filled after; a taker waits for the
// slot's nonzero entry (an entry always has l >= 2).  Which wave sorts which
// disjoint range does not change the result.
constexpr int kPoolCap = 128;
constexpr int kPushT = 128;
struct Pool {
    unsigned int e[kPoolCap];
    int head, tail, active;
};
__device__ __forceinline__ int ld_vol(const int* p) { return *(volatile const int*)p; }
// lane 0 of the calling wave pushes e if there is room for it and for a
// concurrent push by each other wave; returns whether it did (wave-uniform)
__device__ __forceinline__ bool pool_push(Pool* pool, unsigned int e, int W) {
    int ok = 0;
    if ((threadIdx.x & 63) == 0 && ld_vol(&pool->tail) < kPoolCap - W) {
        const int t = atomicAdd(&pool->tail, 1);
        // release: the range's items, as this wave left them, before its entry
        __hip_atomic_store(&pool->e[t], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        ok = 1;
    }
    return __builtin_amdgcn_readfirstlane(ok) != 0;
}

// one step of [f, l) by the calling wave, the variant its size picks
template <class It>
__device__ __forceinline__ int wave_step_any(It* items, unsigned short* tbl, int f, int l) {
    const int len = l - f;
    return len - 1 <= 64 ? wave_step<1>(items, tbl, f, l)
         : len - 1 <= 128 ? wave_step<2>(items, tbl, f, l) : stream_step(items, tbl, f, l);
}

// Sorts items[f0, l0) (LDS, positions < 8192, l0 - f0 <= 4097) into exactly
// std::sort's order for a range that the introsort loop reaches with `depth`
// levels of budget (2 * lg(n) for a whole array).  Called by all 64 lanes of
// one wave; tbl holds an entry per two positions: a step of [f, l) swaps m
// <= (l - f - 1) / 2 pairs and writes tbl[f / 2 .. f / 2 + m), which ends
// before (l - 1) / 2 <= the next range's f / 2, so waves on disjoint ranges
// share it.  *err (if given) counts ranges
// handed to a lane for a reason other than their size (must stay 0).
// prof (if given): cycles in [0] streamed steps, [1] register steps, [2] small ranges and heapsorts;
// [3] items heapsorted (wave_heap_sort)
template <int TLANE, class It>
__device__ __forceinline__ void wave_sort_range(It* items, int f0, int l0, int depth, unsigned short* tbl,
                                                WaveSmem& ws, int* err = nullptr, long long* prof = nullptr,
                                                Pool* pool = nullptr, int W = 1) {
    static_assert(TLANE >= 16 && TLANE <= 64, "ranges of <= TLANE items go to wave_small_sort");
    const int lane = threadIdx.x & 63;
    if (l0 - f0 <= 1) return;
    int sp = 0, nq = 0, f = f0, l = l0, d = depth;
    for (;;) {
        const int len = l - f;
        bool task = len <= TLANE || d == 0, stepped = false;
        int cut = 0;
        if (!task && sp == kStack) {   // cannot happen (sp <= the depth budget); exact anyway
            task = true;
            if (err && lane == 0) atomicAdd(err, 1);
        }
        if (!task) {
            const long long t0 = prof ? clock64() : 0;
            cut = wave_step_any(items, tbl, f, l);
            if (prof) prof[len - 1 <= 128] += clock64() - t0;
            if (cut <= f || cut >= l) {   // cannot happen; sorted (not std::sort's order) rather than a hang
                task = stepped = true;
                if (err && lane == 0) atomicAdd(err, 1);
            }
        }
        if (task) {
            // a spent depth budget (heapsort) or a step that failed: a lane task;
            // otherwise a range of <= 64 items in registers, its spent-depth
            // segments (if any) queued as lane tasks
            unsigned long long hs = 0;
            int hend = 0;
            const long long t0 = prof ? clock64() : 0;
            const bool small = len >= 2 && len <= 64 && d > 0 && !stepped;
            const bool heap = !small && !stepped && d == 0 && len > 16;   // introsort_range's heapsort, by the wave
            int ln = l;   // the end of the ranges sorted together
            if (small) {
                // the stack's top ranges that follow this one (depth first, left half first: its right
                // sibling, then the right siblings of its ancestors) join it while the whole stays within
                // 64 items: one register sort for several small ranges (most are leaves of <= 16)
                int mlo = 0, mhi = len, mdd = d;
                wave_fence();
                while (sp > 0) {
                    const unsigned int e2 = __builtin_amdgcn_readfirstlane(ws.stk[sp - 1]);
                    const int f2 = (int)(e2 & 0x1fffu), l2 = (int)((e2 >> 13) & 0x1fffu), d2 = (int)(e2 >> 26);
                    if (f2 != ln || d2 == 0 || l2 - f > 64) break;
                    --sp;
                    if (lane >= f2 - f && lane < l2 - f) { mlo = f2 - f; mhi = l2 - f; mdd = d2; }
                    ln = l2;
                }
                hs = wave_small_sort(items, f, ln - f, mlo, mhi, mdd, ws.tw, &hend);
            }
            else if (heap) wave_heap_sort(items + f, len);
            else if (len >= 2) hs = 1ull;   // the whole range
            if (prof) {
                prof[2] += clock64() - t0;
                if (heap) prof[3] += len;   // items heapsorted by the wave
            }
            while (hs) {
                const int b = __builtin_ctzll(hs);
                hs &= hs - 1;
                const int e0 = small ? f + b : f;
                const int e1 = small ? f + __shfl(hend, b, 64) : l;
                const int de = small ? 0 : d;
                if (lane == 0) ws.q[nq] = renc(e0, e1, de);
                if (++nq == kQ) {
                    lane_flush(items, ws.q, nq);
                    nq = 0;
                }
            }
            if (sp == 0) break;
            wave_fence();
            const unsigned int e = __builtin_amdgcn_readfirstlane(ws.stk[--sp]);
            f = (int)(e & 0x1fffu);
            l = (int)((e >> 13) & 0x1fffu);
            d = (int)(e >> 26);
            continue;
        }
        if (!(pool && l - cut > kPushT && pool_push(pool, renc(cut, l, d - 1), W))) {
            if (lane == 0) ws.stk[sp] = renc(cut, l, d - 1);
            ++sp;
        }
        l = cut;
        --d;
    }
    if (nq) {
        const long long t0 = prof ? clock64() : 0;
        lane_flush(items, ws.q, nq);
        if (prof) prof[2] += clock64() - t0;
    }
}

template <int TLANE, class It>
__device__ __forceinline__ void wave_sort(It* items, int n, int depth, unsigned short* tbl, WaveSmem& ws,
                                          int* err = nullptr, long long* prof = nullptr) {
    wave_sort_range<TLANE>(items, 0, n, depth, tbl, ws, err, prof);
}

// one introsort step of [f, l) (l - f - 1 <= 4096) by a group of gw waves of
// the workgroup (waves gw * g .. gw * g + gw - 1; every wave of the workgroup
// calls this, each group with its own range and BlockStepSm, so the groups of
// one level step their ranges side by side): stream_step with its rows dealt
// round-robin to the group's waves — the per-row stopper counts in LDS, m and
// the cuts by the group's first wave from the row prefixes (one row per lane,
// as stream_step keeps them), workgroup barriers between the passes (four,
// whatever the group does, so every wave meets every barrier).  Every swapped
// left stopper lies before the crossing and every partner at or after it, so
// a wave reads no position another wave writes except partners past the
// crossing, whose left-stopper flags can only turn on (a right stopper's
// place takes a left stopper's item): the prefixes of the positions that swap
// stay exact.  mode 0: the group has nothing to step; 1: its first wave takes
// the (<= 129-item) range's step alone (wave_step_any); 2: the group's step.
// Returns the cut (modes 1, 2).
struct BlockStepSm {
    int rl[65], rr[65];   // per row stopper counts, then exclusive prefixes
    int m, cutA, cutB, rA, rB;
};
template <class It>
__device__ __forceinline__ int group_step(It* items, unsigned short* tbl, int f, int l, int mode, BlockStepSm& bs,
                                          int gw) {
    const int lane = threadIdx.x & 63, lw = (threadIdx.x >> 6) & (gw - 1);
    constexpr int INF = 0x7fffffff;
    const bool big = mode == 2;
    const int mid = f + (l - f) / 2;
    It a0 = 0, pit = 0;
    unsigned int p = 0, k0 = 0;
    int med = 0;
    if (big) {
        a0 = items[f];
        const It a1 = items[f + 1], a2 = items[mid], a3 = items[l - 1];
        const int w = median3(vkey(a1), vkey(a2), vkey(a3));
        med = w == 0 ? f + 1 : (w == 1 ? mid : l - 1);
        pit = w == 0 ? a1 : (w == 1 ? a2 : a3);
        p = vkey(pit);
        k0 = vkey(a0);
    }
    const int b0 = f + 1, R = big ? (l - b0 + 63) >> 6 : 0;
    // (1) stopper counts per row (the median swap virtual)
    for (int r0 = lw; r0 < R; r0 += 4 * gw) {
        unsigned int kk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) kk[u] = key_at(items, min(b0 + 64 * (r0 + u * gw) + lane, l - 1));
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int r = r0 + u * gw;
            if (r < R) {
                const int x = b0 + 64 * r + lane;
                const unsigned int k = x == med ? k0 : kk[u];
                const int cl = __popcll(__ballot(x < l && !(k < p))), cr = __popcll(__ballot(x < l && !(p < k)));
                if (lane == 0) { bs.rl[r] = cl; bs.rr[r] = cr; }
            }
        }
    }
    __syncthreads();
    if (lw == 0 && mode == 1) {
        bs.cutA = wave_step_any(items, tbl, f, l);
        bs.m = 0;
    } else if (lw == 0 && big) {   // (2) the prefixes (lane r = row r), m, the cuts; the median swap made real
        const int cl = lane < R ? bs.rl[lane] : 0, cr = lane < R ? bs.rr[lane] : 0;
        int il = cl, ir = cr;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int yl = __shfl_up(il, o, 64), yr = __shfl_up(ir, o, 64);
            if (lane >= o) { il += yl; ir += yr; }
        }
        const int rowL = il - cl, rowR = ir - cr;
        const int TL = __shfl(il, 63, 64), TR = __shfl(ir, 63, 64);
        int eL = il, eR = ir;   // stoppers before the row's end
        const int c = __builtin_ctzll(__ballot(lane < R && eL >= TR - eR));
        auto row_flags = [&](int r, bool& iL, bool& iR, int& pl, int& pr) {
            const int x = b0 + 64 * r + lane;
            unsigned int k = key_at(items, min(x, l - 1));
            k = x == med ? k0 : k;
            const bool act = x < l;
            iL = act && !(k < p);
            iR = act && !(p < k);
            pl = __builtin_amdgcn_readlane(rowL, r) + lane_prefix(__ballot(iL));
            pr = __builtin_amdgcn_readlane(rowR, r) + lane_prefix(__ballot(iR));
        };
        int m;
        {
            bool iL, iR;
            int pl, pr;
            row_flags(c, iL, iR, pl, pr);
            const int bc = b0 + 64 * c;
            const unsigned long long fx = __ballot(bc + lane < l && pl >= TR - pr);
            if (fx) {
                const int xl = __builtin_ctzll(fx);
                m = TR - __builtin_amdgcn_readlane(pr, xl);
                if (xl > 0) m = max(m, __builtin_amdgcn_readlane(pl, xl - 1));
            } else {
                const int last = min(63, l - 1 - bc);
                m = max(TR - __builtin_amdgcn_readlane(eR, c), __builtin_amdgcn_readlane(pl, last));
            }
        }
        int cutA = INF, cutB = INF, rA = R - 1, rB = 0;
        if (m < TL) {
            rA = __builtin_ctzll(__ballot(lane < R && rowL <= m && m < eL));
            bool iL, iR;
            int pl, pr;
            row_flags(rA, iL, iR, pl, pr);
            cutA = b0 + 64 * rA + __builtin_ctzll(__ballot(iL && pl == m));
        }
        if (m > 0) {
            const int t = TR - m;
            rB = __builtin_ctzll(__ballot(lane < R && rowR <= t && t < eR));
            bool iL, iR;
            int pl, pr;
            row_flags(rB, iL, iR, pl, pr);
            cutB = b0 + 64 * rB + __builtin_ctzll(__ballot(iR && pr == t));
        }
        if (lane < R) { bs.rl[lane] = rowL; bs.rr[lane] = rowR; }
        if (lane == 0) {
            bs.m = m; bs.cutA = cutA; bs.cutB = cutB; bs.rA = m < TL ? rA : R - 1; bs.rB = rB;
            items[f] = pit;
            items[med] = a0;
        }
        bs.rl[64] = TR;   // (every lane writes the same value)
    }
    __syncthreads();
    const int m = big ? bs.m : 0, TR = big ? bs.rl[64] : 0;
    if (m > 0) {   // (3) the m last right stoppers, by rank from the right
        for (int r = bs.rB + lw; r < R; r += gw) {
            const int x = b0 + 64 * r + lane;
            const bool iR = x < l && !(p < key_at(items, min(x, l - 1)));
            const int kr = TR - 1 - (bs.rr[r] + lane_prefix(__ballot(iR)));
            if (iR && kr < m) tbl[(f >> 1) + kr] = (unsigned short)x;
        }
    }
    __syncthreads();
    if (m > 0) {   // (4) the m first left stoppers swap with their partners
        const int rEnd = bs.rA;
        for (int r = lw; r <= rEnd; r += gw) {
            const int x = b0 + 64 * r + lane;
            const It it = items[min(x, l - 1)];
            const bool iL = x < l && !(vkey(it) < p);
            const int pl = bs.rl[r] + lane_prefix(__ballot(iL));
            if (iL && pl < m) {
                const int y = tbl[(f >> 1) + pl];
                const It py = items[y];
                items[x] = py;
                items[y] = it;
            }
        }
    }
    __syncthreads();
    return mode == 0 ? 0 : min(bs.cutA, m > 0 ? bs.cutB : INF);
}

// W waves on one range: the first levels breadth first — while a level has
// at most W / 2 ranges, each range is stepped by a group of W / G waves (G
// the level's ranges rounded up to a power of two; group_step), the groups
// side by side — then the ranges go to the workgroup's pool (Pool), from
// which the waves take them and sort them depth first, handing the right
// halves of large steps back to the pool.
template <int W>
struct BlockQ {
    unsigned int cur[W], nxt[W];
    int ncur;
    BlockStepSm bs[W > 1 ? W / 2 : 1];
    Pool pool;
};

template <int TLANE, int W, class It>
__device__ __forceinline__ void block_sort(It* items, int n, int depth, unsigned short* tbl, WaveSmem* ws,
                                           BlockQ<W>& bq, int* err = nullptr, long long* prof = nullptr) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (W == 1) {
        wave_sort_range<TLANE>(items, 0, n, depth, tbl, ws[0], err, prof);
        return;
    }
    long long tph = prof ? clock64() : 0;   // prof[4..7] (thread 0's): group levels, -, pool entry, pool
    auto phase = [&](int k) {
        if (prof) {
            const long long t = clock64();
            prof[k] += t - tph;
            tph = t;
        }
    };
    Pool& pool = bq.pool;
    for (int i = threadIdx.x; i < kPoolCap; i += 64 * W) pool.e[i] = 0u;
    if (threadIdx.x == 0) {
        bq.cur[0] = renc(0, n, depth);
        bq.ncur = n >= 2 ? 1 : 0;
        pool.head = pool.tail = 0;
        pool.active = W;
    }
    __syncthreads();
    // the first levels (at most W / 2 ranges, the largest steps): wave groups
    for (;;) {
        const int nc = bq.ncur;
        if (2 * nc > W || nc == 0) break;
        bool more = false;   // a range of this level still needs a step
        for (int i = 0; i < nc; ++i) {
            const unsigned int e = bq.cur[i];
            more |= (int)((e >> 13) & 0x1fffu) - (int)(e & 0x1fffu) > TLANE && (int)(e >> 26) > 0;
        }
        if (!more) break;
        int G = 1;
        while (G < nc) G <<= 1;
        const int gw = W / G, g = wv / gw;
        unsigned int e = 0;
        int f = 0, l = 0, d = 0, mode = 0;
        if (g < nc) {
            e = bq.cur[g];
            f = (int)(e & 0x1fffu);
            l = (int)((e >> 13) & 0x1fffu);
            d = (int)(e >> 26);
            if (l - f > TLANE && d > 0) mode = l - f - 1 > 128 ? 2 : 1;
        }
        const long long t0 = prof ? clock64() : 0;
        const int cut = group_step(items, tbl, f, l, mode, bq.bs[g < nc ? g : 0], gw);
        if (prof && mode) prof[mode == 1] += clock64() - t0;
        if (g < nc && wv % gw == 0 && lane == 0) {
            unsigned int a = e, b = 0;
            if (mode) {
                if (cut > f && cut < l) {
                    a = renc(f, cut, d - 1);
                    b = renc(cut, l, d - 1);
                } else if (err) {
                    atomicAdd(err, 1);
                }
            }
            bq.nxt[2 * g] = a;
            bq.nxt[2 * g + 1] = b;
        }
        __syncthreads();
        if (threadIdx.x == 0) {   // the next level's ranges of two or more items
            int c = 0;
            for (int i = 0; i < 2 * nc; ++i) {
                const unsigned int x = bq.nxt[i];
                if ((int)((x >> 13) & 0x1fffu) - (int)(x & 0x1fffu) >= 2) bq.cur[c++] = x;
            }
            bq.ncur = c;
        }
        __syncthreads();
    }
    phase(4);
    // the pool: the level's ranges first, then whatever the waves hand in
    if (threadIdx.x == 0) {
        for (int i = 0; i < bq.ncur; ++i) pool.e[i] = bq.cur[i];
        pool.tail = bq.ncur;
    }
    __syncthreads();
    phase(6);
    for (;;) {
        unsigned int e = 0;
        if (lane == 0) {
            for (;;) {   // claim the next slot, if any
                const int h = ld_vol(&pool.head);
                if (h >= ld_vol(&pool.tail)) break;
                if (atomicCAS(&pool.head, h, h + 1) == h) {
                    while ((e = __hip_atomic_load(&pool.e[h], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0u)
                        __builtin_amdgcn_s_sleep(1);
                    break;
                }
            }
        }
        e = __builtin_amdgcn_readfirstlane(e);
        if (e) {
            wave_sort_range<TLANE>(items, (int)(e & 0x1fffu), (int)((e >> 13) & 0x1fffu), (int)(e >> 26), tbl, ws[wv],
                                   err, prof, &pool, W);
            continue;
        }
        // idle: done once no wave holds a range and the pool is empty (only
        // a wave holding a range hands one in)
        int done = 0;
        if (lane == 0) {
            atomicSub(&pool.active, 1);
            for (;;) {
                if (ld_vol(&pool.head) < ld_vol(&pool.tail)) {
                    atomicAdd(&pool.active, 1);
                    break;
                }
                if (ld_vol(&pool.active) == 0) {
                    done = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        if (__builtin_amdgcn_readfirstlane(done)) break;
    }
    phase(6);
    __syncthreads();
    phase(7);
}

}  // namespace slo_pcl
