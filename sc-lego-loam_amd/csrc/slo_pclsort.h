// slo_pclsort.h — PCL's VoxelGrid order, computed in parallel.
//
// VoxelGrid<PointXYZI>::applyFilter (PCL 1.8; the reference calls it at
// featureAssociation.cpp:779-780 and mapOptmization.cpp:1224-1262) sorts the
// (voxel index, point index) pairs of the cloud with std::sort, comparing the
// voxel index only, and sums each voxel's points in the order that leaves.
// std::sort is not stable, so that order — and with it every centroid's
// float sum — is whatever libstdc++'s introsort makes of the input order.
// This header computes exactly that order with a workgroup instead of one
// thread.
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
// Here (pcl_block_sort): the items of one range sit in LDS as 64-bit words
// (voxel index << 32 | point index).  All ranges of a level larger than BT
// are stepped together by the whole workgroup (one block scan of the packed
// left / right stopper counts, per-range prefixes at the range ends, m by
// LDS atomicMax, a position table of the right stoppers by rank, then the
// swaps).  Ranges of <= BT items, and any range whose depth budget is spent,
// are finished by one lane each with the sequential restatement
// (slo_sort::introsort_range).
#pragma once

#include "slo_introsort.h"

namespace slo_pcl {

typedef unsigned long long u64;

__host__ __device__ inline unsigned int vkey(u64 it) { return (unsigned int)(it >> 32); }
struct Less {
    __host__ __device__ bool operator()(const u64& a, const u64& b) const { return (a >> 32) < (b >> 32); }
};

__host__ __device__ inline int lg2(int n) {
    int r = 0;
    while (n > 1) { n >>= 1; ++r; }
    return r;
}

constexpr unsigned short kNone = 0xffff;
constexpr unsigned char kNoStart = 0xff;

// LDS of pcl_block_sort for up to NMAX items (NMAX <= 32768: the packed
// counts of the scan hold 16 bits each).  The items themselves are the
// caller's LDS array.
template <int NT, int NMAX, int BT>
struct BlockSmem {
    static constexpr int MAXSEG = NMAX / (BT + 1) + 2;   // disjoint ranges of > BT items, + slack
    unsigned short seg_of[NMAX];   // the active range a position belongs to (kNone: none)
    unsigned short tblB[NMAX];     // right stoppers by rank from the right, at f + rank
    unsigned char dep[NMAX];       // the depth budget of a finished range, at its first position
    int f[2][MAXSEG], l[2][MAXSEG], d[2][MAXSEG];
    unsigned int piv[MAXSEG];
    int sL[MAXSEG], eR[MAXSEG], m[MAXSEG], cutA[MAXSEG], cutB[MAXSEG], nidL[MAXSEG], nidR[MAXSEG];
    int nseg[2];
    unsigned int wsum[NT / 64];
};

// exclusive block scan of a packed pair of 16-bit counts
template <int NT>
__device__ inline unsigned int pcl_block_scan(unsigned int x, unsigned int* wsum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned int incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    unsigned int before = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k)
        if (k < w) before += wsum[k];
    __syncthreads();
    return before + incl - x;
}

// Sorts items[0, n) (LDS, n <= NMAX) into exactly std::sort's order for a
// range that the introsort loop reaches with `depth` levels of budget
// (2 * lg(n) for a whole array).  All NT threads of the workgroup call it.
template <int NT, int NMAX, int BT>
__device__ void pcl_block_sort(u64* items, int n, int depth, BlockSmem<NT, NMAX, BT>& sm) {
    static_assert(NMAX % NT == 0 && NMAX <= 32768 && BT >= 16, "pcl_block_sort layout");
    constexpr int IPT = NMAX / NT;
    constexpr int MAXSEG = BlockSmem<NT, NMAX, BT>::MAXSEG;
    const int tid = threadIdx.x;
    const int x0 = tid * IPT;   // this thread's positions [x0, x0 + IPT)
    const bool block_tier = n > BT && depth > 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const int x = x0 + j;
        sm.seg_of[x] = block_tier ? 0 : kNone;
        sm.dep[x] = (!block_tier && x == 0 && n > 0) ? (unsigned char)depth : kNoStart;
    }
    if (tid == 0) {
        sm.nseg[0] = block_tier ? 1 : 0;
        sm.nseg[1] = 0;
        sm.f[0][0] = 0; sm.l[0][0] = n; sm.d[0][0] = depth;
    }
    __syncthreads();
    int c = 0;
    for (;;) {
        const int ns = sm.nseg[c];
        if (ns == 0) break;
        // (1) median of three to the front; the pivot
        for (int s = tid; s < ns; s += NT) {
            const int F = sm.f[c][s], L = sm.l[c][s];
            u64* a = items + F;
            slo_sort::move_median_to_first_(a, a + 1, a + (L - F) / 2, a + (L - F - 1), Less());
            sm.piv[s] = vkey(a[0]);
            sm.m[s] = 0;
            sm.cutA[s] = 0x7fffffff;
            sm.cutB[s] = 0x7fffffff;
        }
        __syncthreads();
        // (2) stopper flags of this thread's positions and their block prefix
        u64 it[IPT];
        unsigned short so[IPT];
        unsigned int fl = 0, fr = 0;   // bit j: position x0 + j is a left / right stopper
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int x = x0 + j;
            so[j] = x < n ? sm.seg_of[x] : kNone;
            it[j] = x < n ? items[x] : 0ull;
            if (so[j] != kNone && x != sm.f[c][so[j]]) {
                const unsigned int k = vkey(it[j]), p = sm.piv[so[j]];
                fl |= (unsigned int)!(k < p) << j;
                fr |= (unsigned int)!(p < k) << j;
            }
        }
        const unsigned int ex = pcl_block_scan<NT>((unsigned int)__popc(fl) | ((unsigned int)__popc(fr) << 16), sm.wsum);
        const int bl = (int)(ex & 0xffffu), br = (int)(ex >> 16);
        {
            int rl = bl, rr = br;
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int x = x0 + j;
                const int s = so[j];
                if (s != kNone && x == sm.f[c][s] + 1) sm.sL[s] = rl;   // left stoppers before the range
                rl += (fl >> j) & 1;
                rr += (fr >> j) & 1;
                if (s != kNone && x == sm.l[c][s] - 1) sm.eR[s] = rr;   // right stoppers up to its end
            }
        }
        __syncthreads();
        // (3) m of every range: the max over its boundaries of min(left before, right at or after)
        {
            int rl = bl, rr = br, cur = kNone, g = 0;
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int x = x0 + j;
                const int s = so[j];
                if (s != kNone && x > sm.f[c][s]) {
                    const int v = min(rl - sm.sL[s], sm.eR[s] - rr);
                    if (s != cur) {
                        if (cur != kNone) atomicMax(&sm.m[cur], g);
                        cur = s; g = v;
                    } else {
                        g = max(g, v);
                    }
                }
                rl += (fl >> j) & 1;
                rr += (fr >> j) & 1;
            }
            if (cur != kNone) atomicMax(&sm.m[cur], g);
        }
        __syncthreads();
        // (4) right stoppers by rank from the right; the cut candidates
        {
            int rl = bl, rr = br;
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int x = x0 + j;
                const int s = so[j];
                if ((fl >> j) & 1) {
                    if (rl - sm.sL[s] == sm.m[s]) sm.cutA[s] = x;      // i_{m+1}
                    ++rl;
                }
                if ((fr >> j) & 1) {
                    ++rr;
                    const int kr = sm.eR[s] - rr;                        // right stoppers after x
                    if (kr < sm.m[s]) sm.tblB[sm.f[c][s] + kr] = (unsigned short)x;
                    if (kr == sm.m[s] - 1) sm.cutB[s] = x;               // j_m
                }
            }
        }
        __syncthreads();
        // (5) the swaps: left stopper of rank k < m <-> right stopper of rank k
        {
            u64 pit[IPT];
            unsigned short py[IPT];
            unsigned int sw = 0;
            int rl = bl;
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                if ((fl >> j) & 1) {
                    const int s = so[j];
                    const int k = rl - sm.sL[s];
                    if (k < sm.m[s]) {
                        py[j] = sm.tblB[sm.f[c][s] + k];
                        pit[j] = items[py[j]];
                        sw |= 1u << j;
                    }
                    ++rl;
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < IPT; ++j)
                if ((sw >> j) & 1) {
                    items[x0 + j] = pit[j];
                    items[py[j]] = it[j];
                }
        }
        // (6) the halves: ranges of > BT items with budget left stay in the block tier
        for (int s = tid; s < ns; s += NT) {
            const int F = sm.f[c][s], L = sm.l[c][s], D = sm.d[c][s] - 1;
            const int cut = min(sm.cutA[s], sm.m[s] > 0 ? sm.cutB[s] : 0x7fffffff);
            sm.cutA[s] = cut;
            const int lo[2] = {F, cut}, hi[2] = {cut, L};
            for (int h = 0; h < 2; ++h) {
                int id = kNone;
                if (hi[h] - lo[h] > BT && D > 0) {
                    id = atomicAdd(&sm.nseg[c ^ 1], 1);
                    sm.f[c ^ 1][id] = lo[h]; sm.l[c ^ 1][id] = hi[h]; sm.d[c ^ 1][id] = D;
                } else if (hi[h] > lo[h]) {
                    sm.dep[lo[h]] = (unsigned char)D;   // finished by one lane
                }
                (h ? sm.nidR : sm.nidL)[s] = id;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int s = so[j];
            if (s != kNone) sm.seg_of[x0 + j] = (unsigned short)(x0 + j < sm.cutA[s] ? sm.nidL[s] : sm.nidR[s]);
        }
        if (tid == 0) sm.nseg[c] = 0;
        c ^= 1;
        __syncthreads();
        (void)MAXSEG;
    }
    // lane tier: the thread holding a finished range's first position sorts it
#pragma unroll 1
    for (int j = 0; j < IPT; ++j) {
        const int x = x0 + j;
        if (x >= n || sm.dep[x] == kNoStart) continue;
        int e = x + 1;
        while (e < n && sm.dep[e] == kNoStart) ++e;
        slo_sort::introsort_range(items + x, e - x, (int)sm.dep[x], Less());
    }
    __syncthreads();
}

}  // namespace slo_pcl
