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
// (voxel index << 32 | point index); all ranges of a level over 16 items are
// stepped together by the whole workgroup (ballot prefixes of the left /
// right stoppers, per-range prefixes at the range ends, m where the left
// and right counts cross, a position table of the right stoppers by rank,
// the swaps).  A range of <= 16 items is a leaf: the final insertion sort makes it the
// stable order of its items, so every item's place is its rank in the leaf by
// (key, position) — one lane per item.  A range whose depth budget is spent
// (only adversarial inputs) is heapsorted by one lane (slo_sort::heap_sort_,
// the restated libstdc++ heap).
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

constexpr unsigned char kDone = 0xff;
constexpr unsigned char kHeap = 0xff;

// LDS of pcl_block_sort for up to NMAX items (NMAX <= 4096: range ids fit
// 8 bits).  The items themselves are the caller's LDS array.
template <int NT, int NMAX>
struct BlockSmem {
    static constexpr int MAXSEG = NMAX / 17 + 2;   // disjoint ranges of > 16 items, + slack
    unsigned short tblB[NMAX];     // right stoppers by rank from the right, at f + rank
    unsigned short f[2][MAXSEG], l[2][MAXSEG];
    unsigned char d[2][MAXSEG];
    unsigned int piv[MAXSEG];
    int sL[MAXSEG], eR[MAXSEG], m[MAXSEG], cutA[MAXSEG], cutB[MAXSEG];
    short nidL[MAXSEG], nidR[MAXSEG];
    unsigned short hf[MAXSEG], hl[MAXSEG];   // heapsort ranges
    int nseg[2], nheap;
    unsigned int wsum[NT / 64];
};

// Sorts items[0, n) (LDS, n <= NMAX) into exactly std::sort's order for a
// range that the introsort loop reaches with `depth` levels of budget
// (2 * lg(n) for a whole array).  All NT threads of the workgroup call it.
//
// Positions are wave-striped: wave w, row j, lane t owns position
// x = w * 64 * IPT + j * 64 + t for the whole sort, so each position's state
// (its active range, or its leaf) lives in the owner's registers, each LDS
// access of a row is 64 consecutive words (no bank conflicts) and every
// prefix count is a ballot.  Every step issues all of a thread's loads
// before it uses any (indices clamped, no loads behind branches), so a step
// costs one LDS round trip, not one per row.  Returns the levels run.
template <int NT, int NMAX>
__device__ __forceinline__ int pcl_block_sort(u64* items, int n, int depth, BlockSmem<NT, NMAX>& sm) {
    static_assert(NMAX % NT == 0 && NMAX <= 4096 && NT % 64 == 0, "pcl_block_sort layout");
    constexpr int IPT = NMAX / NT, NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int xw = w * 64 * IPT + lane;   // position of row j: xw + 64 j
    const unsigned long long lt = (1ull << lane) - 1ull;
    // per position, packed: bits 0-7 the active range (kDone once finished),
    // 8-15 its leaf's size (kHeap: a heapsort range), 16-31 its leaf's start
    unsigned int st[IPT];
    const bool act0 = n > 16 && depth > 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const int x = xw + 64 * j;
        st[j] = (unsigned int)((act0 && x < n) ? 0 : kDone) | ((unsigned int)(n <= 16 ? n : kHeap) << 8);
    }
    if (tid == 0) {
        sm.nseg[0] = act0 ? 1 : 0;
        sm.nseg[1] = 0;
        sm.nheap = (!act0 && n > 16) ? 1 : 0;
        sm.f[0][0] = 0; sm.l[0][0] = (unsigned short)n; sm.d[0][0] = (unsigned char)depth;
        sm.hf[0] = 0; sm.hl[0] = (unsigned short)n;
    }
    __syncthreads();
    int c = 0, levels = 0;
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
        // (2) every row's range bounds, pivot and item (all loads first), stopper ballots
        u64 it[IPT];
        int rf[IPT], rl[IPT];
        unsigned long long bL[IPT], bR[IPT];
        {
            unsigned int pv[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int sc = (st[j] & 0xff) == kDone ? 0 : (int)(st[j] & 0xff);
                rf[j] = sm.f[c][sc];
                rl[j] = sm.l[c][sc];
                pv[j] = sm.piv[sc];
                it[j] = items[min(xw + 64 * j, NMAX - 1)];
            }
            int cL = 0, cR = 0;
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int x = xw + 64 * j;
                const bool act = (st[j] & 0xff) != kDone && x != rf[j];
                const unsigned int k = vkey(it[j]);
                bL[j] = __ballot(act && !(k < pv[j]));
                bR[j] = __ballot(act && !(pv[j] < k));
                cL += __popcll(bL[j]);
                cR += __popcll(bR[j]);
            }
            if (lane == 0) sm.wsum[w] = (unsigned int)cL | ((unsigned int)cR << 16);
        }
        __syncthreads();
        int pl[IPT], pr[IPT];   // stoppers before each row's position (exclusive prefixes)
        {
            unsigned int ws[NW];
#pragma unroll
            for (int q = 0; q < NW; ++q) ws[q] = sm.wsum[q];
            int bl = 0, br = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q)
                if (q < w) { bl += (int)(ws[q] & 0xffffu); br += (int)(ws[q] >> 16); }
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                pl[j] = bl + __popcll(bL[j] & lt);
                pr[j] = br + __popcll(bR[j] & lt);
                bl += __popcll(bL[j]);
                br += __popcll(bR[j]);
            }
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                if ((st[j] & 0xff) == kDone) continue;
                const int x = xw + 64 * j, s = st[j] & 0xff;
                if (x == rf[j] + 1) sm.sL[s] = pl[j];
                if (x == rl[j] - 1) sm.eR[s] = pr[j] + (int)((bR[j] >> lane) & 1);
            }
        }
        __syncthreads();
        // (3) m of every range: with Lb = left stoppers before a boundary and
        // Rb = right stoppers at or after it, max(min(Lb, Rb)) sits where
        // Lb >= Rb first holds; only the positions around that crossing post
        // it (a wave-block edge, whose neighbour is another wave's, posts its
        // own value: any min(Lb, Rb) is <= m)
        int rsL[IPT], reR[IPT];
        {
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int sc = (st[j] & 0xff) == kDone ? 0 : (int)(st[j] & 0xff);
                rsL[j] = sm.sL[sc];
                reR[j] = sm.eR[sc];
            }
            unsigned long long bF[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int x = xw + 64 * j;
                const bool act = (st[j] & 0xff) != kDone && x > rf[j];
                bF[j] = __ballot(act && pl[j] - rsL[j] >= reR[j] - pr[j]);
            }
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int x = xw + 64 * j;
                if ((st[j] & 0xff) == kDone || x <= rf[j]) continue;
                const int s = st[j] & 0xff;
                const int lb = pl[j] - rsL[j], rb = reR[j] - pr[j];
                const bool fl = (bF[j] >> lane) & 1;
                const bool prevF = lane > 0 ? (bF[j] >> (lane - 1)) & 1 : (j > 0 ? (bF[j - 1] >> 63) & 1 : 0);
                const bool nextF = lane < 63 ? (bF[j] >> (lane + 1)) & 1 : (j + 1 < IPT ? bF[j + 1] & 1 : 1);
                const bool first = x == rf[j] + 1, last = x == rl[j] - 1;
                if (fl && (first || !prevF) && rb > 0) atomicMax(&sm.m[s], rb);
                if (!fl && (last || nextF) && lb > 0) atomicMax(&sm.m[s], lb);
            }
        }
        __syncthreads();
        // (4) right stoppers by rank from the right; the cut candidates
        int rm[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int sc = (st[j] & 0xff) == kDone ? 0 : (int)(st[j] & 0xff);
            rm[j] = sm.m[sc];
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            if ((st[j] & 0xff) == kDone) continue;
            const int x = xw + 64 * j, s = st[j] & 0xff;
            if (((bL[j] >> lane) & 1) && pl[j] - rsL[j] == rm[j]) sm.cutA[s] = x;   // i_{m+1}
            if ((bR[j] >> lane) & 1) {
                const int kr = reR[j] - pr[j] - 1;                                  // right stoppers after x
                if (kr < rm[j]) sm.tblB[rf[j] + kr] = (unsigned short)x;
                if (kr == rm[j] - 1) sm.cutB[s] = x;                                 // j_m
            }
        }
        __syncthreads();
        // (5a) swap partners (left stopper of rank k < m <-> right stopper of rank k)
        u64 pit[IPT];
        int py[IPT];
        unsigned int sw = 0;
        {
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int k = pl[j] - rsL[j];
                const bool swp = ((bL[j] >> lane) & 1) && k < rm[j];
                sw |= (unsigned int)swp << j;
                py[j] = sm.tblB[min(max(rf[j] + k, 0), NMAX - 1)];
            }
#pragma unroll
            for (int j = 0; j < IPT; ++j) pit[j] = items[((sw >> j) & 1) ? py[j] : 0];
        }
        // (6) the halves: ranges of > 16 items with budget left stay active
        for (int s = tid; s < ns; s += NT) {
            const int F = sm.f[c][s], L = sm.l[c][s], D = sm.d[c][s] - 1;
            const int cut = min(sm.cutA[s], sm.m[s] > 0 ? sm.cutB[s] : 0x7fffffff);
            sm.cutA[s] = cut;
            const int lo[2] = {F, cut}, hi[2] = {cut, L};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                short id = -1;
                if (hi[h] - lo[h] > 16) {
                    if (D > 0) {
                        id = (short)atomicAdd(&sm.nseg[c ^ 1], 1);
                        sm.f[c ^ 1][id] = (unsigned short)lo[h]; sm.l[c ^ 1][id] = (unsigned short)hi[h];
                        sm.d[c ^ 1][id] = (unsigned char)D;
                    } else {   // depth spent: heapsort
                        const int q = atomicAdd(&sm.nheap, 1);
                        sm.hf[q] = (unsigned short)lo[h]; sm.hl[q] = (unsigned short)hi[h];
                    }
                }
                (h ? sm.nidR : sm.nidL)[s] = id;
            }
        }
        __syncthreads();
        // (5b) the swaps; (7) every position's next range or leaf (state in registers)
#pragma unroll
        for (int j = 0; j < IPT; ++j)
            if ((sw >> j) & 1) {
                items[xw + 64 * j] = pit[j];
                items[py[j]] = it[j];
            }
        {
            int ct[IPT], iL[IPT], iR[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int sc = (st[j] & 0xff) == kDone ? 0 : (int)(st[j] & 0xff);
                ct[j] = sm.cutA[sc];
                iL[j] = sm.nidL[sc];
                iR[j] = sm.nidR[sc];
            }
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                if ((st[j] & 0xff) == kDone) continue;
                const int x = xw + 64 * j;
                const bool left = x < ct[j];
                const int id = left ? iL[j] : iR[j];
                if (id >= 0) {
                    st[j] = (st[j] & ~0xffu) | (unsigned int)id;
                } else {
                    const int lo = left ? rf[j] : ct[j], hi = left ? ct[j] : rl[j];
                    st[j] = (unsigned int)kDone | ((unsigned int)(hi - lo <= 16 ? hi - lo : kHeap) << 8) |
                            ((unsigned int)lo << 16);
                }
            }
        }
        if (tid == 0) sm.nseg[c] = 0;
        c ^= 1;
        ++levels;
        __syncthreads();
    }
    // heapsort ranges (depth spent), one lane each
    for (int q = tid; q < sm.nheap; q += NT)
        slo_sort::heap_sort_(items + sm.hf[q], sm.hl[q] - sm.hf[q], Less());
    __syncthreads();
    // leaves: the final insertion sort = each item's rank in its leaf by (key, position)
    u64 own[IPT];
    int dst[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const int x = xw + 64 * j;
        own[j] = items[min(x, NMAX - 1)];
        const int lo = (int)(st[j] >> 16), sz = (int)((st[j] >> 8) & 0xff);
        dst[j] = -1;
        if (x >= n || sz == kHeap) continue;
        const unsigned int k = vkey(own[j]);
        unsigned int ky[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) ky[t] = vkey(items[lo + min(t, sz - 1)]);
        int r = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) r += (t < sz) & ((ky[t] < k) | ((ky[t] == k) & (lo + t < x)));
        dst[j] = lo + r;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IPT; ++j)
        if (dst[j] >= 0) items[dst[j]] = own[j];
    __syncthreads();
    return levels;
}

}  // namespace slo_pcl
