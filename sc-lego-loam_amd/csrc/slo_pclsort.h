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
// Here: the items of one range sit in LDS as 64-bit words (voxel index << 32
// | point index).  Two tiers, both computing every step of every range of a
// level at once:
//   * block tier (pcl_block_sort): all ranges of a level over kWT items,
//     stepped by the whole workgroup (block prefix of the packed left / right
//     stopper counts, per-range prefixes at the range ends, m by LDS
//     atomicMax, a position table of the right stoppers by rank, the swaps);
//   * wave tier (pcl_wave_sort): a range of at most kWT items is finished by
//     one wave alone — its positions' state in registers, prefixes by
//     ballots, no workgroup barrier.
// A range of <= 16 items is a leaf: the final insertion sort makes it the
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

constexpr int kWT = 512;               // a range of at most kWT items is finished by one wave
constexpr int kWRows = kWT / 64;
constexpr int kWSub = 32;              // active sub-ranges of a wave range (<= kWT / 17)
constexpr unsigned char kDone = 0xff;
constexpr unsigned char kHeap = 0xff;

__device__ inline void wave_sync() {   // this wave's LDS traffic drained and visible to its lanes
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// per-wave LDS of pcl_wave_sort: the next level's sub-ranges and the heapsort ranges
struct WaveSmem {
    unsigned short sf[kWSub], sl[kWSub];
    unsigned char sd[kWSub];
    unsigned short hf[kWSub], hl[kWSub];
};

// The wave's rows of stopper flags: row j = positions F + 64 j .. + 63, its
// 64-bit ballot held by lane j (bd) and cd in lane j = the flags in rows
// before j (lane kWRows: all of them); cum[] is the same, uniform.  The
// number of flags before a range-relative position r, and the position of
// the k-th flag, from registers and lane shuffles (no memory: dynamic
// indices into register arrays would go to scratch).
__device__ __forceinline__ unsigned long long shfl64(unsigned long long v, int src) {
    const int lo = __shfl((int)(unsigned int)v, src, 64), hi = __shfl((int)(unsigned int)(v >> 32), src, 64);
    return ((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo;
}
__device__ __forceinline__ int wv_prefix(unsigned long long bd, int cd, int r) {
    const int row = r >> 6;
    const unsigned long long m = shfl64(bd, row & (kWRows - 1));
    const int base = __shfl(cd, row, 64);
    return base + (row < kWRows ? __popcll(m & ((1ull << (r & 63)) - 1ull)) : 0);
}
__device__ __forceinline__ int wv_select(unsigned long long bd, int cd, const int (&cum)[kWRows + 1], int k) {
    int row = 0;
#pragma unroll
    for (int j = 1; j < kWRows; ++j) row += k >= cum[j];
    unsigned long long x = shfl64(bd, row);
    int kk = k - __shfl(cd, row, 64), p = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const int c = __popcll(x & ((1ull << w) - 1ull));
        if (kk >= c) { kk -= c; x >>= w; p += w; }
    }
    return row * 64 + p;
}

// Sorts items[F, F + n) (LDS, n <= kWT) into std::sort's order for a range
// the introsort loop reaches with `depth` levels of budget.  One whole wave
// calls it with uniform arguments; it touches only its range and `ws`.
// Position F + 64 j + lane is row j of this lane.  Lane s < ns holds active
// sub-range s (tf, tl, td, its pivot, prefix bases, m, cut, child ids); a
// position reaches its sub-range's values by shuffles.  Prefixes, m, the
// cut and every swap partner come from the rows' ballots (wv_prefix /
// wv_select): per level only the medians, the swapped items and the next
// level's table go through LDS.
__device__ __forceinline__ int pcl_wave_sort(u64* items, int F, int n, int depth, WaveSmem& ws) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int E = F + n;
    // per position (row j of this lane), packed: bits 0-7 the active
    // sub-range (kDone once finished), 8-15 the leaf's size (kHeap: a
    // heapsort range), 16-31 the leaf's start
    unsigned int st[kWRows];
    const bool act0 = n > 16 && depth > 0;
#pragma unroll
    for (int j = 0; j < kWRows; ++j) {
        const int x = F + 64 * j + lane;
        st[j] = (unsigned int)((act0 && x < E) ? 0 : kDone) | ((unsigned int)(n <= 16 ? n : kHeap) << 8) |
                ((unsigned int)F << 16);
    }
    int ns = act0 ? 1 : 0, nheap = (!act0 && n > 16) ? 1 : 0;
    int tf = F, tl = E, td = depth;   // lane s < ns: sub-range s
    if (lane == 0) { ws.hf[0] = (unsigned short)F; ws.hl[0] = (unsigned short)E; }
    int levels = 0;
    while (ns > 0) {
        // (1) median of three to the front; the pivot
        unsigned int tpiv = 0;
        if (lane < ns) {
            u64* a = items + tf;
            slo_sort::move_median_to_first_(a, a + 1, a + (tl - tf) / 2, a + (tl - tf - 1), Less());
            tpiv = vkey(a[0]);
        }
        wave_sync();
        // (2) stopper flags by row ballots (all loads first)
        u64 it[kWRows];
        int pf[kWRows];
        unsigned int pp[kWRows];
#pragma unroll
        for (int j = 0; j < kWRows; ++j) {
            const int s = st[j] & 31;
            pf[j] = __shfl(tf, s, 64);
            pp[j] = (unsigned int)__shfl((int)tpiv, s, 64);
            it[j] = items[min(F + 64 * j + lane, E - 1)];
        }
        unsigned long long bL[kWRows], bR[kWRows], bLd = 0, bRd = 0;
        int cL[kWRows + 1], cR[kWRows + 1];
        cL[0] = 0; cR[0] = 0;
#pragma unroll
        for (int j = 0; j < kWRows; ++j) {
            const int x = F + 64 * j + lane;
            const bool act = (st[j] & 0xff) != kDone && x != pf[j];
            const unsigned int k = vkey(it[j]);
            bL[j] = __ballot(act && !(k < pp[j]));
            bR[j] = __ballot(act && !(pp[j] < k));
            cL[j + 1] = cL[j] + __popcll(bL[j]);
            cR[j + 1] = cR[j] + __popcll(bR[j]);
            if (lane == j) { bLd = bL[j]; bRd = bR[j]; }
        }
        int cLd = 0, cRd = 0;
#pragma unroll
        for (int j = 0; j <= kWRows; ++j)
            if (lane == j) { cLd = cL[j]; cRd = cR[j]; }
        // (3) lane s: its sub-range's prefix bases, m at the crossing, the cut.
        // Every lane runs it (lanes >= ns on an empty range): the shuffles
        // read other lanes' registers, which must all be active
        int tsL, teR, tm, tcut;
        {
            const bool mine = lane < ns;
            const int r0 = mine ? tf + 1 - F : 0, r1 = mine ? tl - F : 0;
            tsL = wv_prefix(bLd, cLd, r0);
            teR = wv_prefix(bRd, cRd, r1);
            const int key = tsL + teR;   // the first boundary r with prefL(r) + prefR(r) >= key
            int lo = r0, hi = r1;
#pragma unroll
            for (int i = 0; i < 10; ++i) {   // 2^10 > kWT + 1 boundaries
                const int mid = (lo + hi) >> 1;
                const bool ge = wv_prefix(bLd, cLd, mid) + wv_prefix(bRd, cRd, mid) >= key;
                if (lo < hi) { if (ge) hi = mid; else lo = mid + 1; }
            }
            const int rlo = wv_prefix(bRd, cRd, lo), llo1 = wv_prefix(bLd, cLd, max(lo - 1, 0));
            tm = lo < r1 ? teR - rlo : 0;
            if (lo > r0) tm = max(tm, llo1 - tsL);
            const int tL = wv_prefix(bLd, cLd, r1);
            const int sa = wv_select(bLd, cLd, cL, min(tsL + tm, max(cL[kWRows] - 1, 0)));
            const int sb = wv_select(bRd, cRd, cR, max(min(teR - tm, cR[kWRows] - 1), 0));
            const int cutA = tsL + tm < tL ? F + sa : 0x7fffffff;   // i_{m+1}
            const int cutB = tm > 0 ? F + sb : 0x7fffffff;          // j_m
            tcut = min(cutA, cutB);
        }
        // (4) swaps: left stopper of rank k < m <-> right stopper of rank k from the right
        {
            u64 pit[kWRows];
            int py[kWRows];
            unsigned int sw = 0;
#pragma unroll
            for (int j = 0; j < kWRows; ++j) {
                const int s = st[j] & 31;
                const int sL = __shfl(tsL, s, 64), eR = __shfl(teR, s, 64), m = __shfl(tm, s, 64);
                const int k = cL[j] + __popcll(bL[j] & lt) - sL;
                const bool swp = ((bL[j] >> lane) & 1) && k < m;
                const int q = wv_select(bRd, cRd, cR, max(min(eR - 1 - k, cR[kWRows] - 1), 0));
                py[j] = swp ? F + q : F;
                sw |= (unsigned int)swp << j;
            }
#pragma unroll
            for (int j = 0; j < kWRows; ++j) pit[j] = items[py[j]];
            wave_sync();
#pragma unroll
            for (int j = 0; j < kWRows; ++j)
                if ((sw >> j) & 1) {
                    items[F + 64 * j + lane] = pit[j];
                    items[py[j]] = it[j];
                }
        }
        // (5) the halves: ids by ballot ranks; the next level's table through LDS
        bool wantL = false, wantR = false, heapL = false, heapR = false;
        const int D = td - 1;
        if (lane < ns) {
            wantL = tcut - tf > 16 && D > 0;
            wantR = tl - tcut > 16 && D > 0;
            heapL = tcut - tf > 16 && D == 0;
            heapR = tl - tcut > 16 && D == 0;
        }
        const unsigned long long bwl = __ballot(wantL), bwr = __ballot(wantR);
        const unsigned long long bhl = __ballot(heapL), bhr = __ballot(heapR);
        const int idL = __popcll(bwl & lt) + __popcll(bwr & lt), idR = idL + (int)wantL;
        if (lane < ns) {
            if (wantL) { ws.sf[idL] = (unsigned short)tf; ws.sl[idL] = (unsigned short)tcut; ws.sd[idL] = (unsigned char)D; }
            if (wantR) { ws.sf[idR] = (unsigned short)tcut; ws.sl[idR] = (unsigned short)tl; ws.sd[idR] = (unsigned char)D; }
            const int hL = nheap + __popcll(bhl & lt) + __popcll(bhr & lt), hR = hL + (int)heapL;
            if (heapL) { ws.hf[hL] = (unsigned short)tf; ws.hl[hL] = (unsigned short)tcut; }
            if (heapR) { ws.hf[hR] = (unsigned short)tcut; ws.hl[hR] = (unsigned short)tl; }
        }
        const int nidL = wantL ? idL : -1, nidR = wantR ? idR : -1;
#pragma unroll
        for (int j = 0; j < kWRows; ++j) {
            const int s = st[j] & 31;
            const int x = F + 64 * j + lane;
            const int ct = __shfl(tcut, s, 64), f0 = __shfl(tf, s, 64), l0 = __shfl(tl, s, 64);
            const int iL = __shfl(nidL, s, 64), iR = __shfl(nidR, s, 64);
            if ((st[j] & 0xff) == kDone) continue;
            const bool left = x < ct;
            const int id = left ? iL : iR;
            if (id >= 0) {
                st[j] = (st[j] & ~0xffu) | (unsigned int)id;
            } else {
                const int lo = left ? f0 : ct, hi = left ? ct : l0;
                st[j] = (unsigned int)kDone | ((unsigned int)(hi - lo <= 16 ? hi - lo : kHeap) << 8) | ((unsigned int)lo << 16);
            }
        }
        ns = __popcll(bwl) + __popcll(bwr);
        nheap += __popcll(bhl) + __popcll(bhr);
        wave_sync();
        if (lane < ns) { tf = ws.sf[lane]; tl = ws.sl[lane]; td = ws.sd[lane]; }
        ++levels;
        wave_sync();   // the table is rewritten by the next level
    }
    if (lane < nheap) slo_sort::heap_sort_(items + ws.hf[lane], ws.hl[lane] - ws.hf[lane], Less());
    wave_sync();
    // leaves: the final insertion sort = each item's rank in its leaf by (key, position)
    u64 own[kWRows];
    int dst[kWRows];
#pragma unroll
    for (int j = 0; j < kWRows; ++j) {
        const int x = F + 64 * j + lane;
        own[j] = items[min(x, E - 1)];
        dst[j] = -1;
        const int lo = (int)(st[j] >> 16), sz = (int)((st[j] >> 8) & 0xff);
        if (x >= E || sz == kHeap) continue;
        const unsigned int k = vkey(own[j]);
        unsigned int ky[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) ky[t] = vkey(items[lo + min(t, sz - 1)]);
        int r = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) r += (t < sz) & ((ky[t] < k) | ((ky[t] == k) & (lo + t < x)));
        dst[j] = lo + r;
    }
    wave_sync();
#pragma unroll
    for (int j = 0; j < kWRows; ++j)
        if (dst[j] >= 0) items[dst[j]] = own[j];
    wave_sync();
    return levels;
}

// LDS of pcl_block_sort for up to NMAX items (NMAX <= 32768).  The items
// themselves are the caller's LDS array.
template <int NT, int NMAX>
struct BlockSmem {
    static constexpr int MAXSEG = NMAX / (kWT + 1) + 2;      // disjoint ranges of > kWT items, + slack
    static constexpr int MAXW = 2 * 2 * 16 * MAXSEG + 32;    // ranges handed to the wave tier
    unsigned short seg_of[NMAX];   // the active range a position belongs to (kNone: handed on)
    unsigned short tblB[NMAX];     // right stoppers by rank from the right, at f + rank
    unsigned short f[2][MAXSEG], l[2][MAXSEG];
    unsigned char d[2][MAXSEG];
    unsigned int piv[MAXSEG];
    int sL[MAXSEG], eR[MAXSEG], m[MAXSEG], cutA[MAXSEG], cutB[MAXSEG];
    unsigned short nidL[MAXSEG], nidR[MAXSEG];
    unsigned short hf[MAXSEG], hl[MAXSEG];   // heapsort ranges over kWT items
    unsigned short wf[MAXW], wl[MAXW];       // wave-tier ranges
    unsigned char wd[MAXW];
    int nseg[2], nheap, nw;
    unsigned int wsum[NT / 64];
};

// The block tier on items[0, n) (LDS, n <= NMAX) of a range the introsort
// loop reaches with `depth` levels of budget (2 * lg(n) for a whole array):
// on return every range over kWT items is split down or heapsorted, and the
// ranges of 2..kWT items that remain are listed in sm.wf / wl / wd (sm.nw)
// for the wave tier (pcl_wave_sort), which the caller runs — in the same
// workgroup, or from a global list.  All NT threads call it.
//
// Block-tier positions are wave-striped: wave w, row j, lane t owns position
// x = w * 64 * IPT + j * 64 + t, so each LDS access of a row is 64
// consecutive words (no bank conflicts) and every prefix count is a ballot.
template <int NT, int NMAX>
__device__ __forceinline__ int pcl_block_sort(u64* items, int n, int depth, BlockSmem<NT, NMAX>& sm) {
    int levels = 0;
    static_assert(NMAX % NT == 0 && NMAX <= 32768 && NT % 64 == 0, "pcl_block_sort layout");
    constexpr int IPT = NMAX / NT, NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int xw = w * 64 * IPT + lane;   // position of row j: xw + 64 j
    const unsigned long long lt = (1ull << lane) - 1ull;
    const bool active0 = n > kWT && depth > 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const int x = xw + 64 * j;
        sm.seg_of[x] = (active0 && x < n) ? 0 : kNone;
    }
    if (tid == 0) {
        sm.nseg[0] = active0 ? 1 : 0;
        sm.nseg[1] = 0;
        sm.nheap = 0;
        sm.nw = 0;
        sm.f[0][0] = 0; sm.l[0][0] = (unsigned short)n; sm.d[0][0] = (unsigned char)depth;
        if (!active0 && n > kWT) { sm.hf[0] = 0; sm.hl[0] = (unsigned short)n; sm.nheap = 1; }
        if (n <= kWT && n > 1) { sm.wf[0] = 0; sm.wl[0] = (unsigned short)n; sm.wd[0] = (unsigned char)depth; sm.nw = 1; }
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
        // (2) stopper flags: per row a ballot of left and of right stoppers
        u64 it[IPT];
        unsigned short so[IPT];
        unsigned long long bL[IPT], bR[IPT];
        int rf[IPT];
        int cL = 0, cR = 0;
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int x = xw + 64 * j;
            so[j] = sm.seg_of[x];
            bool isL = false, isR = false;
            rf[j] = -1;
            if (so[j] != kNone) {
                rf[j] = sm.f[c][so[j]];
                if (x != rf[j]) {
                    it[j] = items[x];
                    const unsigned int k = vkey(it[j]), p = sm.piv[so[j]];
                    isL = !(k < p);
                    isR = !(p < k);
                }
            }
            bL[j] = __ballot(isL);
            bR[j] = __ballot(isR);
            cL += __popcll(bL[j]);
            cR += __popcll(bR[j]);
        }
        if (lane == 0) sm.wsum[w] = (unsigned int)cL | ((unsigned int)cR << 16);
        __syncthreads();
        int bl = 0, br = 0;   // stoppers before this wave's block
#pragma unroll
        for (int q = 0; q < NW; ++q)
            if (q < w) { const unsigned int v = sm.wsum[q]; bl += (int)(v & 0xffffu); br += (int)(v >> 16); }
        int pl[IPT], pr[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            pl[j] = bl + __popcll(bL[j] & lt);
            pr[j] = br + __popcll(bR[j] & lt);
            bl += __popcll(bL[j]);
            br += __popcll(bR[j]);
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int s = so[j];
            if (s == kNone) continue;
            const int x = xw + 64 * j;
            if (x == rf[j] + 1) sm.sL[s] = pl[j];
            if (x == sm.l[c][s] - 1) sm.eR[s] = pr[j] + (int)((bR[j] >> lane) & 1);
        }
        __syncthreads();
        // (3) m of every range: max over its boundaries of min(left before,
        // right at or after); posted only around the crossing (as in the wave
        // tier) and at the edges of each wave's block, whose neighbours are
        // another wave's
        {
            int lb[IPT], rb[IPT];
            unsigned long long bF[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int s = so[j];
                const int x = xw + 64 * j;
                bool fl = false;
                lb[j] = 0; rb[j] = 0;
                if (s != kNone && x > rf[j]) {
                    lb[j] = pl[j] - sm.sL[s];
                    rb[j] = sm.eR[s] - pr[j];
                    fl = lb[j] >= rb[j];
                }
                bF[j] = __ballot(fl);
            }
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int s = so[j];
                const int x = xw + 64 * j;
                if (s == kNone || x <= rf[j]) continue;
                const bool fl = (bF[j] >> lane) & 1;
                const bool edgeP = lane == 0 && j == 0, edgeN = lane == 63 && j == IPT - 1;
                const bool prevF = lane > 0 ? (bF[j] >> (lane - 1)) & 1 : (j > 0 ? (bF[j - 1] >> 63) & 1 : 0);
                const bool nextF = lane < 63 ? (bF[j] >> (lane + 1)) & 1 : (j + 1 < IPT ? bF[j + 1] & 1 : 1);
                const bool first = x == rf[j] + 1, last = x == sm.l[c][s] - 1;
                if (edgeP || edgeN) {
                    const int g = min(lb[j], rb[j]);
                    if (g > 0) atomicMax(&sm.m[s], g);
                }
                if (fl && (first || !prevF) && rb[j] > 0) atomicMax(&sm.m[s], rb[j]);
                if (!fl && (last || nextF) && lb[j] > 0) atomicMax(&sm.m[s], lb[j]);
            }
        }
        __syncthreads();
        // (4) right stoppers by rank from the right; the cut candidates
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int s = so[j];
            if (s == kNone) continue;
            const int x = xw + 64 * j;
            const int m = sm.m[s];
            if (((bL[j] >> lane) & 1) && pl[j] - sm.sL[s] == m) sm.cutA[s] = x;   // i_{m+1}
            if ((bR[j] >> lane) & 1) {
                const int kr = sm.eR[s] - pr[j] - 1;                                // right stoppers after x
                if (kr < m) sm.tblB[rf[j] + kr] = (unsigned short)x;
                if (kr == m - 1) sm.cutB[s] = x;                                     // j_m
            }
        }
        __syncthreads();
        // (5) the swaps: left stopper of rank k < m <-> right stopper of rank k
        {
            u64 pit[IPT];
            unsigned short py[IPT];
            unsigned int sw = 0;
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                if (!((bL[j] >> lane) & 1)) continue;
                const int s = so[j];
                const int k = pl[j] - sm.sL[s];
                if (k < sm.m[s]) {
                    py[j] = sm.tblB[rf[j] + k];
                    pit[j] = items[py[j]];
                    sw |= 1u << j;
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < IPT; ++j)
                if ((sw >> j) & 1) {
                    items[xw + 64 * j] = pit[j];
                    items[py[j]] = it[j];
                }
        }
        // (6) the halves: over kWT items with budget left stay in the block
        // tier; smaller ones go to the wave tier; spent budget: heapsort
        for (int s = tid; s < ns; s += NT) {
            const int F = sm.f[c][s], L = sm.l[c][s], D = sm.d[c][s] - 1;
            const int cut = min(sm.cutA[s], sm.m[s] > 0 ? sm.cutB[s] : 0x7fffffff);
            sm.cutA[s] = cut;
            const int lo[2] = {F, cut}, hi[2] = {cut, L};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                unsigned short id = kNone;
                const int sz = hi[h] - lo[h];
                if (sz > kWT && D > 0) {
                    id = (unsigned short)atomicAdd(&sm.nseg[c ^ 1], 1);
                    sm.f[c ^ 1][id] = (unsigned short)lo[h]; sm.l[c ^ 1][id] = (unsigned short)hi[h];
                    sm.d[c ^ 1][id] = (unsigned char)D;
                } else if (sz > kWT) {
                    const int q = atomicAdd(&sm.nheap, 1);
                    sm.hf[q] = (unsigned short)lo[h]; sm.hl[q] = (unsigned short)hi[h];
                } else if (sz > 1) {
                    const int q = atomicAdd(&sm.nw, 1);
                    sm.wf[q] = (unsigned short)lo[h]; sm.wl[q] = (unsigned short)hi[h]; sm.wd[q] = (unsigned char)D;
                }
                (h ? sm.nidR : sm.nidL)[s] = id;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int s = so[j];
            if (s == kNone) continue;
            sm.seg_of[xw + 64 * j] = xw + 64 * j < sm.cutA[s] ? sm.nidL[s] : sm.nidR[s];
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
    return levels;
}

}  // namespace slo_pcl
