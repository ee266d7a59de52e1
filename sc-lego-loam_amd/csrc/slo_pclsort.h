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
constexpr unsigned char kWave = 0xfe;   // the position's range went to the wave tier
constexpr int kWaveMax = 128;           // ranges of at most this many items go to the wave tier

// ---- wave tier: one wave takes a range of at most kWaveMax items to the
// end (its introsort steps, heapsorts and leaves) with no workgroup barrier.
// Control flow is wave-uniform throughout (every lane runs every step), so
// the cross-lane reductions see all 64 lanes.  LDS operations of one wave
// complete in order; the fences keep the compiler from reordering them.
__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
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

// one introsort step of [f, l) (l - f - 1 <= 64 R): the formulation of the
// header comment with the range's positions f + 1 + 64 r + lane in R rows.
// The median swap is taken virtually while the rows are read (one LDS round
// trip), m comes from the ballot of the crossing and two lane reads, and the
// LDS sees the median swap, the right-stopper table, its reads, the partner
// reads and the swaps: five dependent steps.  Returns the cut.
template <int R>
__device__ __forceinline__ int wave_step(u64* items, unsigned short* tbl, int f, int l) {
    const int lane = threadIdx.x & 63;
    constexpr int INF = 0x7fffffff;
    const int mid = f + (l - f) / 2;
    const u64 a0 = items[f], a1 = items[f + 1], a2 = items[mid], a3 = items[l - 1];
    u64 it[R];
#pragma unroll
    for (int r = 0; r < R; ++r) it[r] = items[min(f + 1 + 64 * r + lane, l - 1)];
    const int w = median3(vkey(a1), vkey(a2), vkey(a3));
    const int med = w == 0 ? f + 1 : (w == 1 ? mid : l - 1);
    const u64 pit = w == 0 ? a1 : (w == 1 ? a2 : a3);
    const unsigned int p = vkey(pit);
    bool iL[R], iR[R];
    int pl[R], pr[R];
    unsigned long long bl[R], br[R];
    int cl = 0, cr = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int x = f + 1 + 64 * r + lane;
        if (x == med) it[r] = a0;   // the item the median swap leaves there
        const bool act = x < l;
        const unsigned int k = vkey(it[r]);
        iL[r] = act && !(k < p);
        iR[r] = act && !(p < k);
        bl[r] = __ballot(iL[r]);
        br[r] = __ballot(iR[r]);
        pl[r] = cl + lane_prefix(bl[r]);
        pr[r] = cr + lane_prefix(br[r]);
        cl += __popcll(bl[r]);
        cr += __popcll(br[r]);
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
        if (iR[r] && kr < m) tbl[f + kr] = (unsigned short)(f + 1 + 64 * r + lane);
    }
    wave_fence();
    int y[R];
    u64 py[R];
#pragma unroll
    for (int r = 0; r < R; ++r) y[r] = (iL[r] && pl[r] < m) ? (int)tbl[f + pl[r]] : -1;
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

// [F, L) with `depth` levels of budget, to the end, by the calling wave
// (every lane); stk: 32 words of this wave's LDS.  Steps go depth first; a
// leaf (<= 16 items, which the final insertion sort leaves stably sorted)
// only marks its positions in tbl (offset in the leaf | size << 5: a
// position's tbl word is free once its range is a leaf), a heapsorted range
// marks them 0xffff; one pass over [F, L) at the end ranks every leaf's
// items at once.
__device__ __forceinline__ void wave_range(u64* items, unsigned short* tbl, unsigned int* stk, int F, int L,
                                           int depth) {
    const int lane = threadIdx.x & 63;
    int sp = 0, f = F, l = L;
    for (;;) {
        const int n = l - f;
        bool pop = true;
        if (n <= 16) {
            if (lane < n) tbl[f + lane] = (unsigned short)(lane | (n << 5));
        } else if (depth == 0) {
            if (lane == 0) slo_sort::heap_sort_(items + f, n, Less());
            for (int x = f + lane; x < l; x += 64) tbl[x] = 0xffff;
        } else {
            const int cut = n - 1 <= 64 ? wave_step<1>(items, tbl, f, l) : wave_step<kWaveMax / 64>(items, tbl, f, l);
            if (lane == 0) stk[sp] = (unsigned int)cut | ((unsigned int)l << 13) | ((unsigned int)(depth - 1) << 26);
            ++sp;
            l = cut;
            depth -= 1;
            pop = false;
        }
        wave_fence();
        if (pop) {
            if (sp == 0) break;
            --sp;
            const unsigned int e = __builtin_amdgcn_readfirstlane(stk[sp]);
            f = (int)(e & 0x1fffu);
            l = (int)((e >> 13) & 0x1fffu);
            depth = (int)(e >> 26);
        }
    }
    // every leaf at once: an item's place is its rank in the leaf by (key, position)
    constexpr int RR = kWaveMax / 64;
    u64 own[RR];
    int dst[RR];
#pragma unroll
    for (int r = 0; r < RR; ++r) {
        const int x = F + 64 * r + lane;
        own[r] = items[min(x, L - 1)];
        const unsigned int info = tbl[min(x, L - 1)];
        dst[r] = -1;
        if (x >= L || info == 0xffffu) continue;
        const int o = (int)(info & 31u), sz = (int)(info >> 5), lo = x - o;
        const unsigned int k = vkey(own[r]);
        unsigned int ky[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) ky[t] = vkey(items[lo + min(t, sz - 1)]);
        int rk = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) rk += (t < sz) & ((ky[t] < k) | ((ky[t] == k) & (t < o)));
        dst[r] = lo + rk;
    }
    wave_fence();
#pragma unroll
    for (int r = 0; r < RR; ++r)
        if (dst[r] >= 0) items[dst[r]] = own[r];
    wave_fence();
}

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
    unsigned int wq[MAXSEG];                 // wave-tier ranges: first | end << 13 | depth << 26
    unsigned int stk[NT / 64][32];           // wave-tier stacks
    int nseg[2], nheap, nwq, wq_next;
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
__device__ __forceinline__ int pcl_block_sort(u64* items, int n, int depth, BlockSmem<NT, NMAX>& sm,
                                              unsigned long long* prof = nullptr) {   // [4] thread 0: phase cycles, wave ranges
    const long long pt0 = clock64();
    static_assert(NMAX % NT == 0 && NMAX <= 4096 && NT % 64 == 0, "pcl_block_sort layout");
    constexpr int IPT = NMAX / NT, NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int xw = w * 64 * IPT + lane;   // position of row j: xw + 64 j
    const unsigned long long lt = (1ull << lane) - 1ull;
    // per position, packed: bits 0-7 the active range (kDone once finished),
    // 8-15 its leaf's size (kHeap: a heapsort range), 16-31 its leaf's start
    unsigned int st[IPT];
    const bool wave0 = n > 16 && depth > 0 && n <= kWaveMax;
    const bool act0 = n > 16 && depth > 0 && !wave0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const int x = xw + 64 * j;
        st[j] = (unsigned int)((act0 && x < n) ? 0 : kDone) |
                ((unsigned int)(n <= 16 ? n : wave0 ? kWave : kHeap) << 8);
    }
    if (tid == 0) {
        sm.nseg[0] = act0 ? 1 : 0;
        sm.nseg[1] = 0;
        sm.nheap = (n > 16 && depth == 0) ? 1 : 0;
        sm.nwq = wave0 ? 1 : 0;
        sm.wq_next = 0;
        sm.f[0][0] = 0; sm.l[0][0] = (unsigned short)n; sm.d[0][0] = (unsigned char)depth;
        sm.hf[0] = 0; sm.hl[0] = (unsigned short)n;
        sm.wq[0] = (unsigned int)n << 13 | (unsigned int)depth << 26;
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
                    if (D > 0 && hi[h] - lo[h] <= kWaveMax) {   // to the wave tier
                        const int q = atomicAdd(&sm.nwq, 1);
                        sm.wq[q] = (unsigned int)lo[h] | ((unsigned int)hi[h] << 13) | ((unsigned int)D << 26);
                        id = -2;
                    } else if (D > 0) {
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
                } else if (id == -2) {
                    st[j] = (unsigned int)kDone | ((unsigned int)kWave << 8);
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
    const long long pt1 = clock64();
    // heapsort ranges (depth spent), one lane each
    for (int q = tid; q < sm.nheap; q += NT)
        slo_sort::heap_sort_(items + sm.hf[q], sm.hl[q] - sm.hf[q], Less());
    // wave tier: every wave takes queued ranges until none is left
    for (;;) {
        int q = 0;
        if (lane == 0) q = atomicAdd(&sm.wq_next, 1);
        q = __builtin_amdgcn_readfirstlane(q);
        if (q >= sm.nwq) break;
        const unsigned int e = __builtin_amdgcn_readfirstlane(sm.wq[q]);
        wave_range(items, sm.tblB, sm.stk[w], (int)(e & 0x1fffu), (int)((e >> 13) & 0x1fffu), (int)(e >> 26));
    }
    __syncthreads();
    const long long pt2 = clock64();
    // leaves: the final insertion sort = each item's rank in its leaf by (key, position)
    u64 own[IPT];
    int dst[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const int x = xw + 64 * j;
        own[j] = items[min(x, NMAX - 1)];
        const int lo = (int)(st[j] >> 16), sz = (int)((st[j] >> 8) & 0xff);
        dst[j] = -1;
        if (x >= n || sz == kHeap || sz == kWave) continue;
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
    if (prof && tid == 0) {
        const long long pt3 = clock64();
        prof[0] += (unsigned long long)(pt1 - pt0);
        prof[1] += (unsigned long long)(pt2 - pt1);
        prof[2] += (unsigned long long)(pt3 - pt2);
        prof[3] += (unsigned long long)sm.nwq;
    }
    return levels;
}

}  // namespace slo_pcl
