// slo_vgpcl.hip — the batched VoxelGrid sort in PCL's own order
// (cfg.voxel_order == SLO_VOXEL_PCL, the default).
//
// PCL's VoxelGrid::applyFilter (featureAssociation.cpp:779-780,
// mapOptmization.cpp:1224-1262) collects (voxel index, point index) pairs of
// the finite points in input order and sorts them with std::sort by voxel
// index; each voxel's centroid is summed in the resulting order.  This file
// produces that order exactly (slo_pclsort.h states the formulation) for S
// streams at once; the voxel heads and centroid sums of slo_vg.hip then read
// it as they read the radix sort's.
//
// Pipeline per call (all sizes from the input strides, counts on the device):
//   k_pc_count, k_pc_scan, k_pc_write: the finite points' items, compacted in
//     input order (the raw cloud is not dense, MO:1236; the other clouds are
//     finite), the non-finite ones after them with the "none" key; each
//     stream's range becomes the first introsort range: a global range
//     (> PC_TAIL items) or a list entry;
//   G global levels, one introsort step of every global range per level:
//     k_pc_lcount  per chunk of PC_CH positions: stopper counts (the median of
//                  three is taken virtually: every chunk derives it alone);
//     k_pc_lscan   per range: chunk prefixes, m from the chunk where the
//                  left / right counts cross;
//     k_pc_lrank   per chunk: the positions of the left stoppers of rank < m
//                  and of the right stoppers of rank < m (from the right), the
//                  cut candidates; chunk 0 makes the median swap real;
//     k_pc_lpairs  the swaps;
//     k_pc_lsplit  per range: the halves — over PC_TAIL items back to the
//                  next level, otherwise (or at the last level) a list entry.
//   (Folding the per-range steps into the last chunk's workgroup, by a
//   done counter, measured 20x slower: the device-scope fence each chunk
//   then needs writes the XCD's L2 back.)
//   k_pc_tail: one workgroup per range of more than PC_T items, depth first
//     down to ranges of at most PC_T (the same step, barriers for launches);
//   k_pc_finish: one wave per range of at most PC_T items sorts it in LDS to
//     the end (slo_pcl::wave_sort);
//   pc_fallback_entry: a range over PC_T items with its depth budget spent
//     (counted in vg_stats) is heapsorted by one wave, inside k_pc_finish32.
#include "slo_vgcommon.h"
#include "slo_pclsort.h"

namespace slo {

using slo_pcl::u64;

#define PC_CH 4096        // positions per chunk of the global levels (256 threads x 16)
#define PC_CT 256
#ifndef PC_T
#define PC_T 4096         // a range of at most PC_T items is finished in LDS
#define PC_ST 2048        // finish size classes: <= PC_WT, <= PC_ST, <= PC_T items (LDS per entry)
#define PC_WT 512
#endif
#ifndef PC_TAIL
#define PC_TAIL 65536     // the global levels take ranges of more than PC_TAIL items, k_pc_tail the rest
#endif
#ifndef PC_FEW
#define PC_FEW 8          // at most this many streams: PC_TAIL_FEW, and 16 / 8 waves per finish entry
#endif
#ifndef PC_TAIL_FEW
#define PC_TAIL_FEW 16384
#endif
#define PC_G 2048         // workgroups of the grid-stride level kernels
#ifndef PC_G_FEW
#define PC_G_FEW PC_G     // the same with a few streams
#endif
#ifndef PC_XLEV
#define PC_XLEV 9         // global levels past log2(stride / tail size), for the uneven splits median-of-three leaves:
                          // 3 / 6 / 9 / 12: the tail 39.9 / 27.1 / 21.3 / 21.1 ms, the levels 21.0 / 23.3 / 24.9 /
                          // 26.4 ms per 6 mapping steps; 18.8k / 19.0k / 19.1k / 19.0k scans/s
#endif
#ifndef PC_XLEV_FEW
#define PC_XLEV_FEW 3     // a few streams: 0 extra levels shortened the sorts of young local maps (2.27 -> 2.02 ms per
                          // mapping step over scans 0-200) but not steady-state ones (the bench's one-stream legs
                          // after its 210-scan pre-roll: 569 / 731 / 1 155 scans/s against 578 / 765 / 1 240 with 3)
#endif
#ifndef PC_LOCC
#define PC_LOCC 8         // waves per SIMD k_pc_lrank is built for (latency-bound streaming)
#endif
#ifndef PC_WOCC
#define PC_WOCC 6         // k_pc_write (8 would spill 12 VGPRs)
#endif
// PclWs::pstat, cumulative work counters (slo_get "pcl_work"; the bench
// prices the kernels' algorithmic bytes with them): [0] items of the ranges
// stepped by the global levels, [1] pairs they swapped, [2..4] items of
// finish lists 0..2, [5] VoxelGrid input points, [6] finish entries, [7]
// items of the ranges k_pc_tail stepped, [8] pairs it swapped, [9 + 3 list + q]
// finish cycles of list `list` in streamed steps, register steps, lane tasks
enum { PW_ACTIVE = 0, PW_PAIRS = 1, PW_FIN = 2, PW_INPUT = 5, PW_ENTRIES = 6, PW_TAIL = 7, PW_TAIL_PAIRS = 8, PW_PROF = 9,
       PW_FINX = 20,     // [20]: items of list 5 (the 4 Ki entries too wide for 32-bit items, k_pc_finish on 64-bit)
       PW_FALL = 21 };   // [21]: items of the spent-depth ranges pc_fallback_entry heapsorts

struct PSeg { int f, l, d, c0; };
struct PRes { unsigned int piv, vmed; int med, m, TR, cutA, cutB; };

// counters (PclWs::ctr)
enum { PCC_NSEG = 0, PCC_NCH = 2, PCC_NW = 6 };   // [cur] per level parity; PCC_NW + k: range list k

// Range lists: finish entries by size class, list 0 <= PC_WT items, 1 <= PC_ST,
// 2 <= PC_T (k_pc_finish32, then k_pc_finish<size>); 3 larger (k_pc_tail); 4 a spent depth budget
// over PC_T items (pc_fallback_entry: heapsort); 5 the list-2 entries whose keys span 2^20 or more (filled by
// k_pc_finish32, sorted by k_pc_finish on 64-bit items); 6 the list-3 ranges over PT_SMAXT tiles (filled by the
// small-table k_pc_tail, stepped by the large-table one).  An entry is (first position, size | depth << 24).
struct PcLists { int2* l[7]; };
__device__ inline void pc_push(const PcLists& L, int* ctr, int f, int n, int d) {
    const int k = n <= PC_WT ? 0 : n <= PC_ST ? 1 : n <= PC_T ? 2 : 3;
    const int i = atomicAdd(&ctr[PCC_NW + k], 1);
    L.l[k][i] = make_int2(f, n | (d << 24));
}

// the pivot of range [f, l), the position swapped with f, and the key that
// lands there (the one at f)
__device__ inline void pc_median(const unsigned int* K, int f, int l, unsigned int& piv, int& med, unsigned int& vmed) {
    const int pos[3] = {f + 1, f + (l - f) / 2, l - 1};
    const unsigned int k0 = K[pos[0]], k1 = K[pos[1]], k2 = K[pos[2]], kf = K[f];
    const int w = slo_pcl::median3(k0, k1, k2);
    med = pos[w];
    piv = w == 0 ? k0 : (w == 1 ? k1 : k2);
    vmed = kf;
}

// the stream whose item range [off[s], off[s + 1]) holds position pos (a
// guard's range, to flag that stream: PclWs::serr)
__device__ inline int pc_stream_of(const int32_t* off, int S, int pos) {
    int lo = 0, hi = S - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= pos) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
__device__ inline void pc_flag(int32_t* serr, const int32_t* off, int S, int pos, int bit) {
    atomicOr(&serr[pc_stream_of(off, S, pos)], bit);
}

__device__ __forceinline__ int lane_prefix64(unsigned long long b) {   // set bits of b below this lane
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned int)(b >> 32), __builtin_amdgcn_mbcnt_lo((unsigned int)b, 0u));
}

// ---- items: finite points first, in input order
__global__ void __launch_bounds__(VG_T) k_pc_count(VgSrc src, const int32_t* off,
                                                    const VgParams* prm, int* tcnt, int maxT, int S, int* ctr) {
    __shared__ unsigned int wsum[VG_W];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 16) ctr[threadIdx.x] = 0;
    const int s = blockIdx.y;
    if (s >= S) return;
    const VgParams p = prm[s];
    const int n = off[s + 1] - off[s];
    const float4* in = src.row(s);
    for (int t = blockIdx.x; t < p.ntiles; t += gridDim.x) {
        const int a = t * VG_TILE, m = min(VG_TILE, n - a);
        float4 q[VG_IPT];
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) q[k] = in[a + min(k * VG_T + (int)threadIdx.x, m - 1)];
        unsigned int c = 0;
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k)
            c += (k * VG_T + (int)threadIdx.x < m) & isfinite(q[k].x) & isfinite(q[k].y) & isfinite(q[k].z);
        unsigned int total;
        vg_block_scan<VG_W>(c, wsum, &total);
        if (threadIdx.x == 0) tcnt[(size_t)s * maxT + t] = (int)total;
    }
}

// per stream: tile prefix of the finite counts, and the stream's first range
__global__ void __launch_bounds__(1024) k_pc_scan(int tail_min, const int32_t* off, const VgParams* prm, int* tcnt, int maxT,
                                                  PSeg* seg0, int* cseg0, PcLists wl, int* ctr, int32_t* nfin,
                                                  unsigned long long* pst, int32_t* serr) {
    __shared__ int wsum[16];
    __shared__ int slot_c0[2];
    const int s = blockIdx.x, tid = threadIdx.x;
    const VgParams p = prm[s];
    const int nt = p.ntiles;
    int* h = tcnt + (size_t)s * maxT;
    const int L = (nt + 1023) / 1024, t0 = min(nt, tid * L), t1 = min(nt, t0 + L);
    int sum = 0;
    for (int t = t0; t < t1; ++t) sum += h[t];
    int total;
    int run = vg_block_scan<16>(sum, wsum, &total);
    for (int t = t0; t < t1; ++t) {
        const int x = h[t];
        h[t] = run;
        run += x;
    }
    const int f = off[s], n = total;
    if (tid == 0) {
        nfin[s] = n;
        atomicAdd(&pst[PW_INPUT], (unsigned long long)(off[s + 1] - off[s]));
        slot_c0[0] = -1;
        // a range's size is kept in 24 bits of its list entry: a larger
        // stream is left unsorted and flagged (never at the configs' sizes)
        if (n >= (1 << 24)) atomicOr(&serr[s], SLO_ERR_MAP_CAPACITY);
        // overflow keys are the positions: already in order
        else if (!p.overflow && n >= 2) {
            const int d = 2 * slo_pcl::lg2(n);
            if (n > tail_min) {
                const int nch = (n - 1 + PC_CH - 1) / PC_CH;
                const int slot = atomicAdd(&ctr[PCC_NSEG], 1);
                const int c0 = atomicAdd(&ctr[PCC_NCH], nch);
                seg0[slot] = PSeg{f, f + n, d, c0};
                slot_c0[0] = slot; slot_c0[1] = c0;
            } else {
                pc_push(wl, ctr, f, n, d);
            }
        }
    }
    __syncthreads();
    if (slot_c0[0] >= 0) {
        const int nch = (n - 1 + PC_CH - 1) / PC_CH;
        for (int c = tid; c < nch; c += 1024) cseg0[slot_c0[1] + c] = slot_c0[0];
    }
}

// Striped: thread tid takes items a + k * VG_T + tid (k = 0 .. VG_IPT - 1),
// so every load and store instruction of a wave touches 64 consecutive items
// (the blocked layout, a + tid * VG_IPT + k, made each instruction 64 separate
// lines: k_pc_write waited on instruction issue 80 % of its cycles).  The
// tile's input order is k-major, then wave, then lane: per (stripe, wave)
// finite counts by ballot, one prefix over them, and the lane's rank by mbcnt.
__global__ void __launch_bounds__(VG_T) __attribute__((amdgpu_waves_per_eu(PC_WOCC))) k_pc_write(VgSrc src, const int32_t* off,
                                                    const VgParams* prm, const int* tcnt, const int32_t* nfin,
                                                    int maxT, unsigned int* K, unsigned int* V, int S) {
    __shared__ int wc[VG_IPT * VG_W];   // finite items per (stripe, wave), then their exclusive prefixes
    const int s = blockIdx.y;
    if (s >= S) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const VgParams p = prm[s];
    const int base = off[s], n = off[s + 1] - base, nf = nfin[s];
    const float4* in = src.row(s);
    for (int t = blockIdx.x; t < p.ntiles; t += gridDim.x) {
        const int a = t * VG_TILE, m = min(VG_TILE, n - a);
        float4 q[VG_IPT];
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) q[k] = in[a + min(k * VG_T + tid, m - 1)];
        unsigned int key[VG_IPT], fin = 0;
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            key[k] = vg_key(q[k], p, a + k * VG_T + tid);
            const bool ok = k * VG_T + tid < m && key[k] != vg_none(p);
            fin |= (unsigned int)ok << k;
            const unsigned long long b = __ballot(ok);
            if (lane == 0) wc[k * VG_W + w] = __popcll(b);
        }
        __syncthreads();
        if (tid < 64) {   // exclusive prefix over the VG_IPT * VG_W (stripe, wave) counts, in input order
            static_assert(VG_IPT * VG_W == 64, "one lane per (stripe, wave)");
            const int x = wc[tid];
            int incl = x;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            wc[tid] = incl - x;
        }
        __syncthreads();
        const int r0 = tcnt[(size_t)s * maxT + t];   // finite items of the stream before the tile
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            const int j = k * VG_T + tid;
            const bool ok = (fin >> k) & 1u;
            const int fb = r0 + wc[k * VG_W + w] + lane_prefix64(__ballot(ok));   // finite items before item j
            if (j < m) {
                const int o = ok ? fb : nf + (a + j) - fb;
                K[base + o] = key[k];
                V[base + o] = (unsigned int)(a + j);
            }
        }
        __syncthreads();   // wc is the next tile's
    }
}

// ---- global levels
__device__ inline void pc_chunk(const PSeg& g, int c, int& a, int& b) {
    a = g.f + 1 + (c - g.c0) * PC_CH;
    b = min(g.l, a + PC_CH);
}

__global__ void __launch_bounds__(PC_CT) k_pc_lcount(const unsigned int* K, const PSeg* seg, const int* cseg,
                                                      int2* ccnt, int* ctr, int cur) {
    __shared__ unsigned int wsum[PC_CT / 64];
    const int nch = ctr[PCC_NCH + cur];
    for (int c = blockIdx.x; c < nch; c += gridDim.x) {
        const PSeg g = seg[cseg[c]];
        unsigned int piv, vmed;
        int med;
        pc_median(K, g.f, g.l, piv, med, vmed);
        int a, b;
        pc_chunk(g, c, a, b);
        unsigned int kk[PC_CH / PC_CT];
#pragma unroll
        for (int q = 0; q < PC_CH / PC_CT; ++q) kk[q] = K[min(a + q * PC_CT + (int)threadIdx.x, b - 1)];
        unsigned int cl = 0, cr = 0;
#pragma unroll
        for (int q = 0; q < PC_CH / PC_CT; ++q) {
            const int x = a + q * PC_CT + (int)threadIdx.x;
            const unsigned int k = x == med ? vmed : kk[q];
            const bool in = x < b;
            cl += in & !(k < piv);
            cr += in & !(piv < k);
        }
        unsigned int total;
        vg_block_scan<PC_CT / 64>(cl | (cr << 16), wsum, &total);
        if (threadIdx.x == 0) ccnt[c] = make_int2((int)(total & 0xffffu), (int)(total >> 16));
    }
}

// per range: pivot record, chunk prefixes, m
__global__ void __launch_bounds__(PC_CT) k_pc_lscan(const unsigned int* K, const PSeg* seg, int2* ccnt, PRes* res,
                                                     int* ctr, int cur, unsigned long long* pst) {
    __shared__ unsigned int wsum[PC_CT / 64];
    __shared__ int cstar_s, mx_s;
    unsigned long long wact = 0, wpairs = 0;   // work counters, one atomic per block
    if (blockIdx.x == 0 && threadIdx.x == 0) { ctr[PCC_NSEG + (cur ^ 1)] = 0; ctr[PCC_NCH + (cur ^ 1)] = 0; }
    const int ns = ctr[PCC_NSEG + cur];
    const int tid = threadIdx.x;
    for (int s = blockIdx.x; s < ns; s += gridDim.x) {
        const PSeg g = seg[s];
        unsigned int piv, vmed;
        int med;
        pc_median(K, g.f, g.l, piv, med, vmed);
        const int nch = (g.l - g.f - 1 + PC_CH - 1) / PC_CH;
        // exclusive prefix of the chunk counts, in place (chunks in rounds of PC_CT)
        int runL = 0, runR = 0;
        for (int c0 = 0; c0 < nch; c0 += PC_CT) {
            const int c = c0 + tid;
            const int2 x = c < nch ? ccnt[g.c0 + c] : make_int2(0, 0);
            int totL, totR;
            const int exL = vg_block_scan<PC_CT / 64>(x.x, (int*)wsum, &totL);
            const int exR = vg_block_scan<PC_CT / 64>(x.y, (int*)wsum, &totR);
            if (c < nch) ccnt[g.c0 + c] = make_int2(runL + exL, runR + exR);
            runL += totL;
            runR += totR;
        }
        const int TR = runR;
        __syncthreads();   // the prefixes are visible to the block
        // the crossing chunk: the first whose end boundary has left >= right-at-or-after
        if (tid == 0) cstar_s = nch - 1;
        __syncthreads();
        for (int c = tid; c < nch; c += PC_CT) {
            const int2 pre = ccnt[g.c0 + c];
            const int2 nxt = c + 1 < nch ? ccnt[g.c0 + c + 1] : make_int2(runL, runR);
            (void)pre;
            if (nxt.x >= TR - nxt.y) atomicMin(&cstar_s, c);
        }
        __syncthreads();
        const int cs = cstar_s;
        // exact m over the boundaries of the crossing chunk (its end included)
        int a, b;
        pc_chunk(g, g.c0 + cs, a, b);
        const int2 pre = ccnt[g.c0 + cs];
        constexpr int Q = PC_CH / PC_CT;
        const int j0 = tid * Q;   // blocked positions a + j0 ..
        unsigned int kk[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) kk[q] = K[min(a + j0 + q, b - 1)];
        unsigned int fl = 0, fr = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int x = a + j0 + q;
            const unsigned int k = x == med ? vmed : kk[q];
            if (x < b) {
                fl |= (unsigned int)!(k < piv) << q;
                fr |= (unsigned int)!(piv < k) << q;
            }
        }
        unsigned int tot;
        const unsigned int ex = vg_block_scan<PC_CT / 64>((unsigned int)__popc(fl) | ((unsigned int)__popc(fr) << 16),
                                                          wsum, &tot);
        int rl = pre.x + (int)(ex & 0xffffu), rr = pre.y + (int)(ex >> 16);
        int g_best = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int x = a + j0 + q;
            if (x < b) g_best = max(g_best, min(rl, TR - rr));
            rl += (fl >> q) & 1;
            rr += (fr >> q) & 1;
        }
        if (a + j0 < b && a + j0 + Q >= b) g_best = max(g_best, min(rl, TR - rr));   // the end boundary b
        if (tid == 0) mx_s = 0;
        __syncthreads();
        atomicMax(&mx_s, g_best);
        __syncthreads();
        const int m = mx_s;
        if (tid == 0) {
            res[s] = PRes{piv, vmed, med, m, TR, 0x7fffffff, 0x7fffffff};
            wact += (unsigned long long)(g.l - g.f);
            wpairs += (unsigned long long)m;
        }
        __syncthreads();   // shared scalars reused by the next range
    }
    if (tid == 0 && wact) {
        atomicAdd(&pst[PW_ACTIVE], wact);
        atomicAdd(&pst[PW_PAIRS], wpairs);
    }
}

// ranks by ballots on striped rows: position a + q * PC_CT + tid is row q,
// wave w, lane t; the stoppers before it are the chunk's prefix + the
// (row, wave) pairs before (q, w) + the lanes below t
__global__ void __launch_bounds__(PC_CT) __attribute__((amdgpu_waves_per_eu(PC_LOCC))) k_pc_lrank(unsigned int* K, unsigned int* V, const PSeg* seg, const int* cseg,
                                                     const int2* ccnt, PRes* res, unsigned int* PA, unsigned int* PB,
                                                     const int* ctr, int cur) {
    constexpr int Q = PC_CH / PC_CT, NWV = PC_CT / 64;
    static_assert(Q * NWV <= 64, "one lane per (row, wave) pair");
    __shared__ unsigned int rc[Q * NWV];   // packed left | right << 16 counts per (row, wave), then their prefixes
    const int nch = ctr[PCC_NCH + cur];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int c = blockIdx.x; c < nch; c += gridDim.x) {
        const int si = cseg[c];
        const PSeg g = seg[si];
        const PRes r = res[si];
        int a, b;
        pc_chunk(g, c, a, b);
        unsigned int kk[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) kk[q] = K[min(a + q * PC_CT + (int)threadIdx.x, b - 1)];
        unsigned long long bl[Q], br[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int x = a + q * PC_CT + (int)threadIdx.x;
            const unsigned int k = x == r.med ? r.vmed : kk[q];
            bl[q] = __ballot(x < b && !(k < r.piv));
            br[q] = __ballot(x < b && !(r.piv < k));
            if (lane == 0) rc[q * NWV + w] = (unsigned int)__popcll(bl[q]) | ((unsigned int)__popcll(br[q]) << 16);
        }
        __syncthreads();
        if (w == 0) {   // exclusive scan of the (row, wave) counts in position order
            const unsigned int v = lane < Q * NWV ? rc[lane] : 0u;
            unsigned int incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            if (lane < Q * NWV) rc[lane] = incl - v;
        }
        __syncthreads();
        const int2 pre = ccnt[c];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int x = a + q * PC_CT + (int)threadIdx.x;
            const unsigned int p = rc[q * NWV + w];
            if ((bl[q] >> lane) & 1) {
                const int rl = pre.x + (int)(p & 0xffffu) + __popcll(bl[q] & lt);
                if (rl < r.m) PA[g.f + rl] = (unsigned int)x;
                else if (rl == r.m) res[si].cutA = x;          // i_{m+1}
            }
            if ((br[q] >> lane) & 1) {
                const int rr = pre.y + (int)(p >> 16) + __popcll(br[q] & lt);
                const int kr = r.TR - 1 - rr;                   // rank from the right
                if (kr < r.m) PB[g.f + kr] = (unsigned int)x;
                if (kr == r.m - 1) res[si].cutB = x;            // j_m
            }
        }
        if (c == g.c0 && threadIdx.x == 0 && r.med != g.f) {    // the median swap, made real
            const unsigned int kf = K[g.f], vf = V[g.f], km = K[r.med], vm = V[r.med];
            K[g.f] = km; V[g.f] = vm; K[r.med] = kf; V[r.med] = vf;
        }
        __syncthreads();   // rc reused by the next chunk
    }
}

// the swaps: chunk c of a range takes the pair ranks [(c - c0) PC_CH, + PC_CH)
// (m < the range's size); each thread's four pairs are loaded before any is
// written (the pairs are disjoint)
__global__ void __launch_bounds__(256) k_pc_lpairs(unsigned int* K, unsigned int* V, const PSeg* seg, const int* cseg,
                                                    const PRes* res, const unsigned int* PA, const unsigned int* PB,
                                                    const int* ctr, int cur) {
    const int nch = ctr[PCC_NCH + cur];
    for (int c = blockIdx.x; c < nch; c += gridDim.x) {
        const int si = cseg[c];
        const int f = seg[si].f, c0 = seg[si].c0;
        const int m = res[si].m;
        const int k0 = (c - c0) * PC_CH, k1 = min(m, k0 + PC_CH);
        for (int k = k0 + (int)threadIdx.x; k < k1; k += 1024) {
            unsigned int x[4], y[4], kx[4], vx[4], ky[4], vy[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int kk = f + min(k + 256 * u, k1 - 1);
                x[u] = PA[kk];
                y[u] = PB[kk];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                kx[u] = K[x[u]]; vx[u] = V[x[u]];
                ky[u] = K[y[u]]; vy[u] = V[y[u]];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (k + 256 * u < k1) {
                    K[x[u]] = ky[u]; V[x[u]] = vy[u];
                    K[y[u]] = kx[u]; V[y[u]] = vx[u];
                }
        }
    }
}

// the halves of every range, a thread per range: the block's new ranges,
// chunks and finish entries are counted by block scans and claimed with one
// atomic per counter (the device-wide counters live in memory shared by all
// XCDs: an atomic per range serialises there)
__global__ void __launch_bounds__(256) k_pc_lsplit(int tail_min, const PSeg* seg, const PRes* res, PSeg* nseg, int* ncseg,
                                                    PcLists wl, int* ctr, int cur, int last) {
    __shared__ unsigned int wsum[4];
    __shared__ int base_s[6];
    const int ns = ctr[PCC_NSEG + cur];
    for (int s0 = blockIdx.x * 256; s0 < ns; s0 += gridDim.x * 256) {
        const int s = s0 + (int)threadIdx.x;
        int lo[2] = {0, 0}, hi[2] = {0, 0}, kind[2] = {-1, -1}, nch[2] = {0, 0}, D = 0;
        if (s < ns) {
            const PSeg g = seg[s];
            const PRes r = res[s];
            const int cut = min(r.cutA, r.m > 0 ? r.cutB : 0x7fffffff);
            D = g.d - 1;
            lo[0] = g.f; hi[0] = cut; lo[1] = cut; hi[1] = g.l;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int n = hi[h] - lo[h];
                if (n <= 1) continue;
                if (n > tail_min && D > 0 && !last) {
                    kind[h] = 4;
                    nch[h] = (n - 1 + PC_CH - 1) / PC_CH;
                } else {
                    kind[h] = n <= PC_WT ? 0 : n <= PC_ST ? 1 : n <= PC_T ? 2 : 3;
                }
            }
        }
        // counts: new ranges | list 0 << 10 | list 1 << 20, list 2 | list 3 << 10, chunks
        unsigned int ca = 0, cb = 0, cc = (unsigned int)(nch[0] + nch[1]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (kind[h] == 4) ca += 1u;
            if (kind[h] == 0) ca += 1u << 10;
            if (kind[h] == 1) ca += 1u << 20;
            if (kind[h] == 2) cb += 1u;
            if (kind[h] == 3) cb += 1u << 10;
        }
        unsigned int ta, tb, tc;
        const unsigned int ea = vg_block_scan<4>(ca, wsum, &ta);
        const unsigned int eb = vg_block_scan<4>(cb, wsum, &tb);
        const unsigned int ec = vg_block_scan<4>(cc, wsum, &tc);
        if (threadIdx.x == 0) {
            const int tot[6] = {(int)(ta & 1023u), (int)((ta >> 10) & 1023u), (int)(ta >> 20), (int)(tb & 1023u),
                                (int)(tb >> 10), (int)tc};
            int* dst[6] = {&ctr[PCC_NSEG + (cur ^ 1)], &ctr[PCC_NW + 0], &ctr[PCC_NW + 1], &ctr[PCC_NW + 2],
                           &ctr[PCC_NW + 3], &ctr[PCC_NCH + (cur ^ 1)]};
#pragma unroll
            for (int q = 0; q < 6; ++q) base_s[q] = tot[q] ? atomicAdd(dst[q], tot[q]) : 0;
        }
        __syncthreads();
        int o[6] = {base_s[0] + (int)(ea & 1023u), base_s[1] + (int)((ea >> 10) & 1023u), base_s[2] + (int)(ea >> 20),
                    base_s[3] + (int)(eb & 1023u), base_s[4] + (int)(eb >> 10), base_s[5] + (int)ec};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int n = hi[h] - lo[h];
            if (kind[h] == 4) {
                const int slot = o[0]++, c0 = o[5];
                o[5] += nch[h];
                nseg[slot] = PSeg{lo[h], hi[h], D, c0};
                for (int i = 0; i < nch[h]; ++i) ncseg[c0 + i] = slot;
            } else if (kind[h] >= 0) {
                const int i = o[1 + kind[h]]++;
                wl.l[kind[h]][i] = make_int2(lo[h], n | (D << 24));
            }
        }
        __syncthreads();   // base_s reused
    }
}

// list 4 — a range over PC_T items whose depth budget is spent (std::sort's
// heapsort; the dense C5 maps send a few hundred per run here, two or three
// per sort): taken first by the low workgroups of the 4 Ki finish
// (k_pc_finish32<PC_T>, one range per workgroup, so the ranges run side by side
// and beside the finish entries instead of in a launch of their own before
// them — round 5's k_pc_fallback was 11.4 % of C5's device time on the
// mapping step's critical path); the first wave heapsorts it in global memory, the heap's
// levels 6 .. 10 cached in the finish's 16 KB item array (slo_pclsort.h wave_heap_sort_cached:
// per pop one LDS and one L2 round trip for the path below the register
// levels, instead of two L2 round trips).  (Staging whole ranges in LDS —
// 96 KB in round 4, 64 KB of 32-bit items in round 5 — held every launch of
// the kernel, nearly always empty, until a CU had that much free beside the
// other contexts' finish kernels: 3-4 ms per launch, and on a graph branch of
// its own the join stalled the context instead: C3 19.2 k -> 16.1 k scans/s.)
// A range that came here for another reason (over PT_MAXT tiles,
// a full stack; never seen) is finished by one lane with the sequential
// restatement.
__device__ __forceinline__ void pc_fallback_entry(unsigned int* K, unsigned int* V, int2 w, int* cstat, u64* scratch,
                                                  unsigned long long* pst, u64* mid) {
    const int f = w.x, n = w.y & 0xffffff, d = w.y >> 24, NT = blockDim.x;
    if (threadIdx.x == 0) atomicAdd(&pst[PW_FALL], (unsigned long long)n);
    for (int i = threadIdx.x; i < n; i += NT) scratch[f + i] = ((u64)K[f + i] << 32) | V[f + i];
    __syncthreads();
    if (d == 0 && n > 16) {
        if (threadIdx.x < 64) slo_pcl::wave_heap_sort_cached<u64>(scratch + f, n, mid);
        if (threadIdx.x == 0) atomicAdd(&cstat[0], 1);
    } else if (threadIdx.x == 0) {
        atomicAdd(&cstat[0], 1);
        __shared__ int st_lo[64], st_hi[64], st_d[64];   // any n (a range over PT_MAXT tiles)
        slo_sort::introsort_range_ws(scratch + f, n, d, slo_pcl::Less(), st_lo, st_hi, st_d);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += NT) {
        const u64 it = scratch[f + i];
        K[f + i] = (unsigned int)(it >> 32);
        V[f + i] = (unsigned int)it;
    }
    __syncthreads();
}

// ---- finish: PC_FW waves per entry (slo_pcl::block_sort; one for the
// smallest class), the entry's items staged in LDS; lane tasks take the
// ranges of <= PC_TLANE items
#ifndef PC_TLANE
#define PC_TLANE 64
#endif
#ifndef PC_FW
#define PC_FW 4           // waves per entry of the two larger size classes
#endif
#ifndef PC_PROF
#define PC_PROF 0         // 1: the finishes count their cycles per step kind (pcl_work [9..17], a diagnostic build:
                          // the clock reads wait for the wave's LDS traffic at every step)
#endif
template <int NMAX, int W>
__global__ void __launch_bounds__(64 * W) k_pc_finish(unsigned int* K, unsigned int* V, PcLists wl, int* ctr, int list,
                                                       unsigned long long* pst, int* cstat, const int32_t* off,
                                                       int S, int32_t* serr) {
    __shared__ u64 items[NMAX];
    __shared__ unsigned short tbl[NMAX / 2 + 1];
    __shared__ slo_pcl::WaveSmem ws[W];
    __shared__ slo_pcl::BlockQ<W> bq;
    __shared__ int ferr;   // the entry's inconsistent steps (slo_pclsort.h guards)
    const int nw = ctr[PCC_NW + list], tid = threadIdx.x;
    unsigned long long wn = 0, we = 0;   // work counters, one atomic per wave
    long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int e = blockIdx.x; e < nw; e += gridDim.x) {
        const int2 w = wl.l[list][e];
        const int f = w.x, n = min(w.y & 0xffffff, NMAX), d = w.y >> 24;
        if (tid == 0) ferr = 0;
        for (int i0 = 0; i0 < n; i0 += 8 * 64 * W) {   // eight loads of each array in flight
            unsigned int kk[8], vv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = min(i0 + u * 64 * W + tid, n - 1);
                kk[u] = K[f + i];
                vv[u] = V[f + i];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (i0 + u * 64 * W + tid < n) items[i0 + u * 64 * W + tid] = ((u64)kk[u] << 32) | vv[u];
        }
        __syncthreads();
        slo_pcl::block_sort<PC_TLANE, W>(items, n, d, tbl, ws, bq, &ferr, PC_PROF ? prof : nullptr);
        __syncthreads();
        if (tid == 0 && ferr) {   // never expected: counted and the stream flagged
            atomicAdd(&cstat[1], ferr);
            pc_flag(serr, off, S, f, SLO_ERR_SORT);
        }
        for (int i = tid; i < n; i += 64 * W) {
            const u64 it = items[i];
            K[f + i] = (unsigned int)(it >> 32);
            V[f + i] = (unsigned int)it;
        }
        __syncthreads();
        wn += (unsigned long long)n;
        we += 1ull;
    }
    if ((tid & 63) == 0 && we) {
        const int sl = list == 5 ? 2 : list;   // list 5: list-2 entries
        if (tid == 0) {
            atomicAdd(&pst[list == 5 ? PW_FINX : PW_FIN + list], wn);
            atomicAdd(&pst[PW_ENTRIES], we);
        }
        for (int q = 0; q < 3; ++q) atomicAdd(&pst[PW_PROF + 3 * sl + q], (unsigned long long)prof[q]);
    }
}

// ---- the same with 32-bit items: (key - min) << 12 | position in the entry
// (slo_pclsort.h kPosBits) for an entry whose keys span less than 2^20.
// Half the LDS of the 64-bit items — 25 KB per 4 Ki entry at four waves, six
// workgroups per CU instead of three — and the same comparisons, so the same
// order.  The point indices stay in global memory and follow their items at
// the write-back (gathered into the items' LDS slots, written back after a
// barrier).  A wider entry (sparse map regions: a range of 4 Ki items over
// several z slabs of a 0.4 m grid) takes the keys' ranks instead of the keys:
// a bitonic sort of its raw keys in the items' LDS, then each position's rank
// = the first sorted index of its key (a binary search), which orders the
// items exactly as their keys do, in 12 bits; the original keys then follow
// their items at the write-back like the point indices.  (Round 4 sent such
// entries to a 64-bit finish kernel, k_pc_finish — 41 KB of LDS, three
// workgroups per CU: 6.9 % of C2's and 8.3 % of C5's device time.)
#ifndef PC_F32_OCC
#define PC_F32_OCC 6      // waves per SIMD k_pc_finish32 is built for (25 KB of LDS: six 4-wave workgroups per CU;
                          // pc_finish_b 32.0 -> 31.0 ms per 6 mapping steps against five)
#endif
template <int NMAX, int W>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(W >= 4 ? PC_F32_OCC : 1))) k_pc_finish32(unsigned int* K, unsigned int* V, PcLists wl, int* ctr,
                                                         int list, unsigned long long* pst, int* cstat,
                                                         const int32_t* off, int S, int32_t* serr, u64* fall) {
    constexpr int NT = 64 * W;
    static_assert(NMAX <= (1 << slo_pcl::kPosBits), "positions fit kPosBits");
    __shared__ __attribute__((aligned(16))) unsigned int items[NMAX];
    __shared__ unsigned short tbl[NMAX / 2 + 1];
    __shared__ slo_pcl::WaveSmem ws[W];
    __shared__ slo_pcl::BlockQ<W> bq;
    __shared__ int ferr;
    __shared__ unsigned int kmn[W], kmx[W];
    const int nw = ctr[PCC_NW + list], tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    unsigned long long wn = 0, we = 0;
    long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (NMAX * sizeof(unsigned int) >= slo_pcl::kMidN * sizeof(u64)) {
        if (fall) {   // list 4 first (the spent-depth ranges: heapsort, the item array as its LDS cache)
            const int n4 = ctr[PCC_NW + 4];
            for (int e = blockIdx.x; e < n4; e += gridDim.x)
                pc_fallback_entry(K, V, wl.l[4][e], cstat, fall, pst, reinterpret_cast<u64*>(items));
        }
    }
    for (int e = blockIdx.x; e < nw; e += gridDim.x) {
        const int2 w = wl.l[list][e];
        const int f = w.x, n = min(w.y & 0xffffff, NMAX), d = w.y >> 24;
        if (tid == 0) ferr = 0;
        unsigned int mn = 0xffffffffu, mx = 0u;
        for (int i0 = 0; i0 < n; i0 += 4 * NT) {   // the raw keys into LDS, four loads in flight
            unsigned int kk[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) kk[u] = K[f + min(i0 + u * NT + tid, n - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + u * NT + tid;
                mn = min(mn, kk[u]);
                mx = max(mx, kk[u]);
                if (i < n) items[i] = kk[u];
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            mn = min(mn, (unsigned int)__shfl_xor((int)mn, o, 64));
            mx = max(mx, (unsigned int)__shfl_xor((int)mx, o, 64));
        }
        if (lane == 0) { kmn[wv] = mn; kmx[wv] = mx; }
        __syncthreads();
        for (int q = 0; q < W; ++q) { mn = min(mn, kmn[q]); mx = max(mx, kmx[q]); }
        const bool wide = mx - mn >= (1u << (32 - slo_pcl::kPosBits));   // uniform
        if (wide) {
            // ranks: the raw keys sorted (bitonic, padded to a power of two
            // with the largest key), then each position's key searched
            int np = 1;
            while (np < n) np <<= 1;
            for (int i = n + tid; i < np; i += NT) items[i] = 0xffffffffu;
            __syncthreads();
            for (int size = 2; size <= np; size <<= 1)
                for (int stride = size >> 1; stride > 0; stride >>= 1) {
                    for (int t = tid; t < np / 2; t += NT) {
                        const int lo = 2 * stride * (t / stride) + (t % stride), hi = lo + stride;
                        const unsigned int a = items[lo], b = items[hi];
                        if ((a > b) == ((lo & size) == 0)) { items[lo] = b; items[hi] = a; }
                    }
                    __syncthreads();
                }
            constexpr int RK = (NMAX + NT - 1) / NT;   // positions per thread
            unsigned int rk[RK];
#pragma unroll
            for (int u = 0; u < RK; ++u) {   // lower_bound of each position's key, all searches side by side
                const int i = u * NT + tid;
                const unsigned int key = K[f + min(i, n - 1)];
                int lo = 0;
#pragma unroll
                for (int step = NMAX >> 1; step > 0; step >>= 1)
                    if (lo + step <= np && items[lo + step - 1] < key) lo += step;
                rk[u] = (unsigned int)lo;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < RK; ++u) {
                const int i = u * NT + tid;
                if (i < n) items[i] = (rk[u] << slo_pcl::kPosBits) | (unsigned int)i;
            }
        } else {
            for (int i = tid; i < n; i += NT) items[i] = ((items[i] - mn) << slo_pcl::kPosBits) | (unsigned int)i;
        }
        __syncthreads();
        slo_pcl::block_sort<PC_TLANE, W>(items, n, d, tbl, ws, bq, &ferr, PC_PROF ? prof : nullptr);
        __syncthreads();
        if (tid == 0 && ferr) {   // never expected: counted and the stream flagged
            atomicAdd(&cstat[1], ferr);
            pc_flag(serr, off, S, f, SLO_ERR_SORT);
        }
        if (wide) {   // the keys and the point indices gathered by position (all reads before any write)
            constexpr int RK = (NMAX + NT - 1) / NT;
            unsigned int pos[RK];
#pragma unroll
            for (int u = 0; u < RK; ++u) {
                const int i = u * NT + tid;
                pos[u] = i < n ? items[i] & ((1u << slo_pcl::kPosBits) - 1u) : 0u;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < RK; ++u)
                if (u * NT + tid < n) items[u * NT + tid] = K[f + pos[u]];
            __syncthreads();
            for (int i = tid; i < n; i += NT) K[f + i] = items[i];
            __syncthreads();
#pragma unroll
            for (int u = 0; u < RK; ++u)
                if (u * NT + tid < n) items[u * NT + tid] = V[f + pos[u]];
        } else {
            // the keys out at once; each position's point index gathered into its
            // LDS slot, written out only after every gather of the entry is done
            for (int i = tid; i < n; i += NT) {
                const unsigned int it = items[i];
                K[f + i] = (it >> slo_pcl::kPosBits) + mn;
                items[i] = V[f + (it & ((1u << slo_pcl::kPosBits) - 1u))];
            }
        }
        __syncthreads();
        for (int i = tid; i < n; i += NT) V[f + i] = items[i];
        __syncthreads();
        wn += (unsigned long long)n;
        we += 1ull;
    }
    if ((tid & 63) == 0 && we) {
        if (tid == 0) {
            atomicAdd(&pst[PW_FIN + list], wn);
            atomicAdd(&pst[PW_ENTRIES], we);
        }
        for (int q = 0; q < 3; ++q) atomicAdd(&pst[PW_PROF + 3 * list + q], (unsigned long long)prof[q]);
#if PC_PROF
        // block_sort's phases (thread 0 of each workgroup): group levels, -, pool entry, pool ([22 + q])
        if (tid == 0)
            for (int q = 4; q < 8; ++q) atomicAdd(&pst[22 + q - 4], (unsigned long long)prof[q]);
#endif
    }
}

// ---- the tail: the ranges of more than PC_T items the global levels leave
// (list 3: up to PC_TAIL items, or whatever is left after the G levels), one
// workgroup per range, depth first.  A step is the global levels' step with
// the workgroup in place of the grid: a tile of PT_TILE positions is one
// wave's (PT_ROWS rows of 64), the tile counts and their prefixes sit in LDS,
// and barriers separate the passes instead of launches.  Halves of at most
// PC_T items go to the finish lists, larger ones onto the workgroup's stack;
// a range whose depth budget is spent goes to list 4 (pc_fallback_entry,
// heapsort).  Ranges over PT_MAXT tiles go to list 4 as well (one lane
// finishes them exactly; never seen: the map clouds' strides are ~1.6 M).

#define PT_ROWS 16
#define PT_TILE (64 * PT_ROWS)
#define PT_MAXT 4096
#define PT_SMAXT 256      // tiles of the small-table tail (4-wave workgroups, 256 Ki items)
#ifndef PT_OCC
#define PT_OCC 8          // waves per SIMD k_pc_tail is built for
#endif
template <int PT_NW, int MAXT>
struct TailSm {
    int tl[MAXT + 1], tr[MAXT + 1];   // per tile stopper counts, then exclusive prefixes (+ totals)
    int sf[64], sl[64], sd[64];             // the stack of ranges still over PC_T
    int f, l, d, sp, have;                  // the range in hand (have: one is)
    unsigned int piv, k0;
    int med, c, m, cutA, cutB, tA, tB;
    int wsum[PT_NW];
};

// (A small-table shape — four waves, tile tables for 64 or 256 tiles, eight
// ranges in flight per CU, the longer ranges handed to list 6 for this one —
// measured slower: 19.6 + 25.2 and 37.1 + 19.8 ms against 40.3 ms per 6
// mapping steps.  The launch is bounded by the few ranges the global levels
// leave far over PC_TAIL, each stepped depth first by one workgroup.)
template <int PT_NT, int MAXT, int LIST>
__global__ void __launch_bounds__(PT_NT) __attribute__((amdgpu_waves_per_eu(PT_OCC))) k_pc_tail(unsigned int* K, unsigned int* V, unsigned int* PB, PcLists wl,
                                                    int* ctr, unsigned long long* pst, int* cstat, const int32_t* off,
                                                    int S, int32_t* serr) {
    constexpr int PT_NW = PT_NT / 64;
    __shared__ TailSm<PT_NW, MAXT> sm;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int INF = 0x7fffffff;
    const int nw = ctr[PCC_NW + LIST];
    unsigned long long wact = 0, wpairs = 0;
    // tid 0 pops the next range into sm.f / sm.l / sm.d with its pivot (the
    // median swap taken virtually until the swaps); sm.have is read by every
    // thread after a barrier and written again only before the next one
    auto pop = [&]() {
        if (sm.sp == 0) { sm.have = 0; return; }
        const int q = --sm.sp, f = sm.sf[q], l = sm.sl[q];
        sm.f = f; sm.l = l; sm.d = sm.sd[q];
        const int mid = f + (l - f) / 2;
        const unsigned int kf = K[f], k1 = K[f + 1], k2 = K[mid], k3 = K[l - 1];
        const int w = slo_pcl::median3(k1, k2, k3);
        sm.med = w == 0 ? f + 1 : (w == 1 ? mid : l - 1);
        sm.piv = w == 0 ? k1 : (w == 1 ? k2 : k3);
        sm.k0 = kf;
        sm.c = INF;
        sm.have = 1;
    };
    for (int e = blockIdx.x; e < nw; e += gridDim.x) {
        if (tid == 0) {
            const int2 w = wl.l[LIST][e];
            sm.sf[0] = w.x; sm.sl[0] = w.x + (w.y & 0xffffff); sm.sd[0] = w.y >> 24;
            sm.sp = 1;
            pop();
        }
        __syncthreads();
        while (sm.have) {
            const int f = sm.f, l = sm.l, d = sm.d, med = sm.med;
            const unsigned int p = sm.piv, k0 = sm.k0;
            const int b0 = f + 1, nt = (l - b0 + PT_TILE - 1) / PT_TILE;
            if (d == 0 || nt > MAXT) {   // heapsort: list 4; too long for the tile table: list 6 (or 4)
                if (tid == 0) {
                    const int to = d == 0 ? 4 : (MAXT < PT_MAXT ? 6 : 4);
                    const int i = atomicAdd(&ctr[PCC_NW + to], 1);
                    wl.l[to][i] = make_int2(f, (l - f) | (d << 24));
                    pop();
                }
                __syncthreads();
                continue;
            }
            // (A) stopper counts per tile, a wave per tile
            for (int t = wv; t < nt; t += PT_NW) {
                const int a = b0 + t * PT_TILE;
                unsigned int kk[PT_ROWS];
#pragma unroll
                for (int r = 0; r < PT_ROWS; ++r) kk[r] = K[min(a + 64 * r + lane, l - 1)];
                int cl = 0, cr = 0;
#pragma unroll
                for (int r = 0; r < PT_ROWS; ++r) {
                    const int x = a + 64 * r + lane;
                    const unsigned int k = x == med ? k0 : kk[r];
                    cl += __popcll(__ballot(x < l && !(k < p)));
                    cr += __popcll(__ballot(x < l && !(p < k)));
                }
                if (lane == 0) { sm.tl[t] = cl; sm.tr[t] = cr; }
            }
            __syncthreads();
            {   // exclusive prefixes over the tiles, totals at [nt]
                const int per = (nt + PT_NT - 1) / PT_NT, t0 = min(nt, tid * per), t1 = min(nt, t0 + per);
                int sl_ = 0, sr_ = 0;
                for (int t = t0; t < t1; ++t) { sl_ += sm.tl[t]; sr_ += sm.tr[t]; }
                int totl, totr;
                int rl = vg_block_scan<PT_NW>(sl_, sm.wsum, &totl);
                int rr = vg_block_scan<PT_NW>(sr_, sm.wsum, &totr);
                for (int t = t0; t < t1; ++t) {
                    const int xl = sm.tl[t], xr = sm.tr[t];
                    sm.tl[t] = rl; sm.tr[t] = rr;
                    rl += xl; rr += xr;
                }
                if (tid == 0) { sm.tl[nt] = totl; sm.tr[nt] = totr; }
            }
            __syncthreads();
            const int TL = sm.tl[nt], TR = sm.tr[nt];
            // the crossing tile: the first whose end boundary has Lb >= Rb (the last one's always has)
            for (int t = tid; t < nt; t += PT_NT)
                if (sm.tl[t + 1] >= TR - sm.tr[t + 1]) atomicMin(&sm.c, t);
            __syncthreads();
            // a tile's rows in order, the tile's keys loaded at once: per lane the
            // exclusive prefixes; fn(x, act, iL, iR, pl, pr) -> stop
            auto rows = [&](int t, auto&& fn) {
                const int a = b0 + t * PT_TILE;
                unsigned int kk[PT_ROWS];
#pragma unroll
                for (int r = 0; r < PT_ROWS; ++r) kk[r] = K[min(a + 64 * r + lane, l - 1)];
                int runL = sm.tl[t], runR = sm.tr[t];
#pragma unroll
                for (int r = 0; r < PT_ROWS; ++r) {
                    if (a + 64 * r >= l) return;
                    const int x = a + 64 * r + lane;
                    const unsigned int k = x == med ? k0 : kk[r];
                    const bool act = x < l, iL = act && !(k < p), iR = act && !(p < k);
                    const unsigned long long bl = __ballot(iL), br = __ballot(iR);
                    const int pl = runL + slo_pcl::lane_prefix(bl), pr = runR + slo_pcl::lane_prefix(br);
                    if (fn(x, act, iL, iR, pl, pr)) return;
                    runL += __popcll(bl);
                    runR += __popcll(br);
                }
            };
            if (wv == 0) {   // m, by the first wave, from the crossing tile
                const int c = sm.c;
                int m = -1, lastPl = 0;
                rows(c, [&](int x, bool act, bool, bool, int pl, int pr) {
                    const unsigned long long fx = __ballot(act && pl >= TR - pr);
                    if (fx) {
                        const int xl = __builtin_ctzll(fx);
                        m = TR - __builtin_amdgcn_readlane(pr, xl);                          // Rb(X)
                        if (xl > 0) m = max(m, __builtin_amdgcn_readlane(pl, xl - 1));       // Lb(X - 1)
                        else if (x - lane > b0) m = max(m, lastPl);                          // X - 1 in the row before
                        return true;
                    }
                    lastPl = __builtin_amdgcn_readlane(pl, min(63, l - 1 - (x - lane)));
                    return false;
                });
                if (m < 0) m = max(TR - sm.tr[c + 1], lastPl);   // X = the tile's end boundary
                if (lane == 0) { sm.m = m; sm.cutA = INF; sm.cutB = INF; sm.tA = nt - 1; sm.tB = 0; }
            }
            __syncthreads();
            const int m = sm.m;
            if (wv == 0 && m < TL) {   // i_{m+1}: the left stopper of rank m
                int tA = nt - 1, cutA = INF;
                for (int t0 = 0; t0 < nt; t0 += 64) {
                    const int t = t0 + lane;
                    const unsigned long long b = __ballot(t < nt && sm.tl[min(t, nt - 1)] <= m && m < sm.tl[min(t, nt - 1) + 1]);
                    if (b) { tA = t0 + __builtin_ctzll(b); break; }
                }
                rows(tA, [&](int x, bool, bool iL, bool, int pl, int) {
                    const unsigned long long b = __ballot(iL && pl == m);
                    if (b) cutA = x - lane + __builtin_ctzll(b);
                    return b != 0;
                });
                if (lane == 0) { sm.cutA = cutA; sm.tA = tA; }
            }
            if (wv == 1 && m > 0) {    // j_m: the right stopper with TR - m right stoppers before it
                const int tq = TR - m;
                int tB = 0, cutB = INF;
                for (int t0 = 0; t0 < nt; t0 += 64) {
                    const int t = t0 + lane;
                    const unsigned long long b = __ballot(t < nt && sm.tr[min(t, nt - 1)] <= tq && tq < sm.tr[min(t, nt - 1) + 1]);
                    if (b) { tB = t0 + __builtin_ctzll(b); break; }
                }
                rows(tB, [&](int x, bool, bool, bool iR, int, int pr) {
                    const unsigned long long b = __ballot(iR && pr == tq);
                    if (b) cutB = x - lane + __builtin_ctzll(b);
                    return b != 0;
                });
                if (lane == 0) { sm.cutB = cutB; sm.tB = tB; }
            }
            __syncthreads();
            if (tid == 0 && med != f) {   // the median swap, made real
                const unsigned int vf = V[f], vm = V[med];
                K[f] = p; V[f] = vm;
                K[med] = k0; V[med] = vf;
            }
            __threadfence_block();
            __syncthreads();
            if (m > 0) {
                // (B) the m last right stoppers (tiles tB ..), by rank from the right
                for (int t = sm.tB + wv; t < nt; t += PT_NW) {
                    const int a = b0 + t * PT_TILE;
                    unsigned int kk[PT_ROWS];
#pragma unroll
                    for (int r = 0; r < PT_ROWS; ++r) kk[r] = K[min(a + 64 * r + lane, l - 1)];
                    int runR = sm.tr[t];
#pragma unroll
                    for (int r = 0; r < PT_ROWS; ++r) {
                        const int x = a + 64 * r + lane;
                        const bool iR = x < l && !(p < kk[r]);
                        const unsigned long long br = __ballot(iR);
                        const int kr = TR - 1 - (runR + slo_pcl::lane_prefix(br));
                        if (iR && kr < m) PB[f + kr] = (unsigned int)x;
                        runR += __popcll(br);
                    }
                }
                __threadfence_block();
                __syncthreads();
                // (C) the m first left stoppers (tiles .. tA) swap with their partners:
                // every swapped left stopper lies before the crossing and every
                // partner at or after it, so no wave reads what another writes
                const int tEnd = m < TL ? sm.tA : nt - 1;
                for (int t = wv; t <= tEnd; t += PT_NW) {
                    const int a = b0 + t * PT_TILE;
                    int runL = sm.tl[t];
                    for (int r0 = 0; r0 < PT_ROWS && a + 64 * r0 < l; r0 += 4) {
                        unsigned int kx[4], vx[4], ky[4], vy[4];
                        int y[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int x = min(a + 64 * (r0 + u) + lane, l - 1);
                            kx[u] = K[x];
                            vx[u] = V[x];
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int x = a + 64 * (r0 + u) + lane;
                            const bool iL = x < l && !(kx[u] < p);
                            const unsigned long long bl = __ballot(iL);
                            const int pl = runL + slo_pcl::lane_prefix(bl);
                            y[u] = (iL && pl < m) ? pl : -1;
                            runL += __popcll(bl);
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            y[u] = y[u] >= 0 ? (int)PB[f + y[u]] : -1;
                            if (y[u] >= l || (y[u] >= 0 && y[u] <= f)) {   // cannot happen: counted, not followed
                                atomicAdd(&cstat[3], 1);
                                pc_flag(serr, off, S, f, SLO_ERR_SORT);
                                y[u] = -1;
                            }
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int yy = y[u] >= 0 ? y[u] : f;
                            ky[u] = K[yy];
                            vy[u] = V[yy];
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (y[u] >= 0) {
                                const int x = a + 64 * (r0 + u) + lane;
                                K[x] = ky[u]; V[x] = vy[u];
                                K[y[u]] = kx[u]; V[y[u]] = vx[u];
                            }
                    }
                }
                __threadfence_block();
            }
            __syncthreads();   // every swap is done before tid 0 reads the next range's pivot
            if (tid == 0) {   // the halves
                int cut = min(sm.cutA, m > 0 ? sm.cutB : INF);
                if (cut <= f || cut >= l) {   // cannot happen: counted, the stream flagged; the range is left as it is
                    atomicAdd(&cstat[2], 1);
                    pc_flag(serr, off, S, f, SLO_ERR_SORT);
                    cut = l;
                }
                wact += (unsigned long long)(l - f);
                wpairs += (unsigned long long)m;
                const int lo[2] = {f, cut}, hi[2] = {cut, l};
                for (int h = 0; h < 2; ++h) {
                    const int n = hi[h] - lo[h];
                    if (n <= 1) continue;
                    if (n <= PC_T) {
                        pc_push(wl, ctr, lo[h], n, d - 1);
                    } else if (sm.sp < 64) {   // the stack holds at most one range per depth level (+ 1)
                        sm.sf[sm.sp] = lo[h]; sm.sl[sm.sp] = hi[h]; sm.sd[sm.sp] = d - 1; ++sm.sp;
                    } else {                   // cannot happen; one lane finishes it exactly
                        const int i = atomicAdd(&ctr[PCC_NW + 4], 1);
                        wl.l[4][i] = make_int2(lo[h], n | ((d - 1) << 24));
                    }
                }
                pop();
            }
            __syncthreads();
        }
        __syncthreads();   // every thread has read sm.have == 0 before the next entry is pushed
    }
    if (tid == 0 && wact) {
        atomicAdd(&pst[PW_TAIL], wact);
        atomicAdd(&pst[PW_TAIL_PAIRS], wpairs);
    }
}

// ---- workspace and driver
static int pcl_ws(slo_ctx* ctx, int SV, size_t items, size_t maxT) {
    PclWs& w = ctx->pws;
    const size_t S = (size_t)VG_MAXG * ctx->S;   // per virtual stream (vg_run_groups)
    if (!w.ctr) {
        SLO_CHECK(hipMalloc(&w.ctr, 16 * sizeof(int)));
        SLO_CHECK(hipMemset(w.ctr, 0, 16 * sizeof(int)));
        SLO_CHECK(hipMalloc(&w.nfin, S * sizeof(int32_t)));
        SLO_CHECK(hipMalloc(&w.cstat, 16 * sizeof(int)));
        SLO_CHECK(hipMemset(w.cstat, 0, 16 * sizeof(int)));
        SLO_CHECK(hipMalloc(&w.pstat, 32 * sizeof(unsigned long long)));
        SLO_CHECK(hipMemset(w.pstat, 0, 32 * sizeof(unsigned long long)));
        SLO_CHECK(hipMalloc(&w.serr, S * sizeof(int32_t)));
        SLO_CHECK(hipMemset(w.serr, 0, S * sizeof(int32_t)));
    }
    if (items > w.items) {
        const size_t it = std::max(items, w.items + w.items / 2);
        void* old[] = {w.seg[0], w.seg[1], w.res, w.cseg[0], w.cseg[1], w.ccnt, w.wl};
        for (void* q : old) if (q) hipFree(q);
        w.items = it;
        const size_t segcap = S + it / PC_T + 2;   // S >= the call's virtual streams
        const size_t chcap = it / PC_CH + segcap;
        const size_t wcap0 = it / 2 + S + 2, wcapk = it / PC_WT + S + 2;   // disjoint entries of >= 2 / > PC_WT items
        ++ctx->ws_gen;
        SLO_CHECK(hipMalloc(&w.seg[0], sizeof(PSeg) * segcap));
        SLO_CHECK(hipMalloc(&w.seg[1], sizeof(PSeg) * segcap));
        SLO_CHECK(hipMalloc(&w.res, sizeof(PRes) * segcap));
        SLO_CHECK(hipMalloc(&w.cseg[0], sizeof(int) * chcap));
        SLO_CHECK(hipMalloc(&w.cseg[1], sizeof(int) * chcap));
        SLO_CHECK(hipMalloc(&w.ccnt, sizeof(int2) * chcap));
        SLO_CHECK(hipMalloc(&w.wl, sizeof(int2) * (wcap0 + 6 * wcapk)));
        w.wcap0 = wcap0;
        w.wcapk = wcapk;
    }
    if ((size_t)SV * maxT > w.tiles) {
        if (w.tcnt) hipFree(w.tcnt);
        w.tiles = std::max((size_t)SV * maxT, w.tiles + w.tiles / 2);
        ++ctx->ws_gen;
        SLO_CHECK(hipMalloc(&w.tcnt, sizeof(int) * w.tiles));
    }
    return 0;
}

int pcl_presize(slo_ctx* ctx, int SV, size_t items, size_t maxT) { return pcl_ws(ctx, SV, items, maxT); }

// global levels for ranges of up to `stride` items: enough that what is left
// is mostly at most PC_TAIL items (median-of-three quicksort's depth runs to
// ~1.5 log2(n / PC_TAIL) on the configs' clouds); whatever is larger after the
// G levels is stepped by k_pc_tail like the rest, only with one workgroup.  An
// empty level still costs its five launches.
static int pcl_levels(size_t stride, int tail_min, bool few) {
    int g = 0;
    size_t x = (size_t)tail_min;
    while (x < stride) { x <<= 1; ++g; }
    return g ? g + (few ? PC_XLEV_FEW : PC_XLEV) : 0;   // (a few streams: each level is five launches of latency)
}

int vg_pcl_sort(slo_ctx* ctx, const VgSrc& src, size_t in_stride, size_t items, const VgParams* prm,
                const int32_t* off, unsigned int* K, unsigned int* V, unsigned int* spare) {
    const int S = src.nv();   // virtual streams: (filter, stream) pairs
    if (items > (size_t)INT32_MAX) {   // item positions are 32-bit
        ctx->err = "PCL-order VoxelGrid: n_streams * in_stride exceeds INT32_MAX items";
        return SLO_E_CAPACITY;
    }
    const int maxT = std::max(1, (int)((in_stride + VG_TILE - 1) / VG_TILE));
    if (int r = pcl_ws(ctx, S, items, (size_t)maxT)) return r;
    PclWs& w = ctx->pws;
    const int GX = std::max(1, std::min(maxT, std::max(4, 2048 / S)));
    PcLists L;
    L.l[0] = w.wl;
    for (int k = 1; k < 7; ++k) L.l[k] = w.wl + w.wcap0 + (size_t)(k - 1) * w.wcapk;
    // the pair positions of a step: the left stoppers' (PA) and their partners
    // (PB), in the VoxelGrid workspace's spare halves (2 * items words)
    unsigned int* PA = spare;
    unsigned int* PB = spare + items;
    SLO_LAUNCH(ctx, "pc_count", k_pc_count, dim3(GX, S), dim3(VG_T), 0, src, off, prm, w.tcnt, maxT, S,
               w.ctr);
    // a few streams leave most of the chip idle: smaller tail ranges (more
    // global levels, each parallel within a range) and more waves per finish
    // entry cut the latency of the one range a workgroup works through
    const bool few = S <= PC_FEW;
    const int tail_min = few ? PC_TAIL_FEW : PC_TAIL;
    SLO_LAUNCH(ctx, "pc_scan", k_pc_scan, dim3(S), dim3(1024), 0, tail_min, off, prm, w.tcnt, maxT, w.seg[0], w.cseg[0], L,
               w.ctr, w.nfin, w.pstat, w.serr);
    SLO_LAUNCH(ctx, "pc_write", k_pc_write, dim3(GX, S), dim3(VG_T), 0, src, off, prm, w.tcnt, w.nfin,
               maxT, K, V, S);
    const int G = pcl_levels(in_stride, tail_min, few);
    for (int lv = 0; lv < G; ++lv) {
        const int cur = lv & 1;
        // the grid-stride kernels take whatever the level holds; past the first
        // levels most items have left for the finish lists: smaller grids
        const int G0 = few ? PC_G_FEW : PC_G;
        const int GG = lv < 8 ? G0 : G0 / 4, GS = G0 / 4;
        SLO_LAUNCH(ctx, "pc_lcount", k_pc_lcount, dim3(GG), dim3(PC_CT), 0, K, w.seg[cur], w.cseg[cur], w.ccnt,
                   w.ctr, cur);
        SLO_LAUNCH(ctx, "pc_lscan", k_pc_lscan, dim3(GS), dim3(PC_CT), 0, K, w.seg[cur], w.ccnt, w.res, w.ctr, cur,
                   w.pstat);
        SLO_LAUNCH(ctx, "pc_lrank", k_pc_lrank, dim3(GG), dim3(PC_CT), 0, K, V, w.seg[cur], w.cseg[cur], w.ccnt,
                   w.res, PA, PB, w.ctr, cur);
        SLO_LAUNCH(ctx, "pc_lpairs", k_pc_lpairs, dim3(GG), dim3(256), 0, K, V, w.seg[cur], w.cseg[cur], w.res, PA, PB,
                   w.ctr, cur);
        SLO_LAUNCH(ctx, "pc_lsplit", k_pc_lsplit, dim3(std::max(1, GS / 4)), dim3(256), 0, tail_min, w.seg[cur], w.res, w.seg[cur ^ 1],
                   w.cseg[cur ^ 1], L, w.ctr, cur, (int)(lv == G - 1));
    }
    // a workgroup per entry, grid-stride: enough to fill the chip at the LDS
    // each size class takes (43 / 23 / 5.6 KB per entry)
    const int FG = std::max(256, std::min(8192, S * 16));
    SLO_LAUNCH(ctx, "pc_tail", (k_pc_tail<512, PT_MAXT, 3>), dim3(std::max(64, std::min(4096, S * 8))), dim3(512), 0,
               K, V, PB, L, w.ctr, w.pstat, w.cstat, off, S, w.serr);
    // 32-bit items (lists 2 and 1; entries whose keys span 2^20 or more take their keys' ranks)
    if (few) {
        SLO_LAUNCH(ctx, "pc_finish_b", (k_pc_finish32<PC_T, 16>), dim3(FG), dim3(64 * 16), 0, K, V, L, w.ctr, 2, w.pstat,
                   w.cstat, off, S, w.serr, (u64*)spare);
        SLO_LAUNCH(ctx, "pc_finish_s", (k_pc_finish32<PC_ST, 8>), dim3(FG), dim3(64 * 8), 0, K, V, L, w.ctr, 1, w.pstat,
                   w.cstat, off, S, w.serr, (u64*)nullptr);
    } else {
        SLO_LAUNCH(ctx, "pc_finish_b", (k_pc_finish32<PC_T, PC_FW>), dim3(FG), dim3(64 * PC_FW), 0, K, V, L, w.ctr, 2,
                   w.pstat, w.cstat, off, S, w.serr, (u64*)spare);
        SLO_LAUNCH(ctx, "pc_finish_s", (k_pc_finish32<PC_ST, PC_FW>), dim3(FG), dim3(64 * PC_FW), 0, K, V, L, w.ctr, 1,
                   w.pstat, w.cstat, off, S, w.serr, (u64*)nullptr);
    }
    SLO_LAUNCH(ctx, "pc_finish_w", (k_pc_finish<PC_WT, 1>), dim3(FG), dim3(64), 0, K, V, L, w.ctr, 0, w.pstat, w.cstat, off, S, w.serr);
    SLO_CHECK(hipGetLastError());
    return 0;
}

// the sort's per-stream flags into StreamState::err (records, bench and
// slo_get see them; slo_get also reads PclWs::serr itself)
__global__ void k_pc_fold_err(StreamState* st, const int32_t* e0, const int32_t* e1, int S) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    int32_t e = 0;
    for (int g = 0; g < VG_MAXG; ++g)   // every filter's virtual stream of stream s
        e |= (e0 ? e0[g * S + s] : 0) | (e1 ? e1[g * S + s] : 0);
    if (e) st[s].err |= e;
}
int pcl_fold_err(slo_ctx* ctx) {
    if (!ctx->pws.serr && !ctx->pws2.serr) return 0;
    SLO_LAUNCH(ctx, "pc_fold_err", k_pc_fold_err, dim3((ctx->S + 255) / 256), dim3(256), 0, ctx->v.st, ctx->pws.serr,
               ctx->pws2.serr, ctx->S);
    SLO_CHECK(hipGetLastError());
    return 0;
}

void pcl_free(slo_ctx* ctx) {
    PclWs& w = ctx->pws;
    void* ps[] = {w.serr, w.ctr, w.nfin, w.cstat, w.pstat, w.seg[0], w.seg[1], w.res, w.cseg[0], w.cseg[1], w.ccnt, w.wl,
                  w.tcnt};
    for (void* p : ps) if (p) hipFree(p);
    w = PclWs();
}

}  // namespace slo
