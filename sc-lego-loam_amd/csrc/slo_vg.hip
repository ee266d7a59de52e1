// slo_vg.hip — batched PCL VoxelGrid and the 1 m hash grid used for the
// mapping 5-NN.
//
// VoxelGrid (PCL 1.8 VoxelGrid<PointXYZI>::applyFilter + CentroidPoint, the
// filter the reference calls at featureAssociation.cpp:779 and
// mapOptmization.cpp:1224-1262): per stream the bounds give min_b and the
// x-fastest linear voxel index; each stream's (idx, point) pairs are sorted
// by a hand-written segmented LSD radix sort (as many passes of <= VG_DMAX
// bits as the stream's key width needs, at most four; stable, so the points
// of a voxel stay in input order; no stream bits in the key), every voxel's
// centroid is summed in that order and written at its rank -> output sorted by voxel index exactly like PCL.  Non-finite
// points are skipped (the raw cloud is not dense, MO:1236); the int32
// overflow guard returns the input unchanged, as PCL does.  All sizes come
// from the input strides and device-side counts: no host round trip.
//
// Hash grid: power-of-two cells, counting sort of the points into hashed
// buckets [S][T + 1] (the last bucket of each stream stays empty, so a run of
// consecutive buckets ends at off[h + 1]); queried by grid_ball
// (slo_internal.h).
#include "slo_vgcommon.h"
#include <float.h>
#include <string>

namespace slo {

// stream offsets of the concatenated input (block scan), bounds init, and the
// meta words [total, max cell count, long-voxel count]
// A count above the stream's input stride (a caller's io->npts: nothing else
// bounds it) is clamped to the stride — the workspace is sized from the
// strides — and flagged (errflag bit 4, slo_get "vg_stats").  S here and in
// every VoxelGrid kernel counts virtual streams (VgSrc).
__global__ void __launch_bounds__(1024) k_vg_prefix(VgSrc src, int S, int32_t* off, unsigned int* bounds,
                                                    int32_t* meta, int32_t* osw, int tile, int32_t* errflag) {
    __shared__ int wsum[16];
    __shared__ int carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int b0 = 0; b0 < S; b0 += 1024) {
        const int s = b0 + tid;
        const int x0 = s < S ? src.count(s) : 0;
        const int x = s < S ? max(0, min(x0, (int)min(src.grp(s).stride, (size_t)0x7fffffff))) : 0;
        if (x != x0) atomicOr(errflag, 4);
        int incl = x;   // inclusive wave scan
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        int before = carry;
        for (int k = 0; k < w; ++k) before += wsum[k];
        if (s < S) off[s] = before + incl - x;
        __syncthreads();
        if (tid == 1023) carry = before + incl;
        __syncthreads();
    }
    if (tid == 0) { off[S] = carry; meta[0] = carry; meta[1] = 0; meta[2] = 0; meta[3] += 1; }
    for (int s = tid; s < S; s += 1024)
        for (int k = 0; k < 3; ++k) { bounds[6 * s + k] = 0xffffffffu; bounds[6 * s + 3 + k] = 0u; }
    if (osw) {   // single-pass scatter: tickets reset, stream s's tiles dealt to XCD s & 7 in stream order
        __syncthreads();   // off[] of this block visible
        if (tid < 32) osw[tid] = 0;
        if (tid < 8) {
            int run = 0;
            for (int s = tid; s < S; s += 8) {
                osw[40 + s] = run;
                run += (off[s + 1] - off[s] + tile - 1) / tile;
            }
            osw[32 + tid] = run;
        }
    }
}

__global__ void __launch_bounds__(256) k_vg_bounds(VgSrc src, const int32_t* off, unsigned int* bounds) {
    const int s = blockIdx.y;
    const int n = off[s + 1] - off[s];
    unsigned int mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
    const float4* pts = src.row(s);
    const int step = gridDim.x * blockDim.x;
    for (int i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += 8 * step) {   // eight loads in flight
        float4 pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pp[u] = pts[min(i0 + u * step, n - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float4 p = pp[u];
            if (i0 + u * step >= n || !(isfinite(p.x) & isfinite(p.y) & isfinite(p.z))) continue;
            const unsigned int q[3] = {f2ord(p.x), f2ord(p.y), f2ord(p.z)};
            for (int k = 0; k < 3; ++k) { mn[k] = min(mn[k], q[k]); mx[k] = max(mx[k], q[k]); }
        }
    }
    for (int o = 32; o > 0; o >>= 1)
        for (int k = 0; k < 3; ++k) {
            mn[k] = min(mn[k], (unsigned int)__shfl_xor((int)mn[k], o, 64));
            mx[k] = max(mx[k], (unsigned int)__shfl_xor((int)mx[k], o, 64));
        }
    __shared__ unsigned int red[16][6];   // up to 16 waves
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 3; ++k) { red[w][k] = mn[k]; red[w][3 + k] = mx[k]; }
    __syncthreads();
    if (threadIdx.x < 6) {   // one atomic per component per workgroup
        const int k = threadIdx.x;
        unsigned int r = red[0][k];
        for (int ww = 1; ww < (int)(blockDim.x >> 6); ++ww) r = k < 3 ? min(r, red[ww][k]) : max(r, red[ww][k]);
        if (k < 3) { if (r != 0xffffffffu) atomicMin(&bounds[6 * s + k], r); }
        else if (r != 0u) atomicMax(&bounds[6 * s + k], r);
    }
}

// Tile kernels run on a (GX, S8) grid, S8 = S rounded up to 8.  With VG_XCD
// the linear workgroup id is split XCD-aware (xcd_stream_chunk): all GX
// workgroups of a stream land on one XCD, so a stream's tiles share that
// XCD's L2 (its scatter runs, its sorted keys, the points its voxels gather).
#ifndef VG_XCD
#define VG_XCD 1
#endif
__device__ inline bool vg_block(int S, int& s, int& chunk) {
#if VG_XCD
    xcd_stream_chunk(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x, s, chunk);
#else
    s = blockIdx.y; chunk = blockIdx.x;
#endif
    return s < S;
}
static inline dim3 vg_tile_grid(int GX, int S) { return dim3(GX, (S + 7) / 8 * 8); }

__global__ void k_vg_params(VgSrc src, const unsigned int* bounds, const int32_t* off, int S, VgParams* prm) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    VgParams p;
    p.inv = 1.0f / src.grp(s).leaf;   // Array4f::Ones() / leaf_size_
    p.overflow = 0;
    const int n = off[s + 1] - off[s];
    p.ntiles = (n + VG_TILE - 1) / VG_TILE;
    if (n == 0 || bounds[6 * s] == 0xffffffffu) {   // empty, or no finite point: every key is "none"
        p.minb[0] = p.minb[1] = p.minb[2] = 0; p.mul1 = p.mul2 = 0;
        p.vbits = 1; p.dbits = 1; p.npass = 1;
        prm[s] = p;
        return;
    }
    float mn[3], mx[3];
    for (int k = 0; k < 3; ++k) { mn[k] = ord2f(bounds[6 * s + k]); mx[k] = ord2f(bounds[6 * s + 3 + k]); }
    long long dx = (long long)((mx[0] - mn[0]) * p.inv) + 1, dy = (long long)((mx[1] - mn[1]) * p.inv) + 1,
              dz = (long long)((mx[2] - mn[2]) * p.inv) + 1;
    if (dx * dy * dz > 2147483647LL) p.overflow = 1;
    for (int k = 0; k < 3; ++k) p.minb[k] = (int)floorf(mn[k] * p.inv);
    int maxbx = (int)floorf(mx[0] * p.inv), maxby = (int)floorf(mx[1] * p.inv), maxbz = (int)floorf(mx[2] * p.inv);
    int divx = maxbx - p.minb[0] + 1, divy = maxby - p.minb[1] + 1, divz = maxbz - p.minb[2] + 1;
    p.mul1 = divx;
    p.mul2 = divx * divy;
    // indices are < divx*divy*divz (or < n: the overflow keys are positions)
    const long long cells = p.overflow ? (long long)n : (long long)divx * divy * divz;
    int vb = 1;
    while (vb < 32 && (1LL << vb) <= cells) ++vb;
    if (cells >= (1LL << 30)) vb = 32;   // int index arithmetic may wrap, as in PCL
    p.vbits = vb;
    p.npass = (vb + VG_DMAX - 1) / VG_DMAX;
    p.dbits = (vb + p.npass - 1) / p.npass;
    prm[s] = p;
}

// ---- LSD radix passes.  The items of stream s occupy [off[s], off[s+1]) of
// the workspace; tile t of the stream is items [t*VG_TILE, (t+1)*VG_TILE),
// read as 4 wave slices of 1024 (item j = w*1024 + k*64 + lane).  Per pass:
// k_vg_hist counts each tile's digits, k_vg_scan turns the counts of a
// stream into global scatter bases (digit-major, tile-minor: the positions a
// stable sort gives), k_vg_scatter ranks each tile's items by digit (wave
// ballots: the lanes holding the same digit, then per-wave running counts in
// LDS; stable), reorders the tile through LDS and writes each digit's run at
// its base.  Pass 0 computes the keys from the points (vals = the point's
// index in its stream).  A stream runs npass passes and skips the rest; its
// passes alternate between the buffer pairs A and B so that the last one
// always writes B (vg_out_b).

// the pair pass `pass` of a stream writes: the last pass writes B
__device__ inline bool vg_out_b(const VgParams& p, int pass) { return ((p.npass - 1 - pass) & 1) == 0; }

// lanes of this wave whose digit equals mine (among `act` lanes), dbits <= VG_DMAX
__device__ inline unsigned long long vg_peers(unsigned int d, int dbits, unsigned long long act) {
    unsigned long long pe = act;
    for (int b = 0; b < dbits; ++b) {
        const bool x = (d >> b) & 1u;
        const unsigned long long bb = __ballot(x);
        pe &= x ? bb : ~bb;
    }
    return pe;
}

// A tile's items of one pass: item k of this thread is j = j0 + 64 k (its wave
// slice).  Every load is issued before the first use: pass 0 loads the points
// VG_LB at a time (their keys need the whole point) and keeps only the keys;
// later passes load all keys at once (their values: vg_tile_vals).
#define VG_LB 8
template <bool FIRST>
__device__ inline void vg_tile_load(const float4* row, const VgParams& p, int base, int a, int m, int j0,
                                    const unsigned int* kin, const unsigned int* vin, unsigned int (&key)[VG_IPT],
                                    unsigned int (&val)[VG_IPT]) {
    if (FIRST) {
        const float4* src = row + a;
#pragma unroll
        for (int h = 0; h < VG_IPT; h += VG_LB) {
            float4 q[VG_LB];
#pragma unroll
            for (int u = 0; u < VG_LB; ++u) {
                const int j = j0 + (h + u) * 64;
                q[u] = j < m ? src[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < VG_LB; ++u) {
                const int j = j0 + (h + u) * 64;
                key[h + u] = j < m ? vg_key(q[u], p, a + j) : 0u;
                val[h + u] = (unsigned int)(a + j);
            }
        }
    } else if (m == VG_TILE) {   // a full tile: straight-line loads at immediate offsets
        const unsigned int* src = kin + base + a + j0;
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) key[k] = src[k * 64];
    } else {
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            const int j = j0 + k * 64;
            key[k] = j < m ? kin[base + a + j] : 0u;
        }
    }
}
// the values of a later pass, loaded once the keys are ranked (fewer live registers while ranking)
__device__ inline void vg_tile_vals(int base, int a, int m, int j0, const unsigned int* vin,
                                    unsigned int (&val)[VG_IPT]) {
    if (m == VG_TILE) {
        const unsigned int* src = vin + base + a + j0;
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) val[k] = src[k * 64];
        return;
    }
#pragma unroll
    for (int k = 0; k < VG_IPT; ++k) {
        const int j = j0 + k * 64;
        val[k] = j < m ? vin[base + a + j] : 0u;
    }
}

template <bool FIRST>
__global__ void __launch_bounds__(VG_T) k_vg_hist(VgSrc src, const int32_t* off, const VgParams* prm, int pass,
                                                  const unsigned int* ka, const unsigned int* kb, int* cnt, int maxT,
                                                  int S) {
    __shared__ int h[VG_NB];
    int s, chunk;
    if (!vg_block(S, s, chunk)) return;
    const float4* in = FIRST ? src.row(s) : nullptr;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const VgParams p = prm[s];
    if (pass >= p.npass) return;
    const unsigned int* kin = vg_out_b(p, pass - 1) ? kb : ka;
    const int base = off[s], n = off[s + 1] - base, shift = pass * p.dbits, nb = 1 << p.dbits;
    const unsigned int mask = (unsigned int)nb - 1u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int t = chunk; t < p.ntiles; t += gridDim.x) {
        for (int d = tid; d < nb; d += VG_T) h[d] = 0;
        __syncthreads();
        const int a = t * VG_TILE, m = min(VG_TILE, n - a);
        unsigned int key[VG_IPT], val[VG_IPT];
        vg_tile_load<FIRST>(in, p, base, a, m, w * (VG_TILE / VG_W) + lane, kin, nullptr, key, val);
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            const int j = w * (VG_TILE / VG_W) + k * 64 + lane;
            const bool ok = j < m;
            const unsigned int d = (key[k] >> shift) & mask;
            const unsigned long long pe = vg_peers(d, p.dbits, __ballot(ok));
            if (ok && (pe & lt) == 0) atomicAdd(&h[d], __popcll(pe));   // one add per digit per wave slice
        }
        __syncthreads();
        for (int d = tid; d < nb; d += VG_T) cnt[((size_t)s * VG_NB + d) * maxT + t] = h[d];
        __syncthreads();
    }
}

__global__ void __launch_bounds__(1024) k_vg_scan(const int32_t* off, const VgParams* prm, int pass, int* cnt,
                                                   int maxT) {
    __shared__ int wsum[16];
    const int s = blockIdx.x, tid = threadIdx.x;
    const VgParams p = prm[s];
    if (pass >= p.npass) return;
    const int nt = p.ntiles, F = (1 << p.dbits) * nt;
    if (F == 0) return;
    int* c = cnt + (size_t)s * VG_NB * maxT;
    // chunks of 4 096 (digit, tile) counts, 4 consecutive per thread: a wave
    // reads 256 consecutive counts of a digit row (coalesced), the block scan
    // carries the running base from chunk to chunk
    int run = off[s];
    for (int f0 = 0; f0 < F; f0 += 4096) {
        int x[4], sum = 0;
        size_t idx[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int f = f0 + tid * 4 + k;
            idx[k] = (size_t)(f / nt) * maxT + f % nt;
            x[k] = f < F ? c[idx[k]] : 0;
            sum += x[k];
        }
        int total;
        int ex = run + vg_block_scan<16>(sum, wsum, &total);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (f0 + tid * 4 + k < F) { c[idx[k]] = ex; ex += x[k]; }
        run += total;
    }
}

template <bool FIRST>
__global__ void __launch_bounds__(VG_T) __attribute__((amdgpu_waves_per_eu(VG_SCATTER_OCC))) k_vg_scatter(VgSrc src, const int32_t* off,
                                                     const VgParams* prm, int pass, unsigned int* ka,
                                                     unsigned int* va, unsigned int* kb, unsigned int* vb,
                                                     const int* cnt, int maxT, int S) {
    __shared__ unsigned int lk[VG_TILE], lv[VG_TILE];
    __shared__ int wc[VG_W][VG_NB];   // per wave slice: running digit counts, then the slice's digit offsets
    __shared__ int lb[VG_NB];         // global base of each digit minus its first position in the tile
    __shared__ int wsum[VG_W];
    int s, chunk;
    if (!vg_block(S, s, chunk)) return;
    const float4* in = FIRST ? src.row(s) : nullptr;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const VgParams p = prm[s];
    if (pass >= p.npass) return;
    const bool ob = vg_out_b(p, pass);
    const unsigned int* kin = ob ? ka : kb;
    const unsigned int* vin = ob ? va : vb;
    unsigned int* kout = ob ? kb : ka;
    unsigned int* vout = ob ? vb : va;
    const int base = off[s], n = off[s + 1] - base, shift = pass * p.dbits, nb = 1 << p.dbits;
    const unsigned int mask = (unsigned int)nb - 1u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int t = chunk; t < p.ntiles; t += gridDim.x) {
        const int a = t * VG_TILE, m = min(VG_TILE, n - a);
        for (int d = tid; d < VG_W * VG_NB; d += VG_T) (&wc[0][0])[d] = 0;
        __syncthreads();
        unsigned int key[VG_IPT], val[VG_IPT];
        int rk[VG_IPT];
        vg_tile_load<FIRST>(in, p, base, a, m, w * (VG_TILE / VG_W) + lane, kin, vin, key, val);
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            const int j = w * (VG_TILE / VG_W) + k * 64 + lane;
            const bool ok = j < m;
            const unsigned int d = (key[k] >> shift) & mask;
            const unsigned long long pe = vg_peers(d, p.dbits, __ballot(ok));
            int before = 0;
            if (ok) before = wc[w][d];   // all lanes read before the leader writes (in-order LDS of one wave)
            rk[k] = before + __popcll(pe & lt);
            if (ok && (pe & lt) == 0) wc[w][d] = before + __popcll(pe);
        }
        if (!FIRST) vg_tile_vals(base, a, m, w * (VG_TILE / VG_W) + lane, vin, val);   // in flight over the scan
        __syncthreads();
        // digit-major, slice-minor exclusive scan of the counts: the tile-local
        // position of each (digit, slice) run
        {
            constexpr int DPT = VG_NB >= VG_T ? VG_NB / VG_T : 1;   // consecutive digits per thread
            const int d0 = tid * DPT;
            int c[DPT][VG_W], tot = 0;
#pragma unroll
            for (int e = 0; e < DPT; ++e)
#pragma unroll
                for (int q = 0; q < VG_W; ++q) { c[e][q] = d0 + e < nb ? wc[q][d0 + e] : 0; tot += c[e][q]; }
            int total;
            int run = vg_block_scan<VG_W>(tot, wsum, &total);
#pragma unroll
            for (int e = 0; e < DPT; ++e) {
                const int d = d0 + e;
                if (d < nb) {
                    const int start = run;
#pragma unroll
                    for (int q = 0; q < VG_W; ++q) { wc[q][d] = run; run += c[e][q]; }
                    if (run != start) lb[d] = cnt[((size_t)s * VG_NB + d) * maxT + t] - start;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            const int j = w * (VG_TILE / VG_W) + k * 64 + lane;
            if (j < m) {
                const int pos = wc[w][(key[k] >> shift) & mask] + rk[k];
                lk[pos] = key[k];
                lv[pos] = val[k];
            }
        }
        __syncthreads();
#pragma unroll 4
        for (int k = 0; k < VG_IPT; ++k) {   // each digit's run is contiguous: coalesced writes
            const int j = k * VG_T + tid;
            if (j < m) {
                const unsigned int key2 = lk[j];
                const int o = lb[(key2 >> shift) & mask] + j;
                kout[o] = key2;
                vout[o] = lv[j];
            }
        }
        __syncthreads();   // LDS reused by the next tile
    }
}

// ---- Single-pass scatter (env SLO_VG_ONESWEEP=1 at context creation; Merrill & Garland's decoupled
// look-back as in "Onesweep"): the digit counts of every pass are taken in
// one read of the points (k_vg_ghist: the per-stream histograms do not depend
// on the order the items are in), k_vg_gscan turns them into each digit's
// first output position, and each pass is then one kernel: a workgroup takes
// the next tile of its XCD's streams by ticket, ranks the tile's items, posts
// its digit counts, adds up its predecessors' posts walking back until one
// carries an inclusive prefix, posts its own inclusive prefix and scatters.
// Tickets are taken in order, so every tile a workgroup waits on is held by a
// running workgroup: no deadlock.  Posts are 64-bit words (tag, inclusive
// flag, count); the tag names the sort call (an epoch k_vg_prefix counts in
// meta[3]) and the pass, so no clearing pass is needed.
#define VG_OSW_G 1024   // persistent single-pass workgroups (128 per XCD)
static_assert(VG_NB <= VG_T, "one look-back thread per digit");

template <bool FIRST>
__global__ void __launch_bounds__(VG_T) k_vg_ghist(VgSrc src, const int32_t* off, const VgParams* prm, int32_t* gh,
                                                   int S) {
    __shared__ int h[VG_PASSES][VG_NB];
    int s, chunk;
    if (!vg_block(S, s, chunk)) return;
    const float4* in = src.row(s);
    const int tid = threadIdx.x;
    const VgParams p = prm[s];
    const int base = off[s], n = off[s + 1] - base, nb = 1 << p.dbits;
    const unsigned int mask = (unsigned int)nb - 1u;
    for (int d = tid; d < VG_PASSES * VG_NB; d += VG_T) (&h[0][0])[d] = 0;
    __syncthreads();
    for (int t = chunk; t < p.ntiles; t += gridDim.x) {
        const int a = t * VG_TILE, m = min(VG_TILE, n - a);
        unsigned int key[VG_IPT];
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            const int j = k * VG_T + tid;
            key[k] = j < m ? vg_key(in[a + j], p, a + j) : 0u;
        }
        const unsigned long long lt = (1ull << (tid & 63)) - 1ull;
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            const bool ok = k * VG_T + tid < m;
            const unsigned long long act = __ballot(ok);
            for (int q = 0; q < p.npass; ++q) {   // one LDS add per digit per wave (neighbouring points share digits)
                const unsigned int d = (key[k] >> (q * p.dbits)) & mask;
                const unsigned long long pe = vg_peers(d, p.dbits, act);
                if (ok && (pe & lt) == 0) atomicAdd(&h[q][d], __popcll(pe));
            }
        }
    }
    __syncthreads();
    for (int q = 0; q < p.npass; ++q)
        for (int d = tid; d < nb; d += VG_T)
            if (h[q][d]) atomicAdd(&gh[((size_t)s * VG_PASSES + q) * VG_NB + d], h[q][d]);
}

__global__ void __launch_bounds__(VG_T) k_vg_gscan(const int32_t* off, const VgParams* prm, int32_t* gh,
                                                   int32_t* gbase) {
    __shared__ int wsum[VG_W];
    const int s = blockIdx.x, tid = threadIdx.x;
    const VgParams p = prm[s];
    for (int q = 0; q < p.npass; ++q) {
        const size_t i = ((size_t)s * VG_PASSES + q) * VG_NB + tid;
        const int x = tid < VG_NB ? gh[i] : 0;
        int total;
        const int ex = vg_block_scan<VG_W>(x, wsum, &total);
        if (tid < VG_NB) { gbase[i] = off[s] + ex; gh[i] = 0; }
    }
}

__device__ inline unsigned long long vg_post(unsigned int tag, bool incl, int c) {
    return ((unsigned long long)tag << 32) | (incl ? 0x80000000ull : 0ull) | (unsigned int)c;
}

template <bool FIRST>
__global__ void __launch_bounds__(VG_T) __attribute__((amdgpu_waves_per_eu(VG_SCATTER_OCC))) k_vg_onesweep(
        VgSrc src, const int32_t* off, const VgParams* prm, int pass, unsigned int* ka,
        unsigned int* va, unsigned int* kb, unsigned int* vb, const int32_t* gbase, int32_t* osw,
        unsigned long long* lbk, const int32_t* meta, int maxT, int S, int32_t* errflag) {
    __shared__ unsigned int lk[VG_TILE], lv[VG_TILE];
    __shared__ int wc[VG_W][VG_NB];
    __shared__ int lb[VG_NB];
    __shared__ int wsum[VG_W];
    __shared__ int tk_s;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int x = blockIdx.x & 7;                 // the XCD this workgroup runs on (round-robin dispatch)
    const int ntx = osw[32 + x], J = (S - x + 7) >> 3;
    const unsigned int tag = ((unsigned int)meta[3] << 2 | (unsigned int)pass) + 1u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (;;) {
        if (tid == 0) tk_s = atomicAdd(&osw[pass * 8 + x], 1);
        __syncthreads();
        const int tk = tk_s;
        if (tk >= ntx) break;
        int lo = 0, hi = J - 1;                   // the last stream of this XCD whose tiles start at or before tk
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (osw[40 + x + 8 * mid] <= tk) lo = mid; else hi = mid - 1;
        }
        const int s = x + 8 * lo, t = tk - osw[40 + s];
        const float4* in = FIRST ? src.row(s) : nullptr;
        const VgParams p = prm[s];
        if (pass >= p.npass) { __syncthreads(); continue; }
        const bool ob = vg_out_b(p, pass);
        const unsigned int* kin = ob ? ka : kb;
        const unsigned int* vin = ob ? va : vb;
        unsigned int* kout = ob ? kb : ka;
        unsigned int* vout = ob ? vb : va;
        const int base = off[s], n = off[s + 1] - base, shift = pass * p.dbits, nb = 1 << p.dbits;
        const unsigned int mask = (unsigned int)nb - 1u;
        const int a = t * VG_TILE, m = min(VG_TILE, n - a);
        for (int d = tid; d < VG_W * VG_NB; d += VG_T) (&wc[0][0])[d] = 0;
        __syncthreads();
        unsigned int key[VG_IPT], val[VG_IPT];
        int rk[VG_IPT];
        vg_tile_load<FIRST>(in, p, base, a, m, w * (VG_TILE / VG_W) + lane, kin, vin, key, val);
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            const int j = w * (VG_TILE / VG_W) + k * 64 + lane;
            const bool ok = j < m;
            const unsigned int d = (key[k] >> shift) & mask;
            const unsigned long long pe = vg_peers(d, p.dbits, __ballot(ok));
            int before = 0;
            if (ok) before = wc[w][d];
            rk[k] = before + __popcll(pe & lt);
            if (ok && (pe & lt) == 0) wc[w][d] = before + __popcll(pe);
        }
        if (!FIRST) vg_tile_vals(base, a, m, w * (VG_TILE / VG_W) + lane, vin, val);   // in flight over the scan
        __syncthreads();
        {
            const int d = tid;   // one digit per thread (VG_NB <= VG_T)
            int c[VG_W], tot = 0;
#pragma unroll
            for (int q = 0; q < VG_W; ++q) { c[q] = d < nb ? wc[q][d] : 0; tot += c[q]; }
            int total;
            int run = vg_block_scan<VG_W>(tot, wsum, &total);
            const int start = run;
            if (d < nb) {
#pragma unroll
                for (int q = 0; q < VG_W; ++q) { wc[q][d] = run; run += c[q]; }
                // post this tile's count, then walk back over the stream's earlier tiles
                unsigned long long* L = lbk + ((size_t)s * maxT) * VG_NB + d;
                int excl = 0;
                if (t > 0) {
                    __hip_atomic_store(L + (size_t)t * VG_NB, vg_post(tag, false, tot), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    int tt = t - 1;
                    long spins = 0;
                    for (;;) {
                        const unsigned long long v =
                            __hip_atomic_load(L + (size_t)tt * VG_NB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((unsigned int)(v >> 32) != tag) {
                            if (++spins > (1l << 22)) { atomicOr(errflag, 2); break; }   // never: a bound, not a hang
                            __builtin_amdgcn_s_sleep(1);
                            continue;
                        }
                        excl += (int)(v & 0x7fffffffull);
                        if (v & 0x80000000ull) break;
                        if (--tt < 0) break;
                    }
                }
                __hip_atomic_store(L + (size_t)t * VG_NB, vg_post(tag, true, excl + tot), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                lb[d] = gbase[((size_t)s * VG_PASSES + pass) * VG_NB + d] + excl - start;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < VG_IPT; ++k) {
            const int j = w * (VG_TILE / VG_W) + k * 64 + lane;
            if (j < m) {
                const int pos = wc[w][(key[k] >> shift) & mask] + rk[k];
                lk[pos] = key[k];
                lv[pos] = val[k];
            }
        }
        __syncthreads();
#pragma unroll 4
        for (int k = 0; k < VG_IPT; ++k) {
            const int j = k * VG_T + tid;
            if (j < m) {
                const unsigned int key2 = lk[j];
                const int o = lb[(key2 >> shift) & mask] + j;
                kout[o] = key2;
                vout[o] = lv[j];
            }
        }
        __syncthreads();   // LDS and tk_s reused by the next tile
    }
}

// ---- voxels of the sorted items: a voxel starts at each key change (the
// "none" key of non-finite points is no voxel).  k_vg_heads counts the starts
// per tile, k_vg_hscan ranks the tiles (and sets the output counts), then
// k_vg_reduce (default) sums each voxel's points at its rank (= its output
// position: the voxels are in index order).  SLO_VG_FUSED=0 builds the
// two-kernel form instead: k_vg_ranges writes each voxel's item range
// [starts[r], ends[r]) at its rank and k_vg_centroid sums it.
__device__ inline bool vg_head(const unsigned int* k, int j, unsigned int none) {
    const unsigned int x = k[j];
    return x != none && (j == 0 || k[j - 1] != x);
}

__global__ void __launch_bounds__(VG_T) k_vg_heads(const unsigned int* keys, const int32_t* off, const VgParams* prm,
                                                   int* hcnt, int maxT, int S) {
    __shared__ int wsum[VG_W];
    int s, chunk;
    if (!vg_block(S, s, chunk)) return;
    const int tid = threadIdx.x;
    const VgParams p = prm[s];
    const int base = off[s], n = off[s + 1] - base;
    const unsigned int none = vg_none(p);
    const unsigned int* k = keys + base;
    for (int t = chunk; t < p.ntiles; t += gridDim.x) {
        const int a = t * VG_TILE, m = min(VG_TILE, n - a);
        unsigned int cur[VG_IPT], prv[VG_IPT];   // every load in flight before the first compare
#pragma unroll
        for (int q = 0; q < VG_IPT; ++q) {
            const int j = q * VG_T + tid, i = a + j;
            cur[q] = j < m ? k[i] : none;
            prv[q] = (j < m && i > 0) ? k[i - 1] : ~cur[q];
        }
        int c = 0;
#pragma unroll
        for (int q = 0; q < VG_IPT; ++q) c += cur[q] != none && prv[q] != cur[q];
        int total;
        vg_block_scan<VG_W>(c, wsum, &total);
        if (tid == 0) hcnt[(size_t)s * maxT + t] = total;
    }
}

// 256 threads: a 1024-thread block needs 16 free wave slots on one CU, which
// the other contexts' LDS-heavy sort blocks rarely leave (1.1 ms per launch
// in the live window against 8 us isolated, round-5 C3 profile)
__global__ void __launch_bounds__(256) k_vg_hscan(VgSrc src, const VgParams* prm, int* hcnt, int maxT, int32_t* nvox,
                                                  int32_t* errflag) {
    __shared__ int wsum[4];
    const int s = blockIdx.x, tid = threadIdx.x;
    const int nt = prm[s].ntiles;
    int* h = hcnt + (size_t)s * maxT;
    const int L = (nt + 255) / 256, t0 = min(nt, tid * L), t1 = min(nt, t0 + L);
    int sum = 0;
    for (int t = t0; t < t1; ++t) sum += h[t];
    int total;
    int run = vg_block_scan<4>(sum, wsum, &total);
    for (int t = t0; t < t1; ++t) {
        const int x = h[t];
        h[t] = run;
        run += x;
    }
    if (tid == 0) {
        const VgGroup& q = src.grp(s);
        nvox[s] = total;
        int c = total;
        if (c > q.out_cap) { c = q.out_cap; atomicOr(errflag, 1); }
        q.nout[(size_t)(s % src.S) * q.nout_stride] = c;
    }
}

// the item range of every voxel, at the voxel's rank (items in wave slices,
// as the scatter reads them; ranks by ballot prefix counts)
__global__ void __launch_bounds__(VG_T) k_vg_ranges(const unsigned int* keys, const int32_t* off, const VgParams* prm,
                                                    const int* hcnt, int maxT, int* starts, int* ends) {
    __shared__ int wsum[VG_W];
    const int s = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const VgParams p = prm[s];
    const int base = off[s], n = off[s + 1] - base;
    const unsigned int none = vg_none(p);
    const unsigned int* k = keys + base;
    const unsigned long long le = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
    for (int t = blockIdx.x; t < p.ntiles; t += gridDim.x) {
        const int a = t * VG_TILE, m = min(VG_TILE, n - a);
        unsigned long long hm[VG_IPT];
        int wrun = 0;
#pragma unroll
        for (int q = 0; q < VG_IPT; ++q) {
            const int j = w * (VG_TILE / VG_W) + q * 64 + lane;
            hm[q] = __ballot(j < m && vg_head(k, a + j, none));
            wrun += __popcll(hm[q]);
        }
        if (lane == 0) wsum[w] = wrun;
        __syncthreads();
        int r = hcnt[(size_t)s * maxT + t];
        for (int q = 0; q < w; ++q) r += wsum[q];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < VG_IPT; ++q) {
            const int j = w * (VG_TILE / VG_W) + q * 64 + lane, i = a + j;
            const int incl = r + __popcll(hm[q] & le);   // voxels started at or before item i
            r += __popcll(hm[q]);
            if (j < m) {
                const unsigned int x = k[i];
                if (x == none) continue;
                if ((hm[q] >> lane) & 1ull) starts[base + incl - 1] = i;
                if (i + 1 == n || k[i + 1] != x) ends[base + incl - 1] = i + 1;
            }
        }
    }
}

// Centroid of one voxel: the points are summed in input order (the sort is
// stable), one float chain per component as PCL's CentroidPoint.  Voxels of
// up to VG_SHORT points: one thread each, loads issued 4 at a time ahead of
// the chain.  Longer ones are listed for k_vg_long.
#define VG_SHORT 32

__device__ inline void vg_store(const VgOut& o, int r, float sx, float sy, float sz, float si, int cnt) {
    const float c = (float)cnt;
    if (r < o.cap) o.out[r] = make_float4(sx / c, sy / c, sz / c, si / c);
}

__global__ void __launch_bounds__(VG_T) k_vg_centroid(VgSrc srcv, const unsigned int* vals, const int32_t* off,
                                                      const int32_t* nvox, const int* starts, const int* ends,
                                                      int32_t* meta, int4* longv, int nlong_cap) {
    const int s = blockIdx.y;
    const VgOut o = srcv.out_row(s);
    const int base = off[s], nv = min(nvox[s], o.cap);
    const unsigned int* v = vals + base;
    const float4* src = srcv.row(s);
    for (int r = blockIdx.x * VG_T + threadIdx.x; r < nv; r += gridDim.x * VG_T) {
        const int j = starts[base + r], e = ends[base + r];
        if (e - j > VG_SHORT) {
            const int li = atomicAdd(&meta[2], 1);
            if (li < nlong_cap) longv[li] = make_int4(s, j, r, e);
            continue;
        }
        float sx = 0, sy = 0, sz = 0, si = 0;
        for (int i = j; i < e; i += 4) {
            float4 q4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) q4[u] = i + u < e ? src[v[i + u]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u < e) { sx += q4[u].x; sy += q4[u].y; sz += q4[u].z; si += q4[u].w; }
        }
        vg_store(o, r, sx, sy, sz, si, e - j);
    }
}

// Long voxels, one wave each (persistent grid over the list).  The wave
// gathers 256 points at a time into LDS — the next chunk's index and point
// loads are issued before the current chunk is summed (two LDS buffers per
// wave), so the gathers' latency hides behind the chains — and lanes 0..3 run
// the x, y, z and intensity chains over the chunk in order, eight LDS values
// loaded ahead of each eight dependent adds.  (A wave's LDS operations run in
// program order, so one buffer per wave serves both chunks.)  The sum is
// PCL's in-order float chain (CentroidPoint), exactly.
#define VG_LONG_G 1024   // workgroups of k_vg_long (4 waves each, 16 KB of LDS)
__global__ void __launch_bounds__(256) k_vg_long(VgSrc srcv, const unsigned int* vals, const int32_t* off,
                                                 const int32_t* meta, const int4* longv, int nlong_cap,
                                                 unsigned long long* work) {
    __shared__ float4 buf[4][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nlong = min(meta[2], nlong_cap);
    unsigned long long witems = 0, wvox = 0;   // this wave's work, added to DevView::wctr once at the end
    for (int t = blockIdx.x * 4 + w; t < nlong; t += gridDim.x * 4) {
        const int4 L = longv[t];
        const int s = L.x, a = L.y, r = L.z, e = L.w;
        const unsigned int* v = vals + off[s];
        const float4* src = srcv.row(s);
        float acc = 0.0f;
        // a chunk of 256 items from c0: its indices, then its points, all loads in flight
        auto gather = [&](int c0, float4& p0, float4& p1, float4& p2, float4& p3) {
            const int mg = min(256, e - c0);
            const unsigned int i0 = v[c0 + min(lane, mg - 1)], i1 = v[c0 + min(64 + lane, mg - 1)],
                               i2 = v[c0 + min(128 + lane, mg - 1)], i3 = v[c0 + min(192 + lane, mg - 1)];
            p0 = src[i0]; p1 = src[i1]; p2 = src[i2]; p3 = src[i3];
        };
        float4 p0, p1, p2, p3;
        gather(a, p0, p1, p2, p3);
        float4* b = buf[w];
        for (int c0 = a; c0 < e; c0 += 256) {
            const int m = min(256, e - c0);
            if (lane < m) b[lane] = p0;
            if (64 + lane < m) b[64 + lane] = p1;
            if (128 + lane < m) b[128 + lane] = p2;
            if (192 + lane < m) b[192 + lane] = p3;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // this wave's LDS traffic drained
            __builtin_amdgcn_wave_barrier();
            if (c0 + 256 < e) gather(c0 + 256, p0, p1, p2, p3);   // the next chunk's loads, in flight during the chains
            if (lane < 4) {
                const float* f = reinterpret_cast<const float*>(b) + lane;
                int q = 0;
                for (; q + 8 <= m; q += 8) {
                    const float x0 = f[4 * q], x1 = f[4 * q + 4], x2 = f[4 * q + 8], x3 = f[4 * q + 12],
                                x4 = f[4 * q + 16], x5 = f[4 * q + 20], x6 = f[4 * q + 24], x7 = f[4 * q + 28];
                    acc += x0; acc += x1; acc += x2; acc += x3; acc += x4; acc += x5; acc += x6; acc += x7;
                }
                for (; q < m; ++q) acc += f[4 * q];
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
        }
        const float sx = __shfl(acc, 0, 64), sy = __shfl(acc, 1, 64), sz = __shfl(acc, 2, 64),
                    si = __shfl(acc, 3, 64);
        if (lane == 0) vg_store(srcv.out_row(s), r, sx, sy, sz, si, e - a);
        witems += (unsigned long long)(e - a);
        ++wvox;
    }
    if (lane == 0 && wvox) {   // DevView::wctr [1] long-voxel items, [2] voxels (one atomic per wave: a
        atomicAdd(&work[1], witems);   // device-scope atomic per voxel on one address serialises)
        atomicAdd(&work[2], wvox);
    }
}

// The ranges and the centroids in one pass (SLO_VG_FUSED): each wave takes its
// slice of a tile (1024 consecutive sorted items at VG_T = 256), lists the
// slice's key changes in LDS (voxel heads in order, then possibly the start of
// the "none" items), and its lanes then take the heads in turn: head h's
// voxel is [list[h], list[h + 1]), the last one running past the slice to the
// next key change (found by a wave-wide ballot walk).  Its rank is the
// tile's rank base plus the heads before it; the sum is the same in-order
// float chain as k_vg_centroid, voxels over VG_SHORT points go to k_vg_long.
#ifndef SLO_VG_FUSED
#define SLO_VG_FUSED 1
#endif
#ifndef SLO_VG_LV
#define SLO_VG_LV 1   // the slice's point indices staged in LDS for the gathers (32.8 KB, four waves per SIMD; without
                      // them eight, measured slower: 13.8 against 12.6 ms per 6 mapping steps; r05, live
                      // in the mix: 20.50 k / 20.19 k against 20.19 k / 20.18 k scans/s, not taken)
#endif
__global__ void __launch_bounds__(VG_T) k_vg_reduce(VgSrc srcv, const unsigned int* keys, const unsigned int* vals,
                                                    const int32_t* off, const VgParams* prm, const int* hcnt, int maxT,
                                                    int32_t* meta, int4* longv, int nlong_cap, int S) {
    constexpr int SL = VG_TILE / VG_W;   // items per wave slice
    __shared__ int lst[VG_W][SL + 1];
#if SLO_VG_LV
    __shared__ unsigned int lvv[VG_W][SL];   // the slice's point indices (the gathers read them from LDS)
#endif
    __shared__ int wsum[VG_W];
    int s, chunk;
    if (!vg_block(S, s, chunk)) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const VgParams p = prm[s];
    const int base = off[s], n = off[s + 1] - base;
    const unsigned int none = vg_none(p);
    const unsigned int* k = keys + base;
    const unsigned int* v = vals + base;
    const float4* src = srcv.row(s);
    const VgOut o = srcv.out_row(s);
    const unsigned long long lt = (1ull << lane) - 1ull;
    int* L = lst[w];
    for (int t = chunk; t < p.ntiles; t += gridDim.x) {
        const int a = t * VG_TILE, m = min(VG_TILE, n - a);
        const int j0 = w * SL, i0 = a + j0;                 // this wave's slice: items [i0, i0 + ms)
        const int ms = max(0, min(SL, m - j0));
        int nh = 0, nc = 0, lasth = 0;                      // heads / key changes listed so far, the last head
        // the slice's keys, all loads in flight at once; each item's predecessor
        // comes from the lane below (lane 0: the previous row's lane 63, or the
        // item before the slice)
        unsigned int kk[SL / 64];
#if SLO_VG_LV
        unsigned int* LV = lvv[w];
#endif
        if (ms == SL) {
#pragma unroll
            for (int q = 0; q < SL / 64; ++q) kk[q] = k[i0 + q * 64 + lane];
#if SLO_VG_LV
#pragma unroll
            for (int q = 0; q < SL / 64; ++q) LV[q * 64 + lane] = v[i0 + q * 64 + lane];
#endif
        } else {
#pragma unroll
            for (int q = 0; q < SL / 64; ++q) kk[q] = q * 64 + lane < ms ? k[i0 + q * 64 + lane] : 0u;
#if SLO_VG_LV
#pragma unroll
            for (int q = 0; q < SL / 64; ++q)
                if (q * 64 + lane < ms) LV[q * 64 + lane] = v[i0 + q * 64 + lane];
#endif
        }
        unsigned int before = (ms > 0 && i0 > 0) ? k[i0 - 1] : 0u;
#pragma unroll
        for (int q = 0; q < SL / 64; ++q) {
            const int j = q * 64 + lane, i = i0 + j;
            const unsigned int x = kk[q];
            const unsigned int up = __shfl_up(x, 1, 64);
            const unsigned int pv = lane == 0 ? before : up;
            before = __shfl(x, 63, 64);
            bool chg = false, head = false;
            if (j < ms) {
                chg = i == 0 || pv != x;
                head = chg && x != none;
            }
            const unsigned long long cm = __ballot(chg);
            if (chg) L[nc + __popcll(cm & lt)] = i;
            const unsigned long long hb = __ballot(head);
            if (hb) lasth = i0 + q * 64 + 63 - __clzll((long long)hb);
            nh += __popcll(hb);
            nc += __popcll(cm);
        }
        // the end of the slice's last run: the next key change at or after the slice end
        int eend = i0 + ms;
        if (nh > 0 && nh == nc) {   // the last change listed is a head (not the "none" start)
            const unsigned int x = k[lasth];
            for (;;) {
                const int i = eend + lane;
                const bool stop = i >= n || k[i] != x;
                const unsigned long long sb = __ballot(stop);
                if (sb) { eend += __ffsll((long long)sb) - 1; break; }
                eend += 64;
            }
        }
        if (lane == 0) wsum[w] = nh;
        __syncthreads();
        int r0 = hcnt[(size_t)s * maxT + t];
        for (int q = 0; q < w; ++q) r0 += wsum[q];
        for (int h = lane; h < nh; h += 64) {
            const int r = r0 + h;
            if (r >= o.cap) break;
            const int j = L[h], e = h + 1 < nc ? L[h + 1] : eend;
            if (e - j > VG_SHORT) {
                const int li = atomicAdd(&meta[2], 1);
                if (li < nlong_cap) longv[li] = make_int4(s, j, r, e);
                continue;
            }
            float sx = 0, sy = 0, sz = 0, si = 0;
            for (int i = j; i < e; i += 4) {
                float4 q4[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {   // indices inside the slice from LDS, past its end from HBM
                    const int ii = i + u;
#if SLO_VG_LV
                    q4[u] = ii < e ? src[ii - i0 < ms ? LV[ii - i0] : v[ii]] : make_float4(0.f, 0.f, 0.f, 0.f);
#else
                    q4[u] = ii < e ? src[v[ii]] : make_float4(0.f, 0.f, 0.f, 0.f);
#endif
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (i + u < e) { sx += q4[u].x; sy += q4[u].y; sz += q4[u].z; si += q4[u].w; }
            }
            vg_store(o, r, sx, sy, sz, si, e - j);
        }
        __syncthreads();   // wsum and the lists are reused by the next tile
    }
}

// workspace for `items` items (the sum over the call's filters of S * stride)
// in tiles of at most maxT per virtual stream: allocated on the host from the
// strides alone (never from a device count), grown geometrically
static int ensure_ws(slo_ctx* ctx, size_t items, size_t tiles) {
    MapWs& w = ctx->mws;
    if (items > w.items) {
        const size_t it = std::max(items, w.items + w.items / 2);
        void* old[] = {w.keys, w.keys2, w.vals, w.longv};   // (vals2 lives in keys2's allocation)
        for (void* q : old) if (q) hipFree(q);
        w.items = it;
        w.nlong_cap = it / VG_SHORT + 1;
        ++ctx->ws_gen;
        SLO_CHECK(hipMalloc(&w.keys, 4 * it));
        // keys2 | vals2 as one allocation: the PCL-order sort uses it as its
        // pair positions and, whole, as the heapsort fallback's 8-byte scratch
        SLO_CHECK(hipMalloc(&w.keys2, 8 * it));
        w.vals2 = w.keys2 + it;
        SLO_CHECK(hipMalloc(&w.vals, 4 * it));
        SLO_CHECK(hipMalloc(&w.longv, sizeof(int4) * w.nlong_cap));
    }
    if (tiles > w.tiles) {
        const size_t tt = std::max(tiles, w.tiles + w.tiles / 2);
        if (w.cnt) hipFree(w.cnt);
        if (w.hcnt) hipFree(w.hcnt);
        if (w.lbk) hipFree(w.lbk);
        w.tiles = tt;
        ++ctx->ws_gen;
        SLO_CHECK(hipMalloc(&w.cnt, sizeof(int) * VG_NB * tt));
        SLO_CHECK(hipMalloc(&w.hcnt, sizeof(int) * tt));
        // look-back posts: zero is no sort call's tag (tags start at 1)
        SLO_CHECK(hipMalloc(&w.lbk, sizeof(unsigned long long) * VG_NB * tt));
        SLO_CHECK(hipMemsetAsync(w.lbk, 0, sizeof(unsigned long long) * VG_NB * tt, ctx->stream));
    }
    return 0;
}

// the host-side shape of a call: virtual streams, the largest stride, the
// workspace bound and the tiles per virtual stream
struct VgShape {
    int SV;
    size_t max_stride, items;
    int maxT;
};
static VgShape vg_shape(const VgSrc& src) {
    VgShape h{src.nv(), 1, 0, 1};
    for (int g = 0; g < src.G; ++g) {
        h.max_stride = std::max(h.max_stride, src.g[g].stride);
        h.items += (size_t)src.S * src.g[g].stride;
    }
    h.maxT = std::max(1, (int)((h.max_stride + VG_TILE - 1) / VG_TILE));
    return h;
}

// The segmented sort of the call's virtual streams' (key, point index)
// items: virtual stream v = g * S + s holds filter g's stream s, keyed by its
// PCL voxel index at the filter's leaf.  On return *keys / *vals hold the
// sorted items of virtual stream v at [off[v], off[v + 1]) of the workspace,
// *spare_k / *spare_v the free ping-pong halves.
static int vg_sort(slo_ctx* ctx, const char* tag, const VgSrc& src, const VgShape& h, unsigned int** keys,
                   unsigned int** vals, unsigned int** spare_k, unsigned int** spare_v) {
    MapWs& w = ctx->mws;
    const int S = h.SV;
    if (S > VG_MAXG * ctx->S) { ctx->err = "VoxelGrid: too many filters in one call"; return SLO_E_ARG; }
    if (int r = ensure_ws(ctx, h.items, (size_t)S * h.maxT)) return r;
    const int maxT = h.maxT;
    const int GX = std::max(1, std::min(maxT, std::max(4, 2048 / S)));
    const int bx = std::max(1, std::min(64, (int)((h.max_stride + 255) / 256)));
    const dim3 grid = vg_tile_grid(GX, S);
    SLO_LAUNCH(ctx, "vg_prefix", k_vg_prefix, dim3(1), dim3(1024), 0, src, S, w.off, w.bounds, w.meta,
               ctx->vg_onesweep ? w.osw : nullptr, VG_TILE, w.errflag);
    SLO_LAUNCH(ctx, "vg_bounds", k_vg_bounds, dim3(bx, S), dim3(256), 0, src, w.off, w.bounds);
    SLO_LAUNCH(ctx, "vg_params", k_vg_params, dim3((S + 63) / 64), dim3(64), 0, src, w.bounds, w.off, S, w.prm);
    hipEvent_t ev = nullptr;
    const std::string sort_name = std::string("vg_sort:") + tag;   // per filter in the timing table
    const bool tm = ctx->timing && timing_on(ctx, sort_name.c_str());
    if (tm) timing_begin(ctx, sort_name.c_str(), &ev);
    if (ctx->cfg.voxel_order == SLO_VOXEL_PCL) {   // the reference's order (slo_vgpcl.hip)
        if (int r = vg_pcl_sort(ctx, src, h.max_stride, h.items, w.prm, w.off, w.keys, w.vals, w.keys2)) return r;
        if (tm) timing_end(ctx, sort_name.c_str(), ev);
        *keys = w.keys; *vals = w.vals; *spare_k = w.keys2; *spare_v = w.vals2;
        return 0;
    }
    // pair A = keys2/vals2, pair B = keys/vals (every stream's last pass writes B)
    unsigned int *ka = w.keys2, *va = w.vals2, *kb = w.keys, *vb = w.vals;
    if (ctx->vg_onesweep) {
        SLO_LAUNCH(ctx, "vg_ghist", k_vg_ghist<true>, grid, dim3(VG_T), 0, src, w.off, w.prm, w.gh, S);
        SLO_LAUNCH(ctx, "vg_gscan", k_vg_gscan, dim3(S), dim3(VG_T), 0, w.off, w.prm, w.gh, w.gbase);
        for (int pass = 0; pass < VG_PASSES; ++pass) {
            if (pass == 0) {
                SLO_LAUNCH(ctx, "vg_onesweep", k_vg_onesweep<true>, dim3(VG_OSW_G), dim3(VG_T), 0, src, w.off, w.prm,
                           pass, ka, va, kb, vb, w.gbase, w.osw, w.lbk, w.meta, maxT, S, w.errflag);
            } else {
                SLO_LAUNCH(ctx, "vg_onesweep", k_vg_onesweep<false>, dim3(VG_OSW_G), dim3(VG_T), 0, src, w.off, w.prm,
                           pass, ka, va, kb, vb, w.gbase, w.osw, w.lbk, w.meta, maxT, S, w.errflag);
            }
        }
        if (tm) timing_end(ctx, sort_name.c_str(), ev);
        *keys = kb; *vals = vb; *spare_k = ka; *spare_v = va;
        return 0;
    }
    for (int pass = 0; pass < VG_PASSES; ++pass) {
        if (pass == 0) {
            SLO_LAUNCH(ctx, "vg_hist", k_vg_hist<true>, grid, dim3(VG_T), 0, src, w.off, w.prm, pass, ka, kb, w.cnt,
                       maxT, S);
        } else {
            SLO_LAUNCH(ctx, "vg_hist", k_vg_hist<false>, grid, dim3(VG_T), 0, src, w.off, w.prm, pass, ka, kb, w.cnt,
                       maxT, S);
        }
        SLO_LAUNCH(ctx, "vg_scan", k_vg_scan, dim3(S), dim3(1024), 0, w.off, w.prm, pass, w.cnt, maxT);
        if (pass == 0) {
            SLO_LAUNCH(ctx, "vg_scatter", k_vg_scatter<true>, grid, dim3(VG_T), 0, src, w.off, w.prm, pass, ka, va, kb,
                       vb, w.cnt, maxT, S);
        } else {
            SLO_LAUNCH(ctx, "vg_scatter", k_vg_scatter<false>, grid, dim3(VG_T), 0, src, w.off, w.prm, pass, ka, va,
                       kb, vb, w.cnt, maxT, S);
        }
    }
    if (tm) timing_end(ctx, sort_name.c_str(), ev);
    *keys = kb; *vals = vb; *spare_k = ka; *spare_v = va;
    return 0;
}

// G batched VoxelGrid filters (VgGroup, at most VG_MAXG) over the context's S
// streams in one launch sequence.  Everything is sized from the strides, so
// the host only issues launches (no round trip).
int vg_run_groups(slo_ctx* ctx, const char* tag, const VgGroup* groups, int G) {
    if (G < 1 || G > VG_MAXG) { ctx->err = "vg_run_groups: 1..VG_MAXG filters"; return SLO_E_ARG; }
    MapWs& w = ctx->mws;
    VgSrc src;
    src.io = ctx->v.io;
    src.S = ctx->S;
    src.G = G;
    for (int g = 0; g < VG_MAXG; ++g) src.g[g] = groups[std::min(g, G - 1)];
    const VgShape h = vg_shape(src);
    const int S = h.SV;
    unsigned int *k0, *v0, *k1, *v1;
    if (int r = vg_sort(ctx, tag, src, h, &k0, &v0, &k1, &v1)) return r;
    const int maxT = h.maxT;
    const int GX = std::max(1, std::min(maxT, std::max(4, 2048 / S)));
    const dim3 grid = vg_tile_grid(GX, S);
    int out_cap = 0;
    for (int g = 0; g < G; ++g) out_cap = std::max(out_cap, groups[g].out_cap);
    // the ping-pong buffers the sort is done with hold the voxel ranges
    int* starts = (int*)k1;
    int* ends = (int*)v1;
    SLO_LAUNCH(ctx, "vg_heads", k_vg_heads, grid, dim3(VG_T), 0, k0, w.off, w.prm, w.hcnt, maxT, S);
    SLO_LAUNCH(ctx, "vg_hscan", k_vg_hscan, dim3(S), dim3(256), 0, src, w.prm, w.hcnt, maxT, w.nvox, w.errflag);
    if (SLO_VG_FUSED) {
        SLO_LAUNCH(ctx, "vg_reduce", k_vg_reduce, grid, dim3(VG_T), 0, src, k0, v0, w.off, w.prm, w.hcnt, maxT, w.meta,
                   w.longv, (int)w.nlong_cap, S);
    } else {
        SLO_LAUNCH(ctx, "vg_ranges", k_vg_ranges, dim3(GX, S), dim3(VG_T), 0, k0, w.off, w.prm, w.hcnt, maxT, starts, ends);
        SLO_LAUNCH(ctx, "vg_centroid", k_vg_centroid,
                   dim3(std::max(1, std::min(64, (int)((out_cap + VG_T - 1) / VG_T))), S), dim3(VG_T), 0, src, v0,
                   w.off, w.nvox, starts, ends, w.meta, w.longv, (int)w.nlong_cap);
    }
    SLO_LAUNCH(ctx, "vg_long", k_vg_long, dim3(VG_LONG_G), dim3(256), 0, src, v0, w.off, w.meta, w.longv, (int)w.nlong_cap,
               ctx->v.wctr);
    SLO_CHECK(hipGetLastError());
    return 0;
}

// The workspaces a vg_run_groups call over these groups needs, allocated now
// (sizes from the strides alone; map_ws_presize at context creation)
int vg_presize(slo_ctx* ctx, const VgGroup* groups, int G) {
    if (G < 1 || G > VG_MAXG) { ctx->err = "vg_presize: 1..VG_MAXG filters"; return SLO_E_ARG; }
    VgSrc src;
    src.io = ctx->v.io;
    src.S = ctx->S;
    src.G = G;
    for (int g = 0; g < VG_MAXG; ++g) src.g[g] = groups[std::min(g, G - 1)];
    const VgShape h = vg_shape(src);
    if (int r = ensure_ws(ctx, h.items, (size_t)h.SV * h.maxT)) return r;
    if (ctx->cfg.voxel_order == SLO_VOXEL_PCL && h.items <= (size_t)INT32_MAX)
        return pcl_presize(ctx, h.SV, h.items, (size_t)h.maxT);
    return 0;
}

// One batched VoxelGrid over S streams: stream s's n = d_n[s * n_stride]
// points at in + s * in_stride (in == nullptr: the context's input scan,
// DevView::io); its centroids go to out + s * out_stride (at most out_cap;
// more sets errflag and is clipped) and their count to d_nout[s * nout_stride].
int vg_run(slo_ctx* ctx, const char* tag, const float4* in, size_t in_stride, const int32_t* d_n, int n_stride,
           float leaf, float4* out, size_t out_stride, int32_t* d_nout, int nout_stride, int out_cap) {
    const VgGroup g{in, in_stride, d_n, n_stride, leaf, out, out_stride, d_nout, nout_stride, out_cap};
    return vg_run_groups(ctx, tag, &g, 1);
}

// ---------------------------------------------------------------- spatial hash grid
// Global hash-grid build (T > SLO_GRID_LDS_T buckets), three passes over the
// points and one over the buckets: k_grid_count (bucket counts by device-scope
// atomics; each workgroup also sums its points per block of VG_TILE buckets
// in LDS and adds those block sums once), k_seg_top + k_seg_down (the
// per-stream exclusive scan of the counts from the block sums; down clears
// each block sum for the next build), k_grid_scatter (each point's slot by an
// atomic decrement of its bucket count, which so returns to zero for the next
// build — no clearing pass).  Entries inside a bucket are unordered; every
// reader is order-independent.
#define GRID_MAX_BLK 1024   // block sums per stream held in LDS: T + 1 <= 1024 * VG_TILE
__global__ void __launch_bounds__(256) k_grid_count(const float4* pts, size_t stride, const int32_t* n, int n_stride,
                                                    int T, float inv, int32_t* cnt, int nblk, int32_t* bsum) {
    __shared__ int bl[GRID_MAX_BLK];
    const int s = blockIdx.y;
    const int m = n[(size_t)s * n_stride];
    for (int k = threadIdx.x; k < nblk; k += blockDim.x) bl[k] = 0;
    __syncthreads();
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const float4 p = pts[(size_t)s * stride + i];
        const unsigned int b = grid_hash(grid_cell(p.x, inv), grid_cell(p.y, inv), grid_cell(p.z, inv), T);
        atomicAdd(&cnt[(size_t)s * (T + 1) + b], 1);
        atomicAdd(&bl[b / VG_TILE], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nblk; k += blockDim.x)
        if (bl[k]) atomicAdd(&bsum[(size_t)s * nblk + k], bl[k]);
}

__global__ void k_grid_scatter(const float4* pts, size_t stride, const int32_t* n, int n_stride, int T, float inv,
                               const int32_t* off, int32_t* cnt, float4* ent, size_t ent_stride) {
    const int s = blockIdx.y;
    const int m = n[(size_t)s * n_stride];
    const int base = off[(size_t)s * (T + 1)];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const float4 p = pts[(size_t)s * stride + i];
        const unsigned int b = grid_hash(grid_cell(p.x, inv), grid_cell(p.y, inv), grid_cell(p.z, inv), T);
        const size_t sb = (size_t)s * (T + 1) + b;
        const int pos = off[sb] - base + atomicSub(&cnt[sb], 1) - 1;
        ent[(size_t)s * ent_stride + pos] = make_float4(p.x, p.y, p.z, __int_as_float(i));
    }
}

// Small grids (T <= SLO_GRID_LDS_T buckets): one workgroup per stream builds
// the whole grid in LDS — bucket counts by LDS atomics, the stream's
// exclusive scan as a block scan (written to off), then the scatter with LDS
// rank counters — with no device-scope atomics and no global scan.
#define SLO_GRID_LDS_T 32768
// H > 1: the buckets in H parts of T / H, each counted, scanned and
// scattered in turn from one LDS table of SLO_GRID_LDS_T / H counters (the
// points are read H times): a smaller table lets the workgroup start on a CU
// that other workgroups still share.  Entries land where H = 1 puts them.
#ifndef SLO_GRID_LDS_H
#define SLO_GRID_LDS_H 2   // 64 KB instead of 128: 2.12 -> 2.02 ms per 24 launches alone, live within noise (r05)
#endif
template <int H>
__global__ void __launch_bounds__(1024) k_grid_build_lds(const float4* pts, size_t stride, const int32_t* n,
                                                         int n_stride, int T, float inv, int32_t* off, float4* ent,
                                                         size_t ent_stride) {
    __shared__ int cnt[SLO_GRID_LDS_T / H];
    __shared__ int wsum[16];
    __shared__ int s_base;
    const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m = n[(size_t)s * n_stride];
    const float4* P = pts + (size_t)s * stride;
    int32_t* O = off + (size_t)s * (T + 1);
    const int TH = T / H;   // T is a power of two >= H
    // GB_U points per thread in flight: the loop was one dependent global load
    // per iteration (97 us per launch isolated at C3's ~20k points)
    constexpr int GB_U = 8;
    int base = 0;
    for (int h = 0; h < H; ++h) {
        const int b0 = h * TH;
        for (int k = tid; k < TH; k += 1024) cnt[k] = 0;
        __syncthreads();
        for (int i0 = 0; i0 < m; i0 += 1024 * GB_U) {
            float4 q[GB_U];
#pragma unroll
            for (int u = 0; u < GB_U; ++u) {
                const int i = i0 + u * 1024 + tid;
                if (i < m) q[u] = P[i];
            }
#pragma unroll
            for (int u = 0; u < GB_U; ++u)
                if (i0 + u * 1024 + tid < m) {
                    const int b = (int)grid_hash(grid_cell(q[u].x, inv), grid_cell(q[u].y, inv), grid_cell(q[u].z, inv), T) - b0;
                    if (H == 1 || (unsigned)b < (unsigned)TH) atomicAdd(&cnt[b], 1);
                }
        }
        __syncthreads();
        const int per = (TH + 1023) / 1024, k0 = tid * per, k1 = min(TH, k0 + per);
        int sum = 0;
        for (int k = k0; k < k1; ++k) sum += cnt[k];
        int incl = sum;   // block exclusive scan of the per-thread sums
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        int run = base + incl - sum;
        for (int k = 0; k < w; ++k) run += wsum[k];
        for (int k = k0; k < k1; ++k) {
            const int c = cnt[k];
            cnt[k] = run;   // bucket start, then the scatter's running position
            O[b0 + k] = run;
            run += c;
        }
        if (tid == 1023) s_base = run;
        __syncthreads();
        for (int i0 = 0; i0 < m; i0 += 1024 * GB_U) {
            float4 q[GB_U];
#pragma unroll
            for (int u = 0; u < GB_U; ++u) {
                const int i = i0 + u * 1024 + tid;
                if (i < m) q[u] = P[i];
            }
#pragma unroll
            for (int u = 0; u < GB_U; ++u) {
                const int i = i0 + u * 1024 + tid;
                if (i < m) {
                    const int b = (int)grid_hash(grid_cell(q[u].x, inv), grid_cell(q[u].y, inv), grid_cell(q[u].z, inv), T) - b0;
                    if (H == 1 || (unsigned)b < (unsigned)TH)
                        ent[(size_t)s * ent_stride + atomicAdd(&cnt[b], 1)] = make_float4(q[u].x, q[u].y, q[u].z, __int_as_float(i));
                }
            }
        }
        base = s_base;
        __syncthreads();   // the next part zeroes cnt
    }
    if (tid == 0) O[T] = base;   // == m: the stream's closing (empty) bucket
}

// Per-stream exclusive scan of the bucket counts [S][N = T + 1] (offsets
// relative to the stream's first entry), reduce-then-scan over blocks of
// VG_TILE counts: block sums, a scan of each stream's block sums, then each
// block rescanned from its base (coalesced loads / stores through LDS).
__global__ void k_seg_top(int nblk, int32_t* bsum) {   // one wave per stream
    const int s = blockIdx.x, lane = threadIdx.x;
    int32_t* bs = bsum + (size_t)s * nblk;
    int run = 0;
    for (int b0 = 0; b0 < nblk; b0 += 64) {
        const int b = b0 + lane;
        const int x = b < nblk ? bs[b] : 0;
        int incl = x;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (b < nblk) bs[b] = run + incl - x;
        run += __shfl(incl, 63, 64);
    }
}

__global__ void __launch_bounds__(VG_T) k_seg_down(const int32_t* in, int N, int nblk, int32_t* bsum,
                                                   int32_t* out) {
    __shared__ int l[VG_TILE + VG_TILE / 16];
    __shared__ int wsum[VG_W];
    const int s = blockIdx.y, tid = threadIdx.x;
    const int32_t* c = in + (size_t)s * N;
    int32_t* o = out + (size_t)s * N;
    for (int b = blockIdx.x; b < nblk; b += gridDim.x) {
        const int a = b * VG_TILE, m = min(VG_TILE, N - a);
#pragma unroll 4
        for (int q = 0; q < VG_IPT; ++q) {
            const int j = q * VG_T + tid;
            l[VG_PAD(j)] = j < m ? c[a + j] : 0;
        }
        __syncthreads();
        int x[VG_IPT], sum = 0;
#pragma unroll
        for (int q = 0; q < VG_IPT; ++q) { x[q] = l[VG_PAD(tid * VG_IPT + q)]; sum += x[q]; }
        int total;
        const int top = bsum[(size_t)s * nblk + b];
        int run = top + vg_block_scan<VG_W>(sum, wsum, &total);
#pragma unroll
        for (int q = 0; q < VG_IPT; ++q) { l[VG_PAD(tid * VG_IPT + q)] = run; run += x[q]; }
        __syncthreads();
#pragma unroll 4
        for (int q = 0; q < VG_IPT; ++q) {
            const int j = q * VG_T + tid;
            if (j < m) o[a + j] = l[VG_PAD(j)];
        }
        __syncthreads();
        if (tid == 0) bsum[(size_t)s * nblk + b] = 0;   // read by this block only (after the barrier): next build
    }
}

int grid_build(slo_ctx* ctx, HashGrid& g, const float4* pts, size_t stride, const int32_t* n, int n_stride) {
    const int S = ctx->S;
    const float inv = 1.0f / g.cell;   // buckets [S][T + 1]: a zero bucket ends each stream
    if (g.T <= SLO_GRID_LDS_T) {
        SLO_LAUNCH(ctx, "grid_build_lds", (k_grid_build_lds<SLO_GRID_LDS_H>), dim3(S), dim3(1024), 0, pts, stride, n,
                   n_stride, g.T, inv,
                   g.off, g.ent, g.ent_stride);
        SLO_CHECK(hipGetLastError());
        return 0;
    }
    const int bx = std::max(1, std::min(128, (int)((stride + 255) / 256)));
    const int N = g.T + 1, nblk = (N + VG_TILE - 1) / VG_TILE;
    SLO_LAUNCH(ctx, "grid_count", k_grid_count, dim3(bx, S), dim3(256), 0, pts, stride, n, n_stride, g.T, inv, g.cnt,
               nblk, g.bsum);
    const dim3 sg(std::min(nblk, std::max(4, 2048 / S)), S);
    SLO_LAUNCH(ctx, "grid_scan", k_seg_top, dim3(S), dim3(64), 0, nblk, g.bsum);
    SLO_LAUNCH(ctx, "grid_scan", k_seg_down, sg, dim3(VG_T), 0, g.cnt, N, nblk, g.bsum, g.off);
    SLO_LAUNCH(ctx, "grid_scatter", k_grid_scatter, dim3(bx, S), dim3(256), 0, pts, stride, n, n_stride, g.T, inv,
               g.off, g.cnt, g.ent, g.ent_stride);
    SLO_CHECK(hipGetLastError());
    return 0;
}

// cell: power-of-two edge length in metres (exact floor(x / cell), GridView)
int grid_alloc(slo_ctx* ctx, HashGrid& g, int T, size_t ent_stride, float cell) {
    const int S = ctx->S;
    int e2;
    if (T <= 0 || (T & (T - 1)) || !(cell > 0) || frexpf(cell, &e2) != 0.5f) {
        ctx->err = "grid_alloc: T and cell must be powers of two";
        return SLO_E_ARG;
    }
    g.T = T;
    g.cell = cell;
    g.ent_stride = ent_stride;
    const size_t nb = (size_t)S * (T + 1);
    const size_t nblk = (T + 1 + VG_TILE - 1) / VG_TILE;
    if (nblk > GRID_MAX_BLK) {
        ctx->err = "grid_alloc: too many buckets";
        return SLO_E_ARG;
    }
    SLO_CHECK(hipMalloc(&g.cnt, sizeof(int32_t) * nb));
    SLO_CHECK(hipMalloc(&g.off, sizeof(int32_t) * nb));
    SLO_CHECK(hipMemset(g.cnt, 0, sizeof(int32_t) * nb));   // back to zero after each build (k_grid_scatter)
    SLO_CHECK(hipMalloc(&g.ent, sizeof(float4) * (size_t)S * ent_stride));
    SLO_CHECK(hipMalloc(&g.bsum, sizeof(int32_t) * (size_t)S * nblk));
    SLO_CHECK(hipMemset(g.bsum, 0, sizeof(int32_t) * (size_t)S * nblk));   // cleared by k_seg_down
    return 0;
}

GridView grid_view(const HashGrid& g) {
    GridView v;
    v.T = g.T;
    v.cell = g.cell;
    v.inv = 1.0f / g.cell;
    v.es = g.ent_stride;
    v.cnt = g.cnt;
    v.off = g.off;
    v.ent = g.ent;
    return v;
}

void grid_free(HashGrid& g) {
    if (g.cnt) hipFree(g.cnt);
    if (g.off) hipFree(g.off);
    if (g.ent) hipFree(g.ent);
    if (g.bsum) hipFree(g.bsum);
    g = HashGrid();
}

int vg_alloc(slo_ctx* ctx) {
    MapWs& w = ctx->mws;
    const int S = VG_MAXG * ctx->S;   // per virtual stream (vg_run_groups: up to VG_MAXG filters per call)
    SLO_CHECK(hipMalloc(&w.off, sizeof(int32_t) * (S + 1)));
    SLO_CHECK(hipMalloc(&w.bounds, sizeof(unsigned int) * 6 * S));
    SLO_CHECK(hipMalloc(&w.prm, sizeof(VgParams) * S));
    SLO_CHECK(hipMalloc(&w.errflag, sizeof(int32_t)));
    SLO_CHECK(hipMemset(w.errflag, 0, sizeof(int32_t)));
    SLO_CHECK(hipMalloc(&w.meta, 4 * sizeof(int32_t)));
    SLO_CHECK(hipMemset(w.meta, 0, 4 * sizeof(int32_t)));
    SLO_CHECK(hipMalloc(&w.nvox, sizeof(int32_t) * S));
    SLO_CHECK(hipMalloc(&w.gh, sizeof(int32_t) * S * VG_PASSES * VG_NB));
    SLO_CHECK(hipMemset(w.gh, 0, sizeof(int32_t) * S * VG_PASSES * VG_NB));
    SLO_CHECK(hipMalloc(&w.gbase, sizeof(int32_t) * S * VG_PASSES * VG_NB));
    SLO_CHECK(hipMalloc(&w.osw, sizeof(int32_t) * (40 + S)));
    return 0;
}

// the look-back posts of both VoxelGrid workspaces back to zero (ensure_ws
// zeroes them on ctx->stream when they are allocated; after a graph capture
// that allocated them, that memset is in the discarded graph)
int vg_ws_reinit(slo_ctx* ctx) {
    for (MapWs* w : {&ctx->mws, &ctx->mws2})
        if (w->lbk) SLO_CHECK(hipMemsetAsync(w->lbk, 0, sizeof(unsigned long long) * VG_NB * w->tiles, ctx->stream));
    return 0;
}

int vg_side_ready(slo_ctx* ctx) {
    if (ctx->side) return 0;
    SLO_CHECK(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
    SLO_CHECK(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    SLO_CHECK(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
    VgSide sc(ctx);
    return vg_alloc(ctx);
}

void vg_side_free(slo_ctx* ctx) {
    if (!ctx->side) return;
    hipStreamSynchronize(ctx->side);
    {
        VgSide sc(ctx);
        vg_free(ctx);
        pcl_free(ctx);
    }
    hipEventDestroy(ctx->ev_fork);
    hipEventDestroy(ctx->ev_join);
    hipStreamDestroy(ctx->side);
    ctx->side = nullptr;
}

void vg_free(slo_ctx* ctx) {
    MapWs& w = ctx->mws;
    void* ps[] = {w.keys, w.keys2, w.vals, w.cnt, w.hcnt, w.longv, w.off, w.bounds, w.prm, w.errflag, w.meta,
                  w.nvox, w.gh, w.gbase, w.osw, w.lbk};
    for (void* p : ps) if (p) hipFree(p);
    w = MapWs();
}

}  // namespace slo
