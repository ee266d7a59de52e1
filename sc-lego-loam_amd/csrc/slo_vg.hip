// slo_vg.hip — batched PCL VoxelGrid and the 1 m hash grid used for the
// mapping 5-NN.
//
// VoxelGrid (PCL 1.8 VoxelGrid<PointXYZI>::applyFilter + CentroidPoint, the
// filter the reference calls at featureAssociation.cpp:779 and
// mapOptmization.cpp:1224-1262): per stream the bounds give min_b and the
// x-fastest linear voxel index; all streams' (stream<<32 | idx, point) pairs
// are radix sorted together (stable, so the points of a voxel stay in input
// order), every voxel's centroid is summed in that order by one thread and
// written at its rank -> output sorted by voxel index exactly like PCL.
// Non-finite points are skipped (the raw cloud is not dense, MO:1236); the
// int32 overflow guard returns the input unchanged, as PCL does.
//
// Hash grid: power-of-two cells, counting sort of the points into hashed
// buckets [S][T + 1] (the last bucket of each stream stays empty, so a run of
// consecutive buckets ends at off[h + 1]); queried by grid_ball
// (slo_internal.h).
#include "slo_internal.h"
#include <hipcub/hipcub.hpp>
#include <float.h>

// a filter whose voxel indices need more than this many bits sorts 64-bit
// keys in one sort; up to it, groups of 2^(32 - vbits) >= 8 streams sort
// 32-bit keys (vg_sorted)
#define SLO_VG_GROUP_MAX_VBITS 29

namespace slo {

__device__ inline unsigned int f2ord(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float ord2f(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// stream offsets of the concatenated input (block scan), bounds init, and the
// meta words [total, max cell count, long-voxel count]
__global__ void __launch_bounds__(1024) k_vg_prefix(const int32_t* n, int n_stride, int S, int32_t* off,
                                                    unsigned int* bounds, int32_t* meta) {
    __shared__ int wsum[16];
    __shared__ int carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int b0 = 0; b0 < S; b0 += 1024) {
        const int s = b0 + tid;
        const int x = s < S ? n[(size_t)s * n_stride] : 0;
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
    if (tid == 0) { off[S] = carry; meta[0] = carry; meta[1] = 0; meta[2] = 0; }
    for (int s = tid; s < S; s += 1024)
        for (int k = 0; k < 3; ++k) { bounds[6 * s + k] = 0xffffffffu; bounds[6 * s + 3 + k] = 0u; }
}

__global__ void __launch_bounds__(256) k_vg_bounds(const float4* in, size_t in_stride, const int32_t* off,
                                                   unsigned int* bounds) {
    const int s = blockIdx.y;
    const int n = off[s + 1] - off[s];
    unsigned int mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        float4 p = in[(size_t)s * in_stride + i];
        if (!(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) continue;
        unsigned int q[3] = {f2ord(p.x), f2ord(p.y), f2ord(p.z)};
        for (int k = 0; k < 3; ++k) { mn[k] = min(mn[k], q[k]); mx[k] = max(mx[k], q[k]); }
    }
    for (int o = 32; o > 0; o >>= 1)
        for (int k = 0; k < 3; ++k) {
            mn[k] = min(mn[k], (unsigned int)__shfl_xor((int)mn[k], o, 64));
            mx[k] = max(mx[k], (unsigned int)__shfl_xor((int)mx[k], o, 64));
        }
    __shared__ unsigned int red[4][6];
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

// voxel-index parameters (PCL applyFilter) and the largest cell count over
// the streams (meta[1]), which sizes the sort keys
struct VgParams { int minb[3]; int mul1, mul2; int overflow; float inv; };

__global__ void k_vg_params(const unsigned int* bounds, const int32_t* off, int S, float leaf, VgParams* prm,
                            int32_t* meta) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    VgParams p;
    p.inv = 1.0f / leaf;
    p.overflow = 0;
    const int n = off[s + 1] - off[s];
    if (n == 0 || bounds[6 * s] == 0xffffffffu) {
        p.minb[0] = p.minb[1] = p.minb[2] = 0; p.mul1 = p.mul2 = 0;
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
    prm[s] = p;
    // indices are < divx*divy*divz (or < n: the overflow keys are positions)
    const long long cells = p.overflow ? (long long)n : (long long)divx * divy * divz;
    atomicMax(&meta[1], (int)min(cells, 2147483647LL));
}

// keys: (stream << vbits) | voxel index; non-finite points get the all-ones
// index, which sorts after every voxel of the stream and is never a voxel
template <class K>
__global__ void k_vg_keys(const float4* in, size_t in_stride, const int32_t* off, const VgParams* prm, int vbits,
                          int G, K* keys, unsigned int* vals) {
    const int s = blockIdx.y;
    const int base = off[s], n = off[s + 1] - base;
    const VgParams p = prm[s];
    const K hi = (K)(s % G) << vbits, none = ((K)1 << vbits) - 1;   // stream bits local to its sort group
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        float4 q = in[(size_t)s * in_stride + i];
        K k;
        if (!(isfinite(q.x) && isfinite(q.y) && isfinite(q.z))) {
            k = hi | none;
        } else if (p.overflow) {
            k = hi | (K)(unsigned int)i;
        } else {
            int ijk0 = (int)(floorf(q.x * p.inv) - (float)p.minb[0]);
            int ijk1 = (int)(floorf(q.y * p.inv) - (float)p.minb[1]);
            int ijk2 = (int)(floorf(q.z * p.inv) - (float)p.minb[2]);
            k = hi | (K)(unsigned int)(ijk0 + ijk1 * p.mul1 + ijk2 * p.mul2);
        }
        keys[base + i] = k;
        vals[base + i] = (unsigned int)i;
    }
}

// item j starts a sort group (G < S: the keys of two groups are not comparable)
__device__ inline bool vg_group_start(const int32_t* off, int S, int G, int j) {
    for (int g = G; g < S; g += G)
        if (off[g] == j) return true;
    return false;
}

template <class K>
__global__ void k_vg_heads(const K* keys, int total, int vbits, const int32_t* off, int S, int G, int* flags) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > total) return;
    if (j == total) { flags[j] = 0; return; }
    const K k = keys[j], none = ((K)1 << vbits) - 1;
    flags[j] = (k & none) != none && (j == 0 || k != keys[j - 1] || vg_group_start(off, S, G, j));
}

// voxel r = rank of its first item: its item range [starts[r], ends[r])
template <class K>
__global__ void k_vg_runs(const K* keys, const int* rank, int total, int vbits, const int32_t* off, int S, int G,
                          int* starts, int* ends) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= total) return;
    const K k = keys[j], none = ((K)1 << vbits) - 1;
    if ((k & none) == none) return;
    const bool head = j == 0 || keys[j - 1] != k || vg_group_start(off, S, G, j);
    const int r = head ? rank[j] : rank[j] - 1;   // rank = heads strictly before j
    if (head) starts[r] = j;
    if (j + 1 == total || keys[j + 1] != k || vg_group_start(off, S, G, j + 1)) ends[r] = j + 1;
}

// the stream of sorted item a whose key carries the group-local stream l:
// sort group g holds the items of streams [g*G, (g+1)*G), i.e. positions
// [off[g*G], off[(g+1)*G])
__device__ inline int vg_stream(const int32_t* off, int S, int G, int l, int a) {
    int g = 0;
    while ((g + 1) * G < S && off[(g + 1) * G] <= a) ++g;
    return g * G + l;
}

// Centroid of one voxel: the points are summed in input order (the sort is
// stable), one float chain per component as PCL's CentroidPoint.  Voxels of
// up to VG_SHORT points: one thread each, loads issued 4 at a time ahead of
// the chain.  Longer ones are listed for k_vg_long.
#define VG_SHORT 32
struct VgOut { float4* out; size_t stride; int cap; };

__device__ inline void vg_store(const VgOut& o, const int* rank, const int32_t* off, int s, int r, float sx, float sy,
                                float sz, float si, int cnt) {
    const int pos = r - rank[off[s]];
    const float c = (float)cnt;
    if (pos < o.cap) o.out[(size_t)s * o.stride + pos] = make_float4(sx / c, sy / c, sz / c, si / c);
}

template <class K>
__global__ void k_vg_centroid(const float4* in, size_t in_stride, const K* keys, const unsigned int* vals,
                              const int* rank, const int32_t* off, int total, int vbits, int S, int G,
                              const int* starts, const int* ends, int32_t* meta, int* longv, VgOut o) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rank[total]) return;
    const int a = starts[r], e = ends[r];
    if (e - a > VG_SHORT) {
        longv[atomicAdd(&meta[2], 1)] = r;
        return;
    }
    const int s = vg_stream(off, S, G, (int)(keys[a] >> vbits), a);
    const float4* src = in + (size_t)s * in_stride;
    float sx = 0, sy = 0, sz = 0, si = 0;
    for (int j = a; j < e; j += 4) {
        float4 p[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) p[u] = j + u < e ? src[vals[j + u]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (j + u < e) { sx += p[u].x; sy += p[u].y; sz += p[u].z; si += p[u].w; }
    }
    vg_store(o, rank, off, s, r, sx, sy, sz, si, e - a);
}

// Long voxels, one wave each (persistent grid over the list): the wave
// stages 256 points at a time in LDS and lanes 0..3 run the x, y, z and
// intensity chains over them in order.
template <class K>
__global__ void __launch_bounds__(256) k_vg_long(const float4* in, size_t in_stride, const K* keys,
                                                 const unsigned int* vals, const int* rank, const int32_t* off,
                                                 int vbits, int S, int G, const int* starts, const int* ends,
                                                 const int32_t* meta, const int* longv, VgOut o) {
    __shared__ float4 buf[4][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nlong = meta[2];
    float4* b = buf[w];
    for (int t = blockIdx.x * 4 + w; t < nlong; t += gridDim.x * 4) {
        const int r = longv[t], a = starts[r], e = ends[r];
        const int s = vg_stream(off, S, G, (int)(keys[a] >> vbits), a);
        const float4* src = in + (size_t)s * in_stride;
        float acc = 0.0f;
        for (int c0 = a; c0 < e; c0 += 256) {
            const int m = min(256, e - c0);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = u * 64 + lane;
                if (k < m) b[k] = src[vals[c0 + k]];
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // this wave's LDS traffic drained
            __builtin_amdgcn_wave_barrier();
            if (lane < 4) {
                const float* f = reinterpret_cast<const float*>(b) + lane;
                for (int k = 0; k < m; ++k) acc += f[4 * k];
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // this wave's LDS traffic drained
            __builtin_amdgcn_wave_barrier();
        }
        const float sx = __shfl(acc, 0, 64), sy = __shfl(acc, 1, 64), sz = __shfl(acc, 2, 64),
                    si = __shfl(acc, 3, 64);
        if (lane == 0) vg_store(o, rank, off, s, r, sx, sy, sz, si, e - a);
    }
}

__global__ void k_vg_count(const int* rank, const int32_t* off, int S, int32_t* nout, int nout_stride, int out_cap,
                           int32_t* errflag) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    int c = rank[off[s + 1]] - rank[off[s]];
    if (c > out_cap) { c = out_cap; atomicOr(errflag, 1); }
    nout[(size_t)s * nout_stride] = c;
}

static int ensure_ws(slo_ctx* ctx, size_t items) {
    MapWs& w = ctx->mws;
    if (items <= w.items) return 0;
    // grow geometrically: a local map creeping up by a few points per mapping
    // step must not reallocate (a device-wide synchronisation) every time
    items = std::max(items, w.items + w.items / 2);
    void* old[] = {w.keys, w.keys2, w.vals, w.vals2, w.flags, w.rank, w.starts, w.ends, w.longv, w.temp};
    for (void* p : old) if (p) hipFree(p);
    w.items = items;
    SLO_CHECK(hipMalloc(&w.keys, 8 * items));
    SLO_CHECK(hipMalloc(&w.keys2, 8 * items));
    SLO_CHECK(hipMalloc(&w.vals, 4 * items));
    SLO_CHECK(hipMalloc(&w.vals2, 4 * items));
    SLO_CHECK(hipMalloc(&w.flags, 4 * (items + 1)));
    SLO_CHECK(hipMalloc(&w.rank, 4 * (items + 1)));
    SLO_CHECK(hipMalloc(&w.starts, 4 * items));
    SLO_CHECK(hipMalloc(&w.ends, 4 * items));
    SLO_CHECK(hipMalloc(&w.longv, 4 * items));
    size_t t1 = 0, t2 = 0, t3 = 0;
    SLO_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, t1, (unsigned long long*)w.keys,
                                                 (unsigned long long*)w.keys2, w.vals, w.vals2, (int)items, 0, 64,
                                                 ctx->stream));
    SLO_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, t3, (unsigned int*)w.keys, (unsigned int*)w.keys2, w.vals,
                                                 w.vals2, (int)items, 0, 32, ctx->stream));
    SLO_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, w.flags, w.rank, (int)items + 1, ctx->stream));
    w.temp_bytes = std::max(std::max(t1, t2), t3);
    SLO_CHECK(hipMalloc(&w.temp, w.temp_bytes));
    return 0;
}

// G streams per sort group: the (group-local stream, voxel) keys of group g
// occupy the item range [off[g*G], off[(g+1)*G]), sorted on their own, so a
// filter whose voxel index and stream count need more than 32 bits together
// still sorts 32-bit keys (a third less traffic per pass than 64-bit keys,
// and one pass fewer)
template <class K>
static int vg_sorted(slo_ctx* ctx, const char* tag, const float4* in, size_t in_stride, int total, int vbits, int sbits,
                     int G, const VgOut& o) {
    MapWs& w = ctx->mws;
    const int S = ctx->S, T = 256;
    const int bx = std::max(1, std::min(64, (int)((in_stride + T - 1) / T)));
    K* keys = (K*)w.keys;
    K* keys2 = (K*)w.keys2;
    SLO_LAUNCH(ctx, "vg_keys", k_vg_keys<K>, dim3(bx, S), dim3(T), 0, in, in_stride, w.off, w.prm, vbits, G, keys,
               w.vals);
    size_t tb = w.temp_bytes;
    hipEvent_t ev = nullptr;
    const std::string sort_name = std::string("vg_sort:") + tag;   // per filter in the timing table
    const bool tm = ctx->timing && timing_on(ctx, sort_name.c_str());
    if (tm) timing_begin(ctx, sort_name.c_str(), &ev);
    for (int g0 = 0; g0 < S; g0 += G) {   // one sort per group (G = S: one sort)
        const int a = G >= S ? 0 : w.h_off[g0], e = G >= S ? total : w.h_off[std::min(S, g0 + G)];
        if (e <= a) continue;
        tb = w.temp_bytes;
        SLO_CHECK(hipcub::DeviceRadixSort::SortPairs(w.temp, tb, keys + a, keys2 + a, w.vals + a, w.vals2 + a, e - a, 0,
                                                     vbits + sbits, ctx->stream));
    }
    if (tm) timing_end(ctx, sort_name.c_str(), ev);
    const int gi = (total + T - 1) / T;
    SLO_LAUNCH(ctx, "vg_heads", k_vg_heads<K>, dim3((total + 1 + T - 1) / T), dim3(T), 0, keys2, total, vbits, w.off,
               S, G, w.flags);
    tb = w.temp_bytes;
    SLO_CHECK(hipcub::DeviceScan::ExclusiveSum(w.temp, tb, w.flags, w.rank, total + 1, ctx->stream));
    SLO_LAUNCH(ctx, "vg_runs", k_vg_runs<K>, dim3(gi), dim3(T), 0, keys2, w.rank, total, vbits, w.off, S, G, w.starts,
               w.ends);
    SLO_LAUNCH(ctx, "vg_centroid", k_vg_centroid<K>, dim3(gi), dim3(T), 0, in, in_stride, keys2, w.vals2, w.rank,
               w.off, total, vbits, S, G, w.starts, w.ends, w.meta, w.longv, o);
    SLO_LAUNCH(ctx, "vg_long", k_vg_long<K>, dim3(std::min(1024, gi)), dim3(T), 0, in, in_stride, keys2, w.vals2,
               w.rank, w.off, vbits, S, G, w.starts, w.ends, w.meta, w.longv, o);
    return 0;
}

int vg_run(slo_ctx* ctx, const char* tag, const float4* in, size_t in_stride, const int32_t* d_n, int n_stride,
           float leaf, float4* out, size_t out_stride, int32_t* d_nout, int nout_stride, int out_cap) {
    MapWs& w = ctx->mws;
    const int S = ctx->S;
    const int T = 256;
    const int bx = std::max(1, std::min(64, (int)((in_stride + T - 1) / T)));
    SLO_LAUNCH(ctx, "vg_prefix", k_vg_prefix, dim3(1), dim3(1024), 0, d_n, n_stride, S, w.off, w.bounds, w.meta);
    SLO_LAUNCH(ctx, "vg_bounds", k_vg_bounds, dim3(bx, S), dim3(T), 0, in, in_stride, w.off, w.bounds);
    SLO_LAUNCH(ctx, "vg_params", k_vg_params, dim3((S + 63) / 64), dim3(64), 0, w.bounds, w.off, S, leaf, w.prm,
               w.meta);
    // one host round trip per filter: the item count, the key width and the
    // stream offsets (the sort groups' item ranges)
    SLO_CHECK(hipMemcpyAsync(w.h_meta, w.meta, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    SLO_CHECK(hipMemcpyAsync(w.h_off, w.off, (S + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    const int total = w.h_meta[0];
    int vbits = 1;   // every index < 2^vbits - 1 (the all-ones index marks non-finite points)
    while (vbits < 32 && (1LL << vbits) <= (long long)w.h_meta[1]) ++vbits;
    if (w.h_meta[1] >= (1 << 30)) vbits = 32;   // int index arithmetic may wrap, as in PCL
    int sbits = 0;
    while ((1 << sbits) < S) ++sbits;
    if (int r = ensure_ws(ctx, (size_t)total + 1)) return r;
    if (total > 0) {
        const VgOut o{out, out_stride, out_cap};
        int r;
        if (vbits + sbits <= 32 && vbits < 32) {
            r = vg_sorted<unsigned int>(ctx, tag, in, in_stride, total, vbits, sbits, S, o);
        } else if (vbits <= SLO_VG_GROUP_MAX_VBITS) {   // groups of G streams on 32-bit keys
            const int gbits = 32 - vbits;
            r = vg_sorted<unsigned int>(ctx, tag, in, in_stride, total, vbits, gbits, 1 << gbits, o);
        } else {
            r = vg_sorted<unsigned long long>(ctx, tag, in, in_stride, total, vbits, sbits, S, o);
        }
        if (r) return r;
    } else {
        SLO_CHECK(hipMemsetAsync(w.rank, 0, sizeof(int), ctx->stream));
    }
    SLO_LAUNCH(ctx, "vg_count", k_vg_count, dim3((S + 63) / 64), dim3(64), 0, w.rank, w.off, S, d_nout, nout_stride,
               out_cap, w.errflag);
    SLO_CHECK(hipGetLastError());
    return 0;
}

// ---------------------------------------------------------------- spatial hash grid
__global__ void k_grid_count(const float4* pts, size_t stride, const int32_t* n, int n_stride, int T, float inv,
                             int32_t* cnt) {
    const int s = blockIdx.y;
    const int m = n[(size_t)s * n_stride];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const float4 p = pts[(size_t)s * stride + i];
        const unsigned int b = grid_hash(grid_cell(p.x, inv), grid_cell(p.y, inv), grid_cell(p.z, inv), T);
        atomicAdd(&cnt[(size_t)s * (T + 1) + b], 1);
    }
}

__global__ void k_grid_scatter(const float4* pts, size_t stride, const int32_t* n, int n_stride, int T, float inv,
                               const int32_t* off, int32_t* cur, float4* ent, size_t ent_stride) {
    const int s = blockIdx.y;
    const int m = n[(size_t)s * n_stride];
    const int base = off[(size_t)s * (T + 1)];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const float4 p = pts[(size_t)s * stride + i];
        const unsigned int b = grid_hash(grid_cell(p.x, inv), grid_cell(p.y, inv), grid_cell(p.z, inv), T);
        const int pos = off[(size_t)s * (T + 1) + b] - base + atomicAdd(&cur[(size_t)s * (T + 1) + b], 1);
        ent[(size_t)s * ent_stride + pos] = make_float4(p.x, p.y, p.z, __int_as_float(i));
    }
}

// cnt / cur back to zero for the next build: only the buckets the points hit
// are non-zero, so clearing those replaces two memsets of the whole [S][T + 1]
// arrays (grid_alloc zeroes them once)
__global__ void k_grid_clear(const float4* pts, size_t stride, const int32_t* n, int n_stride, int T, float inv,
                             int32_t* cnt, int32_t* cur) {
    const int s = blockIdx.y;
    const int m = n[(size_t)s * n_stride];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const float4 p = pts[(size_t)s * stride + i];
        const size_t b = (size_t)s * (T + 1) + grid_hash(grid_cell(p.x, inv), grid_cell(p.y, inv), grid_cell(p.z, inv), T);
        cnt[b] = 0;
        cur[b] = 0;
    }
}

// Small grids (T <= SLO_GRID_LDS_T buckets): one workgroup per stream builds
// the whole grid in LDS — bucket counts by LDS atomics, the stream's
// exclusive scan as a block scan (written to off), then the scatter with LDS
// rank counters — with no device-scope atomics and no global scan.
#define SLO_GRID_LDS_T 32768
__global__ void __launch_bounds__(1024) k_grid_build_lds(const float4* pts, size_t stride, const int32_t* n,
                                                         int n_stride, int T, float inv, int32_t* off, float4* ent,
                                                         size_t ent_stride) {
    __shared__ int cnt[SLO_GRID_LDS_T];
    __shared__ int wsum[16];
    const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m = n[(size_t)s * n_stride];
    const float4* P = pts + (size_t)s * stride;
    int32_t* O = off + (size_t)s * (T + 1);
    for (int k = tid; k < T; k += 1024) cnt[k] = 0;
    __syncthreads();
    for (int i = tid; i < m; i += 1024) {
        const float4 p = P[i];
        atomicAdd(&cnt[grid_hash(grid_cell(p.x, inv), grid_cell(p.y, inv), grid_cell(p.z, inv), T)], 1);
    }
    __syncthreads();
    const int per = (T + 1023) / 1024, k0 = tid * per, k1 = min(T, k0 + per);
    int sum = 0;
    for (int k = k0; k < k1; ++k) sum += cnt[k];
    int incl = sum;   // block exclusive scan of the per-thread sums
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int run = incl - sum;
    for (int k = 0; k < w; ++k) run += wsum[k];
    for (int k = k0; k < k1; ++k) {
        const int c = cnt[k];
        cnt[k] = run;   // bucket start, then the scatter's running position
        O[k] = run;
        run += c;
    }
    if (tid == 1023) O[T] = run;   // == m: the stream's closing (empty) bucket
    __syncthreads();
    for (int i = tid; i < m; i += 1024) {
        const float4 p = P[i];
        const int b = (int)grid_hash(grid_cell(p.x, inv), grid_cell(p.y, inv), grid_cell(p.z, inv), T);
        ent[(size_t)s * ent_stride + atomicAdd(&cnt[b], 1)] = make_float4(p.x, p.y, p.z, __int_as_float(i));
    }
}

int grid_build(slo_ctx* ctx, HashGrid& g, const float4* pts, size_t stride, const int32_t* n, int n_stride) {
    const int S = ctx->S;
    const float inv = 1.0f / g.cell;
    const size_t nb = (size_t)S * (g.T + 1);   // [S][T + 1]: a zero bucket ends each stream
    if (g.T <= SLO_GRID_LDS_T) {
        SLO_LAUNCH(ctx, "grid_build_lds", k_grid_build_lds, dim3(S), dim3(1024), 0, pts, stride, n, n_stride, g.T, inv,
                   g.off, g.ent, g.ent_stride);
        SLO_CHECK(hipGetLastError());
        return 0;
    }
    const int bx = std::max(1, std::min(128, (int)((stride + 255) / 256)));
    SLO_LAUNCH(ctx, "grid_count", k_grid_count, dim3(bx, S), dim3(256), 0, pts, stride, n, n_stride, g.T, inv, g.cnt);
    size_t tb = g.temp_bytes;
    SLO_CHECK(hipcub::DeviceScan::ExclusiveSum(g.temp, tb, g.cnt, g.off, (int)nb, ctx->stream));
    SLO_LAUNCH(ctx, "grid_scatter", k_grid_scatter, dim3(bx, S), dim3(256), 0, pts, stride, n, n_stride, g.T, inv,
               g.off, g.cur, g.ent, g.ent_stride);
    SLO_LAUNCH(ctx, "grid_clear", k_grid_clear, dim3(bx, S), dim3(256), 0, pts, stride, n, n_stride, g.T, inv, g.cnt,
               g.cur);
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
    SLO_CHECK(hipMalloc(&g.cnt, sizeof(int32_t) * nb));
    SLO_CHECK(hipMalloc(&g.cur, sizeof(int32_t) * nb));
    SLO_CHECK(hipMalloc(&g.off, sizeof(int32_t) * nb));
    SLO_CHECK(hipMemset(g.cnt, 0, sizeof(int32_t) * nb));   // kept zero between builds (k_grid_clear)
    SLO_CHECK(hipMemset(g.cur, 0, sizeof(int32_t) * nb));
    SLO_CHECK(hipMalloc(&g.ent, sizeof(float4) * (size_t)S * ent_stride));
    size_t tb = 0;
    SLO_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, g.cnt, g.off, (int)nb, ctx->stream));
    g.temp_bytes = tb;
    SLO_CHECK(hipMalloc(&g.temp, tb));
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
    if (g.cur) hipFree(g.cur);
    if (g.off) hipFree(g.off);
    if (g.ent) hipFree(g.ent);
    if (g.temp) hipFree(g.temp);
    g = HashGrid();
}

int vg_alloc(slo_ctx* ctx) {
    MapWs& w = ctx->mws;
    const int S = ctx->S;
    SLO_CHECK(hipMalloc(&w.off, sizeof(int32_t) * (S + 1)));
    SLO_CHECK(hipMalloc(&w.bounds, sizeof(unsigned int) * 6 * S));
    SLO_CHECK(hipMalloc(&w.prm, sizeof(VgParams) * S));
    SLO_CHECK(hipMalloc(&w.errflag, sizeof(int32_t)));
    SLO_CHECK(hipMemset(w.errflag, 0, sizeof(int32_t)));
    SLO_CHECK(hipMalloc(&w.meta, 4 * sizeof(int32_t)));
    SLO_CHECK(hipHostMalloc((void**)&w.h_meta, 4 * sizeof(int32_t)));
    SLO_CHECK(hipHostMalloc((void**)&w.h_off, (S + 1) * sizeof(int32_t)));
    return 0;
}

void vg_free(slo_ctx* ctx) {
    MapWs& w = ctx->mws;
    void* ps[] = {w.keys, w.keys2, w.vals, w.vals2, w.flags, w.rank, w.starts, w.ends, w.longv,
                  w.temp, w.off, w.bounds, w.prm, w.errflag, w.meta};
    for (void* p : ps) if (p) hipFree(p);
    if (w.h_meta) hipHostFree(w.h_meta);
    if (w.h_off) hipHostFree(w.h_off);
    w = MapWs();
}

}  // namespace slo
