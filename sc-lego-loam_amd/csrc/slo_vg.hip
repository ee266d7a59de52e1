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

namespace slo {

__device__ inline unsigned int f2ord(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float ord2f(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__global__ void k_vg_prefix(const int32_t* n, int n_stride, const int32_t* active, int S, int32_t* off,
                            unsigned int* bounds) {
    // one thread: stream offsets (tiny S); bounds init
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        int a = 0;
        for (int s = 0; s < S; ++s) {
            off[s] = a;
            a += (active == nullptr || active[s]) ? n[(size_t)s * n_stride] : 0;
        }
        off[S] = a;
    }
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
        for (int k = 0; k < 3; ++k) { bounds[6 * s + k] = 0xffffffffu; bounds[6 * s + 3 + k] = 0u; }
    }
}

__global__ void k_vg_bounds(const float4* in, size_t in_stride, const int32_t* off, unsigned int* bounds) {
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
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 3; ++k) {
            atomicMin(&bounds[6 * s + k], mn[k]);
            atomicMax(&bounds[6 * s + 3 + k], mx[k]);
        }
}

struct VgParams { int minb[3]; int mul1, mul2; int overflow; float inv; };

__global__ void k_vg_params(const unsigned int* bounds, const int32_t* off, int S, float leaf, VgParams* prm) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    VgParams p;
    p.inv = 1.0f / leaf;
    p.overflow = 0;
    if (off[s + 1] - off[s] == 0 || bounds[6 * s] == 0xffffffffu) {
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
    int maxbx = (int)floorf(mx[0] * p.inv), maxby = (int)floorf(mx[1] * p.inv);
    int divx = maxbx - p.minb[0] + 1, divy = maxby - p.minb[1] + 1;
    p.mul1 = divx;
    p.mul2 = divx * divy;
    prm[s] = p;
}

__global__ void k_vg_keys(const float4* in, size_t in_stride, const int32_t* off, const VgParams* prm,
                          unsigned long long* keys, unsigned int* vals) {
    const int s = blockIdx.y;
    const int base = off[s], n = off[s + 1] - base;
    const VgParams p = prm[s];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        float4 q = in[(size_t)s * in_stride + i];
        unsigned long long k;
        if (!(isfinite(q.x) && isfinite(q.y) && isfinite(q.z))) {
            // sorts after every voxel of stream s, keeping the stream's segment contiguous
            k = ((unsigned long long)s << 32) | 0xffffffffull;
        } else if (p.overflow) {
            k = ((unsigned long long)s << 32) | (unsigned int)i;
        } else {
            int ijk0 = (int)(floorf(q.x * p.inv) - (float)p.minb[0]);
            int ijk1 = (int)(floorf(q.y * p.inv) - (float)p.minb[1]);
            int ijk2 = (int)(floorf(q.z * p.inv) - (float)p.minb[2]);
            unsigned int idx = (unsigned int)(ijk0 + ijk1 * p.mul1 + ijk2 * p.mul2);
            k = ((unsigned long long)s << 32) | idx;
        }
        keys[base + i] = k;
        vals[base + i] = (unsigned int)i;
    }
}

__global__ void k_vg_heads(const unsigned long long* keys, int total, int* flags) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > total) return;
    if (j == total) { flags[j] = 0; return; }
    unsigned long long k = keys[j];
    flags[j] = ((unsigned int)k != 0xffffffffu) && (j == 0 || k != keys[j - 1]);
}

__global__ void k_vg_centroid(const float4* in, size_t in_stride, const unsigned long long* keys,
                              const unsigned int* vals, const int* rank, const int32_t* off, int total,
                              float4* out, size_t out_stride, int out_cap) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= total) return;
    const unsigned long long k = keys[j];
    if ((unsigned int)k == 0xffffffffu || (j > 0 && keys[j - 1] == k)) return;
    const int s = (int)(k >> 32);
    const int r = rank[j] - rank[off[s]];
    float sx = 0, sy = 0, sz = 0, si = 0;
    int e = j;
    while (e < total && keys[e] == k) {
        float4 p = in[(size_t)s * in_stride + vals[e]];
        sx += p.x; sy += p.y; sz += p.z; si += p.w;
        ++e;
    }
    float c = (float)(e - j);
    if (r < out_cap) out[(size_t)s * out_stride + r] = make_float4(sx / c, sy / c, sz / c, si / c);
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
    if (w.keys) { hipFree(w.keys); hipFree(w.keys2); hipFree(w.vals); hipFree(w.vals2); hipFree(w.flags); hipFree(w.rank); }
    if (w.temp) hipFree(w.temp);
    w.items = items;
    SLO_CHECK(hipMalloc(&w.keys, 8 * items));
    SLO_CHECK(hipMalloc(&w.keys2, 8 * items));
    SLO_CHECK(hipMalloc(&w.vals, 4 * items));
    SLO_CHECK(hipMalloc(&w.vals2, 4 * items));
    SLO_CHECK(hipMalloc(&w.flags, 4 * (items + 1)));
    SLO_CHECK(hipMalloc(&w.rank, 4 * (items + 1)));
    size_t t1 = 0, t2 = 0;
    SLO_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, t1, w.keys, w.keys2, w.vals, w.vals2, (int)items, 0, 64,
                                                 ctx->stream));
    SLO_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, w.flags, w.rank, (int)items + 1, ctx->stream));
    w.temp_bytes = std::max(t1, t2);
    SLO_CHECK(hipMalloc(&w.temp, w.temp_bytes));
    return 0;
}

int vg_run(slo_ctx* ctx, const char* tag, const float4* in, size_t in_stride, const int32_t* d_n, int n_stride,
           float leaf, float4* out, size_t out_stride, int32_t* d_nout, int nout_stride, int out_cap) {
    MapWs& w = ctx->mws;
    const int S = ctx->S;
    SLO_LAUNCH(ctx, "vg_prefix", k_vg_prefix, dim3(1), dim3(256), 0, d_n, n_stride, (const int32_t*)nullptr, S,
               w.off, w.bounds);
    SLO_CHECK(hipMemcpyAsync(w.h_total, w.off + S, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    const int total = *w.h_total;
    if (int r = ensure_ws(ctx, (size_t)total + 1)) return r;
    const int T = 256;
    const int bx = std::max(1, std::min(64, (int)((in_stride + T - 1) / T)));
    SLO_LAUNCH(ctx, "vg_bounds", k_vg_bounds, dim3(bx, S), dim3(T), 0, in, in_stride, w.off, w.bounds);
    SLO_LAUNCH(ctx, "vg_params", k_vg_params, dim3((S + 63) / 64), dim3(64), 0, w.bounds, w.off, S, leaf, w.prm);
    if (total > 0) {
        SLO_LAUNCH(ctx, "vg_keys", k_vg_keys, dim3(bx, S), dim3(T), 0, in, in_stride, w.off, w.prm, w.keys, w.vals);
        int sbits = 1;
        while ((1 << sbits) < S) ++sbits;
        size_t tb = w.temp_bytes;
        hipEvent_t ev = nullptr;
        if (ctx->timing) timing_begin(ctx, "vg_sort", &ev);
        SLO_CHECK(hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.keys, w.keys2, w.vals, w.vals2, total, 0,
                                                     32 + sbits + 1, ctx->stream));
        if (ctx->timing) timing_end(ctx, "vg_sort", ev);
    }
    SLO_LAUNCH(ctx, "vg_heads", k_vg_heads, dim3((total + 1 + T - 1) / T), dim3(T), 0, w.keys2, total, w.flags);
    {
        size_t tb = w.temp_bytes;
        SLO_CHECK(hipcub::DeviceScan::ExclusiveSum(w.temp, tb, w.flags, w.rank, total + 1, ctx->stream));
    }
    if (total > 0)
        SLO_LAUNCH(ctx, "vg_centroid", k_vg_centroid, dim3((total + T - 1) / T), dim3(T), 0, in, in_stride, w.keys2,
                   w.vals2, w.rank, w.off, total, out, out_stride, out_cap);
    SLO_LAUNCH(ctx, "vg_count", k_vg_count, dim3((S + 63) / 64), dim3(64), 0, w.rank, w.off, S, d_nout, nout_stride,
               out_cap, w.errflag);
    (void)tag;
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

int grid_build(slo_ctx* ctx, HashGrid& g, const float4* pts, size_t stride, const int32_t* n, int n_stride) {
    const int S = ctx->S;
    const float inv = 1.0f / g.cell;
    const size_t nb = (size_t)S * (g.T + 1);   // [S][T + 1]: a zero bucket ends each stream
    SLO_CHECK(hipMemsetAsync(g.cnt, 0, sizeof(int32_t) * nb, ctx->stream));
    SLO_CHECK(hipMemsetAsync(g.cur, 0, sizeof(int32_t) * nb, ctx->stream));
    const int bx = std::max(1, std::min(128, (int)((stride + 255) / 256)));
    SLO_LAUNCH(ctx, "grid_count", k_grid_count, dim3(bx, S), dim3(256), 0, pts, stride, n, n_stride, g.T, inv, g.cnt);
    size_t tb = g.temp_bytes;
    SLO_CHECK(hipcub::DeviceScan::ExclusiveSum(g.temp, tb, g.cnt, g.off, (int)nb, ctx->stream));
    SLO_LAUNCH(ctx, "grid_scatter", k_grid_scatter, dim3(bx, S), dim3(256), 0, pts, stride, n, n_stride, g.T, inv,
               g.off, g.cur, g.ent, g.ent_stride);
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
    SLO_CHECK(hipHostMalloc((void**)&w.h_total, sizeof(int32_t)));
    return 0;
}

void vg_free(slo_ctx* ctx) {
    MapWs& w = ctx->mws;
    void* ps[] = {w.keys, w.keys2, w.vals, w.vals2, w.flags, w.rank, w.temp, w.off, w.bounds, w.prm, w.errflag};
    for (void* p : ps) if (p) hipFree(p);
    if (w.h_total) hipHostFree(w.h_total);
    w = MapWs();
}

}  // namespace slo
