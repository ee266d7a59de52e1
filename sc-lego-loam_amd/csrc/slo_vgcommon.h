// slo_vgcommon.h — what the two VoxelGrid sorts share (slo_vg.hip: the
// stable radix sort; slo_vgpcl.hip: PCL's std::sort order): the input view,
// the per-stream voxel parameters of PCL's applyFilter and the voxel key.
#pragma once
#include "slo_internal.h"
#include <utility>

namespace slo {

// One VoxelGrid filter over the context's S streams: stream s's
// n[s * n_stride] points at in + s * stride (in == nullptr: the context's
// input scan through its io slot, counts io->npts), VoxelGrid(leaf), its
// centroids to out + s * out_stride (at most out_cap, more are clipped and
// flagged) and their count to nout[s * nout_stride].
struct VgGroup {
    const float4* in;
    size_t stride;
    const int32_t* n;
    int n_stride;
    float leaf;
    float4* out;
    size_t out_stride;
    int32_t* nout;
    int nout_stride;
    int out_cap;
};
// A VoxelGrid call (a kernel argument): G filters of S streams each, run as
// G * S virtual streams v = g * S + s.  Every workspace array, tile list and
// sort range is per virtual stream, so the filters of a mapping step
// (MO:1224-1263) sort together in one launch sequence.
struct VgOut { float4* out; int cap; };
struct VgSrc {
    const SloIo* io;
    int S, G;
    VgGroup g[VG_MAXG];
    __host__ __device__ int nv() const { return S * G; }
    __device__ const VgGroup& grp(int v) const { return g[v / S]; }
    __device__ const float4* row(int v) const {   // the virtual stream's input cloud
        const VgGroup& q = g[v / S];
        return (q.in ? q.in : io->pts) + (size_t)(v % S) * q.stride;
    }
    __device__ int count(int v) const {
        const VgGroup& q = g[v / S];
        return q.in ? q.n[(size_t)(v % S) * q.n_stride] : io->npts[v % S];
    }
    __device__ VgOut out_row(int v) const {      // its output row and capacity
        const VgGroup& q = g[v / S];
        return VgOut{q.out + (size_t)(v % S) * q.out_stride, q.out_cap};
    }
};

__device__ inline unsigned int f2ord(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float ord2f(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// voxel-index parameters (PCL applyFilter) per stream, and the stream's key
// width: vbits (every voxel index < 2^vbits - 1, the all-ones key marks a
// non-finite point), split into npass digits of dbits <= VG_DMAX each
struct VgParams { int minb[3]; int mul1, mul2; int overflow; float inv; int vbits, dbits, npass, ntiles; };

#ifndef VG_T
#define VG_T 256                      // threads per tile workgroup
#endif
#define VG_W (VG_T / 64)              // waves per tile workgroup (each owns a slice of the tile)
#ifndef VG_SCATTER_OCC
// vg_scatter waves per SIMD: 3 leaves room (<= 168 VGPRs) for all of a tile's
// key and value loads in flight at once; at 4 the same code spills (measured
// 28.5 k against 27.9 k scans/s, and 26.8 k for 4 waves with one load in flight)
#define VG_SCATTER_OCC (VG_W == 4 ? 3 : 6)
#endif
#ifndef VG_IPT
#define VG_IPT 16                     // items per thread
#endif
#define VG_TILE (VG_T * VG_IPT)       // items per tile
#define VG_PASSES 4                   // LSD radix passes launched (a stream runs npass <= VG_PASSES of them)
#ifndef VG_DMAX
#define VG_DMAX 8                     // digit bits per pass at most; VG_PASSES * VG_DMAX >= 32
#endif
#define VG_NB (1 << VG_DMAX)          // digit bins
static_assert(VG_PASSES * VG_DMAX >= 32 && (VG_NB % VG_T == 0 || VG_T % VG_NB == 0), "VoxelGrid digit layout");
#define VG_PAD(j) ((j) + ((j) >> 4))  // LDS index padded against 16-way bank conflicts (blocked reads)

__device__ inline unsigned int vg_none(const VgParams& p) { return p.vbits >= 32 ? 0xffffffffu : (1u << p.vbits) - 1u; }

// the PCL voxel index of point i of a stream (positions on overflow)
__device__ inline unsigned int vg_key(const float4& q, const VgParams& p, int i) {
    if (!(isfinite(q.x) & isfinite(q.y) & isfinite(q.z))) return vg_none(p);   // no short-circuit: one load
    if (p.overflow) return (unsigned int)i;
    const int ijk0 = (int)(floorf(q.x * p.inv) - (float)p.minb[0]);
    const int ijk1 = (int)(floorf(q.y * p.inv) - (float)p.minb[1]);
    const int ijk2 = (int)(floorf(q.z * p.inv) - (float)p.minb[2]);
    return (unsigned int)(ijk0 + ijk1 * p.mul1 + ijk2 * p.mul2);
}

// exclusive scan over the workgroup (NW waves of 64); *total = the sum
template <int NW, class T>
__device__ inline T vg_block_scan(T x, T* wsum, T* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T incl = x;
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    T before = 0, all = 0;
    for (int k = 0; k < NW; ++k) {
        if (k < w) before += wsum[k];
        all += wsum[k];
    }
    __syncthreads();   // wsum reusable
    *total = all;
    return before + incl - x;
}

// PCL's std::sort order of the call's virtual streams' items
// (slo_vgpcl.hip): K / V receive virtual stream v's sorted (voxel key, point
// index) items at [off[v], off[v + 1]), finite points first, the non-finite
// ones after them with the "none" key.  max_stride: the largest input stride;
// items: the workspace bound, sum over the filters of S * stride.
// spare: 2 * items 32-bit words of scratch (MapWs keys2 | vals2)
int vg_pcl_sort(slo_ctx* ctx, const VgSrc& src, size_t max_stride, size_t items, const VgParams* prm,
                const int32_t* off, unsigned int* K, unsigned int* V, unsigned int* spare);

// G batched VoxelGrid filters over the context's S streams (slo_vg.hip)
int vg_run_groups(slo_ctx* ctx, const char* tag, const VgGroup* groups, int G);

#ifndef SLO_VG_FORK_STREAMS
#define SLO_VG_FORK_STREAMS 8   // contexts of at most this many streams run the local-map VoxelGrids on ctx->side
#endif
// Issues the enclosed launches on ctx->side with the side workspaces: the
// context's stream and VoxelGrid / PCL-sort workspaces are swapped for the
// scope's lifetime (one host thread drives a context).
struct VgSide {
    slo_ctx* c;
    explicit VgSide(slo_ctx* ctx) : c(ctx) { swap_(); }
    ~VgSide() { swap_(); }
    void swap_() {
        std::swap(c->stream, c->side);
        std::swap(c->mws, c->mws2);
        std::swap(c->pws, c->pws2);
    }
};
int vg_side_ready(slo_ctx* ctx);   // creates the side stream, its events and workspaces once

}  // namespace slo
