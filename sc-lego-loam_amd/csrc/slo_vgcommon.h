// slo_vgcommon.h — what the two VoxelGrid sorts share (slo_vg.hip: the
// stable radix sort; slo_vgpcl.hip: PCL's std::sort order): the input view,
// the per-stream voxel parameters of PCL's applyFilter and the voxel key.
#pragma once
#include "slo_internal.h"
#include <utility>

namespace slo {

// a VoxelGrid input: a cloud [S][stride] with counts n[s * n_stride], or
// (in == nullptr) the context's input scan through its io slot
struct VgSrc {
    const float4* in;
    const int32_t* n;
    const SloIo* io;
    __device__ const float4* pts() const { return in ? in : io->pts; }
    __device__ const int32_t* cnt() const { return in ? n : io->npts; }
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

// PCL's std::sort order of S streams' items (slo_vgpcl.hip): K / V receive
// stream s's sorted (voxel key, point index) items at [off[s], off[s + 1]),
// finite points first, the non-finite ones after them with the "none" key
int vg_pcl_sort(slo_ctx* ctx, const VgSrc& src, size_t in_stride, const VgParams* prm, const int32_t* off,
                unsigned int* K, unsigned int* V);

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
