// slo_internal.h — context layout shared by the HIP translation units.
//
// HBM layout: every per-stream array is a [n_streams][capacity] slab carved
// out of one arena (struct-of-arrays, 256-byte aligned), so a batched kernel
// indexes (stream, element) with one multiply and reads each stream's slab
// contiguously.  State that the reference keeps across scans (FA's
// cloudSmoothness / cloudCurvature / cloudNeighborPicked / cloudLabel, the
// cloud_info arrays with their stale tails, *Last clouds, the keyframe ring,
// the Scan Context history) lives here for the lifetime of the context.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>
#include <map>
#include "slo_config.h"
#include "slo_ddsum.h"
#include "../../include/slo_abi.h"

#define SLO_CHECK(x)                                                            \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            ctx->err = std::string(#x) + ": " + hipGetErrorString(e_);            \
            return SLO_E_HIP;                                                     \
        }                                                                         \
    } while (0)

namespace slo {

struct alignas(8) Smooth { float value; int32_t ind; };

// Per-stream scalar state of the FA / MO nodes (one record per stream).
struct StreamState {
    float transformCur[6];
    float transformSum[6];
    float matP_fa[9];
    int32_t isDegenerate_fa;
    int32_t cornerLastNum, surfLastNum;   // laserCloud*LastNum
    int32_t kdCornerNum, kdSurfNum;       // size of the cloud the "tree" was last built on
    int32_t iters_surf, iters_corner;
    int32_t first_half;                   // deskew: first index with halfPassed
    int32_t odo_phase;                    // odometry control between launches (slo_odom.hip)
    int32_t seg_count, outlier_count;
    int32_t n_sharp, n_less_sharp, n_flat, n_less_flat;
    // mapping
    float transformLast[6], transformIncre[6], transformTobeMapped[6];
    float transformBefMapped[6], transformAftMapped[6];
    float mo_sum[6];
    float matP_mo[36];
    int32_t isDegenerate_mo;
    int32_t n_keyframes;
    int32_t latestFrameID;
    int32_t recent_n;                     // deque size
    int32_t recent_ids[64];               // deque of keyframe ids (front first)
    float prevPos[3];
    int32_t mo_ran, kf_saved, mo_iters, mo_converged;
    int32_t n_corner_map, n_surf_map, n_corner_ds, n_surf_total_ds, n_raw_ds;
    int32_t n_surf_ds, n_outl_ds, n_st, n_cmap_ds, n_smap_ds, n_sel, map_ok;
    // scan context
    int32_t sc_count, sc_tree_n, sc_counter;
    int32_t det_valid, det_loop_id, det_nn_idx, det_cand[64];
    float det_yaw;
    double det_min_dist;
    int32_t flags;
    int32_t err;
    unsigned long long dbg[8];            // diagnostic counters (slo_get "dbg"), not part of the algorithm
};

// Spatial hash grid over one [S][es] cloud (built by grid_build): cell edge
// `cell` is a power of two, so floor(x * inv) is floor(x / cell) exactly and
// "a point in a cell r rings away is more than (r-1)*cell away" holds in float
// arithmetic too — the searches rely on it to stop early and stay exact.
// Bucket b of stream s holds ent[s*es + off[s*T+b] - off[s*T] .. + cnt[s*T+b]],
// each entry (x, y, z, point index as int bits).
struct GridView {
    int T;
    float inv, cell;
    size_t es;
    const int32_t *cnt, *off;
    const float4* ent;
};

// kernel-visible view of the context (passed by value)
struct DevView {
    slo_config cfg;
    int S;        // streams
    int P;        // max points per scan
    int H;        // R*C
    int cap_sharp, cap_less_sharp, cap_flat, cap_less_flat;
    // inputs
    const float4* pts;   // [S][P]
    const int32_t* npts; // [S]
    // image projection
    int32_t* owner;      // [S][H]
    int32_t* fl;         // [S][2] first/last finite index
    float* range;        // [S][H]
    float4* full;        // [S][H]
    int8_t* ground;      // [S][H]
    int32_t* label;      // [S][H]
    int32_t* parent;     // [S][H]
    int32_t* csize;      // [S][H]
    unsigned long long* crows;  // [S][H][2]
    int32_t* rowcnt;     // [S][R][2] kept / outlier per row
    float4* seg;         // [S][H]
    uint8_t* seg_ground; // [S][H]
    uint32_t* seg_col;   // [S][H]
    float* seg_range;    // [S][H]
    int32_t* ring_se;    // [S][R][2]
    float* orient;       // [S][3]
    float4* outlier;     // [S][H]
    // feature association
    float4* fpts;        // [S][H] deskewed camera-frame points
    float* curv;         // [S][H]
    int32_t* picked;     // [S][H]
    int32_t* clabel;     // [S][H]
    Smooth* smooth;      // [S][H]
    int32_t* ring_cnt;   // [S][R][4] sharp, less_sharp, flat, less_flat(after DS)
    float4* r_sharp;     // [S][R][12]
    float4* r_less_sharp;// [S][R][120]
    float4* r_flat;      // [S][R][24]
    float4* r_lf_scan;   // [S][R][C] less-flat scan (before DS)
    int32_t* r_lf_n;     // [S][R]
    float4* r_lf_ds;     // [S][R][C]
    float4* sharp;       // [S][cap_sharp]
    float4* less_sharp;  // [S][cap_less_sharp]
    float4* flat;        // [S][cap_flat]
    float4* less_flat;   // [S][cap_less_flat]
    // odometry
    float4* corner_last; // [S][cap_less_sharp]  (previous scan, end-of-sweep)
    float4* surf_last;   // [S][cap_less_flat]
    float4* corner_next; // [S][cap_less_sharp]  (this scan, written by odometry)
    float4* surf_next;   // [S][cap_less_flat]
    float4* kd_corner;   // [S][cap_less_sharp]  copy the "tree" searches (setInputCloud copies)
    float4* kd_surf;     // [S][cap_less_flat]
    int32_t* roff_cur;   // [S][2][R+1] first index of each ring in less_sharp / less_flat
    int16_t* ex_list;    // [S][2][H] per-sector pick candidates (sharp, flat), window offsets
    int32_t* ex_cnt;     // [S][R][6][2] candidate counts
    int32_t* roff_last;  // [S][2][R+1] the same for corner_last / surf_last
    int32_t* ind_surf;   // [S][cap_flat][3]   pointSearchSurfInd1..3 (Q9: exact ints)
    int32_t* ind_corner; // [S][cap_sharp][2]  pointSearchCornerInd1..2
    StreamState* st;     // [S]
    // ---- mapping (mapOptmization.cpp)
    int KFR;             // keyframe cloud ring slots (>= surroundingKeyframeSearchNum + 2)
    int KFMAX;           // keyframe pose / Scan Context history capacity
    int cap_kc, cap_ks, cap_ko, cap_mc, cap_ms, cap_st;
    float4* outl_cam;    // [S][H]          outlier cloud, camera frame (adjustOutlierCloud)
    float4* kf_corner;   // [S][KFR][cap_kc] keyframe clouds, world frame
    float4* kf_surf;     // [S][KFR][cap_ks]
    float4* kf_outl;     // [S][KFR][cap_ko]
    int32_t* kf_n;       // [S][KFR][3]
    float* kf_pose;      // [S][KFMAX][6]   cloudKeyPoses6D (x,y,z,roll,pitch,yaw)
    float4* map_c;       // [S][cap_mc]     laserCloudCornerFromMap
    float4* map_s;       // [S][cap_ms]     laserCloudSurfFromMap
    float4* map_c_ds;    // [S][cap_mc]
    float4* map_s_ds;    // [S][cap_ms]
    float4* cur_raw_ds;  // [S][P]          laserCloudRawDS
    float4* cur_c_ds;    // [S][cap_less_sharp]
    float4* cur_s_ds;    // [S][H]
    float4* cur_o_ds;    // [S][H/5]
    float4* cur_st;      // [S][cap_st]     laserCloudSurfTotalLast
    float4* cur_st_ds;   // [S][cap_st]
    double* mo_part;     // [S][MO_BLOCKS][SLO_MO_PART] partial A^T A / A^T b (double-double) + count
    int cap_q;           // mapping queries per stream: cap_less_sharp + cap_st
    int32_t* mo_nn;      // [S][cap_q][5] 5-NN map indices of each query (-1: rejected)
    // hash grids: odometry "kd-tree" clouds (corner / surf) and the DS maps
    GridView g_oc, g_os, g_mc, g_ms;
    // ---- Scan Context history (Scancontext.h:99-106)
    double* sc_desc;     // [S][KFMAX][NR*NS]
    float* sc_ring;      // [S][KFMAX][NR]   invkeys (float, tree data)
    double* sc_ringd;    // [S][KFMAX][NR]
    double* sc_sect;     // [S][KFMAX][NS]
};

#ifndef SLO_DIAG
#define SLO_DIAG 0              // 1: kernels add phase cycle counts to StreamState::dbg
#endif
#define SLO_MO_BLOCKS 64
#define SLO_MO_PART 55          // 27 double-double sums (21 AtA + 6 AtB) + correspondence count
#define SLO_RECORD_FLOATS 40
#define SLO_KFMAX 4096          // keyframe pose / Scan Context history capacity per stream
#define SLO_SC_MAX_K 64         // NUM_CANDIDATES_FROM_TREE limit (C5 uses 50)
#define SLO_SC_MAX_SECTOR 64
#define SLO_SC_MAX_CELLS 1200   // PC_NUM_RING * PC_NUM_SECTOR limit (20 x 60)
// StreamState::err bits (sticky; read with slo_get(.., "err"))
#define SLO_ERR_KEYFRAMES 1     // keyframe pose history full: keyframe dropped
#define SLO_ERR_SC_HISTORY 2    // Scan Context history full: descriptor dropped
#define SLO_ERR_MAP_CAPACITY 4  // a map / cloud capacity clipped a cloud

// Locality-preserving bucket of cell (x, y, z): x-adjacent cells get adjacent
// buckets, so a ring walk reads each row of cells' bucket words from one cache
// line and their entries (stored in bucket order) as one contiguous run.
// Distinct cells can share a bucket (the index wraps mod T); walkers re-check
// cell membership, so collisions cost time, never correctness.
__host__ __device__ inline unsigned int grid_hash(int x, int y, int z, int T) {
    return ((unsigned int)x + (unsigned int)y * 1031u + (unsigned int)z * 620531u) & (unsigned int)(T - 1);
}
__host__ __device__ inline int grid_cell(float x, float inv) { return (int)floorf(x * inv); }

// XCD-aware 1-D grids for (stream, chunk) work: blocks b and b + 8 share an
// XCD (MI355X_MICROARCH.md "Workgroup dispatch"), so stream s goes to the XCD
// of blocks == s (mod 8) and all NB chunks of a stream share that XCD's L2.
// Grid size xcd_grid(S, NB); blocks with s >= S exit.
__host__ __device__ inline int xcd_grid(int S, int NB) { return ((S + 7) / 8) * 8 * NB; }
__device__ inline void xcd_stream_chunk(int b, int NB, int& s, int& chunk) {
    const int x = b & 7, k = b >> 3;
    s = (k / NB) * 8 + x;
    chunk = k % NB;
}

// Visit every grid point of stream s in the cells at Chebyshev ring r around
// cell (cx, cy, cz): f(point) for points of exactly those cells (buckets are
// shared by hash collisions, so membership is re-checked).
//
// The walk is latency-bound (hash -> bucket (offset, count) -> entries), so
// it is batched for memory-level parallelism: the ring's cells go in groups
// of GRING_BATCH whose bucket words are all loaded before any is used, and the
// group's entries are then visited as one flattened list, GRING_UNROLL
// independent loads at a time.  Visiting order does not matter to the callers
// (their results are order-independent: exact distances, ties by index).
#define GRING_BATCH 4
#define GRING_UNROLL 4
__device__ inline void grid_ring_cell(int r, int c, int& dx, int& dy, int& dz) {
    // c-th cell of Chebyshev ring r (r >= 1): the two full z-faces, then the
    // y-faces of the inner z-slices, then the x-edges of what remains
    const int w = 2 * r + 1, face = w * w;
    if (c < 2 * face) {
        dz = c < face ? -r : r;
        const int q = c % face;
        dy = q / w - r; dx = q % w - r;
        return;
    }
    c -= 2 * face;
    const int inner = 2 * r - 1;             // z-slices strictly inside
    if (c < 2 * w * inner) {
        dy = c < w * inner ? -r : r;
        const int q = c % (w * inner);
        dz = q / w - r + 1; dx = q % w - r;
        return;
    }
    c -= 2 * w * inner;                      // remaining: x = +-r, |y| < r, |z| < r
    dx = c < inner * inner ? -r : r;
    const int q = c % (inner * inner);
    dz = q / inner - r + 1; dy = q % inner - r + 1;
}

template <class F>
__device__ inline void grid_ring(const GridView& g, int s, int cx, int cy, int cz, int r, F&& f) {
    const size_t gb = (size_t)s * g.T;
    const int base = g.off[gb];
    const float4* E = g.ent + (size_t)s * g.es;
    const int ncell = r == 0 ? 1 : (2 * r + 1) * (2 * r + 1) * (2 * r + 1) - (2 * r - 1) * (2 * r - 1) * (2 * r - 1);
    for (int c0 = 0; c0 < ncell; c0 += GRING_BATCH) {
        int tx[GRING_BATCH], ty[GRING_BATCH], tz[GRING_BATCH], st[GRING_BATCH], pre[GRING_BATCH + 1];
#pragma unroll
        for (int k = 0; k < GRING_BATCH; ++k) {
            int dx = 0, dy = 0, dz = 0;
            if (r > 0 && c0 + k < ncell) grid_ring_cell(r, c0 + k, dx, dy, dz);
            tx[k] = cx + dx; ty[k] = cy + dy; tz[k] = cz + dz;
        }
        int m[GRING_BATCH];
#pragma unroll
        for (int k = 0; k < GRING_BATCH; ++k) {   // independent bucket loads
            const bool live = c0 + k < ncell;
            const unsigned int b = grid_hash(tx[k], ty[k], tz[k], g.T);
            m[k] = live ? g.cnt[gb + b] : 0;
            st[k] = live ? g.off[gb + b] - base : 0;
        }
        pre[0] = 0;
#pragma unroll
        for (int k = 0; k < GRING_BATCH; ++k) pre[k + 1] = pre[k] + m[k];
        const int tot = pre[GRING_BATCH];
        for (int t0 = 0; t0 < tot; t0 += GRING_UNROLL) {
            float4 p[GRING_UNROLL];
            int ckx[GRING_UNROLL], cky[GRING_UNROLL], ckz[GRING_UNROLL];
#pragma unroll
            for (int u = 0; u < GRING_UNROLL; ++u) {   // independent entry loads
                const int t = t0 + u;
                // the cell of flattened entry t: the last q with pre[q] <= t
                // (selects, not indexing: the small arrays stay in registers)
                int sk = st[0], pk = 0, ax = tx[0], ay = ty[0], az = tz[0];
#pragma unroll
                for (int q = 1; q < GRING_BATCH; ++q)
                    if (t >= pre[q]) { sk = st[q]; pk = pre[q]; ax = tx[q]; ay = ty[q]; az = tz[q]; }
                ckx[u] = ax; cky[u] = ay; ckz[u] = az;
                p[u] = t < tot ? E[sk + (t - pk)] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < GRING_UNROLL; ++u) {
                if (t0 + u >= tot) break;
                if (grid_cell(p[u].x, g.inv) != ckx[u] || grid_cell(p[u].y, g.inv) != cky[u] ||
                    grid_cell(p[u].z, g.inv) != ckz[u])
                    continue;
                f(p[u]);
            }
        }
    }
}

struct VgParams;
struct MapWs {  // VoxelGrid workspace
    size_t items = 0;
    unsigned long long *keys = nullptr, *keys2 = nullptr;
    unsigned int *vals = nullptr, *vals2 = nullptr;
    int *flags = nullptr, *rank = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    int32_t* off = nullptr;
    unsigned int* bounds = nullptr;
    VgParams* prm = nullptr;
    int32_t* errflag = nullptr;
    int32_t* h_total = nullptr;
};
struct HashGrid {
    int T = 0;
    float cell = 1.0f;
    size_t ent_stride = 0;
    int32_t *cnt = nullptr, *cur = nullptr, *off = nullptr;
    float4* ent = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
};

}  // namespace slo

struct slo_ctx {
    slo_config cfg;
    int dev = 0;
    int S = 0;
    hipStream_t stream = nullptr;
    std::string err;
    void* arena = nullptr;
    size_t arena_bytes = 0;
    slo::DevView v;
    slo::StreamState* h_st = nullptr;   // pinned host mirror
    int scan_index = 0;                 // scans processed by the batched pipeline
    int fa_frame_count = 0;             // FA frameCount (host-known, lockstep streams)
    bool fa_inited = false;
    double t_last_processing = -1;      // MO timeLastProcessing (lockstep streams)
    bool fa_published = false;
    // timing
    bool timing = false;
    struct KT { std::vector<hipEvent_t> ev; double total_ms = 0; int64_t n = 0; };
    std::map<std::string, KT> ktimes;
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
    // host staging for single-scan API
    void* h_stage = nullptr;
    size_t h_stage_bytes = 0;
    std::vector<char> h_view[16];       // backing store of the single-scan views
    int32_t h_ring[2][128];
    float4* d_in = nullptr;   // internal input buffer [S][P]
    int32_t* d_cnt = nullptr;
    // mapping workspaces
    slo::MapWs mws;
    slo::HashGrid grid_c, grid_s, grid_oc, grid_os;
    bool map_ready = false;
};

// launch helpers with optional per-kernel HIP-event timing
namespace slo {
void timing_begin(slo_ctx* ctx, const char* name, hipEvent_t* a);
void timing_end(slo_ctx* ctx, const char* name, hipEvent_t a);
int ip_run(slo_ctx* ctx);
int fa_features_run(slo_ctx* ctx);
int fa_odometry_run(slo_ctx* ctx, bool first_scan);
int vg_alloc(slo_ctx* ctx);
void vg_free(slo_ctx* ctx);
int vg_run(slo_ctx* ctx, const char* tag, const float4* in, size_t in_stride, const int32_t* d_n, int n_stride,
           float leaf, float4* out, size_t out_stride, int32_t* d_nout, int nout_stride, int out_cap);
int grid_alloc(slo_ctx* ctx, HashGrid& g, int T, size_t ent_stride, float cell);
GridView grid_view(const HashGrid& g);
void grid_free(HashGrid& g);
int grid_build(slo_ctx* ctx, HashGrid& g, const float4* pts, size_t stride, const int32_t* n, int n_stride);
int map_run(slo_ctx* ctx, const float4* d_points, const int32_t* d_counts);
int sc_make_run(slo_ctx* ctx, const float4* pts, size_t stride, const int32_t* n, int n_stride, int n_streams);
int sc_detect_run(slo_ctx* ctx);
int sc_detect_run_one(slo_ctx* ctx);
int pack_records_run(slo_ctx* ctx, float* d_out);
}  // namespace slo

#define SLO_LAUNCH(ctx, name, kernel, grid, block, shmem, ...)                        \
    do {                                                                              \
        hipEvent_t ev_a_ = nullptr;                                                   \
        if ((ctx)->timing) slo::timing_begin((ctx), name, &ev_a_);                    \
        hipLaunchKernelGGL(kernel, grid, block, shmem, (ctx)->stream, __VA_ARGS__);   \
        if ((ctx)->timing) slo::timing_end((ctx), name, ev_a_);                       \
    } while (0)
