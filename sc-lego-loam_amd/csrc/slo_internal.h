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

// The scan a batched call works on (device pointers [S][P] points, [S]
// counts), kept in device memory and set by k_set_io at the start of each
// call: kernels read it there, so a captured HIP graph replays on whatever
// buffers the next call names.
struct SloIo { const float4* pts; const int32_t* npts; double t_scan; };

// FeatureAssociation's IMU state of one stream (featureAssociation.cpp:85-158,
// imuQueLength = 200, utility.h:113): the ring of imuHandler messages with the
// shift / velocity / rotation AccumulateIMUShiftAndRotation integrates, and
// the per-scan quantities adjustDistortion, updateInitialGuess,
// TransformToEnd and integrateTransformation exchange.  imuShiftFromStart*Cur
// stays 0: LeGO-LOAM never calls ShiftToStartIMU, so the shift terms are the
// zero the constructor sets (kept literally).
#define SLO_IMU_QUE 200
struct ImuState {
    int32_t last;                       // imuPointerLast (-1: no message yet)
    int32_t last_iter;                  // imuPointerLastIteration
    int32_t iter_scan;                  // the value this scan's deskew starts from
    int32_t pad;
    float rollStart, pitchStart, yawStart;
    float veloStart[3];
    float rollCur, pitchCur, yawCur;    // the last deskewed point's (imu*Cur after adjustDistortion)
    float veloFromStartCur[3];
    float angLast[3], angFromStart[3];  // imuAngularRotation*Last, imuAngularFromStart*
    float rollLast, pitchLast, yawLast; // updateInitialGuess
    float shiftFromStart[3], veloFromStart[3];
    double time[SLO_IMU_QUE];
    float roll[SLO_IMU_QUE], pitch[SLO_IMU_QUE], yaw[SLO_IMU_QUE];
    float acc[3][SLO_IMU_QUE], velo[3][SLO_IMU_QUE], shift[3][SLO_IMU_QUE];
    float angVelo[3][SLO_IMU_QUE], angRot[3][SLO_IMU_QUE];
};

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
    int32_t kd_set;                       // this scan's odometry (re)built the "trees" (k_fa_sx_kd's gate)
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
    // sin/cos of transformTobeMapped (pointAssociateToMap's cRoll .. tZ),
    // kept with the pose by mo_prepare / mo_solve (computed once per pose,
    // not per query)
    float mo_trig[9];
    // transformFusion (transformFusion.cpp): /aft_mapped_to_init as it
    // decodes it (publishTF, MO:680-705) and its /integrated_to_init
    float tf_aft[6], tf_bef[6], integrated[6];
    // the transform a saved keyframe hands to the pose graph
    // (transformTobeMapped for the first, else transformAftMapped before
    // the estimate replaces it, MO:1541-1555)
    float kf_pre[6];
    // scan context
    int32_t sc_count, sc_tree_n, sc_counter;
    int32_t sc_wrote;   // the last makeAndSave stored its descriptor (0: the history was full)
    int32_t det_valid, det_loop_id, det_nn_idx, det_cand[64];
    float det_yaw;
    double det_min_dist;
    // a few streams: detect split over launches (slo_sc.hip) — the candidates'
    // distances, one workgroup each, and whether the pick is still to come
    double det_cdist[64];
    int32_t det_calign[64], det_pending;
    int32_t flags;
    int32_t err;
    int32_t err_map;   // the local-map selection's error bits until k_mo_concat folds them into err
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
    const SloIo* io;     // the input scan: io->pts [S][P], io->npts [S]
    const uint16_t* rings; // [S][P] ring per input point (cfg.use_cloud_ring), else unused
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
    int32_t* ex_cnt;     // [S][R][SLO_EX_CNT]: per sector (sharp, flat) candidate counts, [12] = staged in LDS
    int32_t* roff_last;  // [S][2][R+1] the same for corner_last / surf_last
    // x-sorted surf clouds (k_fa_sx_rings): each ring's segment of surf_last
    // / surf_next sorted by x, w = the point's index in the cloud (int bits)
    float4* sx_surf_last;    // [S][cap_less_flat]
    float4* sx_surf_next;    // [S][cap_less_flat]
    float4* sx_kd_corner;    // [S][cap_less_sharp] the corner "tree" cloud sorted by x (w = index)
    int32_t* sharp_perm;     // [S][cap_sharp] sharp points in x order (query grouping)
    int32_t* ind_surf;   // [S][cap_flat][3]   pointSearchSurfInd1..3 (Q9: exact ints)
    int32_t* ind_corner; // [S][cap_sharp][2]  pointSearchCornerInd1..2
    StreamState* st;     // [S]
    ImuState* imu;       // [S] (slo_batch_imu / slo_imu_handler)
    unsigned long long* wctr;   // [8] cumulative work counters (slo_get "work"): [0] Scan Context pairs whose
                                // distance was evaluated (k_sc_detect; the bench prices sc_detect's MFMA work),
                                // [1] / [2] points / voxels of the VoxelGrids' long voxels (k_vg_long)
    // ---- mapping (mapOptmization.cpp)
    int KFR;             // keyframe cloud ring slots (>= surroundingKeyframeSearchNum + 2)
    int KFMAX;           // keyframe pose / Scan Context history capacity
    int MAPK;            // keyframes the local map may hold (map_ids row length)
    int32_t* map_ids;    // [S][MAPK] loopClosureEnableFlag == false: surroundingExistingKeyPosesID
    int cap_kc, cap_ks, cap_ko, cap_mc, cap_ms, cap_st;
    int cap_kfs, cap_kfo;  // keyframe surf / outlier cloud slots (cfg.keyframe_cloud_cap)
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
    int32_t* tick;       // [S] arrivals of a fused odometry launch's search workgroups (k_fa_fused, 0 between launches)
    int cap_q;           // mapping queries per stream: cap_less_sharp + cap_st
    int32_t* mo_nn;      // [S][cap_q][5] 5-NN map indices of each query (-1: rejected)
    int32_t* mo_perm;    // [S][cap_q] the queries grouped by their body-frame 2 m cell (k_mo_perm): the order
                         // k_mo_knn takes them in (any order gives the same result)
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
#ifndef SLO_MAP_CELL
#define SLO_MAP_CELL 0.5f       // map grid cell (m, power of two): the 5-NN ball of 1 m spans SLO_MAP_R cells
#endif
#ifndef SLO_MAP_R
#define SLO_MAP_R 2
#endif
#ifndef SLO_MAP_TLOG2
#define SLO_MAP_TLOG2 19        // map grid buckets per stream (log2): ~0.2 occupied cells per bucket at
#endif                          // C3's ~145 k-point surf maps, so few hash collisions share a row's run
#define SLO_MO_PART 55          // 27 double-double sums (21 AtA + 6 AtB) + correspondence count
#define SLO_ODO_SURF_CELL 1.0f  // odometry surf grid cell (m, power of two)
#define SLO_ODO_SURF_R 5        // its search box radius in cells: covers sqrt(nearest_feature_search_sq_dist)
#define SLO_EX_CNT 16
#define SLO_KFMAX 4096          // keyframe pose / Scan Context history capacity per stream
#define SLO_SC_MAX_K 64         // NUM_CANDIDATES_FROM_TREE limit (C5 uses 50)
#define SLO_SC_MAX_SECTOR 64
#define SLO_SC_MAX_CELLS 1200   // PC_NUM_RING * PC_NUM_SECTOR limit (20 x 60)
// StreamState::err bits (sticky; read with slo_get(.., "err"))
#define SLO_MAPK_MAX 1024       // map_keyframes bound (radius branch)
#define SLO_ERR_KEYFRAMES 1     // keyframe pose history full: keyframe dropped
#define SLO_ERR_SC_HISTORY 2    // Scan Context history full: descriptor dropped
#define SLO_ERR_MAP_CAPACITY 4  // a map / cloud capacity clipped a cloud
#define SLO_ERR_INPUT 8         // slo_batch_pc2_unpack: a message exceeded max_points
#define SLO_ERR_SORT 16         // PCL-order sort (ring or batched VoxelGrid): an inconsistent step caught by a
                                // guard (slo_pclsort.h, slo_vgpcl.hip; never expected)

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

// Ball queries on a hash grid.  The x coefficient of grid_hash is 1, so the
// cells of one x-row (fixed y, z) occupy consecutive buckets, and the bucket
// offsets are an exclusive prefix sum over [S][T + 1] buckets: a row's cells
// [xa, xb] are ONE contiguous entry range [off[h(xa)], off[h(xb) + 1]) (two
// when the buckets wrap at T).  A ball query therefore walks rows, not cells:
// two offset loads and a run of entries per row.
//
// Rows of the (2R+1)^2 box around the query's cell are visited nearest first
// (GridRows: by gap = max(|dy|-1,0)^2 + max(|dz|-1,0)^2, then dy^2 + dz^2).
// With the caller's current bound b on the squared distance (it tightens as
// points are accepted):
//   * gap * cell^2 > b ends the walk: every later row is at least that far
//     (computed distances are monotone in the coordinate differences, and
//     these bounds are exact in float);
//   * a row whose exact float lower bound ((0 + ey^2) + ez^2) exceeds b is
//     skipped;
//   * within a row only the x cells that can still hold a point within b are
//     taken (with a safety margin: over-inclusion only costs a test).
// Buckets are shared by hash collisions, so cell membership is re-checked
// (each point is then visited at most once).  Callers' results are
// order-independent (exact distances, ties by index).
template <int R>
struct GridRows {
    static constexpr int N = (2 * R + 1) * (2 * R + 1);
    int8_t dy[N], dz[N];
    uint8_t gap[N];
    constexpr GridRows() : dy(), dz(), gap() {
        int k = 0, key[N] = {};
        for (int a = -R; a <= R; ++a)
            for (int b = -R; b <= R; ++b) {
                const int ga = a < 0 ? -a - 1 : (a > 0 ? a - 1 : 0), gb = b < 0 ? -b - 1 : (b > 0 ? b - 1 : 0);
                dy[k] = (int8_t)a; dz[k] = (int8_t)b; gap[k] = (uint8_t)(ga * ga + gb * gb);
                key[k] = gap[k] * 1024 + a * a + b * b;
                ++k;
            }
        for (int i = 1; i < N; ++i)   // insertion sort by key (stable)
            for (int j = i; j > 0 && key[j - 1] > key[j]; --j) {
                int t = key[j]; key[j] = key[j - 1]; key[j - 1] = t;
                int8_t u = dy[j]; dy[j] = dy[j - 1]; dy[j - 1] = u;
                u = dz[j]; dz[j] = dz[j - 1]; dz[j - 1] = u;
                uint8_t w = gap[j]; gap[j] = gap[j - 1]; gap[j - 1] = w;
            }
    }
};
template <int R>
__constant__ GridRows<R> kGridRows = GridRows<R>();

//
// Probe: the query's own cell is visited first, on its own (one bucket), so
// the walk starts with the bound its points give instead of the caller's
// initial radius; the row walk then skips that cell (each point is still
// visited once).
#define GBALL_UNROLL 4
// grid_ball_rows: the same walk restricted to rows k = k0, k0 + ks, ... < k1
// (and the probe cell only if `probe`), so several lanes can share one query
// (each bound by its own best; correct because a point a lane skips is
// farther than that lane's best, hence than the joint best).
template <int R, int U = GBALL_UNROLL, class B, class F>
__device__ inline void grid_ball_rows(const GridView& g, int s, float qx, float qy, float qz, int k0, int k1, int ks,
                                      bool probe, B&& bound, F&& f) {
    const float inv = g.inv, cell = g.cell, c2 = cell * cell;
    const int cx = grid_cell(qx, inv), cy = grid_cell(qy, inv), cz = grid_cell(qz, inv);
    const size_t gb = (size_t)s * (g.T + 1);
    const int base = g.off[gb];
    const float4* E = g.ent + (size_t)s * g.es;
    static_assert(GridRows<R>().dy[0] == 0 && GridRows<R>().dz[0] == 0, "row 0 is the probed cell's row");
    if (probe) {
        const int h0 = (int)grid_hash(cx, cy, cz, g.T);
        const int p0 = g.off[gb + h0] - base, p1 = g.off[gb + h0 + 1] - base;
        for (int e = p0; e < p1; e += U) {
            float4 p[U];
#pragma unroll
            for (int u = 0; u < U; ++u) p[u] = E[min(e + u, p1 - 1)];   // unconditional: all U loads in flight
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (e + u >= p1) break;
                if (grid_cell(p[u].x, inv) != cx || grid_cell(p[u].y, inv) != cy || grid_cell(p[u].z, inv) != cz) continue;
                f(p[u]);
            }
        }
    }
    for (int k = k0; k < min(k1, GridRows<R>::N); k += ks) {
        const float b = bound();
        if ((float)kGridRows<R>.gap[k] * c2 > b) break;
        const int dy = kGridRows<R>.dy[k], dz = kGridRows<R>.dz[k];
        const int yy = cy + dy, zz = cz + dz;
        const float ey = dy > 0 ? (float)yy * cell - qy : (dy < 0 ? qy - (float)(yy + 1) * cell : 0.0f);
        const float ez = dz > 0 ? (float)zz * cell - qz : (dz < 0 ? qz - (float)(zz + 1) * cell : 0.0f);
        float lb = ey * ey;
        lb += ez * ez;
        if (lb > b) continue;
        const float rx = sqrtf((b - lb) * 1.0001f + 1e-5f * b) + 1e-3f;
        const int xa = max(cx - R, grid_cell(qx - rx, inv)), xb = min(cx + R, grid_cell(qx + rx, inv));
        const int h = (int)grid_hash(xa, yy, zz, g.T), len = xb - xa + 1;
        const int h2 = min(h + len, g.T);
        int e0 = g.off[gb + h] - base, e1 = g.off[gb + h2] - base;
        const int w1 = h + len - h2;   // buckets wrapped to the table start
        const int f1 = w1 > 0 ? g.off[gb + w1] - base : 0;
        for (int pass = 0; pass < 2; ++pass) {
            for (int e = e0; e < e1; e += U) {
                float4 p[U];
#pragma unroll
                for (int u = 0; u < U; ++u) p[u] = E[min(e + u, e1 - 1)];   // unconditional: all U loads in flight
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (e + u >= e1) break;
                    const int px = grid_cell(p[u].x, inv);
                    if (grid_cell(p[u].y, inv) != yy || grid_cell(p[u].z, inv) != zz || px < xa || px > xb ||
                        (k == 0 && px == cx)) continue;   // k == 0: the probed cell's row (dy = dz = 0)
                    f(p[u]);
                }
            }
            if (w1 <= 0) break;
            e0 = 0; e1 = f1;
        }
    }
}


template <int R, int U = GBALL_UNROLL, class B, class F>
__device__ inline void grid_ball(const GridView& g, int s, float qx, float qy, float qz, B&& bound, F&& f) {
    grid_ball_rows<R, U>(g, s, qx, qy, qz, 0, GridRows<R>::N, 1, true, bound, f);
}

// ---- loop-closure verification (slo_lc.hip; mapOptmization.cpp:841-1110)
#define SLO_LC_MAX_N 64                      // historyKeyframeSearchNum limit
#define SLO_LC_SEG (2 * SLO_LC_MAX_N + 1)    // submap keyframes id-N .. id+N
// per stream; the int32 counts come first (vg_run / grid_build read them at
// an int32 stride of sizeof(LcState) / 4)
struct LcState {
    int32_t used;                  // archive points in use
    int32_t rs_id, sc_id, latest;  // candidates of the last select; newest keyframe
    int32_t n_src_raw, n_src, n_raw, n_tgt;   // source before / after the intensity filter; submap raw / DS
    int32_t active, iter, converged, pass;
    int32_t nseg, src_off, pad0, pad1;
    int32_t seg_off[SLO_LC_SEG + 1];          // submap prefix: keyframe seg k -> [seg_off[k], seg_off[k+1])
    int32_t seg_src[SLO_LC_SEG];              // its archive offset
    float seg_trig[SLO_LC_SEG][9];            // cos/sin roll, pitch, yaw + x, y, z of its pose
    float src_trig[9];                        // the source's pose (RS: newest keyframe, SC: the candidate)
    float T[16], Ti[16];                      // final transformation, last increment (row-major)
    double prev_mse;
};
struct LcView {
    int A;             // archive / submap capacity per stream (cfg.loop_archive_points)
    int cap_src;       // source capacity per stream
    float4* kfa;       // [S][A] keyframe archive: per keyframe corner DS then surf DS, body frame
    int32_t* kmeta;    // [S][KFMAX][3] archive offset, n corner, n surf
    double* ktime;     // [S][KFMAX] cloudKeyPoses6D.time
    float4* src;       // [S][cap_src] ICP source (input_)
    float4* src_t;     // [S][cap_src] input_transformed
    int32_t* corr_j;   // [S][cap_src] nearest target index (-1: none / rejected)
    float* corr_d;     // [S][cap_src] its squared distance
    float4* raw;       // [S][A] submap before VoxelGrid
    float4* tgt;       // [S][A] submap after VoxelGrid (ICP target)
    LcState* st;       // [S]
    slo_loop_result* res;   // [S][2] RS, SC
    int32_t* n_active; // live ICP jobs
    GridView g;        // hash grid over tgt
};

struct VgParams;
struct MapWs {  // VoxelGrid workspace (slo_vg.hip), sized on the host from the input strides only
    size_t items = 0;             // S * largest input stride so far
    size_t tiles = 0;             // S * largest tile count per stream so far
    unsigned int *keys = nullptr, *keys2 = nullptr;   // radix-pass ping-pong
    unsigned int *vals = nullptr, *vals2 = nullptr;
    int* cnt = nullptr;           // [S][256][maxT] digit counts -> scatter bases
    int* hcnt = nullptr;          // [S][maxT] voxel heads per tile -> ranks
    int4* longv = nullptr;        // long voxels (stream, first item, rank)
    size_t nlong_cap = 0;
    int32_t* meta = nullptr;      // [total, -, long-voxel count]
    int32_t* nvox = nullptr;      // [S] voxels per stream (before the output clip)
    int32_t* off = nullptr;
    unsigned int* bounds = nullptr;
    VgParams* prm = nullptr;
    int32_t* errflag = nullptr;
    // single-pass scatter (ctx->vg_onesweep): per-stream digit histograms of every
    // pass and their bases, tile tickets / per-XCD tile offsets, look-back status
    int32_t* gh = nullptr;        // [S][4][256] digit counts (zeroed again by their scan)
    int32_t* gbase = nullptr;     // [S][4][256] first output position of each digit
    int32_t* osw = nullptr;       // [32] tickets (pass, XCD), [8] tiles per XCD, [S] XCD tile offsets
    unsigned long long* lbk = nullptr;   // [tiles][256] (tag, inclusive flag, count)
};
#define VG_MAXG 8   // VoxelGrid filters one call can batch (vg_run_groups): per-virtual-stream arrays hold VG_MAXG * S
struct PSeg;
struct PRes;
struct PclWs {  // PCL-order VoxelGrid sort (slo_vgpcl.hip), sized from the input strides only
    size_t items = 0, tiles = 0;
    int* ctr = nullptr;           // [16] per-call counters (ranges, chunks, finish entries)
    int* cstat = nullptr;         // [16] cumulative: [0] ranges the one-lane fallback took, [1] inconsistent
                                  // wave-sort steps, [2] / [3] inconsistent tail cuts / partners (1-3 must stay 0)
    int32_t* serr = nullptr;      // [S] sticky per stream: SLO_ERR_SORT (a guard of 1-3 fired on one of its
                                  // ranges), SLO_ERR_MAP_CAPACITY (2^24 or more items: not sorted); folded
                                  // into StreamState::err (k_pc_fold_err, slo_get "err")
    unsigned long long* pstat = nullptr;   // [32] cumulative work counters (slo_vgpcl.hip PW_*)
    int32_t* nfin = nullptr;      // [S] finite points per stream
    PSeg* seg[2] = {nullptr, nullptr};     // ranges of the current / next level
    PRes* res = nullptr;          // per range of the current level: pivot, m, cuts
    int* cseg[2] = {nullptr, nullptr};     // chunk -> range
    int2* ccnt = nullptr;         // per chunk stopper counts -> prefixes
    int2* wl = nullptr;           // finish entries (f, size | depth << 24): four lists by size
    size_t wcap0 = 0, wcapk = 0;  // capacity of list 0 and of lists 1..3
    int* tcnt = nullptr;          // [S][maxT] finite points per tile -> prefixes
};
struct HashGrid {
    int T = 0;
    float cell = 1.0f;
    size_t ent_stride = 0;
    int32_t *cnt = nullptr, *off = nullptr;
    int32_t* bsum = nullptr;   // per-stream block sums of the offset scan
    float4* ent = nullptr;
};

}  // namespace slo

namespace slo { struct SloPipe; }
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
    std::string timing_only;            // non-empty: time only launches of these names (slo_timing_filter)
    std::vector<std::string> stamp_names;   // timing_only split at commas
    struct KT { std::vector<hipEvent_t> ev; double total_ms = 0; int64_t n = 0; };
    std::map<std::string, KT> ktimes;
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
    // with a filter (timing_only), the named kernel is timed by device
    // timestamps written in-stream around each launch (k_stamp: the device's
    // constant-rate wall clock), so the timing survives graph capture
    unsigned long long* d_stamp = nullptr;   // [SLO_STAMP_CAP] (timestamp, name id) + [1] counter
    double stamp_khz = 0;
    // host staging for single-scan API
    void* h_stage = nullptr;
    size_t h_stage_bytes = 0;
    std::vector<char> h_view[16];       // backing store of the single-scan views
    int32_t h_ring[2][128];
    float4* d_in = nullptr;   // internal input buffer [S][P]
    uint16_t* d_ring_in = nullptr;   // internal ring buffer [S][P] (single-scan useCloudRing)
    int32_t* d_cnt = nullptr;
    // mapping workspaces
    slo::MapWs mws;
    slo::PclWs pws;
    // contexts of a few streams run the mapping step's local-map VoxelGrids on
    // a side stream beside the current scan's (slo_map.hip map_run): its own
    // workspaces, swapped in while its launches are issued (VgSide)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    slo::MapWs mws2;
    slo::PclWs pws2;
    slo::HashGrid grid_c, grid_s, grid_oc, grid_os;
    bool map_ready = false;
    // loop-closure verification (cfg.loop_verify)
    slo::LcView lc{};
    slo::HashGrid grid_lc;
    int32_t* h_lc_active = nullptr;     // pinned copy of lc.n_active
    // pose-graph back end (cfg.pose_graph, slo_pgwire.hip)
    std::vector<slo_pg*> pg;            // one graph per stream
    std::vector<char> pg_pending;       // aLoopIsClosed
    std::vector<std::vector<float>> pg_snap;   // key poses of the last save, for correctPoses without a new keyframe
    float* d_pg_poses = nullptr;
    size_t pg_cap = 0;
    bool mapped_now = false;            // this batch step ran the mapping stage
    bool imu_fed = false;               // slo_batch_imu / slo_imu_handler ran on this context
    bool modes_used = false;            // a Mode S entry point ran on it (Mode S carries no IMU ring: the two
                                        // refuse each other, SLO_E_STATE)
    // the input slot (DevView::io) and the captured steps of slo_batch_process
    // (slo_ctx.hip): step kind (0: no mapping, 1: mapping) x the layout of
    // the odometry ping-pong halves (fa_swap_last)
    slo::SloIo* d_io = nullptr;
    bool graphs = true;                 // slo_graph_mode
    int graph_seen[2] = {0, 0};         // the step kind has run once (its workspaces are sized)
    hipGraphExec_t graph_exec[4] = {nullptr, nullptr, nullptr, nullptr};
    slo::DevView graph_v[4];            // the kernel-argument view each graph was captured with
    unsigned int graph_ws[4] = {0, 0, 0, 0};
    unsigned int ws_gen = 0;            // bumped whenever a workspace behind a captured pointer moves
    const float4* pp_corner0 = nullptr; // corner_last of layout 0
    bool vg_onesweep = false;           // VoxelGrid sort by single-pass scatters (env SLO_VG_ONESWEEP=1 at creation)
    // the odometry's preparation of the next scan's search structures (the
    // surf rings' x-order, the corner tree's x-order, the surf hash grid;
    // slo_odom.hip fa_prep_*): a batched step of a few streams defers it to
    // the next step, which runs it on prep_stream beside its projection and
    // features; any other odometry entry runs a pending one in-stream first
    bool prep_pending = false;
    hipStream_t prep_stream = nullptr;
    hipEvent_t ev_pfork = nullptr, ev_pjoin = nullptr;
    // the less-flat VoxelGrids of a batched step of a few streams, forked
    // beside its odometry on ring_stream (fa_features_run) and joined before
    // the odometry's end (fa_ring_join); created with prep_stream
    bool ring_pending = false;
    // the local map's half of this step's mapping, issued on `side` at the
    // step's start (map_side_fork, slo_map.hip); map_run joins it
    bool map_forked = false;
    bool map_fork_ready = false;   // map_fork_prepare made the side stream and sized its workspaces
    hipStream_t ring_stream = nullptr;
    hipEvent_t ev_rfork = nullptr, ev_rjoin = nullptr;
    // the mapping step's workspaces are sized on the first entry that can map
    // (map_ws_ensure), so a Mode S front or odometry context never holds them
    bool map_ws_ready = false;
    // slo_pipeline: the front end and the odometry on two internal contexts,
    // each on its own stream, this context the mapping stage (slo_ctx.hip)
    slo::SloPipe* pipe = nullptr;
};

// With at most SLO_PREP_DEFER_STREAMS streams a batched step defers the
// odometry's preparation of the next scan's searches to the next step, forked
// beside its projection and features (slo_ctx.hip step_launches)
#ifndef SLO_PREP_DEFER_STREAMS
#define SLO_PREP_DEFER_STREAMS 8
#endif
#ifndef SLO_MAP_FORK
#define SLO_MAP_FORK 1   // such a step also issues its mapping's local-map half at its start (map_side_fork)
#endif
#ifndef SLO_MAP_FORK_G
#define SLO_MAP_FORK_G 3   // the forked half's VoxelGrids (map_groups order): both local maps and the raw scan
#endif

// launch helpers with optional per-kernel HIP-event timing
namespace slo {
void timing_begin(slo_ctx* ctx, const char* name, hipEvent_t* a);
bool timing_on(const slo_ctx* ctx, const char* name);
void timing_end(slo_ctx* ctx, const char* name, hipEvent_t a);
struct PgTf { float t[6]; };
int pg_alloc(slo_ctx* ctx);
void pg_free(slo_ctx* ctx);
int pg_after_mapping(slo_ctx* ctx);
int pg_after_loops(slo_ctx* ctx);
int ip_run(slo_ctx* ctx);
int fa_features_run(slo_ctx* ctx, bool fork = false);
int fa_ring_join(slo_ctx* ctx);    // a forked step's less-flat VoxelGrids, joined to ctx->stream
int fa_ring_init(slo_ctx* ctx);    // ring_stream and its events (slo_batch_process, outside captures)
int fa_odometry_run(slo_ctx* ctx, bool first_scan, bool fuse = true, bool defer = false);
void fa_swap_last(slo_ctx* ctx);
int fa_prep_fork(slo_ctx* ctx);    // a pending preparation on prep_stream (forked from / joined to ctx->stream)
int fa_prep_join(slo_ctx* ctx);
void fa_prep_free(slo_ctx* ctx);
int fa_prep_init(slo_ctx* ctx);    // prep_stream and its two events (at creation, never inside a capture)
int vg_alloc(slo_ctx* ctx);
void vg_free(slo_ctx* ctx);
int vg_ws_reinit(slo_ctx* ctx);    // the stream-ordered initialisation of the VoxelGrid workspaces, again
void pcl_free(slo_ctx* ctx);
int pcl_fold_err(slo_ctx* ctx);    // PclWs::serr of both sort workspaces into StreamState::err (slo_vgpcl.hip)
void vg_side_free(slo_ctx* ctx);   // the side stream of map_run and its workspaces (slo_vg.hip)
int vg_run(slo_ctx* ctx, const char* tag, const float4* in, size_t in_stride, const int32_t* d_n, int n_stride,
           float leaf, float4* out, size_t out_stride, int32_t* d_nout, int nout_stride, int out_cap);
int grid_alloc(slo_ctx* ctx, HashGrid& g, int T, size_t ent_stride, float cell);
GridView grid_view(const HashGrid& g);
void grid_free(HashGrid& g);
int grid_build(slo_ctx* ctx, HashGrid& g, const float4* pts, size_t stride, const int32_t* n, int n_stride);
int map_run(slo_ctx* ctx);
bool map_fork_ok(const slo_ctx* ctx);   // a few-stream PCL-order context: its steps fork the local map's half
int map_side_fork(slo_ctx* ctx);        // (step_launches, before the projection)
int map_fork_prepare(slo_ctx* ctx);     // its side stream and workspaces (slo_batch_process, outside captures)
int map_ws_presize(slo_ctx* ctx);  // the mapping step's VoxelGrid / sort workspaces (slo_map.hip)
int map_ws_ensure(slo_ctx* ctx);   // map_ws_presize once, from an entry point that can map, before any capture
// slo_pipeline (slo_ctx.hip): one scan through the three stages; the stage
// contexts; the stage that computes a slo_get field; freeing it all
int pipe_step(slo_ctx* ctx, const void* d_points, const int32_t* d_counts, double t_scan);
std::vector<slo_ctx*> pipe_stages(slo_ctx* ctx);
slo_ctx* pipe_stage_of(slo_ctx* ctx, const std::string& name);
void pipe_free(slo_ctx* ctx);
struct VgGroup;
int vg_presize(slo_ctx* ctx, const VgGroup* groups, int G);
int pcl_presize(slo_ctx* ctx, int SV, size_t items, size_t maxT);
void graphs_drop(slo_ctx* ctx);
int imu_init(slo_ctx* ctx);
int sc_make_run(slo_ctx* ctx, const float4* pts, size_t stride, const int32_t* n, int n_stride, int n_streams);
// the SCManager helpers on device data (slo_map.hip): op 0 make (pts, stride, n -> desc, ring, sector),
// 1 keys (desc -> ring, sector), 2 align (vkey1, vkey2 -> shift), 3 direct (sc1, sc2 -> dist),
// 4 distance (sc1, sc2 -> dist, shift); nitems descriptors / pairs, contiguous
int sc_api_run(slo_ctx* ctx, int op, int nitems, const void* in1, const void* in2, size_t stride, const int32_t* n,
               void* out1, void* out2, void* out3);
int sc_detect_run(slo_ctx* ctx);
int sc_detect_run_one(slo_ctx* ctx);
int pack_records_run(slo_ctx* ctx, float* d_out);
int lc_alloc(slo_ctx* ctx);
void lc_free(slo_ctx* ctx);
int lc_archive_run(slo_ctx* ctx, double t_scan);
int lc_run(slo_ctx* ctx);
int lc_icp_run(slo_ctx* ctx, const float4* src, size_t src_stride, const int32_t* nsrc, const float4* tgt,
               size_t tgt_stride, const int32_t* ntgt);
}  // namespace slo

#define SLO_STAMP_CAP 65536

#define SLO_LAUNCH(ctx, name, kernel, grid, block, shmem, ...)                        \
    do {                                                                              \
        hipEvent_t ev_a_ = nullptr;                                                   \
        const bool tm_ = (ctx)->timing && slo::timing_on((ctx), name);                \
        if (tm_) slo::timing_begin((ctx), name, &ev_a_);                              \
        hipLaunchKernelGGL(kernel, grid, block, shmem, (ctx)->stream, __VA_ARGS__);   \
        if (tm_) slo::timing_end((ctx), name, ev_a_);                                 \
    } while (0)
