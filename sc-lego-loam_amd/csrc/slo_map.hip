// slo_map.hip — scan-to-map optimisation of mapOptmization.cpp for a batch
// of S streams: transformAssociateToMap (MO:397-482), the recent-50 keyframe
// local map (MO:1122-1231, loopClosureEnableFlag branch including its
// latestFrameID bookkeeping), downsampleCurrentScan (MO:1233-1263),
// cornerOptimization / surfOptimization / LMOptimization (MO:1265-1499),
// scan2MapOptimization (MO:1501-1522), transformUpdate (MO:484-517) and
// saveKeyFramesAndFactor (MO:1525-1638, GTSAM replaced by its fixed point:
// with only prior + consistent between-factors the newest estimate is its
// initial value) with the Scan Context descriptor build of the keyframe
// (Scancontext.cpp:151-244).
//
// Layout: keyframe clouds are stored once in their body frame and
// transformed with the current key pose when the local map is assembled
// (transformPointCloud, MO:566-596): between correctPoses the poses do not
// change, so this equals the reference's transform at deque insertion, and a
// correctPoses (slo_set_key_poses) takes effect at the next assembly, as the
// reference's cleared-and-rebuilt deque does (MO:1642-1664).  Each LM iteration is two launches: every
// workgroup of a stream takes a contiguous slice of its corner+surf queries,
// does the exact 5-NN in the hash grid, the 3x3 Jacobi / 5x3 QR of the
// reference and accumulates A^T A, A^T b in double-double (slo_ddsum.h); a
// per-stream lane then merges the slices, rounds once to float and runs the
// 6x6 QR / degeneracy projection.
#include "slo_internal.h"
#include "slo_vgcommon.h"
#include <memory>
#include "slo_libm.h"
#include "slo_pose.h"
#include "slo_pose_wave.h"
#include "slo_linalg.h"
#include "slo_scdist.h"
#include <float.h>

namespace slo {

using slo_pose::P4;
#define ST_STRIDE ((int)(sizeof(StreamState) / sizeof(int32_t)))

// ---------------------------------------------------------------- prepare
// pointAssociateToMap's sin/cos (MO:521-532) of transformTobeMapped into st.mo_trig
__device__ inline void mo_store_trig(StreamState& st) {
    const float* t = st.transformTobeMapped;
    float* o = st.mo_trig;
    o[0] = slo_libm::sinf_(t[0]); o[1] = slo_libm::cosf_(t[0]);
    o[2] = slo_libm::sinf_(t[1]); o[3] = slo_libm::cosf_(t[1]);
    o[4] = slo_libm::sinf_(t[2]); o[5] = slo_libm::cosf_(t[2]);
    o[6] = t[3]; o[7] = t[4]; o[8] = t[5];
}

__device__ inline unsigned int ford(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float unord(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// the keyframe ids of stream s's local map, in concatenation order
__device__ inline const int32_t* mo_map_ids(const DevView& v, int s, const StreamState& st) {
    return v.cfg.loop_closure_enable ? st.recent_ids : v.map_ids + (size_t)s * v.MAPK;
}

// extractSurroundingKeyFrames, loopClosureEnableFlag == false (MO:1167-1222),
// one workgroup per stream:
//  1. radiusSearch(currentRobotPosPoint, surroundingKeyframeSearchRadius) over
//     cloudKeyPoses3D: FLANN's L2 of (query - point), kept when < (float)r^2;
//     currentRobotPosPoint is the last run's transformAftMapped position
//     (MO:1527-1529; the keyframe round trip leaves translations unchanged);
//  2. downSizeFilterSurroundingKeyPoses (VoxelGrid 1.0, intensity = key index):
//     the hits sorted by (voxel index, key index) in LDS; a voxel's id is
//     (int) of the float mean of its members' indices (an exact integer sum);
//     voxels in index order;
//  3. surroundingExistingKeyPosesID: ids no longer present erased in order,
//     new ids appended in voxel order (MO:1181-1214).
// A bounding box of more than INT32_MAX voxels (PCL returns its input then,
// radius >> 1000 leaves) is not supported and flags SLO_ERR_MAP_CAPACITY.
constexpr int kSurrMax = 4096;   // hits sorted in LDS (<= SLO_KFMAX)
__device__ void mo_surrounding_radius(const DevView& v, int s, StreamState& st) {
    __shared__ unsigned long long key[kSurrMax];
    __shared__ int nsel, ds_n, bad;
    __shared__ unsigned int bmin[3], bmax[3];
    __shared__ int ds_id[kSurrMax];
    const int nk = min(st.n_keyframes, v.KFMAX);
    const float qx = st.transformAftMapped[3], qy = st.transformAftMapped[4], qz = st.transformAftMapped[5];
    const float r2 = (float)((double)v.cfg.surrounding_keyframe_search_radius *
                             (double)v.cfg.surrounding_keyframe_search_radius);
    if (threadIdx.x == 0) {
        nsel = 0; bad = 0;
        for (int a = 0; a < 3; ++a) { bmin[a] = ford(FLT_MAX); bmax[a] = ford(-FLT_MAX); }
    }
    __syncthreads();
    const float* kp = v.kf_pose + (size_t)s * v.KFMAX * 6;
    for (int i = threadIdx.x; i < nk; i += blockDim.x) {
        const float px = kp[6 * i], py = kp[6 * i + 1], pz = kp[6 * i + 2];
        const float d0 = qx - px, d1 = qy - py, d2 = qz - pz;
        float d = 0.0f;
        d += d0 * d0;
        d += d1 * d1;
        d += d2 * d2;
        if (d < r2) {
            const int j = atomicAdd(&nsel, 1);
            key[j] = (unsigned long long)i;   // index now, voxel index after the bounds
            atomicMin(&bmin[0], ford(px)); atomicMin(&bmin[1], ford(py)); atomicMin(&bmin[2], ford(pz));
            atomicMax(&bmax[0], ford(px)); atomicMax(&bmax[1], ford(py)); atomicMax(&bmax[2], ford(pz));
        }
    }
    __syncthreads();
    const int n = nsel;
    const float inv = 1.0f / v.cfg.leaf_surrounding_key_poses;
    const float mn[3] = {unord(bmin[0]), unord(bmin[1]), unord(bmin[2])};
    const float mx[3] = {unord(bmax[0]), unord(bmax[1]), unord(bmax[2])};
    const long long dx = (long long)((mx[0] - mn[0]) * inv) + 1, dy = (long long)((mx[1] - mn[1]) * inv) + 1,
                    dz = (long long)((mx[2] - mn[2]) * inv) + 1;
    const int minb0 = (int)floorf(mn[0] * inv), minb1 = (int)floorf(mn[1] * inv), minb2 = (int)floorf(mn[2] * inv);
    const int divx = (int)floorf(mx[0] * inv) - minb0 + 1, divy = (int)floorf(mx[1] * inv) - minb1 + 1;
    if (n > 0 && dx * dy * dz > 2147483647LL) {
        if (threadIdx.x == 0) st.err_map |= SLO_ERR_MAP_CAPACITY;
        bad = 1;
    }
    // (voxel index << 32 | key index), padded to a power of two with ~0
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int j = threadIdx.x; j < n2; j += blockDim.x) {
        if (j < n) {
            const int i = (int)key[j];
            const float px = kp[6 * i], py = kp[6 * i + 1], pz = kp[6 * i + 2];
            const int i0 = (int)(floorf(px * inv) - (float)minb0), i1 = (int)(floorf(py * inv) - (float)minb1),
                      i2 = (int)(floorf(pz * inv) - (float)minb2);
            const unsigned int idx = (unsigned int)(i0 + i1 * divx + i2 * divx * divy);
            key[j] = ((unsigned long long)idx << 32) | (unsigned int)i;
        } else {
            key[j] = ~0ull;
        }
    }
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1)          // bitonic sort, ascending
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < n2; t += blockDim.x) {
                const int u = t ^ j;
                if (u > t) {
                    const unsigned long long a = key[t], b = key[u];
                    if (((t & k) == 0) == (a > b)) { key[t] = b; key[u] = a; }
                }
            }
            __syncthreads();
        }
    if (threadIdx.x == 0) {
        // voxel centroids' intensity, voxels in index order
        int m = 0;
        for (int j = 0; j < n && !bad;) {
            const unsigned int vox = (unsigned int)(key[j] >> 32);
            float sum = 0.0f;
            int c = 0;
            while (j < n && (unsigned int)(key[j] >> 32) == vox) { sum += (float)(unsigned int)key[j]; ++c; ++j; }
            ds_id[m++] = (int)(sum / (float)c);
        }
        ds_n = m;
        // the existing list: erase what left the region, append what entered
        int32_t* ex = v.map_ids + (size_t)s * v.MAPK;
        int ne = st.recent_n, w = 0;
        for (int i = 0; i < ne; ++i) {
            bool keep = false;
            for (int j = 0; j < m; ++j) if (ds_id[j] == ex[i]) { keep = true; break; }
            if (keep) ex[w++] = ex[i];
        }
        ne = w;
        for (int j = 0; j < m; ++j) {
            bool have = false;
            for (int i = 0; i < ne; ++i) if (ex[i] == ds_id[j]) { have = true; break; }
            if (have) continue;
            if (ne < v.MAPK) ex[ne++] = ds_id[j];
            else st.err_map |= SLO_ERR_MAP_CAPACITY;
        }
        st.recent_n = ne;
        // a keyframe whose cloud slot a newer keyframe reused
        for (int i = 0; i < ne; ++i)
            if (ex[i] < nk - v.KFR) st.err_map |= SLO_ERR_MAP_CAPACITY;
    }
}

// part: 1 the current scan's half (the outlier cloud's axes, the odometry
// hand-off and transformAssociateToMap), 2 the local map's half
// (extractSurroundingKeyFrames' selection and the map sizes: state the last
// mapping step left, none of the current scan's), 3 both.  A few-stream step
// runs half 2 on the side stream from its start (map_side_fork); the halves
// write disjoint StreamState fields, the map half's errors into err_map
// (k_mo_concat folds them after the join)
__global__ void k_mo_prepare(DevView v, int part) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    // adjustOutlierCloud (FA:1746-1757): lidar -> camera axes
    if (part & 1)
        for (int i = threadIdx.x; i < st.outlier_count; i += blockDim.x) {
            float4 p = v.outlier[(size_t)s * v.H + i];
            v.outl_cam[(size_t)s * v.H + i] = make_float4(p.y, p.z, p.x, p.w);
        }
    // extractSurroundingKeyFrames without loop closure: the radius branch
    // reads the pose of the last run (transformAftMapped)
    if ((part & 2) && !v.cfg.loop_closure_enable && st.n_keyframes > 0) mo_surrounding_radius(v, s, st);
    if (threadIdx.x >= 64) return;
    // laserOdometryHandler (via the tf round trip), transformAssociateToMap
    // and pointAssociateToMap's sin/cos, their trig side by side on wave 0's
    // lanes (slo_pose_wave.h); lane 0 stores
    if (part & 1) {
        float ts[6], bef[6], aft[6], sum[6], inc[6], tbm[6];
        for (int k = 0; k < 6; ++k) {
            ts[k] = st.transformSum[k]; bef[k] = st.transformBefMapped[k]; aft[k] = st.transformAftMapped[k];
        }
        slo_pose::odom_handoff_w(ts, sum);
        slo_pose::associate_to_map_w(sum, bef, aft, inc, tbm);
        const float a3[3] = {tbm[0], tbm[1], tbm[2]};
        float sn[3], cs[3];
        slo_pose::wave_sincos<3>(a3, sn, cs);
        if (threadIdx.x != 0) return;
        for (int k = 0; k < 6; ++k) {
            st.mo_sum[k] = sum[k]; st.transformTobeMapped[k] = tbm[k];
        }
        for (int k = 3; k < 6; ++k) st.transformIncre[k] = inc[k];   // associate_to_map writes incre[3..5]
        float* o = st.mo_trig;   // mo_store_trig
        o[0] = sn[0]; o[1] = cs[0]; o[2] = sn[1]; o[3] = cs[1]; o[4] = sn[2]; o[5] = cs[2];
        o[6] = tbm[3]; o[7] = tbm[4]; o[8] = tbm[5];
    }
    if (threadIdx.x != 0) return;
    if (part & 1) {
        st.mo_ran = 1;
        st.kf_saved = 0;
        st.mo_iters = 0;
        st.mo_converged = 0;
    }
    if (!(part & 2)) return;
    // extractSurroundingKeyFrames: recent keyframe deque
    const int nk = st.n_keyframes;
    const int N = v.cfg.surrounding_keyframe_search_num;
    if (!v.cfg.loop_closure_enable) {
        // list built above
    } else if (nk > 0) {
        if (st.recent_n < N) {
            int cnt = 0;
            int ids[64];
            for (int i = nk - 1; i >= 0; --i) {
                ids[cnt++] = i;  // push_front order reversed below
                if (cnt >= N) break;
            }
            for (int k = 0; k < cnt; ++k) st.recent_ids[k] = ids[cnt - 1 - k];
            st.recent_n = cnt;
        } else if (st.latestFrameID != nk - 1) {
            for (int k = 1; k < st.recent_n; ++k) st.recent_ids[k - 1] = st.recent_ids[k];
            st.latestFrameID = nk - 1;
            st.recent_ids[st.recent_n - 1] = st.latestFrameID;
        }
    } else {
        st.recent_n = 0;
    }
    const int32_t* ids = mo_map_ids(v, s, st);
    int nc = 0, ns = 0;
    for (int k = 0; k < st.recent_n; ++k) {
        const int slot = ids[k] % v.KFR;
        const int32_t* kn = v.kf_n + ((size_t)s * v.KFR + slot) * 3;
        nc += kn[0];
        ns += kn[1] + kn[2];
    }
    if (nc > v.cap_mc) { nc = v.cap_mc; st.err_map |= SLO_ERR_MAP_CAPACITY; }
    if (ns > v.cap_ms) { ns = v.cap_ms; st.err_map |= SLO_ERR_MAP_CAPACITY; }
    st.n_corner_map = nc;
    st.n_surf_map = ns;
}

// one block per deque entry (blockIdx.x) of stream blockIdx.y (need_ran 0:
// the side stream's, issued before this step's k_mo_prepare sets mo_ran)
__global__ void k_mo_assemble(DevView v, int need_ran) {
    const int s = blockIdx.y, e = blockIdx.x;
    const StreamState& st = v.st[s];
    if ((need_ran && !st.mo_ran) || e >= st.recent_n) return;
    const int32_t* ids = mo_map_ids(v, s, st);
    // the clouds before this keyframe's: their sizes summed by the block
    // (integer sums: any order), not by every thread in a row
    __shared__ int s_oc, s_os;
    __shared__ float tr[9];
    if (threadIdx.x == 0) { s_oc = 0; s_os = 0; }
    __syncthreads();
    {
        int a = 0, b = 0;
        for (int k = threadIdx.x; k < e; k += blockDim.x) {
            const int32_t* kn = v.kf_n + ((size_t)s * v.KFR + ids[k] % v.KFR) * 3;
            a += kn[0];
            b += kn[1] + kn[2];
        }
        if (a) atomicAdd(&s_oc, a);
        if (b) atomicAdd(&s_os, b);
    }
    const int slot = ids[e] % v.KFR;
    const int32_t* kn = v.kf_n + ((size_t)s * v.KFR + slot) * 3;
    const size_t ks = (size_t)s * v.KFR + slot;
    // transformPointCloud with cloudKeyPoses6D[id] (MO:566-596): the ring
    // keeps body-frame clouds, so a pose correctPoses rewrote is used as is;
    // its three sin / cos pairs on three lanes of wave 0 (slo_pose_wave.h)
    if (threadIdx.x < 64) {
        const float* kp = v.kf_pose + ((size_t)s * v.KFMAX + ids[e]) * 6;
        const float a3[3] = {kp[3], kp[4], kp[5]};
        float sn[3], cs[3];
        slo_pose::wave_sincos<3>(a3, sn, cs);
        if (threadIdx.x == 0) {
            tr[0] = cs[0]; tr[1] = sn[0]; tr[2] = cs[1]; tr[3] = sn[1]; tr[4] = cs[2]; tr[5] = sn[2];
            tr[6] = kp[0]; tr[7] = kp[1]; tr[8] = kp[2];
        }
    }
    __syncthreads();
    const int oc = s_oc, os = s_os;
    const float ctRoll = tr[0], stRoll = tr[1], ctPitch = tr[2], stPitch = tr[3], ctYaw = tr[4], stYaw = tr[5];
    auto xf = [&](const float4 p) {
        const float x1 = ctYaw * p.x - stYaw * p.y, y1 = stYaw * p.x + ctYaw * p.y, z1 = p.z;
        const float x2 = x1, y2 = ctRoll * y1 - stRoll * z1, z2 = stRoll * y1 + ctRoll * z1;
        return make_float4(ctPitch * x2 + stPitch * z2 + tr[6], y2 + tr[7], -stPitch * x2 + ctPitch * z2 + tr[8], p.w);
    };
    // eight points per thread (256-thread launch) loaded before the first is transformed
    auto copy = [&](const float4* src, int n, float4* dst, int room) {
        for (int i0 = threadIdx.x; i0 < n; i0 += 8 * 256) {
            float4 q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) q[u] = src[min(i0 + u * 256, n - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u * 256;
                if (i < n && i < room) dst[i] = xf(q[u]);
            }
        }
    };
    copy(v.kf_corner + ks * v.cap_kc, kn[0], v.map_c + (size_t)s * v.cap_mc + oc, v.cap_mc - oc);
    copy(v.kf_surf + ks * v.cap_kfs, kn[1], v.map_s + (size_t)s * v.cap_ms + os, v.cap_ms - os);
    copy(v.kf_outl + ks * v.cap_kfo, kn[2], v.map_s + (size_t)s * v.cap_ms + os + kn[1], v.cap_ms - os - kn[1]);
}

__global__ void k_mo_concat(DevView v) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    const int a = st.n_surf_ds, b = st.n_outl_ds;
    for (int i = threadIdx.x; i < a; i += blockDim.x) v.cur_st[(size_t)s * v.cap_st + i] = v.cur_s_ds[(size_t)s * v.H + i];
    for (int i = threadIdx.x; i < b; i += blockDim.x)
        v.cur_st[(size_t)s * v.cap_st + a + i] = v.cur_o_ds[(size_t)s * v.cap_ko + i];
    if (threadIdx.x == 0) {
        st.n_st = a + b;
        st.map_ok = st.n_cmap_ds > 10 && st.n_smap_ds > 100;
        st.err |= st.err_map;   // the local-map selection's (k_mo_prepare half 2)
        st.err_map = 0;
    }
}

// ---------------------------------------------------------------- 5-NN in the hash grid
__device__ inline float sqd(const P4& q, float x, float y, float z) {
    float d0 = q.x - x, d1 = q.y - y, d2 = q.z - z;
    float r = 0.0f;
    r += d0 * d0;
    r += d1 * d1;
    r += d2 * d2;
    return r;
}

// Exact 5-NN (sorted by (distance, index)) among the map points within 1 m —
// the only ones the reference accepts (pointSearchSqDis[4] < 1.0, MO:1281 /
// 1364).  Rings of cells grow outward; after ring r every unseen point is at
// least r*cell away, so the search stops as soon as the 5th distance is below
// (r*cell)^2, and it never needs rings beyond ceil(1 m / cell).
// The 5 nearest map points of q whose squared distance is below 1 (ties ->
// lowest index), n = how many were found (<= 5).  The residuals only use a
// 5-NN whose 5th squared distance is < 1 (MO:1281 / 1364): when the true
// 5-NN has that, these are the same five points; when it has not, n < 5 or
// od[4] == 1 and the query is rejected either way.  So the search is a ball
// of squared radius 1 — R = 2 cells of 0.5 m — whose bound is the current 5th
// distance.
#ifndef SLO_KNN_UNROLL
#define SLO_KNN_UNROLL 2   // entry loads in flight per walk step: 4 costs occupancy (110 VGPRs -> 4 waves)
#endif
// bw: a bound on the walk known before it starts (the squared distance of
// five map points, so at least the 5th-NN distance; 1 = none): rows and
// cells past it are skipped, every point within it is still visited, so the
// five found are the same.
__device__ inline int knn5(const GridView& g, int s, const P4& q, int* oi, float* od, float bw = 1.0f) {
    // sorted top-5 by (distance, index); empty slots are (1, INT_MAX).
    // Insertion is unrolled with constant indices so the lists stay in
    // registers (a data-dependent index would put them in scratch memory).
#pragma unroll
    for (int k = 0; k < 5; ++k) { od[k] = 1.0f; oi[k] = INT_MAX; }
    if (!(isfinite(q.x) && isfinite(q.y) && isfinite(q.z))) return 0;
    auto less = [](float da, int ia, float db, int ib) { return da < db || (da == db && ia < ib); };
    int n = 0;
    grid_ball<SLO_MAP_R, SLO_KNN_UNROLL>(g, s, q.x, q.y, q.z, [&]() { return fminf(od[4], bw); }, [&](const float4& p) {
        const float d = sqd(q, p.x, p.y, p.z);
        const int idx = __float_as_int(p.w);
        if (!less(d, idx, od[4], oi[4])) return;
        bool placed = false;
#pragma unroll
        for (int k = 4; k >= 1; --k) {
            if (!placed) {
                if (less(d, idx, od[k - 1], oi[k - 1])) { od[k] = od[k - 1]; oi[k] = oi[k - 1]; }
                else { od[k] = d; oi[k] = idx; placed = true; }
            }
        }
        if (!placed) { od[0] = d; oi[0] = idx; }
        n = min(n + 1, 5);
    });
    return n;
}

// ---------------------------------------------------------------- correspondences + partial normal equations
// XCD-aware grid (xcd_stream_chunk): a stream's SLO_MO_BLOCKS workgroups share
// one XCD's L2, and each takes a contiguous run of the (voxel-ordered, hence
// spatially coherent) queries, so the map cells a workgroup walks are mostly
// the ones its neighbours just pulled in.
//
// Per round of 256 queries every thread computes its query's Jacobian row
// (matA row, matB entry; MO:1432-1441) into LDS — a zero row when the query is
// rejected — and the 27 products of the normal equations are then summed from
// LDS in double-double by 216 threads (27 terms x 8 slices of 32 rows) and
// folded into per-term totals.  The query phase so keeps no accumulators in
// registers, which is what bounds its occupancy.
__device__ __constant__ int8_t kMoTermI[27] = {0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 5,
                                               0, 1, 2, 3, 4, 5};
__device__ __constant__ int8_t kMoTermJ[27] = {0, 1, 2, 3, 4, 5, 1, 2, 3, 4, 5, 2, 3, 4, 5, 3, 4, 5, 4, 5, 5,
                                               6, 6, 6, 6, 6, 6};

// query q of stream s (corner queries first, then surf+outlier) and its
// map-frame position (pointAssociateToMap, MO:534-548)
struct MoTrig {
    float srx, crx, sry, cry, srz, crz, tX, tY, tZ;
};
// the stored sin/cos of transformTobeMapped (StreamState::mo_trig)
__device__ inline MoTrig mo_trig_of(const float* t) {
    MoTrig g;
    g.srx = t[0]; g.crx = t[1]; g.sry = t[2]; g.cry = t[3]; g.srz = t[4]; g.crz = t[5];
    g.tX = t[6]; g.tY = t[7]; g.tZ = t[8];
    return g;
}
__device__ inline MoTrig mo_trig(const StreamState& st) { return mo_trig_of(st.mo_trig); }
__device__ inline P4 mo_query(const DevView& v, int s, const StreamState& st, int q, const MoTrig& g, P4& po) {
    const int nc = st.n_corner_ds;
    const float4 po4 = q < nc ? v.cur_c_ds[(size_t)s * v.cap_less_sharp + q] : v.cur_st_ds[(size_t)s * v.cap_st + (q - nc)];
    po = P4{po4.x, po4.y, po4.z, po4.w};
    const float cRoll = g.crx, sRoll = g.srx, cPitch = g.cry, sPitch = g.sry, cYaw = g.crz, sYaw = g.srz;
    const float x1 = cYaw * po.x - sYaw * po.y, y1 = sYaw * po.x + cYaw * po.y, z1 = po.z;
    const float x2 = x1, y2 = cRoll * y1 - sRoll * z1, z2 = sRoll * y1 + cRoll * z1;
    return P4{cPitch * x2 + sPitch * z2 + g.tX, y2 + g.tY, -sPitch * x2 + cPitch * z2 + g.tZ, po.w};
}

// k_mo_knn's query order: a counting sort of the queries by the Morton code
// of their body-frame 4 m cell (corner queries first), in LDS, one workgroup
// per stream — so the lanes of a wave walk neighbouring rows of the map grid.
// Only the work order changes: mo_nn is indexed by query.
#define MO_PERM_B 4096   // buckets per query kind (12-bit Morton codes): 32 KB of LDS, so the
                         // block finds a CU next to the other contexts' sort blocks
#ifndef MO_PERM_INV
#define MO_PERM_INV 0.25f   // 1 / cell edge (4 m)
#endif
#ifndef SLO_MO_PERM
#define SLO_MO_PERM 1
#endif
__global__ void __launch_bounds__(256) k_mo_perm(DevView v) {
    __shared__ int cnt[2 * MO_PERM_B];
    __shared__ int wsum[4];
    const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const StreamState& st = v.st[s];
    if (!st.mo_ran) return;
    const int nc = st.n_corner_ds, nq = nc + st.n_surf_total_ds;
    const float4* qc = v.cur_c_ds + (size_t)s * v.cap_less_sharp;
    const float4* qs = v.cur_st_ds + (size_t)s * v.cap_st;
    // Morton code of the body-frame cell: x, z, y 4 bits each (clamped to
    // +-32 m around the sensor), interleaved x z y from the top -> 12 bits
    auto bucket = [&](int q) {
        const float4 p = q < nc ? qc[q] : qs[q - nc];
        unsigned int h = 0;
        if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
            const unsigned int a = (unsigned int)min(max(grid_cell(p.x, MO_PERM_INV) + 8, 0), 15);
            const unsigned int b = (unsigned int)min(max(grid_cell(p.y, MO_PERM_INV) + 8, 0), 15);
            const unsigned int c = (unsigned int)min(max(grid_cell(p.z, MO_PERM_INV) + 8, 0), 15);
#pragma unroll
            for (int k = 3; k >= 0; --k) {
                h = (h << 1) | ((a >> k) & 1u);
                h = (h << 1) | ((c >> k) & 1u);
                h = (h << 1) | ((b >> k) & 1u);
            }
        }
        return (q < nc ? 0 : MO_PERM_B) + (int)h;
    };
    for (int b = tid; b < 2 * MO_PERM_B; b += 256) cnt[b] = 0;
    __syncthreads();
    for (int q = tid; q < nq; q += 256) atomicAdd(&cnt[bucket(q)], 1);
    __syncthreads();
    constexpr int PER = 2 * MO_PERM_B / 256;
    int c[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) { c[k] = cnt[tid * PER + k]; sum += c[k]; }
    int incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int run = incl - sum;
    for (int k = 0; k < w; ++k) run += wsum[k];
#pragma unroll
    for (int k = 0; k < PER; ++k) { cnt[tid * PER + k] = run; run += c[k]; }
    __syncthreads();
    int32_t* perm = v.mo_perm + (size_t)s * v.cap_q;
    for (int q = tid; q < nq; q += 256) perm[atomicAdd(&cnt[bucket(q)], 1)] = q;
}

// The 5-NN of every query, one thread per query, into mo_nn (index -1 in the
// first slot = rejected: fewer than 5 within 1 m).  A kernel of its own so its
// few registers give full occupancy to the latency-bound grid walk.
__global__ void __launch_bounds__(256) k_mo_knn(DevView v) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, SLO_MO_BLOCKS, s, chunk);
    if (s >= v.S) return;
    const StreamState& st = v.st[s];
    if (!(st.mo_ran && st.map_ok && !st.mo_converged)) return;
    const MoTrig g = mo_trig(st);
    const int nc = st.n_corner_ds, nq = nc + st.n_surf_total_ds, per = (nq + SLO_MO_BLOCKS - 1) / SLO_MO_BLOCKS;
    const int q0 = chunk * per, q1 = min(nq, q0 + per);
    int32_t* nn = v.mo_nn + (size_t)s * v.cap_q * 5;
    const int32_t* perm = v.mo_perm + (size_t)s * v.cap_q;
    for (int qi = q0 + (int)threadIdx.x; qi < q1; qi += blockDim.x) {
#if SLO_MO_PERM
        const int q = perm[qi];   // grouped by 2 m cell: a wave's queries are neighbours
#else
        const int q = qi;
#endif
        P4 po;
        const P4 sel = mo_query(v, s, st, q, g, po);
        int ind[5];
        float dis[5];
        // warm start (LM iterations after the first, same map): the previous
        // iteration's five neighbours, seen from the moved query, bound the
        // walk before it starts
        float bw = 1.0f;
        if (st.mo_iters > 0) {
            int pi[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) pi[k] = nn[(size_t)q * 5 + k];
            if (pi[0] >= 0) {
                const float4* mp = q < nc ? v.map_c_ds + (size_t)s * v.cap_mc : v.map_s_ds + (size_t)s * v.cap_ms;
                float4 m[5];
#pragma unroll
                for (int k = 0; k < 5; ++k) m[k] = mp[pi[k]];
                bw = 0.0f;
#pragma unroll
                for (int k = 0; k < 5; ++k) bw = fmaxf(bw, sqd(sel, m[k].x, m[k].y, m[k].z));
                bw = fminf(bw, 1.0f);
            }
        }
        const int n = q < nc ? knn5(v.g_mc, s, sel, ind, dis, bw) : knn5(v.g_ms, s, sel, ind, dis, bw);
        const bool ok = n == 5 && dis[4] < 1.0;   // MO:1281 / 1364
#pragma unroll
        for (int k = 0; k < 5; ++k) nn[(size_t)q * 5 + k] = ok ? ind[k] : -1;
    }
}

__device__ inline bool mo_row(const DevView& v, int s, const StreamState& st, int q, float* row) {
    const MoTrig g = mo_trig(st);
    const float srx = g.srx, crx = g.crx, sry = g.sry, cry = g.cry, srz = g.srz, crz = g.crz;
    const bool corner = q < st.n_corner_ds;
    P4 po;
    const P4 sel = mo_query(v, s, st, q, g, po);
    const int32_t* nn = v.mo_nn + ((size_t)s * v.cap_q + q) * 5;
    int ind[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) ind[k] = nn[k];
    if (ind[0] < 0) return false;
    float cfx, cfy, cfz, cfw;
    if (corner) {   // cornerOptimization (MO:1265-1346)
        const float4* mc = v.map_c_ds + (size_t)s * v.cap_mc;
        float cx = 0, cy = 0, cz = 0;
        for (int j = 0; j < 5; j++) { float4 m = mc[ind[j]]; cx += m.x; cy += m.y; cz += m.z; }
        cx /= 5; cy /= 5; cz /= 5;
        float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
        for (int j = 0; j < 5; j++) {
            float4 m = mc[ind[j]];
            float ax = m.x - cx, ay = m.y - cy, az = m.z - cz;
            a11 += ax * ax; a12 += ax * ay; a13 += ax * az;
            a22 += ay * ay; a23 += ay * az;
            a33 += az * az;
        }
        a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
        float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33}, D1[3], V1[9];
        slo_la::eigen_sym(A1, 3, D1, V1);
        if (!(D1[0] > 3 * D1[1])) return false;
        const float x0 = sel.x, y0 = sel.y, z0 = sel.z;
        const float xa = (float)(cx + 0.1 * V1[0]), ya = (float)(cy + 0.1 * V1[1]), za = (float)(cz + 0.1 * V1[2]);
        const float xb = (float)(cx - 0.1 * V1[0]), yb = (float)(cy - 0.1 * V1[1]), zb = (float)(cz - 0.1 * V1[2]);
        const float m1 = (x0 - xa) * (y0 - yb) - (x0 - xb) * (y0 - ya);
        const float m2 = (x0 - xa) * (z0 - zb) - (x0 - xb) * (z0 - za);
        const float m3 = (y0 - ya) * (z0 - zb) - (y0 - yb) * (z0 - za);
        const float a012 = sqrtf(m1 * m1 + m2 * m2 + m3 * m3);
        const float l12 = sqrtf((xa - xb) * (xa - xb) + (ya - yb) * (ya - yb) + (za - zb) * (za - zb));
        const float la = ((ya - yb) * m1 + (za - zb) * m2) / a012 / l12;
        const float lb = -((xa - xb) * m1 - (za - zb) * m3) / a012 / l12;
        const float lc = -((xa - xb) * m2 + (ya - yb) * m3) / a012 / l12;
        const float ld2 = a012 / l12;
        const float sw = (float)(1 - 0.9 * fabsf(ld2));
        cfx = sw * la; cfy = sw * lb; cfz = sw * lc; cfw = sw * ld2;
        if (!(sw > 0.1)) return false;
    } else {        // surfOptimization (MO:1348-1399)
        const float4* ms = v.map_s_ds + (size_t)s * v.cap_ms;
        float A0[15], B0[5] = {-1, -1, -1, -1, -1}, X0[3];
        for (int j = 0; j < 5; j++) { float4 m = ms[ind[j]]; A0[j * 3] = m.x; A0[j * 3 + 1] = m.y; A0[j * 3 + 2] = m.z; }
        slo_la::solve_qr(A0, B0, 5, 3, X0);
        float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
        const float ps = sqrtf(pa * pa + pb * pb + pc * pc);
        pa /= ps; pb /= ps; pc /= ps; pd /= ps;
        for (int j = 0; j < 5; j++) {
            float4 m = ms[ind[j]];
            if (fabsf(pa * m.x + pb * m.y + pc * m.z + pd) > 0.2) return false;
        }
        const float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
        const float sw = (float)(1 - 0.9 * fabsf(pd2) / sqrtf(sqrtf(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z)));
        cfx = sw * pa; cfy = sw * pb; cfz = sw * pc; cfw = sw * pd2;
        if (!(sw > 0.1)) return false;
    }
    // LMOptimization rows (MO:1418-1441)
    const P4& p = po;
    row[0] = (crx * sry * srz * p.x + crx * crz * sry * p.y - srx * sry * p.z) * cfx +
             (-srx * srz * p.x - crz * srx * p.y - crx * p.z) * cfy +
             (crx * cry * srz * p.x + crx * cry * crz * p.y - cry * srx * p.z) * cfz;
    row[1] = ((cry * srx * srz - crz * sry) * p.x + (sry * srz + cry * crz * srx) * p.y + crx * cry * p.z) * cfx +
             ((-cry * crz - srx * sry * srz) * p.x + (cry * srz - crz * srx * sry) * p.y - crx * sry * p.z) * cfz;
    row[2] = ((crz * srx * sry - cry * srz) * p.x + (-cry * crz - srx * sry * srz) * p.y) * cfx +
             (crx * crz * p.x - crx * srz * p.y) * cfy +
             ((sry * srz + cry * crz * srx) * p.x + (crz * sry - cry * srx * srz) * p.y) * cfz;
    row[3] = cfx; row[4] = cfy; row[5] = cfz;
    row[6] = -cfw;
    return true;
}

__global__ void __launch_bounds__(256) k_mo_corr(DevView v) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, SLO_MO_BLOCKS, s, chunk);
    if (s >= v.S) return;
    const StreamState& st = v.st[s];
    const int tid = threadIdx.x;
    __shared__ float rows[256][8];
    __shared__ int shn[4];
    const int term = tid >> 3, slice = tid & 7;   // 216 reducing threads: 27 terms x 8 slices
    const int ti = term < 27 ? kMoTermI[term] : 0, tj = term < 27 ? kMoTermJ[term] : 0;
    slo_dd::DD tot = slo_dd::zero();   // per-term total (valid in slice 0)
    int nsel = 0;
    const bool live = st.mo_ran && st.map_ok && !st.mo_converged;
    if (live) {
        const int nq = st.n_corner_ds + st.n_surf_total_ds, per = (nq + SLO_MO_BLOCKS - 1) / SLO_MO_BLOCKS;
        const int q0 = chunk * per, q1 = min(nq, q0 + per);
        for (int qb = q0; qb < q1; qb += 256) {   // uniform trip count
            float row[7] = {0, 0, 0, 0, 0, 0, 0};
            const int q = qb + tid;
#if SLO_DIAG
            const unsigned long long t_row = clock64();
#endif
            const bool okrow = q < q1 && mo_row(v, s, st, q, row);
            if (okrow) ++nsel;
            else for (int k = 0; k < 7; ++k) row[k] = 0.0f;   // rejected: contributes exact zeros
#if SLO_DIAG
            if ((threadIdx.x & 63) == 0) atomicAdd(&v.st[s].dbg[7], clock64() - t_row);   // wave time per round
#endif
            for (int k = 0; k < 7; ++k) rows[tid][k] = row[k];
            __syncthreads();
            if (term < 27) {
                slo_dd::DD acc = slo_dd::zero();
                for (int r = slice * 32; r < slice * 32 + 32; ++r)
                    slo_dd::add(acc, (double)rows[r][ti] * (double)rows[r][tj]);
                for (int o = 4; o > 0; o >>= 1) {   // the 8 slices of a term are 8 adjacent lanes
                    slo_dd::DD y{__shfl_xor(acc.hi, o, 64), __shfl_xor(acc.lo, o, 64)};
                    slo_dd::merge(acc, y);
                }
                slo_dd::merge(tot, acc);
            }
            __syncthreads();
        }
    }
    for (int o = 32; o > 0; o >>= 1) nsel += __shfl_xor(nsel, o, 64);
    if ((tid & 63) == 0) shn[tid >> 6] = nsel;
    __syncthreads();
    double* part = v.mo_part + ((size_t)s * SLO_MO_BLOCKS + chunk) * SLO_MO_PART;
    if (term < 27 && slice == 0) {
        part[2 * term] = tot.hi;
        part[2 * term + 1] = tot.lo;
    }
    if (tid == 0) part[54] = (double)(shn[0] + shn[1] + shn[2] + shn[3]);
}

// LMOptimization tail (MO:1445-1498) for one stream
__global__ void __launch_bounds__(64) k_mo_solve(DevView v, int iterCount) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    if (!(st.mo_ran && st.map_ok && !st.mo_converged)) return;
    // the workgroups' partial sums: lane k < 27 folds term k, lane 27 the
    // correspondence count (double-double: the fold order does not change the
    // rounded result, slo_ddsum.h)
    __shared__ slo_dd::DD s_acc[27];
    __shared__ int s_nsel;
    const int lane = threadIdx.x;
#ifdef SLO_DIAG_FIN   // [4] fold, [5] solve_qr, [6] degeneracy (iteration 0), [7] the rest, cycles
    unsigned long long tq0 = clock64();
#endif
    if (lane < 27) {
        slo_dd::DD a = slo_dd::zero();
        const double* part = v.mo_part + (size_t)s * SLO_MO_BLOCKS * SLO_MO_PART + 2 * lane;
#pragma unroll 8
        for (int b = 0; b < SLO_MO_BLOCKS; ++b)
            slo_dd::merge(a, slo_dd::DD{part[(size_t)b * SLO_MO_PART], part[(size_t)b * SLO_MO_PART + 1]});
        s_acc[lane] = a;
    } else if (lane == 27) {
        int n = 0;
        for (int b = 0; b < SLO_MO_BLOCKS; ++b) n += (int)v.mo_part[((size_t)s * SLO_MO_BLOCKS + b) * SLO_MO_PART + 54];
        s_nsel = n;
    }
    __syncthreads();
    if (lane != 0) return;
    const slo_dd::DD* acc = s_acc;
    const int nsel = s_nsel;
    st.mo_iters = iterCount + 1;
    st.n_sel = nsel;
    if (nsel < 50) return;  // LMOptimization returns false, loop continues
    float AtA[36], AtB[6], X[6];
    int k = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j) {
            const float f = slo_dd::to_float(acc[k++]);
            AtA[i * 6 + j] = f; AtA[j * 6 + i] = f;
        }
    for (int i = 0; i < 6; ++i) AtB[i] = slo_dd::to_float(acc[21 + i]);
#ifdef SLO_DIAG_FIN
    unsigned long long tq1 = clock64();
#endif
    slo_la::solve_qr(AtA, AtB, 6, 6, X);
#ifdef SLO_DIAG_FIN
    unsigned long long tq2 = clock64();
#endif
    if (iterCount == 0) {
        // the data-indexed matrices in LDS (as private arrays they lived in
        // scratch memory: ~100 us of this one lane per mapping step)
        __shared__ float E[6], V[36], V2[36], Vi[36], wa[36], wb[36];
        __shared__ int wr[6], wc[6];
        slo_la::eigen_sym_ws<6>(AtA, E, V, wa, wr, wc);
        for (int i = 0; i < 36; ++i) V2[i] = V[i];
        st.isDegenerate_mo = 0;
        for (int i = 5; i >= 0; i--) {
            if (E[i] < 100.0f) {
                for (int j = 0; j < 6; j++) V2[i * 6 + j] = 0;
                st.isDegenerate_mo = 1;
            } else break;
        }
        slo_la::inv_ws(V, 6, Vi, wa, wb);
        slo_la::mul(Vi, V2, 6, 6, 6, st.matP_mo);
    }
#ifdef SLO_DIAG_FIN
    unsigned long long tq3 = clock64();
#endif
    if (st.isDegenerate_mo) {
        float X2[6];
        for (int i = 0; i < 6; ++i) X2[i] = X[i];
        slo_la::mul(st.matP_mo, X2, 6, 6, 1, X);
    }
    for (int i = 0; i < 6; ++i) st.transformTobeMapped[i] += X[i];
    mo_store_trig(st);
    double r0 = X[0] * 57.29578f, r1 = X[1] * 57.29578f, r2 = X[2] * 57.29578f;
    double t0 = X[3] * 100, t1 = X[4] * 100, t2 = X[5] * 100;
    float deltaR = (float)sqrt(r0 * r0 + r1 * r1 + r2 * r2);
    float deltaT = (float)sqrt(t0 * t0 + t1 * t1 + t2 * t2);
    if (deltaR < 0.05 && deltaT < 0.05) st.mo_converged = 1;
#ifdef SLO_DIAG_FIN
    unsigned long long tq4 = clock64();
    st.dbg[4] += tq1 - tq0; st.dbg[5] += tq2 - tq1; st.dbg[6] += tq3 - tq2; st.dbg[7] += tq4 - tq3;
#endif
}

// ---------------------------------------------------------------- keyframe + Scan Context make
__device__ __forceinline__ void sc_make_block(const DevView& v, int s, const float4* raw, int nraw);
__device__ __forceinline__ void sc_desc_block(const slo_config& cfg, const float4* raw, int nraw, unsigned int* cell, double* desc);


__device__ inline float sc_xy2theta(float x, float y, int atan_float) {
    auto at = [&](float t) -> double { return atan_float ? (double)slo_libm::atanf_(t) : atan((double)t); };
    if ((x >= 0) & (y >= 0)) return (float)((180 / M_PI) * at(y / x));
    if ((x < 0) & (y >= 0)) return (float)(180 - ((180 / M_PI) * at(y / (-x))));
    if ((x < 0) & (y < 0)) return (float)(180 + ((180 / M_PI) * at(y / x)));
    if ((x >= 0) & (y < 0)) return (float)(360 - ((180 / M_PI) * at((-y) / x)));
    return __builtin_nanf("");
}

__global__ void __launch_bounds__(256) k_mo_finish(DevView v) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    __shared__ int save;
    __shared__ float pose[6];
    __shared__ int kfid;
    if (threadIdx.x == 0) {
        save = 0;
        if (st.mo_ran) {
            if (st.map_ok)  // scan2MapOptimization -> transformUpdate
                for (int i = 0; i < 6; i++) { st.transformBefMapped[i] = st.mo_sum[i]; st.transformAftMapped[i] = st.transformTobeMapped[i]; }
            // saveKeyFramesAndFactor
            float cx = st.transformAftMapped[3], cy = st.transformAftMapped[4], cz = st.transformAftMapped[5];
            float dx = st.prevPos[0] - cx, dy = st.prevPos[1] - cy, dz = st.prevPos[2] - cz;
            bool saveThis = !(sqrtf(dx * dx + dy * dy + dz * dz) < 0.3);
            if ((saveThis || st.n_keyframes == 0) && st.n_keyframes >= v.KFMAX) st.err |= SLO_ERR_KEYFRAMES;
            if ((saveThis || st.n_keyframes == 0) && st.n_keyframes < v.KFMAX) {
                st.prevPos[0] = cx; st.prevPos[1] = cy; st.prevPos[2] = cz;
                float est[6];
                for (int i = 0; i < 6; ++i) st.kf_pre[i] = st.n_keyframes == 0 ? st.transformTobeMapped[i] : st.transformAftMapped[i];
                if (st.n_keyframes == 0) {   // iSAM2 estimate = initial value, through Rot3
                    for (int i = 0; i < 6; ++i) st.transformLast[i] = st.transformTobeMapped[i];
                    slo_pose::keyframe_estimate(st.transformTobeMapped, est);
                } else {
                    slo_pose::keyframe_estimate(st.transformAftMapped, est);
                }
                pose[0] = est[3]; pose[1] = est[4]; pose[2] = est[5];
                pose[3] = est[0]; pose[4] = est[1]; pose[5] = est[2];
                kfid = st.n_keyframes;
                float* kp = v.kf_pose + ((size_t)s * v.KFMAX + kfid) * 6;
                for (int i = 0; i < 6; ++i) kp[i] = pose[i];
                st.n_keyframes = kfid + 1;
                if (st.n_keyframes > 1)
                    for (int i = 0; i < 6; ++i) {
                        st.transformAftMapped[i] = est[i]; st.transformLast[i] = est[i]; st.transformTobeMapped[i] = est[i];
                    }
                st.kf_saved = 1;
                save = 1;
            }
            // publishTF (MO:680-705) as transformFusion reads it (TF:222-241)
            slo_pose::odom_handoff(st.transformAftMapped, st.tf_aft);
            for (int i = 0; i < 6; ++i) st.tf_bef[i] = st.transformBefMapped[i];
        }
    }
    __syncthreads();
    if (!save) return;
    // the keyframe's DS clouds, body frame (cornerCloudKeyFrames & co,
    // MO:1634-1636); k_mo_assemble transforms them with the key pose
    const int slot = kfid % v.KFR;
    const size_t ks = (size_t)s * v.KFR + slot;
    const int n3[3] = {min(st.n_corner_ds, v.cap_kc), min(st.n_surf_ds, v.cap_kfs), min(st.n_outl_ds, v.cap_kfo)};
    const float4* src[3] = {v.cur_c_ds + (size_t)s * v.cap_less_sharp, v.cur_s_ds + (size_t)s * v.H,
                            v.cur_o_ds + (size_t)s * v.cap_ko};
    float4* dst[3] = {v.kf_corner + ks * v.cap_kc, v.kf_surf + ks * v.cap_kfs, v.kf_outl + ks * v.cap_kfo};
    for (int c = 0; c < 3; ++c)
        for (int i = threadIdx.x; i < n3[c]; i += blockDim.x) dst[c][i] = src[c][i];
    if (threadIdx.x < 3) v.kf_n[ks * 3 + threadIdx.x] = n3[threadIdx.x];
    if (threadIdx.x == 0 && (n3[0] < st.n_corner_ds || n3[1] < st.n_surf_ds || n3[2] < st.n_outl_ds))
        st.err |= SLO_ERR_MAP_CAPACITY;
    // Scan Context make on laserCloudRawDS (MO:1626-1631)
    sc_make_block(v, s, v.cur_raw_ds + (size_t)s * v.P, st.n_raw_ds);
}

// makeAndSaveScancontextAndKeys on an already downsampled cloud (public SC API)
__global__ void __launch_bounds__(256) k_sc_make(DevView v, const float4* pts, size_t stride, const int32_t* n,
                                                 int n_stride) {
    const int s = blockIdx.x;
    sc_make_block(v, s, pts + (size_t)s * stride, n[(size_t)s * n_stride]);
}

// ---- the public SCManager helpers (Scancontext.h:63-69), batched: item b of
// each launch is one descriptor / pair (slo_sc_* in include/slo_abi.h).
// Descriptors are row-major NR x NS doubles, sector keys NS, ring keys NR.
__device__ inline void sc_keys_block(const slo_config& cfg, const double* desc, double* ring, double* sect) {
    const int NR = cfg.sc_num_ring, NS = cfg.sc_num_sector;
    for (int r = threadIdx.x; r < NR; r += blockDim.x) ring[r] = eigen_sum(desc + r * NS, NS, 1) / (double)NS;   // SCc:198-211
    for (int c = threadIdx.x; c < NS; c += blockDim.x) sect[c] = eigen_sum(desc + c, NR, NS) / (double)NR;       // SCc:214-227
}

__global__ void __launch_bounds__(256) k_sc_api_make(slo_config cfg, const float4* pts, size_t stride, const int32_t* n,
                                                     double* desc, double* ring, double* sect) {
    __shared__ unsigned int cell[20 * 60];
    __shared__ double d[20 * 60];
    const int b = blockIdx.x, NR = cfg.sc_num_ring, NS = cfg.sc_num_sector;
    sc_desc_block(cfg, pts + (size_t)b * stride, n[b], cell, d);
    for (int i = threadIdx.x; i < NR * NS; i += blockDim.x) desc[(size_t)b * NR * NS + i] = d[i];
    sc_keys_block(cfg, d, ring + (size_t)b * NR, sect + (size_t)b * NS);
}

__global__ void __launch_bounds__(64) k_sc_api_keys(slo_config cfg, const double* desc, double* ring, double* sect) {
    const int b = blockIdx.x, NR = cfg.sc_num_ring, NS = cfg.sc_num_sector;
    sc_keys_block(cfg, desc + (size_t)b * NR * NS, ring + (size_t)b * NR, sect + (size_t)b * NS);
}

// fastAlignUsingVkey (SCc:93-113): the first shift of least |vkey1 - circshift(vkey2, shift)|
__global__ void __launch_bounds__(64) k_sc_api_align(slo_config cfg, const double* vk1, const double* vk2,
                                                     int32_t* shift) {
    __shared__ double nrm[SC_NS];
    const int b = blockIdx.x, NS = cfg.sc_num_sector, tid = threadIdx.x;
    const double* a = vk1 + (size_t)b * NS;
    const double* c = vk2 + (size_t)b * NS;
    if (tid < NS) {
        ESum e;
        for (int j = 0; j < NS; ++j) {
            const double d = a[j] - c[((j - tid) % NS + NS) % NS];
            e.add(d * d);
        }
        nrm[tid] = sqrt(e.get());
    }
    __syncthreads();
    if (tid == 0) {
        int am = 0;
        double mn = 10000000;
        for (int sh = 0; sh < NS; ++sh)
            if (nrm[sh] < mn) { am = sh; mn = nrm[sh]; }
        shift[b] = am;
    }
}

// distDirectSC (SCc:69-90): 1 - the mean column cosine over the columns non-zero in both
__global__ void __launch_bounds__(64) k_sc_api_direct(slo_config cfg, const double* sc1, const double* sc2,
                                                      double* dist) {
    __shared__ double sim[SC_NS];
    __shared__ int ok[SC_NS];
    const int b = blockIdx.x, NR = cfg.sc_num_ring, NS = cfg.sc_num_sector, j = threadIdx.x;
    const double* a = sc1 + (size_t)b * NR * NS;
    const double* c = sc2 + (size_t)b * NR * NS;
    if (j < NS) {
        ESum n1, n2, dt;
        for (int r = 0; r < NR; ++r) {
            const double x = a[r * NS + j], y = c[r * NS + j];
            n1.add(x * x); n2.add(y * y); dt.add(x * y);
        }
        const double nn1 = sqrt(n1.get()), nn2 = sqrt(n2.get());
        ok[j] = !((nn1 == 0) | (nn2 == 0));
        sim[j] = ok[j] ? dt.get() / (nn1 * nn2) : 0.0;
    }
    __syncthreads();
    if (j == 0) {
        double sum = 0;
        int ne = 0;
        for (int k = 0; k < NS; ++k)
            if (ok[k]) { sum = sum + sim[k]; ne = ne + 1; }
        dist[b] = 1.0 - sum / ne;
    }
}

// distanceBtnScanContext (SCc:116-148): sector keys, then the shared pair distance
__global__ void __launch_bounds__(256) k_sc_api_dist(slo_config cfg, const double* sc1, const double* sc2,
                                                     double* dist, int32_t* shift) {
    __shared__ double vk[2][SC_NS];
    __shared__ double rk[2][20];
    __shared__ ScPairLds L;
    const int b = blockIdx.x, NR = cfg.sc_num_ring, NS = cfg.sc_num_sector;
    const double* a = sc1 + (size_t)b * NR * NS;
    const double* c = sc2 + (size_t)b * NR * NS;
    sc_keys_block(cfg, a, rk[0], vk[0]);
    sc_keys_block(cfg, c, rk[1], vk[1]);
    __syncthreads();
    double d;
    int al;
    sc_pair_distance(a, vk[0], c, vk[1], NR, NS, cfg.sc_search_ratio, L, &d, &al);
    if (threadIdx.x == 0) { dist[b] = d; shift[b] = al; }
}

int sc_api_run(slo_ctx* ctx, int op, int nitems, const void* in1, const void* in2, size_t stride, const int32_t* n,
               void* out1, void* out2, void* out3) {
    const slo_config& cfg = ctx->cfg;
    if (cfg.sc_num_ring > 20 || cfg.sc_num_sector > SC_NS || nitems <= 0) return SLO_E_ARG;
    switch (op) {
    case 0:
        SLO_LAUNCH(ctx, "sc_api_make", k_sc_api_make, dim3(nitems), dim3(256), 0, cfg, (const float4*)in1, stride, n,
                   (double*)out1, (double*)out2, (double*)out3);
        break;
    case 1:
        SLO_LAUNCH(ctx, "sc_api_keys", k_sc_api_keys, dim3(nitems), dim3(64), 0, cfg, (const double*)in1,
                   (double*)out1, (double*)out2);
        break;
    case 2:
        SLO_LAUNCH(ctx, "sc_api_align", k_sc_api_align, dim3(nitems), dim3(64), 0, cfg, (const double*)in1,
                   (const double*)in2, (int32_t*)out1);
        break;
    case 3:
        SLO_LAUNCH(ctx, "sc_api_direct", k_sc_api_direct, dim3(nitems), dim3(64), 0, cfg, (const double*)in1,
                   (const double*)in2, (double*)out1);
        break;
    default:
        SLO_LAUNCH(ctx, "sc_api_dist", k_sc_api_dist, dim3(nitems), dim3(256), 0, cfg, (const double*)in1,
                   (const double*)in2, (double*)out1, (int32_t*)out2);
    }
    SLO_CHECK(hipGetLastError());
    return 0;
}

int sc_make_run(slo_ctx* ctx, const float4* pts, size_t stride, const int32_t* n, int n_stride, int n_streams) {
    SLO_LAUNCH(ctx, "sc_make", k_sc_make, dim3(n_streams), dim3(256), 0, ctx->v, pts, stride, n, n_stride);
    SLO_CHECK(hipGetLastError());
    return 0;
}

// SCManager::makeScancontext (Scancontext.cpp:151-195) of nraw points into
// desc[NR * NS] (LDS, row-major: ring, sector), one workgroup; cell is LDS
// scratch of the same size
__device__ __forceinline__ void sc_desc_block(const slo_config& cfg, const float4* raw, int nraw, unsigned int* cell, double* desc) {
    const int NR = cfg.sc_num_ring, NS = cfg.sc_num_sector;
    for (int i = threadIdx.x; i < NR * NS; i += blockDim.x) cell[i] = ford(-1000.0f);
    __syncthreads();
    for (int i = threadIdx.x; i < nraw; i += blockDim.x) {
        float4 p0 = raw[i];
        float px = p0.x, py = p0.y;
        float pz = (float)(p0.z + cfg.sc_lidar_height);
        float azim_range = sqrtf(px * px + py * py);
        float azim_angle = sc_xy2theta(px, py, cfg.sc_atan_float);
        if (azim_range > cfg.sc_max_radius) continue;
        int ring_idx = max(min(NR, (int)ceil((azim_range / cfg.sc_max_radius) * NR)), 1);
        double sc = ceil((azim_angle / 360.0) * NS);
        int sraw = isnan(sc) ? INT_MIN : (int)sc;
        int sctor_idx = max(min(NS, sraw), 1);
        atomicMax(&cell[(ring_idx - 1) * NS + (sctor_idx - 1)], ford(pz));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NR * NS; i += blockDim.x) {
        float f = unord(cell[i]);
        desc[i] = (f == -1000.0f) ? 0.0 : (double)f;
    }
    __syncthreads();
}

// SCManager::makeScancontext + makeRingkey/SectorkeyFromScancontext +
// history append (Scancontext.cpp:151-244), one workgroup
// (inlined into its kernels: a call would take the address of the kernel's
// by-value DevView, which then gets a 1.2 KB private copy in scratch memory)
__device__ __forceinline__ void sc_make_block(const DevView& v, int s, const float4* raw, int nraw) {
    StreamState& st = v.st[s];
    const int NR = v.cfg.sc_num_ring, NS = v.cfg.sc_num_sector;
    __shared__ unsigned int cell[20 * 60];
    __shared__ double desc[20 * 60];
    __shared__ int hid;
    if (threadIdx.x == 0) hid = st.sc_count;
    __syncthreads();
    const int kfid = hid;
    if (kfid >= v.KFMAX) {
        if (threadIdx.x == 0) { st.err |= SLO_ERR_SC_HISTORY; st.sc_wrote = 0; }
        return;
    }
    sc_desc_block(v.cfg, raw, nraw, cell, desc);
    double* hd = v.sc_desc + ((size_t)s * v.KFMAX + kfid) * NR * NS;
    for (int i = threadIdx.x; i < NR * NS; i += blockDim.x) hd[i] = desc[i];
    __syncthreads();
    if (threadIdx.x < NR) {
        double rk = eigen_sum(desc + threadIdx.x * NS, NS, 1) / (double)NS;
        v.sc_ringd[((size_t)s * v.KFMAX + kfid) * NR + threadIdx.x] = rk;
        v.sc_ring[((size_t)s * v.KFMAX + kfid) * NR + threadIdx.x] = (float)rk;
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + NS) {
        const int c = threadIdx.x - 64;
        v.sc_sect[((size_t)s * v.KFMAX + kfid) * NS + c] = eigen_sum(desc + c, NR, NS) / (double)NR;
    }
    if (threadIdx.x == 0) { st.sc_count = kfid + 1; st.sc_wrote = 1; }
}

// The mapping step's six VoxelGrid filters (MO:1224-1263) as one batched
// call's groups.  One call sorts S * (sum of the six strides) items; item
// positions are 32-bit, so a context whose sum passes INT32_MAX runs them as
// two calls (the local maps, then the current scan's four): map_vg_split.
static void map_groups(slo_ctx* ctx, VgGroup gs[6]) {
    DevView& v = ctx->v;
    const int SS = ST_STRIDE;
    StreamState* st0 = v.st;
    auto fld = [&](int32_t StreamState::*f) { return &(st0->*f); };
    const VgGroup g[6] = {
        {v.map_c, (size_t)v.cap_mc, fld(&StreamState::n_corner_map), SS, v.cfg.leaf_corner, v.map_c_ds,
         (size_t)v.cap_mc, fld(&StreamState::n_cmap_ds), SS, v.cap_mc},
        {v.map_s, (size_t)v.cap_ms, fld(&StreamState::n_surf_map), SS, v.cfg.leaf_surf, v.map_s_ds,
         (size_t)v.cap_ms, fld(&StreamState::n_smap_ds), SS, v.cap_ms},
        {nullptr, (size_t)v.P, nullptr, 1, v.cfg.leaf_sc, v.cur_raw_ds, (size_t)v.P,
         fld(&StreamState::n_raw_ds), SS, v.P},
        {v.corner_last, (size_t)v.cap_less_sharp, fld(&StreamState::cornerLastNum), SS, v.cfg.leaf_corner,
         v.cur_c_ds, (size_t)v.cap_less_sharp, fld(&StreamState::n_corner_ds), SS, v.cap_less_sharp},
        {v.surf_last, (size_t)v.cap_less_flat, fld(&StreamState::surfLastNum), SS, v.cfg.leaf_surf, v.cur_s_ds,
         (size_t)v.H, fld(&StreamState::n_surf_ds), SS, v.H},
        {v.outl_cam, (size_t)v.H, fld(&StreamState::outlier_count), SS, v.cfg.leaf_outlier, v.cur_o_ds,
         (size_t)v.cap_ko, fld(&StreamState::n_outl_ds), SS, v.cap_ko}};
    for (int k = 0; k < 6; ++k) gs[k] = g[k];
}
static bool map_vg_split(slo_ctx* ctx, const VgGroup gs[6]) {
    size_t items = 0;
    for (int k = 0; k < 6; ++k) items += (size_t)ctx->S * gs[k].stride;
    return items > (size_t)INT32_MAX;
}
static VgGroup map_total_group(slo_ctx* ctx) {
    DevView& v = ctx->v;
    StreamState* st0 = v.st;
    return {v.cur_st, (size_t)v.cap_st, &st0->n_st, ST_STRIDE, v.cfg.leaf_surf, v.cur_st_ds, (size_t)v.cap_st,
            &st0->n_surf_total_ds, ST_STRIDE, v.cap_st};
}

// Every workspace a mapping step's VoxelGrids and sorts will use, allocated
// from the capacities (the sizes depend on the strides alone) by the first
// entry point that can map, before anything is captured (map_ws_ensure), so no
// step allocates: an out-of-memory shows at that call, a captured step
// graph's pointers never move, and a context that never maps (a Mode S front
// or odometry context) never holds them.
int map_ws_presize(slo_ctx* ctx) {
    VgGroup gs[6];
    map_groups(ctx, gs);
    int r;
    if (map_vg_split(ctx, gs)) {
        if ((r = vg_presize(ctx, gs, 2)) || (r = vg_presize(ctx, gs + 2, 4))) return r;
    } else if ((r = vg_presize(ctx, gs, 6))) {
        return r;
    }

    const VgGroup t = map_total_group(ctx);
    return vg_presize(ctx, &t, 1);
}

int map_ws_ensure(slo_ctx* ctx) {
    if (ctx->map_ws_ready) return 0;
    if (int r = map_ws_presize(ctx)) return r;
    ctx->map_ws_ready = true;
    return 0;
}

static int map_run_rest(slo_ctx* ctx, bool grids_built);

bool map_fork_ok(const slo_ctx* ctx) {
    return SLO_MAP_FORK && ctx->S <= SLO_PREP_DEFER_STREAMS && ctx->cfg.voxel_order == SLO_VOXEL_PCL;
}

// the side stream and its workspaces for map_side_fork (slo_batch_process,
// never inside a capture; only contexts that step through it)
int map_fork_prepare(slo_ctx* ctx) {
    if (ctx->map_fork_ready || !map_fork_ok(ctx)) return 0;
    if (int r = map_ws_ensure(ctx)) return r;
    if (int r = vg_side_ready(ctx)) return r;
    VgGroup gs[6];
    map_groups(ctx, gs);
    {
        VgSide sd(ctx);
        if (int r = vg_presize(ctx, gs, SLO_MAP_FORK_G)) return r;
    }
    ctx->map_fork_ready = true;
    return 0;
}

// A few-stream step's mapping half that needs nothing of the current scan's
// odometry, issued on the side stream at the step's start, beside its
// projection, features and odometry: extractSurroundingKeyFrames' selection
// (k_mo_prepare half 2; MO:1127-1166), the local map's assembly (MO:1168-1222)
// and the VoxelGrids of the two local maps and of the raw scan (MO:1224-1230,
// the Scan Context input), then the hash grids over the DS maps.  map_run's
// current-scan half joins it before k_mo_concat.
int map_side_fork(slo_ctx* ctx) {
    DevView& v = ctx->v;
    const int S = ctx->S;
    const int SS = ST_STRIDE;
    StreamState* st0 = v.st;
    auto fld = [&](int32_t StreamState::*f) { return &(st0->*f); };
    int r;
    SLO_CHECK(hipEventRecord(ctx->ev_fork, ctx->stream));   // (side: map_fork_prepare made it)
    SLO_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    {
        VgSide sd(ctx);
        SLO_LAUNCH(ctx, "mo_prepare", k_mo_prepare, dim3(S), dim3(256), 0, v, 2);
        SLO_LAUNCH(ctx, "mo_assemble", k_mo_assemble, dim3(v.MAPK, S), dim3(256), 0, v, 0);
        VgGroup gs[6];
        map_groups(ctx, gs);
        if ((r = vg_run_groups(ctx, "map_local", gs, SLO_MAP_FORK_G))) return r;
        if ((r = grid_build(ctx, ctx->grid_c, v.map_c_ds, v.cap_mc, fld(&StreamState::n_cmap_ds), SS))) return r;
        if ((r = grid_build(ctx, ctx->grid_s, v.map_s_ds, v.cap_ms, fld(&StreamState::n_smap_ds), SS))) return r;
    }
    SLO_CHECK(hipEventRecord(ctx->ev_join, ctx->side));
    ctx->map_forked = true;
    return 0;
}

int map_run(slo_ctx* ctx) {
    DevView& v = ctx->v;
    const int S = ctx->S;
    const int SS = ST_STRIDE;
    StreamState* st0 = v.st;
    auto fld = [&](int32_t StreamState::*f) { return &(st0->*f); };
    const bool forked = ctx->map_forked;   // map_side_fork issued the local map's half
    ctx->map_forked = false;
    SLO_LAUNCH(ctx, "mo_prepare", k_mo_prepare, dim3(S), dim3(256), 0, v, forked ? 1 : 3);
    if (forked) {
        VgGroup gs[6];
        map_groups(ctx, gs);
        int r = vg_run_groups(ctx, "map_step", gs + SLO_MAP_FORK_G, 6 - SLO_MAP_FORK_G);   // corner, surf, outlier (MO:1233-1263)
        if (r) return r;
        SLO_CHECK(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
        return map_run_rest(ctx, true);
    }
    SLO_LAUNCH(ctx, "mo_assemble", k_mo_assemble, dim3(v.MAPK, S), dim3(256), 0, v, 1);
    // local map DS (MO:1224-1230) and current scan DS (MO:1233-1263): the six
    // filters as one batched VoxelGrid call (vg_run_groups: (filter, stream)
    // pairs as the sort's units), so a scan waits for one sort chain, not six
    int r;
#ifndef SLO_MAP_BATCHED_VG
#define SLO_MAP_BATCHED_VG 1
#endif
    const bool fork = !SLO_MAP_BATCHED_VG && S <= SLO_VG_FORK_STREAMS && !(ctx->timing && !ctx->timing_only.empty());
    if (SLO_MAP_BATCHED_VG) {
        VgGroup gs[6];
        map_groups(ctx, gs);
        if (map_vg_split(ctx, gs)) {   // over 2^31 items in one call: the local maps, then the rest
            if ((r = vg_run_groups(ctx, "map_step", gs, 2)) || (r = vg_run_groups(ctx, "map_step", gs + 2, 4))) return r;
        } else if ((r = vg_run_groups(ctx, "map_step", gs, 6))) {
            return r;
        }
    } else {
    // (round 3's form: one call per filter; with a few streams the two
    // local-map filters run on a side stream while the current scan's run here)
    if (fork) {
        if ((r = vg_side_ready(ctx))) return r;
        SLO_CHECK(hipEventRecord(ctx->ev_fork, ctx->stream));
        SLO_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    }
    {
        std::unique_ptr<VgSide> side(fork ? new VgSide(ctx) : nullptr);
        if ((r = vg_run(ctx, "map_corner", v.map_c, v.cap_mc, fld(&StreamState::n_corner_map), SS, v.cfg.leaf_corner,
                        v.map_c_ds, v.cap_mc, fld(&StreamState::n_cmap_ds), SS, v.cap_mc))) return r;
        if ((r = vg_run(ctx, "map_surf", v.map_s, v.cap_ms, fld(&StreamState::n_surf_map), SS, v.cfg.leaf_surf,
                        v.map_s_ds, v.cap_ms, fld(&StreamState::n_smap_ds), SS, v.cap_ms))) return r;
        if (fork) {   // the hash grids over the DS maps follow them on the side stream
            if ((r = grid_build(ctx, ctx->grid_c, v.map_c_ds, v.cap_mc, fld(&StreamState::n_cmap_ds), SS))) return r;
            if ((r = grid_build(ctx, ctx->grid_s, v.map_s_ds, v.cap_ms, fld(&StreamState::n_smap_ds), SS))) return r;
        }
    }
    if (fork) SLO_CHECK(hipEventRecord(ctx->ev_join, ctx->side));
    if ((r = vg_run(ctx, "raw", nullptr, v.P, nullptr, 1, v.cfg.leaf_sc, v.cur_raw_ds, v.P,
                    fld(&StreamState::n_raw_ds), SS, v.P))) return r;
    if ((r = vg_run(ctx, "corner", v.corner_last, v.cap_less_sharp, fld(&StreamState::cornerLastNum), SS,
                    v.cfg.leaf_corner, v.cur_c_ds, v.cap_less_sharp, fld(&StreamState::n_corner_ds), SS,
                    v.cap_less_sharp))) return r;
    if ((r = vg_run(ctx, "surf", v.surf_last, v.cap_less_flat, fld(&StreamState::surfLastNum), SS, v.cfg.leaf_surf,
                    v.cur_s_ds, v.H, fld(&StreamState::n_surf_ds), SS, v.H))) return r;
    if ((r = vg_run(ctx, "outlier", v.outl_cam, v.H, fld(&StreamState::outlier_count), SS, v.cfg.leaf_outlier,
                    v.cur_o_ds, v.cap_ko, fld(&StreamState::n_outl_ds), SS, v.cap_ko))) return r;
    if (fork) SLO_CHECK(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));   // k_mo_concat's map_ok reads the map DS sizes
    }
    return map_run_rest(ctx, fork);
}

// k_mo_concat onwards; grids_built: the hash grids over the DS maps were
// built on the side stream
static int map_run_rest(slo_ctx* ctx, bool grids_built) {
    DevView& v = ctx->v;
    const int S = ctx->S;
    const int SS = ST_STRIDE;
    StreamState* st0 = v.st;
    auto fld = [&](int32_t StreamState::*f) { return &(st0->*f); };
    int r;
    SLO_LAUNCH(ctx, "mo_concat", k_mo_concat, dim3(S), dim3(256), 0, v);
    {
        const VgGroup t = map_total_group(ctx);
        if ((r = vg_run_groups(ctx, "surf_total", &t, 1))) return r;
    }
    if (SLO_MO_PERM) SLO_LAUNCH(ctx, "mo_perm", k_mo_perm, dim3(S), dim3(256), 0, v);
    // hash grids over the DS maps (on the side stream when forked, above)
    if (!grids_built && (r = grid_build(ctx, ctx->grid_c, v.map_c_ds, v.cap_mc, fld(&StreamState::n_cmap_ds), SS))) return r;
    if (!grids_built && (r = grid_build(ctx, ctx->grid_s, v.map_s_ds, v.cap_ms, fld(&StreamState::n_smap_ds), SS))) return r;
    for (int it = 0; it < 10; ++it) {
        SLO_LAUNCH(ctx, "mo_knn", k_mo_knn, dim3(xcd_grid(S, SLO_MO_BLOCKS)), dim3(256), 0, v);
        SLO_LAUNCH(ctx, "mo_corr", k_mo_corr, dim3(xcd_grid(S, SLO_MO_BLOCKS)), dim3(256), 0, v);
        SLO_LAUNCH(ctx, "mo_solve", k_mo_solve, dim3(S), dim3(64), 0, v, it);
    }
    SLO_LAUNCH(ctx, "mo_finish", k_mo_finish, dim3(S), dim3(256), 0, v);
    SLO_CHECK(hipGetLastError());
    return pcl_fold_err(ctx);   // the VoxelGrid sorts' per-stream flags into StreamState::err
}

}  // namespace slo
