// slo_odom.hip — scan-to-scan odometry of featureAssociation.cpp for a batch
// of S streams: updateTransformation (FA:1666-1695) with the surf / corner
// correspondence searches (FA:1044-1268) and 3-DOF Gauss-Newton solvers
// (FA:1270-1478), integrateTransformation (FA:1697-1725) and
// publishCloudsLast (FA:1759-1788) / checkSystemInitialization (FA:1605-1637).
//
// The correspondence searches (every 5th iteration) run one thread per query
// across the whole chip: exact nearest neighbour in a hash grid over the
// "kd-tree" cloud (rebuilt after every scan by fa_odometry_run, like
// setInputCloud), then the ring-ordered walk for the 2nd/3rd points exactly as
// the reference (including Q7's bound).  The iterations run one workgroup per
// stream: every lane accumulates its rows of A^T A / A^T b in double-double
// (slo_ddsum.h); a wave-shuffle + LDS tree reduces them and lane 0 rounds once
// to float and runs the 3x3 QR / Jacobi / degeneracy projection.  No host
// round trip happens per iteration (launch structure below).
// Nearest-neighbour ties resolve to the lowest index (FLANN's tie order is
// traversal dependent).
#include "slo_internal.h"
#include "slo_libm.h"
#include "slo_pose.h"
#include "slo_pose_wave.h"
#include "slo_linalg.h"
#include <float.h>

namespace slo {

using slo_pose::P4;

__device__ inline P4 ld4(const float4* a, int i) { float4 q = a[i]; return P4{q.x, q.y, q.z, q.w}; }

__device__ inline float sq3_ref(const float4& a, const P4& b) {  // (a-b)^2 summed left to right
    return (a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z);
}
__device__ inline float sqdist_flann(const P4& q, const float4& p) {  // ((0+d0^2)+d1^2)+d2^2, d = q - p
    float d0 = q.x - p.x, d1 = q.y - p.y, d2 = q.z - p.z;
    float r = 0.0f;
    r += d0 * d0;
    r += d1 * d1;
    r += d2 * d2;
    return r;
}

// Exact 1-NN in the hash grid of the "tree" cloud: rings of cells at
// Chebyshev distance r = 0,1,..; every point outside rings <= r is more than
// r*cell away, so once the best float distance is < (r*cell)^2 nothing unseen
// can beat or tie it (fl(d) is monotone in the exact distance, GridView).  The
// rings stop where the nearestFeatureSearchSqDist gate lies: anything further
// fails it anyway, as it would after the reference's exact FLANN search.
// Ties -> lowest index.
__device__ inline void nn1_grid(const GridView& g, int s, float gate, const P4& q, int& bi, float& bd) {
    // the nearest point if its squared distance is <= gate (ties -> lowest
    // index); the caller keeps it only when < gate (FA:1009), so the search
    // is a ball of the gate's radius (R cells) bounded by the best so far
    constexpr int R = SLO_ODO_SURF_R;
    bi = INT_MAX; bd = gate;
    if (isfinite(q.x) && isfinite(q.y) && isfinite(q.z))
        grid_ball<R>(g, s, q.x, q.y, q.z, [&]() { return bd; }, [&](const float4& p) {
            const float d = sqdist_flann(q, p);
            const int idx = __float_as_int(p.w);
            if (d < bd || (d == bd && idx < bi)) { bd = d; bi = idx; }
        });
    if (bi == INT_MAX) { bi = -1; bd = FLT_MAX; }
}

// The same 1-NN by an aligned group of G lanes of one query (the few-stream
// surf search, where one stream's queries leave most of the chip idle and a
// query's latency is its chain of dependent loads): the walk of nn1_grid —
// the probed cell, then the rows of the (2R+1)^2 box nearest first — with
// each cell's / row's entry run dealt over the group (G x U loads in flight)
// and the group's best (d, index) taken after each, so every row is cut by
// the bound of all points seen so far.  Exact: rows and points are skipped
// only when strictly farther than a distance already found, and the
// (distance, index) minimum does not depend on the visiting order.
template <int G>
__device__ inline void nn1_grid_group(const GridView& g, int s, float gate, const P4& q, bool act, int sub, int& bi,
                                      float& bd) {
    constexpr int R = SLO_ODO_SURF_R, N = GridRows<R>::N, U = 2;
    bi = INT_MAX; bd = gate;
    if (act && isfinite(q.x) && isfinite(q.y) && isfinite(q.z)) {
        const float inv = g.inv, cell = g.cell, c2 = cell * cell;
        const int cx = grid_cell(q.x, inv), cy = grid_cell(q.y, inv), cz = grid_cell(q.z, inv);
        const size_t gb = (size_t)s * (g.T + 1);
        const int base = g.off[gb];
        const float4* E = g.ent + (size_t)s * g.es;
        auto run = [&](int e0, int e1, int yy, int zz, int xa, int xb, bool skip_cx) {   // entries [e0, e1)
            for (int e = e0 + sub; e < e1; e += G * U) {
                float4 p[U];
#pragma unroll
                for (int u = 0; u < U; ++u) p[u] = E[min(e + u * G, e1 - 1)];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (e + u * G >= e1) break;
                    const int px = grid_cell(p[u].x, inv);
                    if (grid_cell(p[u].y, inv) != yy || grid_cell(p[u].z, inv) != zz || px < xa || px > xb ||
                        (skip_cx && px == cx)) continue;
                    const float d = sqdist_flann(q, p[u]);
                    const int idx = __float_as_int(p[u].w);
                    if (d < bd || (d == bd && idx < bi)) { bd = d; bi = idx; }
                }
            }
#pragma unroll
            for (int o = 1; o < G; o <<= 1) {
                const float d2 = __shfl_xor(bd, o, 64);
                const int i2 = __shfl_xor(bi, o, 64);
                if (d2 < bd || (d2 == bd && i2 < bi)) { bd = d2; bi = i2; }
            }
        };
        {   // the probed cell
            const int h0 = (int)grid_hash(cx, cy, cz, g.T);
            run(g.off[gb + h0] - base, g.off[gb + h0 + 1] - base, cy, cz, cx, cx, false);
        }
        for (int k = 0; k < N; ++k) {   // bd, bi: the same in the group's lanes here
            const float b = bd;
            if ((float)kGridRows<R>.gap[k] * c2 > b) break;
            const int dy = kGridRows<R>.dy[k], dz = kGridRows<R>.dz[k];
            const int yy = cy + dy, zz = cz + dz;
            const float ey = dy > 0 ? (float)yy * cell - q.y : (dy < 0 ? q.y - (float)(yy + 1) * cell : 0.0f);
            const float ez = dz > 0 ? (float)zz * cell - q.z : (dz < 0 ? q.z - (float)(zz + 1) * cell : 0.0f);
            float lb = ey * ey;
            lb += ez * ez;
            if (lb > b) continue;
            const float rx = sqrtf((b - lb) * 1.0001f + 1e-5f * b) + 1e-3f;
            const int xa = max(cx - R, grid_cell(q.x - rx, inv)), xb = min(cx + R, grid_cell(q.x + rx, inv));
            const int h = (int)grid_hash(xa, yy, zz, g.T), len = xb - xa + 1;
            const int h2 = min(h + len, g.T), w1 = h + len - h2;   // w1: buckets wrapped to the table start
            const int e0 = g.off[gb + h] - base, e1 = g.off[gb + h2] - base;
            const int f1 = w1 > 0 ? g.off[gb + w1] - base : 0;
            run(e0, e1, yy, zz, xa, xb, k == 0);   // k == 0: the probed cell's row
            if (w1 > 0) run(0, f1, yy, zz, xa, xb, k == 0);
        }
    }
    if (bi == INT_MAX) { bi = -1; bd = FLT_MAX; }
}

// block-wide double-double sum of NV terms + one int (slo_ddsum.h); result
// valid in lane 0 of wave 0
template <int NV>
__device__ inline void block_reduce(slo_dd::DD* acc, int& cnt, slo_dd::DD* sh, int* shi) {
    for (int o = 32; o > 0; o >>= 1) {
        for (int k = 0; k < NV; ++k) {
            slo_dd::DD y{__shfl_xor(acc[k].hi, o, 64), __shfl_xor(acc[k].lo, o, 64)};
            slo_dd::merge(acc[k], y);
        }
        cnt += __shfl_xor(cnt, o, 64);
    }
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        for (int k = 0; k < NV; ++k) sh[w * NV + k] = acc[k];
        shi[w] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < NV; ++k) acc[k] = sh[k];
        cnt = shi[0];
        for (int ww = 1; ww < nw; ++ww) {
            for (int k = 0; k < NV; ++k) slo_dd::merge(acc[k], sh[ww * NV + k]);
            cnt += shi[ww];
        }
    }
}

// one row of matA / matB into AtA (upper) / AtB; float products are exact in double
__device__ inline void accumulate9(slo_dd::DD* acc, double A0, double A1, double A2, double B) {
    slo_dd::add(acc[0], A0 * A0); slo_dd::add(acc[1], A0 * A1); slo_dd::add(acc[2], A0 * A2);
    slo_dd::add(acc[3], A1 * A1); slo_dd::add(acc[4], A1 * A2); slo_dd::add(acc[5], A2 * A2);
    slo_dd::add(acc[6], A0 * B); slo_dd::add(acc[7], A1 * B); slo_dd::add(acc[8], A2 * B);
}

// lane-0 tail shared by calculateTransformationSurf/Corner (FA:1324-1377)
__device__ inline bool solve_step(StreamState& st, const slo_dd::DD* acc, int iterCount, float* X) {
    // acc: AtA(00,01,02,11,12,22), AtB(0,1,2); matAtA / matAtB are float Mats
    float r[9];
    for (int k = 0; k < 9; ++k) r[k] = slo_dd::to_float(acc[k]);
    float AtA[9] = {r[0], r[1], r[2], r[1], r[3], r[4], r[2], r[4], r[5]};
    float AtB[3] = {r[6], r[7], r[8]};
    slo_la::solve_qr(AtA, AtB, 3, 3, X);
    if (iterCount == 0) {
        // the data-indexed arrays in LDS (private ones went to scratch memory)
        __shared__ float E[3], V[9], V2[9], Vi[9], wa[9];
        __shared__ int wr[6], wc[6];
        slo_la::eigen_sym_ws<3>(AtA, E, V, wa, wr, wc);
        for (int i = 0; i < 9; ++i) V2[i] = V[i];
        st.isDegenerate_fa = 0;
        for (int i = 2; i >= 0; i--) {
            if (E[i] < 10.0f) {
                for (int j = 0; j < 3; j++) V2[i * 3 + j] = 0;
                st.isDegenerate_fa = 1;
            } else break;
        }
        slo_la::inv(V, 3, Vi);
        slo_la::mul(Vi, V2, 3, 3, 3, st.matP_fa);
    }
    if (st.isDegenerate_fa) {
        float X2[3] = {X[0], X[1], X[2]};
        slo_la::mul(st.matP_fa, X2, 3, 3, 1, X);
    }
    return true;
}

// ---------------------------------------------------------------- launch structure
// The 25 + 25 Gauss-Newton iterations of a stream are sequential, the streams
// independent.  Each phase (surf, then corner) runs as 5 rounds of
//   k_fa_search_*   one thread (surf) / 4 waves (corner) per query: the
//                    correspondence search of iteration 5b (findCorresponding*
//                    runs when iterCount % 5 == 0, FA:1157 / 1046) — the
//                    expensive part, spread over the whole chip;
//   k_fa_iter<PH>    one workgroup per stream: iterations 5b .. 5b+4 (residuals,
//                    double-double normal equations, lane-0 solve, convergence).
// StreamState::odo_phase carries the control flow between launches:
// 0 = surf running, 1 = corner running, 2 = solved (or skipped), 3 = init scan.

// the clouds becoming *Last keep the ring structure of less_sharp / less_flat
__device__ inline void copy_ring_offsets(const DevView& v, int s) {
    const int n = 2 * (v.cfg.n_scan + 1);
    for (int k = threadIdx.x; k < n; k += blockDim.x) v.roff_last[(size_t)s * n + k] = v.roff_cur[(size_t)s * n + k];
}

#define SLO_PERM_MAX 2048   // >= cap_sharp = 12 R (R <= 128)
__device__ inline uint64_t sx_key(float x, int idx) {
    uint32_t u = __float_as_uint(x);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((uint64_t)u << 32) | (uint32_t)idx;
}

// sorts key[0..n) ascending in LDS (np = next power of two >= n, padded with ~0)
__device__ inline void lds_bitonic(uint64_t* key, int n, int np) {
    const int tid = threadIdx.x, T = blockDim.x;
    for (int i = n + tid; i < np; i += T) key[i] = ~0ull;
    __syncthreads();
    for (int k = 2; k <= np; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < np; i += T) {
                const int l = i ^ j;
                if (l > i) {
                    const uint64_t x = key[i], y = key[l];
                    if ((x > y) == ((i & k) == 0)) { key[i] = y; key[l] = x; }
                }
            }
            __syncthreads();
        }
}

// The bitonic network over 64 * NE keys in one wave's registers, for the
// slice of positions base .. base + 64 NE - 1 of a longer array: each
// element's direction comes from its position in the whole array (up when
// (position & size) == 0), so the slices come out sorted in alternating
// directions, as the network's later stages need.  sx_chunk_sort runs the
// stages of size 2 .. 64 NE; sx_chunk_merge the strides 32 NE .. 1 of one
// later stage of size `size`.
template <int NE>
__device__ inline void sx_cx(unsigned long long* k, int lane, int base, int size, int stride) {
    if (stride >= 64) {   // partner in the same lane
        const int es = stride >> 6;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            if (e & es) continue;
            const bool up = ((base + e * 64 + lane) & size) == 0;
            const unsigned long long x = k[e], y = k[e | es];
            const bool sw = up ? (x > y) : (x < y);
            k[e] = sw ? y : x;
            k[e | es] = sw ? x : y;
        }
    } else {              // partner in lane ^ stride
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const unsigned long long y = __shfl_xor(k[e], stride, 64);
            const bool up = ((base + e * 64 + lane) & size) == 0;
            const bool take_min = up == ((lane & stride) == 0);
            k[e] = take_min ? (k[e] < y ? k[e] : y) : (k[e] > y ? k[e] : y);
        }
    }
}
template <int NE>
__device__ inline void sx_chunk_sort(unsigned long long* k, int lane, int base) {
#pragma unroll
    for (int size = 2; size <= 64 * NE; size <<= 1)
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) sx_cx<NE>(k, lane, base, size, stride);
}
template <int NE>
__device__ inline void sx_chunk_merge(unsigned long long* k, int lane, int base, int size) {
#pragma unroll
    for (int stride = 32 * NE; stride > 0; stride >>= 1) sx_cx<NE>(k, lane, base, size, stride);
}

// key[0, n) in LDS (capacity >= max(512, n rounded up to a power of two))
// sorted ascending by the workgroup: 512-key slices in the waves' registers,
// then the merge stages as in k_fa_sx_long
__device__ inline void lds_slice_sort(uint64_t* key, int n) {
    constexpr int NE = 8, CH = 64 * NE;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    int np = CH;
    while (np < n) np <<= 1;
    __syncthreads();   // the caller's key writes
    for (int c = wv; c * CH < np; c += nwv) {
        unsigned long long k[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int i = c * CH + e * 64 + lane;
            k[e] = i < n ? key[i] : ~0ull;
        }
        sx_chunk_sort<NE>(k, lane, c * CH);
#pragma unroll
        for (int e = 0; e < NE; ++e) key[c * CH + e * 64 + lane] = k[e];
    }
    __syncthreads();
    for (int size = 2 * CH; size <= np; size <<= 1) {
        for (int stride = size >> 1; stride >= CH; stride >>= 1) {
            for (int i = threadIdx.x; i < np; i += blockDim.x) {
                const int l = i ^ stride;
                if (l > i) {
                    const uint64_t x = key[i], y = key[l];
                    if ((x > y) == ((i & size) == 0)) { key[i] = y; key[l] = x; }
                }
            }
            __syncthreads();
        }
        for (int c = wv; c * CH < np; c += nwv) {
            unsigned long long k[NE];
#pragma unroll
            for (int e = 0; e < NE; ++e) k[e] = key[c * CH + e * 64 + lane];
            sx_chunk_merge<NE>(k, lane, c * CH, size);
#pragma unroll
            for (int e = 0; e < NE; ++e) key[c * CH + e * 64 + lane] = k[e];
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) k_fa_odo_begin(DevView v, int first_scan) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    const int tid = threadIdx.x, T = blockDim.x;
    const int nLS = st.n_less_sharp, nLF = st.n_less_flat;
    if (first_scan) {  // checkSystemInitialization (FA:1605-1637): swap, build trees, no odometry
        const float4* lsharp = v.less_sharp + (size_t)s * v.cap_less_sharp;
        const float4* lflat = v.less_flat + (size_t)s * v.cap_less_flat;
        float4* cnext = v.corner_next + (size_t)s * v.cap_less_sharp;
        float4* snext = v.surf_next + (size_t)s * v.cap_less_flat;
        float4* kdc = v.kd_corner + (size_t)s * v.cap_less_sharp;
        float4* kds = v.kd_surf + (size_t)s * v.cap_less_flat;
        for (int i = tid; i < nLS; i += T) { cnext[i] = lsharp[i]; kdc[i] = lsharp[i]; }
        for (int i = tid; i < nLF; i += T) { snext[i] = lflat[i]; kds[i] = lflat[i]; }
        copy_ring_offsets(v, s);
        if (tid == 0) {
            st.cornerLastNum = nLS; st.surfLastNum = nLF;
            st.kdCornerNum = nLS; st.kdSurfNum = nLF;
            st.kd_set = 1;
            st.iters_surf = st.iters_corner = 0;
            st.odo_phase = 3;
            st.transformSum[0] += v.imu[s].pitchStart;   // FA:1633-1634
            st.transformSum[2] += v.imu[s].rollStart;
        }
        return;
    }
    if (tid == 0) {
        // updateInitialGuess (FA:1639-1664)
        ImuState& m = v.imu[s];
        m.pitchLast = m.pitchCur;
        m.yawLast = m.yawCur;
        m.rollLast = m.rollCur;
        for (int k = 0; k < 3; ++k) {
            m.shiftFromStart[k] = 0.0f;   // imuShiftFromStart*Cur: never set (no ShiftToStartIMU call)
            m.veloFromStart[k] = m.veloFromStartCur[k];
        }
        float* tcur = st.transformCur;
        if (m.angFromStart[0] != 0 || m.angFromStart[1] != 0 || m.angFromStart[2] != 0) {
            tcur[0] = -m.angFromStart[1];
            tcur[1] = -m.angFromStart[2];
            tcur[2] = -m.angFromStart[0];
        }
        if (m.veloFromStart[0] != 0 || m.veloFromStart[1] != 0 || m.veloFromStart[2] != 0) {
            tcur[3] -= m.veloFromStart[0] * v.cfg.scan_period;
            tcur[4] -= m.veloFromStart[1] * v.cfg.scan_period;
            tcur[5] -= m.veloFromStart[2] * v.cfg.scan_period;
        }
        // updateTransformation (FA:1666-1672)
        st.iters_surf = st.iters_corner = 0;
        st.odo_phase = (st.cornerLastNum < 10 || st.surfLastNum < 100) ? 2 : 0;
    }
    // the sharp points in x order: k_fa_search_corner groups its queries by
    // it (a grouping only; results do not depend on it)
    __shared__ uint64_t key[SLO_PERM_MAX];   // (>= 512: lds_slice_sort's slices)
    const int ns = st.n_sharp;
    const float4* sp = v.sharp + (size_t)s * v.cap_sharp;
    for (int i = tid; i < ns; i += T) key[i] = sx_key(sp[i].x, i);
    lds_slice_sort(key, ns);
    for (int i = tid; i < ns; i += T) v.sharp_perm[(size_t)s * v.cap_sharp + i] = (int)(uint32_t)key[i];
}

// ---------------------------------------------------------------- x-sorted clouds
// The correspondence searches are nearest-point queries over (a) the whole
// corner "tree" cloud and (b) single rings of the *Last clouds restricted to
// index ranges (the reference's ring-ordered walks).  Both run as sweeps over
// an x-sorted copy: start at the query's x (binary search) and walk outward in
// both directions until fl((p.x - q.x)^2) exceeds the current bound.  The
// distance expressions add non-negative squares to that first term, and float
// subtraction / squaring are monotone, so every point the sweep stops before
// is strictly farther than the bound: the result (with its tie rule) equals
// the exhaustive walk's.
// one wave per (stream, ring), four rings per workgroup: the ring's segment
// of the cloud becoming surf_last sorted by x — a bitonic network over the
// segment's 64 * NE (x, index) keys held in registers (lane-local stages in
// registers, cross-lane stages by shuffles), NE chosen per ring
template <int NE>
__device__ inline void sx_sort_wave(const float4* in, float4* out, int a, int n, int lane) {
    unsigned long long k[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        const int i = e * 64 + lane;
        k[e] = i < n ? sx_key(in[a + i].x, a + i) : ~0ull;
    }
    constexpr int N = 64 * NE;
#pragma unroll
    for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 64) {   // partner in the same lane
                const int es = stride >> 6;
#pragma unroll
                for (int e = 0; e < NE; ++e) {
                    if (e & es) continue;
                    const bool up = ((e * 64 + lane) & size) == 0;
                    const unsigned long long x = k[e], y = k[e | es];
                    const bool sw = up ? (x > y) : (x < y);
                    k[e] = sw ? y : x;
                    k[e | es] = sw ? x : y;
                }
            } else {              // partner in lane ^ stride
#pragma unroll
                for (int e = 0; e < NE; ++e) {
                    const unsigned long long y = __shfl_xor(k[e], stride, 64);
                    const bool up = ((e * 64 + lane) & size) == 0;
                    const bool take_min = up == ((lane & stride) == 0);
                    k[e] = take_min ? (k[e] < y ? k[e] : y) : (k[e] > y ? k[e] : y);
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        const int i = e * 64 + lane;
        if (i < n) {
            const int idx = (int)(uint32_t)k[e];
            const float4 p = in[idx];
            out[a + i] = make_float4(p.x, p.y, p.z, __int_as_float(idx));
        }
    }
}

#define SLO_SX_RING_MAX 4096   // >= horizon_scan limit (slo_create): a ring holds <= C points
__global__ void __launch_bounds__(256) k_fa_sx_rings(DevView v, int nb) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, nb, s, chunk);
    if (s >= v.S) return;
    const int R = v.cfg.n_scan;
    const int lane = threadIdx.x & 63, r = chunk * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int32_t* rf = v.roff_last + ((size_t)s * 2 + 1) * (R + 1);   // == roff_cur after k_fa_odo_finish
    const int a = rf[r], n = rf[r + 1] - a;
    if (n <= 0) return;
    const float4* in = v.surf_next + (size_t)s * v.cap_less_flat;
    float4* out = v.sx_surf_next + (size_t)s * v.cap_less_flat;
    if (n <= 64) sx_sort_wave<1>(in, out, a, n, lane);
    else if (n <= 128) sx_sort_wave<2>(in, out, a, n, lane);
    else if (n <= 256) sx_sort_wave<4>(in, out, a, n, lane);
    else if (n <= 512) sx_sort_wave<8>(in, out, a, n, lane);
    // longer rings: k_fa_sx_long
}

// rings of more than 512 points, one workgroup of four waves each: every
// 512-key slice sorted in a wave's registers, then the network's merge stages
// (size 1024, 2048, 4096) with the strides of 512 and more through LDS and
// the smaller ones again in registers — five to nine barriers instead of the
// 66-78 of a bitonic sort in LDS (the (x, index) keys are a total order: any
// correct sort gives the same result)
__global__ void __launch_bounds__(256) k_fa_sx_long(DevView v, int nb) {
    int s, r;
    xcd_stream_chunk(blockIdx.x, nb, s, r);
    if (s >= v.S) return;
    const int R = v.cfg.n_scan;
    const int32_t* rf = v.roff_last + ((size_t)s * 2 + 1) * (R + 1);
    const int a = rf[r], n = rf[r + 1] - a;
    if (n <= 512) return;
    const float4* in = v.surf_next + (size_t)s * v.cap_less_flat;
    float4* out = v.sx_surf_next + (size_t)s * v.cap_less_flat;
    __shared__ uint64_t key[SLO_SX_RING_MAX];
    constexpr int NE = 8, CH = 64 * NE;   // a wave's slice
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int np = CH;
    while (np < n) np <<= 1;
    for (int c = wv; c * CH < np; c += 4) {   // the slices, sorted in registers
        unsigned long long k[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int i = c * CH + e * 64 + lane;
            k[e] = i < n ? sx_key(in[a + i].x, a + i) : ~0ull;
        }
        sx_chunk_sort<NE>(k, lane, c * CH);
#pragma unroll
        for (int e = 0; e < NE; ++e) key[c * CH + e * 64 + lane] = k[e];
    }
    __syncthreads();
    for (int size = 2 * CH; size <= np; size <<= 1) {
        for (int stride = size >> 1; stride >= CH; stride >>= 1) {   // across slices: through LDS
            for (int i = threadIdx.x; i < np; i += blockDim.x) {
                const int l = i ^ stride;
                if (l > i) {
                    const uint64_t x = key[i], y = key[l];
                    if ((x > y) == ((i & size) == 0)) { key[i] = y; key[l] = x; }
                }
            }
            __syncthreads();
        }
        for (int c = wv; c * CH < np; c += 4) {   // within a slice: in registers
            unsigned long long k[NE];
#pragma unroll
            for (int e = 0; e < NE; ++e) k[e] = key[c * CH + e * 64 + lane];
            sx_chunk_merge<NE>(k, lane, c * CH, size);
#pragma unroll
            for (int e = 0; e < NE; ++e) key[c * CH + e * 64 + lane] = k[e];
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int idx = (int)(uint32_t)key[i];
        const float4 p = in[idx];
        out[a + i] = make_float4(p.x, p.y, p.z, __int_as_float(idx));
    }
}

// one workgroup per stream: the corner "tree" cloud sorted by x, whenever the
// tree is (re)built (checkSystemInitialization, or publishCloudsLast with
// enough points, FA:1779-1786)
template <int NP>
__global__ void __launch_bounds__(1024) k_fa_sx_kd(DevView v) {
    const int s = blockIdx.x;
    const StreamState& st = v.st[s];
    if (!st.kd_set) return;
    const int n = st.kdCornerNum;
    const float4* in = v.kd_corner + (size_t)s * v.cap_less_sharp;
    float4* out = v.sx_kd_corner + (size_t)s * v.cap_less_sharp;
    __shared__ uint64_t key[NP];
    static_assert(NP >= 512, "lds_slice_sort pads to 512-key slices");
    for (int i = threadIdx.x; i < n; i += blockDim.x) key[i] = sx_key(in[i].x, i);
    lds_slice_sort(key, n);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int idx = (int)(uint32_t)key[i];
        const float4 p = in[idx];
        out[i] = make_float4(p.x, p.y, p.z, __int_as_float(idx));
    }
}

// the same as sx_lower, by a whole wave (every lane gets the result): each
// round loads 64 equally spaced x values and narrows [lo, hi) to one stride
// by a ballot of the (monotone) "x < qx" predicate, so a cloud of <= 4096
// points takes two dependent loads instead of a dozen
__device__ inline int sx_lower_wave(const float4* a, int lo, int hi, float qx) {
    const int lane = threadIdx.x & 63;
    while (hi - lo > 64) {
        const int step = (hi - lo + 63) / 64;
        const int idx = lo + lane * step;
        const bool p = idx < hi && a[idx].x < qx;
        const int c = __popcll(__ballot(p));
        const int nlo = c == 0 ? lo : lo + (c - 1) * step + 1;
        hi = min(hi, lo + c * step);
        lo = nlo;
    }
    const int idx = lo + lane;
    const bool p = idx < hi && a[idx].x < qx;
    return lo + __popcll(__ballot(p));
}

// first position in a[lo, hi) whose x is >= qx
__device__ inline int sx_lower(const float4* a, int lo, int hi, float qx) {
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (a[m].x < qx) lo = m + 1; else hi = m;
    }
    return lo;
}

// sweep a[lo, hi) outward from position j0 (4 loads in flight); visit(p) for
// every point until fl((p.x - qx)^2) > bound()
template <class B, class F>
__device__ inline void sx_sweep(const float4* a, int lo, int hi, int j0, float qx, B&& bound, F&& visit) {
    for (int j = j0; j < hi; j += 4) {
        float4 p[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) p[u] = a[min(j + u, hi - 1)];
        bool stop = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (stop || j + u >= hi) { stop = true; continue; }
            const float dx = p[u].x - qx;
            if (dx * dx > bound()) { stop = true; continue; }
            visit(p[u]);
        }
        if (stop) break;
    }
    for (int j = j0 - 1; j >= lo; j -= 4) {
        float4 p[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) p[u] = a[max(j - u, lo)];
        bool stop = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (stop || j - u < lo) { stop = true; continue; }
            const float dx = p[u].x - qx;
            if (dx * dx > bound()) { stop = true; continue; }
            visit(p[u]);
        }
        if (stop) break;
    }
}

// The reference's 2nd / 3rd point walks (FA:1058-1099, 1169-1225) keep, per
// target, the strict minimum of sq3_ref first over a forward index range
// (ties -> lowest index), then over a backward range (replaced only by a
// strictly smaller distance; ties -> the first met going down = highest
// index), starting from the gate (strict).  As one total order: the smallest
// (d, class, t) with class 0 / t = idx forward, class 1 / t = -idx backward,
// and the gate itself (d = gate, class -1) never beaten by a tie.
struct WalkBest {
    float d; int cls, t;
    __device__ void init(float gate) { d = gate; cls = -1; t = 0; }
    __device__ void offer(float dd, int c, int tt) {
        if (dd < d || (dd == d && (c < cls || (c == cls && tt < t)))) { d = dd; cls = c; t = tt; }
    }
    __device__ int index() const { return cls < 0 ? -1 : (cls == 0 ? t : -t); }
};

// sweep ring r of the x-sorted cloud `sx` (segment [rf[r], rf[r+1])),
// classifying each point by its index: [f0, f1) forward, [b0, b1) backward
__device__ inline void ring_walk(const float4* sx, const int32_t* rf, int R, int r, const P4& q,
                                 int f0, int f1, int b0, int b1, WalkBest& wb) {
    if (r < 0 || r >= R) return;
    const int lo = rf[r], hi = rf[r + 1];
    if (lo >= hi || (max(f0, lo) >= min(f1, hi) && max(b0, lo) >= min(b1, hi))) return;
    const int j0 = sx_lower(sx, lo, hi, q.x);
    sx_sweep(sx, lo, hi, j0, q.x, [&]() { return wb.d; }, [&](const float4& p) {
        const int idx = __float_as_int(p.w);
        const bool fw = idx >= f0 && idx < f1, bw = idx >= b0 && idx < b1;
        if (!fw && !bw) return;
        wb.offer(sq3_ref(p, q), fw ? 0 : 1, fw ? idx : -idx);
    });
}

// the same over ring r of the unsorted cloud, in index order (short rings)
__device__ inline void ring_walk_linear(const float4* a, const int32_t* rf, int R, int r, const P4& q,
                                        int f0, int f1, int b0, int b1, WalkBest& wb) {
    if (r < 0 || r >= R) return;
    const int lo = rf[r], hi = rf[r + 1];
    for (int pass = 0; pass < 2; ++pass) {
        const int j0 = max(lo, pass == 0 ? f0 : b0), j1 = min(hi, pass == 0 ? f1 : b1);
#pragma unroll 4
        for (int j = j0; j < j1; ++j) wb.offer(sq3_ref(a[j], q), pass, pass == 0 ? j : -j);
    }
}

#ifndef SLO_SURF_LINEAR
#define SLO_SURF_LINEAR 0   // 1: surf walks in index order over surf_last (no x-sorted rings)
#endif
#ifndef SLO_DIAG_ODO
#define SLO_DIAG_ODO 0   // 1: k_fa_search_* add per-wave phase cycles to StreamState::dbg[0..3]
#endif
#if SLO_DIAG_ODO
#define ODO_STAMP(k) do { const unsigned long long t_n = clock64(); \
    if ((threadIdx.x & 63) == 0) atomicAdd(&v.st[s].dbg[k], t_n - t_d); t_d = t_n; } while (0)
#else
#define ODO_STAMP(k) do {} while (0)
#endif

// The *Last clouds are concatenated ring by ring, so the reference's walk for
// the 2nd / 3rd points — step away from `closest` until the ring leaves
// [cscan-2, cscan+2], sorting each point into "same/lower ring" or "other
// ring" by its ring — is a minimum over index ranges cut at the ring
// boundaries (roff_last) with the visiting order's tie rule (WalkBest):
// forward over [closest+1, ...) bounded by Q7's min(query count, cloud
// size), then backward from closest-1.

// findCorrespondingSurfFeatures (FA:1155-1268), one thread per query: exact
// 1-NN in the tree cloud through the 1 m hash grid, then the walks for the
// 2nd / 3rd points as x-sweeps over the rings of the x-sorted surf_last.
__global__ void __launch_bounds__(256) k_fa_search_surf(DevView v, int nb) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, nb, s, chunk);
    if (s >= v.S) return;
    const StreamState& st = v.st[s];
    if (st.odo_phase != 0) return;
    const int i = chunk * blockDim.x + threadIdx.x;
    const int nq = st.n_flat;
    if (chunk * (int)blockDim.x >= nq) return;   // uniform
#if SLO_DIAG_ODO
    unsigned long long t_d = clock64();
#endif
    const bool active = i < nq;
    const float gate = v.cfg.nearest_feature_search_sq_dist;
    const int R = v.cfg.n_scan;
    float tc[6];
    for (int k = 0; k < 6; ++k) tc[k] = st.transformCur[k];
    const P4 sel = slo_pose::transform_to_start(ld4(v.flat + (size_t)s * v.cap_flat, active ? i : 0), tc);
    const int32_t* rf = v.roff_last + ((size_t)s * 2 + 1) * (R + 1);
    auto ring_first = [&](int r) { return rf[min(max(r, 0), R)]; };
    int ci = -1; float cd = FLT_MAX;
    if (active) nn1_grid(v.g_os, s, gate, sel, ci, cd);
    ODO_STAMP(0);
    const float4* sx = v.sx_surf_last + (size_t)s * v.cap_less_flat;
    const float4* slast = v.surf_last + (size_t)s * v.cap_less_flat;
    const int surfLastNum = st.surfLastNum;
    int closest = -1, i2 = -1, i3 = -1;
    if (active && cd < gate && ci >= 0 && ci < surfLastNum) {
        closest = ci;
        const int cscan = (int)slast[closest].w;
        const int lim = min(nq, surfLastNum);                        // Q7: bounded by the flat count
        const int e0 = ring_first(cscan + 1), e2 = ring_first(cscan + 3);
        const int b0 = ring_first(cscan), b2 = ring_first(cscan - 2);
        WalkBest w2, w3;
        w2.init(gate); w3.init(gate);
#if SLO_SURF_LINEAR
#define SURF_WALK(...) ring_walk_linear(slast, __VA_ARGS__)
#else
#define SURF_WALK(...) ring_walk(sx, __VA_ARGS__)
#endif
        SURF_WALK(rf, R, cscan, sel, closest + 1, min(e0, lim), b0, closest, w2);   // ring == cscan
        const int f0 = max(closest + 1, e0), f1 = min(e2, lim), bb1 = min(b0, closest);
        for (int r = cscan - 2; r <= cscan + 2; ++r)                              // other rings
            if (r != cscan) SURF_WALK(rf, R, r, sel, f0, f1, b2, bb1, w3);
#undef SURF_WALK
        i2 = w2.index(); i3 = w3.index();
    }
    ODO_STAMP(1);
    if (!active) return;
    int32_t* ind = v.ind_surf + (size_t)s * v.cap_flat * 3;
    ind[3 * i] = closest; ind[3 * i + 1] = i2; ind[3 * i + 2] = i3;
}

// The same for a context of a few streams, where one stream's queries leave
// most of the chip idle and the search is the odometry's latency: eight lanes
// per query.  The lanes find the 1-NN together, eight grid rows per round
// with the bound shared after each (nn1_grid_group; dealing the rows with
// every lane pruning by its own, looser bound measured twice as slow as one
// lane's walk), then the five ring walks run one
// per lane — lane 0 the closest point's ring (the 2nd point), lanes 1-4 rings
// cscan - 2, - 1, + 1, + 2 (the 3rd) — and the 3rd point's four bests merge
// in WalkBest's order, a strict total order on (distance, class, index): the
// minimum over all offers, whatever the order of the rings.  Same results as
// k_fa_search_surf.
#define SURF_QL 8
#ifndef SLO_SURF_GROUP_NN
#define SLO_SURF_GROUP_NN 1   // the 1-NN by the query's eight lanes with a shared bound (nn1_grid_group)
#endif
#ifndef SLO_ODO_FEW
#define SLO_ODO_FEW 8   // at most this many streams: k_fa_search_surf_few
#endif
#ifndef SLO_ODO_FUSED
#define SLO_ODO_FUSED 1   // ... and k_fa_fused (a search and its iterations in one launch)
#endif
__device__ inline bool walk_better(float d, int c, int t, const WalkBest& w) {
    return d < w.d || (d == w.d && (c < w.cls || (c == w.cls && t < w.t)));
}
__device__ __forceinline__ void search_surf_few_block(const DevView& v, int s, int chunk) {
    const StreamState& st = v.st[s];
    if (st.odo_phase != 0) return;
    constexpr int QPB = 256 / SURF_QL;   // queries per workgroup
    const int sub = threadIdx.x & (SURF_QL - 1);
    const int i = chunk * QPB + (int)(threadIdx.x / SURF_QL);
    const int nq = st.n_flat;
    if (chunk * QPB >= nq) return;   // uniform
    const bool active = i < nq;
    const float gate = v.cfg.nearest_feature_search_sq_dist;
    const int R = v.cfg.n_scan;
    float tc[6];
    for (int k = 0; k < 6; ++k) tc[k] = st.transformCur[k];
    const P4 sel = slo_pose::transform_to_start(ld4(v.flat + (size_t)s * v.cap_flat, active ? i : 0), tc);
    const int32_t* rf = v.roff_last + ((size_t)s * 2 + 1) * (R + 1);
    auto ring_first = [&](int r) { return rf[min(max(r, 0), R)]; };
    int ci = -1;
    float cd = FLT_MAX;
#if SLO_DIAG_ODO
    // per wave: [4] / [5] the slowest wave's 1-NN / walk cycles, [6] / [7] their sums, [0] waves
    unsigned long long t_d = clock64(), t_nn = 0;
#endif
#if SLO_SURF_GROUP_NN
    nn1_grid_group<SURF_QL>(v.g_os, s, gate, sel, active, sub, ci, cd);
#else
    if (active) nn1_grid(v.g_os, s, gate, sel, ci, cd);
#endif
#if SLO_DIAG_ODO
    t_nn = clock64() - t_d;
    t_d = clock64();
#endif
    const float4* sx = v.sx_surf_last + (size_t)s * v.cap_less_flat;
    const float4* slast = v.surf_last + (size_t)s * v.cap_less_flat;
    const int surfLastNum = st.surfLastNum;
    const bool found = active && cd < gate && ci >= 0 && ci < surfLastNum;   // the same in the query's eight lanes
    WalkBest w;
    w.init(gate);
    if (found && sub <= 4) {
        const int closest = ci;
        const int cscan = (int)slast[closest].w;
        const int lim = min(nq, surfLastNum);                        // Q7: bounded by the flat count
        const int e0 = ring_first(cscan + 1), e2 = ring_first(cscan + 3);
        const int b0 = ring_first(cscan), b2 = ring_first(cscan - 2);
        if (sub == 0) {
            ring_walk(sx, rf, R, cscan, sel, closest + 1, min(e0, lim), b0, closest, w);   // ring == cscan
        } else {
            const int f0 = max(closest + 1, e0), f1 = min(e2, lim), bb1 = min(b0, closest);
            ring_walk(sx, rf, R, cscan + (sub <= 2 ? sub - 3 : sub - 2), sel, f0, f1, b2, bb1, w);   // other rings
        }
    }
    // the 3rd point: the best of lanes 1-4 (lane 0's walk is the 2nd point's)
    WalkBest w3;
    w3.init(gate);
    if (sub >= 1 && sub <= 4) w3 = w;
#pragma unroll
    for (int o = 1; o < SURF_QL; o <<= 1) {
        const float d2 = __shfl_xor(w3.d, o, 64);
        const int c2 = __shfl_xor(w3.cls, o, 64), t2 = __shfl_xor(w3.t, o, 64);
        if (walk_better(d2, c2, t2, w3)) { w3.d = d2; w3.cls = c2; w3.t = t2; }
    }
#if SLO_DIAG_ODO
    if ((threadIdx.x & 63) == 0) {
        const unsigned long long t_w = clock64() - t_d;
        atomicMax(&v.st[s].dbg[4], t_nn); atomicMax(&v.st[s].dbg[5], t_w);
        atomicAdd(&v.st[s].dbg[6], t_nn); atomicAdd(&v.st[s].dbg[7], t_w); atomicAdd(&v.st[s].dbg[0], 1ull);
    }
#endif
    if (!active || sub != 0) return;
    int32_t* ind = v.ind_surf + (size_t)s * v.cap_flat * 3;
    ind[3 * i] = found ? ci : -1;
    ind[3 * i + 1] = found ? w.index() : -1;
    ind[3 * i + 2] = found ? w3.index() : -1;
}
__global__ void __launch_bounds__(256) k_fa_search_surf_few(DevView v, int nb) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, nb, s, chunk);
    if (s >= v.S) return;
    search_surf_few_block(v, s, chunk);
}

// findCorrespondingCornerFeatures (FA:1044-1153): one workgroup = 64 queries
// (consecutive in x order, sharp_perm) x 4 waves.  1-NN by brute force over
// the x-window of the x-sorted tree cloud that can hold a point within the
// gate of any of the 64 queries (a wider margin than float rounding needs;
// every point outside it is farther than the gate, where the reference
// rejects the neighbour anyway), streamed through LDS: wave w takes a quarter
// of each 256-point tile, every lane keeps four independent minimum chains,
// and the 16 partial minima of a query merge by (distance, index) — the
// result of the reference's exact nearest neighbour with ties to the lowest
// index.  Then the 2nd point: wave w walks ring cscan + {-2, -1, +1, +2}[w]
// and the four WalkBests merge in LDS.
__device__ __forceinline__ void search_corner_block(const DevView& v, int s, int chunk) {
    const StreamState& st = v.st[s];
    if (st.odo_phase != 1) return;
    const int nq = st.n_sharp;
    if (chunk * 64 >= nq) return;   // uniform
#if SLO_DIAG_ODO
    unsigned long long t_d = clock64();
#endif
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int pos = chunk * 64 + lane;
    const bool active = pos < nq;
    const int i = active ? v.sharp_perm[(size_t)s * v.cap_sharp + pos] : 0;
    const float gate = v.cfg.nearest_feature_search_sq_dist;
    const int R = v.cfg.n_scan;
    // TransformToStart of the 64 queries once (wave 0), shared through LDS
    __shared__ float4 s_sel[64];
    if (w == 0) {
        float tc[6];
        for (int k = 0; k < 6; ++k) tc[k] = st.transformCur[k];
        const P4 q = slo_pose::transform_to_start(ld4(v.sharp + (size_t)s * v.cap_sharp, i), tc);
        s_sel[lane] = make_float4(q.x, q.y, q.z, q.w);
    }
    __syncthreads();
    const float4 sel4 = s_sel[lane];
    const P4 sel{sel4.x, sel4.y, sel4.z, sel4.w};
    const bool fin = active && isfinite(sel.x) && isfinite(sel.y) && isfinite(sel.z);
    // the workgroup's x-window (every wave computes the same one)
    float xmin = fin ? sel.x : FLT_MAX, xmax = fin ? sel.x : -FLT_MAX;
    for (int o = 32; o > 0; o >>= 1) {
        xmin = fminf(xmin, __shfl_xor(xmin, o, 64));
        xmax = fmaxf(xmax, __shfl_xor(xmax, o, 64));
    }
    const float4* kx = v.sx_kd_corner + (size_t)s * v.cap_less_sharp;
    const int n = st.kdCornerNum;
    int lo = 0, hi = 0;
    if (xmin <= xmax) {   // wave-uniform: xmin / xmax are wave reductions
        const float rr = sqrtf(gate) * 1.001f + 1e-3f + 1e-5f * fmaxf(fabsf(xmin), fabsf(xmax));
        lo = sx_lower_wave(kx, 0, n, xmin - rr);
        hi = sx_lower_wave(kx, lo, n, xmax + rr);
    }
    __shared__ float4 tile[256];
    __shared__ float s_d[4][64];
    __shared__ int s_i[4][64], s_c[4][64];
    float cd[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
    int ci[4] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX};
    auto take = [&](int c, const float4& p) {
        const float d = sqdist_flann(sel, p);
        const int idx = __float_as_int(p.w);
        if (d < cd[c] || (d == cd[c] && idx < ci[c])) { cd[c] = d; ci[c] = idx; }
    };
    for (int t0 = lo; t0 < hi; t0 += 256) {
        __syncthreads();
        if (t0 + tid < hi) tile[tid] = kx[t0 + tid];
        __syncthreads();
        const int m = min(256, hi - t0) - w * 64;   // this wave's share of the tile: [w*64, w*64 + m)
        if (fin && m > 0) {
            if (m >= 64) {
#pragma unroll 4
                for (int j = 0; j < 64; j += 4)
#pragma unroll
                    for (int c = 0; c < 4; ++c) take(c, tile[w * 64 + j + c]);
            } else {
                for (int j = 0; j < m; ++j) take(j & 3, tile[w * 64 + j]);
            }
        }
    }
    for (int c = 1; c < 4; ++c)
        if (cd[c] < cd[0] || (cd[c] == cd[0] && ci[c] < ci[0])) { cd[0] = cd[c]; ci[0] = ci[c]; }
    s_d[w][lane] = cd[0]; s_i[w][lane] = ci[0];
    __syncthreads();
    float bd = s_d[0][lane];
    int bi = s_i[0][lane];
    for (int k = 1; k < 4; ++k) {
        const float d = s_d[k][lane];
        const int x = s_i[k][lane];
        if (d < bd || (d == bd && x < bi)) { bd = d; bi = x; }
    }
    ODO_STAMP(2);
    const float4* clast = v.corner_last + (size_t)s * v.cap_less_sharp;
    const int32_t* rf = v.roff_last + ((size_t)s * 2 + 0) * (R + 1);
    auto ring_first = [&](int r) { return rf[min(max(r, 0), R)]; };
    const int cornerLastNum = st.cornerLastNum;
    const bool found = fin && bi != INT_MAX && bd < gate && bi < cornerLastNum;
    WalkBest wb;
    wb.init(gate);
    if (found) {
        const int cscan = (int)clast[bi].w;
        const int lim = min(nq, cornerLastNum);                      // Q7: bounded by the sharp count
        const int f0 = max(bi + 1, ring_first(cscan + 1)), f1 = min(ring_first(cscan + 3), lim);
        const int b0 = ring_first(cscan - 2), b1 = min(ring_first(cscan), bi);
        const int r = cscan + (w < 2 ? w - 2 : w - 1);
        ring_walk_linear(clast, rf, R, r, sel, f0, f1, b0, b1, wb);
    }
    __syncthreads();   // s_d / s_i reads above are done
    s_d[w][lane] = wb.d; s_c[w][lane] = wb.cls; s_i[w][lane] = wb.t;
    __syncthreads();
    ODO_STAMP(3);
    if (w != 0 || !active) return;
    for (int k = 1; k < 4; ++k) wb.offer(s_d[k][lane], s_c[k][lane], s_i[k][lane]);
    int32_t* indc = v.ind_corner + (size_t)s * v.cap_sharp * 2;
    indc[2 * i] = found ? bi : -1; indc[2 * i + 1] = found ? wb.index() : -1;
}
__global__ void __launch_bounds__(256) k_fa_search_corner(DevView v, int nb) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, nb, s, chunk);
    if (s >= v.S) return;
    search_corner_block(v, s, chunk);
}

// iterations iter0 .. iter0+4 of calculateTransformationSurf (FA:1270-1377)
// or ...Corner (FA:1379-1478) for one stream
template <int PH>
__device__ __forceinline__ void fa_iter_block(const DevView& v, int s, int iter0) {
    StreamState& st = v.st[s];
    if (st.odo_phase != PH) return;
    const int tid = threadIdx.x, T = blockDim.x;
    __shared__ float tc[6];
    __shared__ int s_ctl;      // 0 = go on, 1 = skip solve (continue), 2 = break
    __shared__ slo_dd::DD sh[4 * 9];
    __shared__ int shi[4];
    if (tid < 6) tc[tid] = st.transformCur[tid];
    if (tid == 0) s_ctl = 0;
    __syncthreads();
    const int nq = PH == 0 ? st.n_flat : st.n_sharp;
    const float4* qp = PH == 0 ? v.flat + (size_t)s * v.cap_flat : v.sharp + (size_t)s * v.cap_sharp;
    const float4* last = PH == 0 ? v.surf_last + (size_t)s * v.cap_less_flat
                                 : v.corner_last + (size_t)s * v.cap_less_sharp;
    const int32_t* ind = PH == 0 ? v.ind_surf + (size_t)s * v.cap_flat * 3 : v.ind_corner + (size_t)s * v.cap_sharp * 2;
    int iterCount = iter0;
    for (; iterCount < iter0 + 5; iterCount++) {
        slo_dd::DD acc[9];
        for (int k = 0; k < 9; ++k) acc[k] = slo_dd::zero();
        int cnt = 0;
        const float srx = slo_libm::sinf_(tc[0]), crx = slo_libm::cosf_(tc[0]);
        const float sry = slo_libm::sinf_(tc[1]), cry = slo_libm::cosf_(tc[1]);
        const float srz = slo_libm::sinf_(tc[2]), crz = slo_libm::cosf_(tc[2]);
        const float tx = tc[3], ty = tc[4], tz = tc[5];
        for (int i = tid; i < nq; i += T) {
            const P4 po = ld4(qp, i);
            const P4 sel = slo_pose::transform_to_start(po, tc);
            const P4& p = po;
            if (PH == 0) {
                const int j1 = ind[3 * i], j2 = ind[3 * i + 1], j3 = ind[3 * i + 2];
                if (!(j2 >= 0 && j3 >= 0)) continue;
                const float4 t1 = last[j1], t2 = last[j2], t3 = last[j3];
                float pa = (t2.y - t1.y) * (t3.z - t1.z) - (t3.y - t1.y) * (t2.z - t1.z);
                float pb = (t2.z - t1.z) * (t3.x - t1.x) - (t3.z - t1.z) * (t2.x - t1.x);
                float pc = (t2.x - t1.x) * (t3.y - t1.y) - (t3.x - t1.x) * (t2.y - t1.y);
                float pd = -(pa * t1.x + pb * t1.y + pc * t1.z);
                const float ps = sqrtf(pa * pa + pb * pb + pc * pc);
                pa /= ps; pb /= ps; pc /= ps; pd /= ps;
                const float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
                float sw = 1;
                if (iterCount >= 5)
                    sw = (float)(1 - 1.8 * fabsf(pd2) / sqrtf(sqrtf(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z)));
                if (!(sw > 0.1 && pd2 != 0)) continue;
                const float cx = sw * pa, cy = sw * pb, cz = sw * pc, cw = sw * pd2;
                // calculateTransformationSurf (FA:1282-1318): rows d/d(rx, rz, ty)
                const float a1 = crx * sry * srz; const float a2 = crx * crz * sry; const float a3 = srx * sry;
                const float a4 = tx * a1 - ty * a2 - tz * a3;
                const float a5 = srx * srz; const float a6 = crz * srx; const float a7 = ty * a6 - tz * crx - tx * a5;
                const float a8 = crx * cry * srz; const float a9 = crx * cry * crz; const float a10 = cry * srx;
                const float a11 = tz * a10 + ty * a9 - tx * a8;
                const float b1 = -crz * sry - cry * srx * srz; const float b2 = cry * crz * srx - sry * srz;
                const float b5 = cry * crz - srx * sry * srz; const float b6 = cry * srz + crz * srx * sry;
                const float c1 = -b6; const float c2 = b5; const float c3 = tx * b6 - ty * b5;
                const float c4 = -crx * crz; const float c5 = crx * srz; const float c6 = ty * c5 + tx * -c4;
                const float c7 = b2; const float c8 = -b1; const float c9 = tx * -b2 - ty * -b1;
                const float arx = (-a1 * p.x + a2 * p.y + a3 * p.z + a4) * cx + (a5 * p.x - a6 * p.y + crx * p.z + a7) * cy +
                                  (a8 * p.x - a9 * p.y - a10 * p.z + a11) * cz;
                const float arz = (c1 * p.x + c2 * p.y + c3) * cx + (c4 * p.x - c5 * p.y + c6) * cy +
                                  (c7 * p.x + c8 * p.y + c9) * cz;
                const float aty = -b6 * cx + c4 * cy + b2 * cz;
                const float bb = (float)(-0.05 * cw);
                accumulate9(acc, arx, arz, aty, bb);
                cnt++;
            } else {
                const int j1 = ind[2 * i], j2 = ind[2 * i + 1];
                if (!(j2 >= 0)) continue;
                const float4 t1 = last[j1], t2 = last[j2];
                const float x0 = sel.x, y0 = sel.y, z0 = sel.z;
                const float x1 = t1.x, y1 = t1.y, z1 = t1.z, x2 = t2.x, y2 = t2.y, z2 = t2.z;
                const float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
                const float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
                const float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
                const float a012 = sqrtf(m11 * m11 + m22 * m22 + m33 * m33);
                const float l12 = sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
                const float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
                const float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
                const float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
                const float ld2 = a012 / l12;
                float sw = 1;
                if (iterCount >= 5) sw = (float)(1 - 1.8 * fabsf(ld2));
                if (!(sw > 0.1 && ld2 != 0)) continue;
                const float cx = sw * la, cy = sw * lb, cz = sw * lc, cw = sw * ld2;
                // calculateTransformationCorner (FA:1391-1421): rows d/d(ry, tx, tz)
                const float b1 = -crz * sry - cry * srx * srz; const float b2 = cry * crz * srx - sry * srz;
                const float b3 = crx * cry; const float b4 = tx * -b1 + ty * -b2 + tz * b3;
                const float b5 = cry * crz - srx * sry * srz; const float b6 = cry * srz + crz * srx * sry;
                const float b7 = crx * sry; const float b8 = tz * b7 - ty * b6 - tx * b5;
                const float c5 = crx * srz;
                const float ary = (b1 * p.x + b2 * p.y - b3 * p.z + b4) * cx + (b5 * p.x + b6 * p.y - b7 * p.z + b8) * cz;
                const float atx = -b5 * cx + c5 * cy + b1 * cz;
                const float atz = b7 * cx - srx * cy - b3 * cz;
                const float bb = (float)(-0.05 * cw);
                accumulate9(acc, ary, atx, atz, bb);
                cnt++;
            }
        }
        block_reduce<9>(acc, cnt, sh, shi);
        if (tid == 0) {
            if (PH == 0) st.iters_surf = iterCount + 1; else st.iters_corner = iterCount + 1;
            s_ctl = 0;
            if (cnt < 10) s_ctl = 1;
            else {
                float X[3];
                solve_step(st, acc, iterCount, X);
                if (PH == 0) { tc[0] += X[0]; tc[2] += X[1]; tc[4] += X[2]; }
                else { tc[1] += X[0]; tc[3] += X[1]; tc[5] += X[2]; }
                for (int k = 0; k < 6; k++) if (isnan(tc[k])) tc[k] = 0;
                float deltaR, deltaT;
                if (PH == 0) {
                    const double r0 = X[0] * 180.0 / M_PI, r1 = X[1] * 180.0 / M_PI;
                    const double t2 = (double)(X[2] * 100);
                    deltaR = (float)sqrt(r0 * r0 + r1 * r1);
                    deltaT = (float)sqrt(t2 * t2);
                } else {
                    const double r0 = X[0] * 180.0 / M_PI;
                    const double t1 = (double)(X[1] * 100), t2 = (double)(X[2] * 100);
                    deltaR = (float)sqrt(r0 * r0);
                    deltaT = (float)sqrt(t1 * t1 + t2 * t2);
                }
                if (deltaR < 0.1 && deltaT < 0.1) s_ctl = 2;
            }
        }
        __syncthreads();
        if (s_ctl == 2) break;
    }
    if (tid == 0) {
        for (int k = 0; k < 6; ++k) st.transformCur[k] = tc[k];
        if (s_ctl == 2 || iterCount >= 25) st.odo_phase = PH + 1;
    }
}
template <int PH>
__global__ void __launch_bounds__(256) k_fa_iter(DevView v, int iter0) {
    fa_iter_block<PH>(v, blockIdx.x, iter0);
}

// A context of a few streams: the correspondence search of iteration iter0
// and the iterations iter0 .. iter0+4 after it in one launch — the stream's
// last search workgroup to finish (a device-scope fence, then a ticket in
// DevView::tick) runs k_fa_iter's workgroup.  Half the odometry's launches,
// most of them empty once the stream has converged (a launch is ~5 us).
template <int PH>
__global__ void __launch_bounds__(256) k_fa_fused(DevView v, int nb, int iter0) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, nb, s, chunk);
    if (s >= v.S) return;
    if (v.st[s].odo_phase != PH) return;   // every workgroup of the stream: the iterations would return too
    if (PH == 0) search_surf_few_block(v, s, chunk);
    else search_corner_block(v, s, chunk);
    __shared__ int last;
    __threadfence();   // this workgroup's correspondences, before its ticket
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(&v.tick[s], 1) == nb - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();   // every workgroup's correspondences, after the last ticket
    if (threadIdx.x == 0) v.tick[s] = 0;   // (the next launch reads it after this one's end)
    fa_iter_block<PH>(v, s, iter0);
}

// integrateTransformation (FA:1697-1725) + publishCloudsLast (FA:1759-1788)
// TransformToEnd (FA:885-953) of the less-sharp / less-flat clouds into the
// next *Last buffers, and into the "trees" when they are rebuilt
// (setInputCloud copies, only when both clouds are big enough): chip-wide,
// SLO_TOEND_BLOCKS workgroups per stream (XCD-aware), sin/cos of the frame
// rotation once per workgroup.
#define SLO_TOEND_BLOCKS 16
__global__ void __launch_bounds__(256) k_fa_to_end(DevView v) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, SLO_TOEND_BLOCKS, s, chunk);
    if (s >= v.S) return;
    const StreamState& st = v.st[s];
    if (st.odo_phase == 3) return;
    __shared__ float tc[6], tct[6];
    __shared__ slo_pose::ImuEnd im;
    if (threadIdx.x < 6) tc[threadIdx.x] = st.transformCur[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        slo_pose::tc_trig(tc, tct);
        // publishCloudsLast: updateImuRollPitchYawStartSinCos, then TransformToEnd (FA:1759-1771)
        const ImuState& m = v.imu[s];
        im = slo_pose::imu_end(m.rollStart, m.pitchStart, m.yawStart, m.shiftFromStart, m.yawLast, m.pitchLast,
                               m.rollLast);
    }
    __syncthreads();
    const int nLS = st.n_less_sharp, nLF = st.n_less_flat;
    const bool rebuild = nLS > 10 && nLF > 100;
    const float4* lsharp = v.less_sharp + (size_t)s * v.cap_less_sharp;
    const float4* lflat = v.less_flat + (size_t)s * v.cap_less_flat;
    float4* cnext = v.corner_next + (size_t)s * v.cap_less_sharp;
    float4* snext = v.surf_next + (size_t)s * v.cap_less_flat;
    float4* kdc = v.kd_corner + (size_t)s * v.cap_less_sharp;
    float4* kds = v.kd_surf + (size_t)s * v.cap_less_flat;
    for (int i = chunk * blockDim.x + threadIdx.x; i < nLS + nLF; i += SLO_TOEND_BLOCKS * blockDim.x) {
        const bool corner = i < nLS;
        const int k = corner ? i : i - nLS;
        const P4 q = slo_pose::transform_to_end(ld4(corner ? lsharp : lflat, k), tc, tct, im);
        const float4 o = make_float4(q.x, q.y, q.z, q.w);
        (corner ? cnext : snext)[k] = o;
        if (rebuild) (corner ? kdc : kds)[k] = o;
    }
}

// integrate (FA:1697-1725) and the *Last / tree bookkeeping, per stream.
// One wave: the trig of integrateTransformation and of transformFusion's
// hand-off runs on its lanes side by side (slo_pose_wave.h; 53 -> ~15 us on
// one stream), lane 0 stores.
__global__ void __launch_bounds__(64) k_fa_odo_finish(DevView v, int fuse) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    if (st.odo_phase == 3) return;
    copy_ring_offsets(v, s);
    const bool w0 = threadIdx.x == 0;
    float tc[6], sum0[6], sum[6];
    for (int k = 0; k < 6; ++k) { tc[k] = st.transformCur[k]; sum0[k] = st.transformSum[k]; }
    const ImuState& m = v.imu[s];
    const float imu[9] = {m.shiftFromStart[0], m.shiftFromStart[1], m.shiftFromStart[2], m.pitchStart, m.yawStart,
                          m.rollStart, m.pitchLast, m.yawLast, m.rollLast};
#ifdef SLO_DIAG_FIN   // [0] integrate, [1] odom_handoff, [2] associate_to_map cycles, [3] calls
    unsigned long long t0 = clock64();
#endif
    slo_pose::integrate_w(sum0, tc, imu, sum);
#ifdef SLO_DIAG_FIN
    unsigned long long t1 = clock64();
    if (w0) { st.dbg[0] += t1 - t0; st.dbg[3] += 1; }
#endif
    // TransformFusion::laserOdometryHandler (TF:186-219): this scan's
    // odometry through the tf round trip, associated to the map with the
    // last published mapping result (this scan's mapping comes after)
    float tbm[6];
    if (fuse) {
        float h[6], incre[6];
#ifdef SLO_DIAG_FIN
        unsigned long long t2 = clock64();
#endif
        slo_pose::odom_handoff_w(sum, h);
#ifdef SLO_DIAG_FIN
        unsigned long long t3 = clock64();
#endif
        slo_pose::associate_to_map_w(h, st.tf_bef, st.tf_aft, incre, tbm);
#ifdef SLO_DIAG_FIN
        unsigned long long t4 = clock64();
        if (w0) { st.dbg[1] += t3 - t2; st.dbg[2] += t4 - t3; }
#endif
    }
    if (w0) {
        for (int k = 0; k < 6; ++k) st.transformSum[k] = sum[k];
        if (fuse)
            for (int k = 0; k < 6; ++k) st.integrated[k] = tbm[k];
        const int nLS = st.n_less_sharp, nLF = st.n_less_flat;
        st.cornerLastNum = nLS;
        st.surfLastNum = nLF;
        st.kd_set = nLS > 10 && nLF > 100;
        if (st.kd_set) { st.kdCornerNum = nLS; st.kdSurfNum = nLF; }
    }
}

// the clouds just written become *Last for the next scan (a host-side swap
// of the ping-pong halves: DevView alternates between two layouts, and a
// captured step graph is kept per layout, slo_ctx.hip)
void fa_swap_last(slo_ctx* ctx) {
    std::swap(ctx->v.corner_last, ctx->v.corner_next);
    std::swap(ctx->v.surf_last, ctx->v.surf_next);
    std::swap(ctx->v.sx_surf_last, ctx->v.sx_surf_next);
}

// The preparation of the next scan's searches: the surf rings' x-order, the
// corner tree's x-order (both read the clouds this scan's odometry wrote: the
// ping-pong halves before fa_swap_last, prep_view) and the hash grid over the
// surf tree cloud (setInputCloud; the corner tree is a windowed brute force
// over its x-sorted copy).  Nothing before the next scan's searches reads
// them, and nothing the next scan's projection and features write feeds them
// (the ring offsets come from roff_last, the gate from StreamState::kd_set).
static DevView prep_view(const DevView& v) {
    DevView p = v;
    std::swap(p.corner_last, p.corner_next);
    std::swap(p.surf_last, p.surf_next);
    std::swap(p.sx_surf_last, p.sx_surf_next);
    return p;
}
static int fa_prep_launch(slo_ctx* ctx) {
    const DevView v = prep_view(ctx->v);
    const int S = ctx->S, R = v.cfg.n_scan;
    ctx->prep_pending = false;
    if (!SLO_SURF_LINEAR) {
        SLO_LAUNCH(ctx, "fa_sx_rings", k_fa_sx_rings, dim3(xcd_grid(S, (R + 3) / 4)), dim3(256), 0, v, (R + 3) / 4);
        if (v.cfg.horizon_scan > 512)
            SLO_LAUNCH(ctx, "fa_sx_long", k_fa_sx_long, dim3(xcd_grid(S, R)), dim3(256), 0, v, R);
    }
    if (v.cap_less_sharp <= 4096) SLO_LAUNCH(ctx, "fa_sx_kd", k_fa_sx_kd<4096>, dim3(S), dim3(1024), 0, v);
    else if (v.cap_less_sharp <= 8192) SLO_LAUNCH(ctx, "fa_sx_kd", k_fa_sx_kd<8192>, dim3(S), dim3(1024), 0, v);
    else SLO_LAUNCH(ctx, "fa_sx_kd", k_fa_sx_kd<16384>, dim3(S), dim3(1024), 0, v);
    SLO_CHECK(hipGetLastError());
    const int SS = (int)(sizeof(StreamState) / sizeof(int32_t));
    return grid_build(ctx, ctx->grid_os, v.kd_surf, v.cap_less_flat, &v.st->kdSurfNum, SS);
}

int fa_prep_init(slo_ctx* ctx) {
    if (ctx->prep_stream) return 0;
    SLO_CHECK(hipStreamCreateWithFlags(&ctx->prep_stream, hipStreamNonBlocking));
    SLO_CHECK(hipEventCreateWithFlags(&ctx->ev_pfork, hipEventDisableTiming));
    SLO_CHECK(hipEventCreateWithFlags(&ctx->ev_pjoin, hipEventDisableTiming));
    return 0;
}

// ring_stream and its events: only a context that steps through
// slo_batch_process makes them (not the stage contexts of Mode S or
// slo_pipeline, whose streams should each keep a hardware queue of their own)
int fa_ring_init(slo_ctx* ctx) {
    if (ctx->ring_stream) return 0;
    SLO_CHECK(hipStreamCreateWithFlags(&ctx->ring_stream, hipStreamNonBlocking));
    SLO_CHECK(hipEventCreateWithFlags(&ctx->ev_rfork, hipEventDisableTiming));
    SLO_CHECK(hipEventCreateWithFlags(&ctx->ev_rjoin, hipEventDisableTiming));
    return 0;
}

// (prep_stream exists from slo_create: only contexts of at most
// SLO_PREP_DEFER_STREAMS streams defer, so nothing is created mid-capture)
int fa_prep_fork(slo_ctx* ctx) {
    if (!ctx->prep_pending) return 0;
    if (int r = fa_prep_init(ctx)) return r;
    SLO_CHECK(hipEventRecord(ctx->ev_pfork, ctx->stream));
    SLO_CHECK(hipStreamWaitEvent(ctx->prep_stream, ctx->ev_pfork, 0));
    std::swap(ctx->stream, ctx->prep_stream);
    const int r = fa_prep_launch(ctx);
    std::swap(ctx->stream, ctx->prep_stream);
    if (r) return r;
    SLO_CHECK(hipEventRecord(ctx->ev_pjoin, ctx->prep_stream));
    return 0;
}

int fa_prep_join(slo_ctx* ctx) {
    if (ctx->prep_stream) SLO_CHECK(hipStreamWaitEvent(ctx->stream, ctx->ev_pjoin, 0));
    return 0;
}

void fa_prep_free(slo_ctx* ctx) {
    if (!ctx->prep_stream) return;
    hipStreamSynchronize(ctx->prep_stream);
    hipEventDestroy(ctx->ev_pfork);
    hipEventDestroy(ctx->ev_pjoin);
    hipStreamDestroy(ctx->prep_stream);
    ctx->prep_stream = nullptr;
    if (ctx->ring_stream) {
        hipStreamSynchronize(ctx->ring_stream);
        hipEventDestroy(ctx->ev_rfork);
        hipEventDestroy(ctx->ev_rjoin);
        hipStreamDestroy(ctx->ring_stream);
        ctx->ring_stream = nullptr;
    }
}

// fuse: transformFusion's /integrated_to_init in k_fa_odo_finish (false on a
// Mode S odometry context, slo_odom_process: the mapping context computes it).
// defer: leave the next scan's preparation pending (the batched step of a few
// streams forks it beside its next projection and features, fa_prep_fork)
int fa_odometry_run(slo_ctx* ctx, bool first_scan, bool fuse, bool defer) {
    if (ctx->prep_pending)
        if (int r = fa_prep_launch(ctx)) return r;   // the last scan's, in-stream
    if (first_scan)   // (k_fa_odo_begin's first-scan branch reads the less-flat cloud)
        if (int r = fa_ring_join(ctx)) return r;
    DevView& v = ctx->v;
    const int S = ctx->S;
    SLO_LAUNCH(ctx, "fa_odo_begin", k_fa_odo_begin, dim3(S), dim3(256), 0, v, first_scan ? 1 : 0);
    if (!first_scan) {
        const bool few = S <= SLO_ODO_FEW && !SLO_SURF_LINEAR;
        const int nbs = few ? (v.cap_flat + 255 / SURF_QL) / (256 / SURF_QL) : (v.cap_flat + 255) / 256;
        const int nbc = (v.cap_sharp + 63) / 64;
        if (few && SLO_ODO_FUSED && !(ctx->timing && !ctx->timing_only.empty())) {   // (a timing filter times each kernel)
            for (int b = 0; b < 5; ++b)
                SLO_LAUNCH(ctx, "fa_surf", k_fa_fused<0>, dim3(xcd_grid(S, nbs)), dim3(256), 0, v, nbs, 5 * b);
            for (int b = 0; b < 5; ++b)
                SLO_LAUNCH(ctx, "fa_corner", k_fa_fused<1>, dim3(xcd_grid(S, nbc)), dim3(256), 0, v, nbc, 5 * b);
        } else {
            for (int b = 0; b < 5; ++b) {
                if (few) SLO_LAUNCH(ctx, "fa_search_surf", k_fa_search_surf_few, dim3(xcd_grid(S, nbs)), dim3(256), 0, v, nbs);
                else SLO_LAUNCH(ctx, "fa_search_surf", k_fa_search_surf, dim3(xcd_grid(S, nbs)), dim3(256), 0, v, nbs);
                SLO_LAUNCH(ctx, "fa_iter_surf", k_fa_iter<0>, dim3(S), dim3(256), 0, v, 5 * b);
            }
            for (int b = 0; b < 5; ++b) {
                SLO_LAUNCH(ctx, "fa_search_corner", k_fa_search_corner, dim3(xcd_grid(S, nbc)), dim3(256), 0, v, nbc);
                SLO_LAUNCH(ctx, "fa_iter_corner", k_fa_iter<1>, dim3(S), dim3(256), 0, v, 5 * b);
            }
        }
    }
    if (int r = fa_ring_join(ctx)) return r;   // the less-flat cloud, forked by fa_features_run
    SLO_LAUNCH(ctx, "fa_to_end", k_fa_to_end, dim3(xcd_grid(S, SLO_TOEND_BLOCKS)), dim3(256), 0, v);
    SLO_LAUNCH(ctx, "fa_odo_finish", k_fa_odo_finish, dim3(S), dim3(64), 0, v, fuse ? 1 : 0);
    SLO_CHECK(hipGetLastError());
    fa_swap_last(ctx);
    ctx->prep_pending = true;
    return defer ? 0 : fa_prep_launch(ctx);
}

}  // namespace slo
