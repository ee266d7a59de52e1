// slo_lc.hip — loop-closure verification on the GPU:
// detectLoopClosure (mapOptmization.cpp:841-962) and performLoopClosure
// (MO:964-1110) minus the GTSAM factors, for every stream whose Scan Context
// detect ran this scan.
//
//   k_lc_archive   keyframe save (MO:1587-1594): the new keyframe's corner and
//                  surf DS clouds (body frame) appended to the stream's
//                  archive — cornerCloudKeyFrames / surfCloudKeyFrames
//   k_lc_select    RS candidate: radius search over the keyframe positions,
//                  oldest id more than 30 s away (MO:856-875); SC candidate =
//                  the detect result (MO:916)
//   per candidate (pass 0 = RS, 1 = SC):
//   k_lc_plan      submap keyframes id-N..id+N and their pose trig
//   k_lc_source    newest keyframe's clouds in the source pose, (int)i >= 0
//                  filter (MO:879-889 / 924-936), order-preserving compaction
//   k_lc_gather    submap concatenation, each keyframe in its own pose
//                  (MO:894-901 / 941-947), chip-wide
//   vg_run         downSizeFilterHistoryKeyFrames (0.3 m, MO:902 / 948)
//   grid_build     0.5 m hash grid over the submap (the ICP "kd-tree")
//   k_lc_corr      ICP correspondences: input_transformed advanced by the
//                  previous increment, exact 1-NN, max distance (chip-wide)
//   k_lc_solve     one workgroup per stream: double-double correspondence
//                  sums, Umeyama (JacobiSVD 3x3), composition, convergence
//   k_lc_fit       getFitnessScore's nearest neighbours (chip-wide)
//   k_lc_finish    fitness, acceptance (MO:1020 / 1071), Euler angles
//
// The arithmetic contract is the oracle's (oracle/oracle_lc.h header): the
// sums are order-independent (every term exact in double, summed in
// double-double), so the GPU's tree and the oracle's loop give the same
// transforms bit for bit.
#include "slo_internal.h"
#include "slo_libm.h"
#include <float.h>
#include <limits.h>

namespace slo {

#define SLO_LC_CELL 0.5f   // submap grid cell (m, power of two): ~1-10 points of a 0.3 m voxelised submap
#define SLO_LC_R 12        // grid walk box radius in cells (6 m); farther neighbours: exhaustive scan

__device__ inline float lc_sqdist(float qx, float qy, float qz, const float4& p) {   // FLANN L2_Simple, d = q - p
    const float d0 = qx - p.x, d1 = qy - p.y, d2 = qz - p.z;
    float r = 0.0f;
    r += d0 * d0;
    r += d1 * d1;
    r += d2 * d2;
    return r;
}

// exact nearest neighbour in tgt[0, n) of stream s (ties -> lowest index):
// the grid walk answers every query with a neighbour within SLO_LC_R cells
// (gate = (R cell)^2, GridView guarantees); the rest scan the submap
__device__ inline void lc_nn(const GridView& g, const float4* tgt, int n, int s, float qx, float qy, float qz,
                             int& bi, float& bd) {
    const float gate = (float)(SLO_LC_R * SLO_LC_R) * g.cell * g.cell;
    bi = INT_MAX; bd = gate;
    grid_ball<SLO_LC_R>(g, s, qx, qy, qz, [&]() { return bd; }, [&](const float4& p) {
        const float d = lc_sqdist(qx, qy, qz, p);
        const int idx = __float_as_int(p.w);
        if (d < bd || (d == bd && idx < bi)) { bd = d; bi = idx; }
    });
    if (bi != INT_MAX) return;
    bi = -1; bd = FLT_MAX;
    for (int j = 0; j < n; ++j) {
        const float d = lc_sqdist(qx, qy, qz, tgt[j]);
        if (d < bd || (bi < 0 && d == bd)) { bd = d; bi = j; }
    }
}

// transformPointCloud (MO:566-596) with precomputed trig t[9] =
// {cos roll, sin roll, cos pitch, sin pitch, cos yaw, sin yaw, x, y, z}
__device__ inline float4 lc_pose_apply(const float* t, const float4& p) {
    const float x1 = t[4] * p.x - t[5] * p.y, y1 = t[5] * p.x + t[4] * p.y, z1 = p.z;
    const float x2 = x1, y2 = t[0] * y1 - t[1] * z1, z2 = t[1] * y1 + t[0] * z1;
    return make_float4(t[2] * x2 + t[3] * z2 + t[6], y2 + t[7], -t[3] * x2 + t[2] * z2 + t[8], p.w);
}
__device__ inline void lc_pose_trig(const float* kp, float* t) {   // kp: x, y, z, roll, pitch, yaw
    using slo_libm::cosf_;
    using slo_libm::sinf_;
    t[0] = cosf_(kp[3]); t[1] = sinf_(kp[3]);
    t[2] = cosf_(kp[4]); t[3] = sinf_(kp[4]);
    t[4] = cosf_(kp[5]); t[5] = sinf_(kp[5]);
    t[6] = kp[0]; t[7] = kp[1]; t[8] = kp[2];
}

// x' = ((r0 x + r1 y) + r2 z) + r3 (ICP transformCloud / pcl::transformPointCloud)
__device__ inline float4 lc_T_apply(const float* T, const float4& p) {
    return make_float4(((T[0] * p.x + T[1] * p.y) + T[2] * p.z) + T[3], ((T[4] * p.x + T[5] * p.y) + T[6] * p.z) + T[7],
                       ((T[8] * p.x + T[9] * p.y) + T[10] * p.z) + T[11], p.w);
}
__device__ inline bool lc_finite(const float4& p) { return isfinite(p.x) && isfinite(p.y) && isfinite(p.z); }
// (int)intensity >= 0 with x86 cvttss2si semantics (NaN / out of range -> INT_MIN)
__device__ inline bool lc_keep(float v) { return v > -1.0f && v < 2147483648.0f; }

// ---------------------------------------------------------------- Eigen JacobiSVD<Matrix3d> (one lane)
struct LcRot { double c, s; };
__device__ inline void lc_make_jacobi(double x, double y, double z, LcRot& r) {
    const double deno = 2.0 * fabs(y);
    if (deno < DBL_MIN) { r.c = 1.0; r.s = 0.0; return; }
    const double tau = (x - z) / deno;
    const double w = sqrt(tau * tau + 1.0);
    const double t = tau > 0.0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
    const double sign_t = t > 0.0 ? 1.0 : -1.0;
    const double n = 1.0 / sqrt(t * t + 1.0);
    r.s = -sign_t * (y / fabs(y)) * fabs(t) * n;
    r.c = n;
}
__device__ inline void lc_rot_rows(double* M, int p, int q, const LcRot& j) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double x = M[p * 3 + i], y = M[q * 3 + i];
        M[p * 3 + i] = j.c * x + j.s * y;
        M[q * 3 + i] = -j.s * x + j.c * y;
    }
}
__device__ inline void lc_rot_cols(double* M, int p, int q, const LcRot& j) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double x = M[i * 3 + p], y = M[i * 3 + q];
        M[i * 3 + p] = j.c * x - j.s * y;
        M[i * 3 + q] = j.s * x + j.c * y;
    }
}
__device__ inline bool lc_svd3(const double* A, double* U, double* S, double* V) {
    double scale = 0.0;
    for (int i = 0; i < 9; ++i) scale = fmax(scale, fabs(A[i]));
    if (!isfinite(scale)) return false;
    if (scale == 0.0) scale = 1.0;
    double W[9];
    for (int i = 0; i < 9; ++i) { W[i] = A[i] / scale; U[i] = V[i] = (i % 4 == 0) ? 1.0 : 0.0; }
    const double precision = 2.0 * DBL_EPSILON, considerAsZero = DBL_MIN;
    double maxDiag = fmax(fabs(W[0]), fmax(fabs(W[4]), fabs(W[8])));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 64; ++sweep) {   // Eigen converges in a few sweeps
        finished = true;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const double threshold = fmax(considerAsZero, precision * maxDiag);
                if (fabs(W[p * 3 + q]) > threshold || fabs(W[q * 3 + p]) > threshold) {
                    finished = false;
                    double m00 = W[p * 3 + p], m01 = W[p * 3 + q], m10 = W[q * 3 + p], m11 = W[q * 3 + q];
                    LcRot rot1;
                    const double t = m00 + m11, d = m10 - m01;
                    if (fabs(d) < DBL_MIN) { rot1.s = 0.0; rot1.c = 1.0; }
                    else {
                        const double u = t / d;
                        const double tmp = sqrt(1.0 + u * u);
                        rot1.s = 1.0 / tmp;
                        rot1.c = u / tmp;
                    }
                    {
                        const double a0 = m00, a1 = m01, b0 = m10, b1 = m11;
                        m00 = rot1.c * a0 + rot1.s * b0; m01 = rot1.c * a1 + rot1.s * b1;
                        m10 = -rot1.s * a0 + rot1.c * b0; m11 = -rot1.s * a1 + rot1.c * b1;
                    }
                    LcRot jr;
                    lc_make_jacobi(m00, m01, m11, jr);
                    const LcRot jrt{jr.c, -jr.s};
                    LcRot jl;
                    jl.c = rot1.c * jrt.c - rot1.s * jrt.s;
                    jl.s = rot1.c * jrt.s + rot1.s * jrt.c;
                    lc_rot_rows(W, p, q, jl);
                    lc_rot_cols(U, p, q, LcRot{jl.c, -jl.s});
                    lc_rot_cols(W, p, q, jr);
                    lc_rot_cols(V, p, q, jr);
                    maxDiag = fmax(maxDiag, fmax(fabs(W[p * 3 + p]), fabs(W[q * 3 + q])));
                }
            }
    }
    for (int i = 0; i < 3; ++i) {
        const double a = W[i * 3 + i];
        S[i] = fabs(a);
        if (a < 0.0) for (int r = 0; r < 3; ++r) U[r * 3 + i] = -U[r * 3 + i];
    }
    for (int i = 0; i < 3; ++i) S[i] *= scale;
    for (int i = 0; i < 3; ++i) {
        int pos = i;
        for (int k = i + 1; k < 3; ++k) if (S[k] > S[pos]) pos = k;
        if (S[pos] == 0.0) break;
        if (pos != i) {
            double x = S[i]; S[i] = S[pos]; S[pos] = x;
            for (int r = 0; r < 3; ++r) {
                x = U[r * 3 + i]; U[r * 3 + i] = U[r * 3 + pos]; U[r * 3 + pos] = x;
                x = V[r * 3 + i]; V[r * 3 + i] = V[r * 3 + pos]; V[r * 3 + pos] = x;
            }
        }
    }
    return true;
}
__device__ inline double lc_det3(const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[3] * (m[1] * m[8] - m[2] * m[7]) + m[6] * (m[1] * m[5] - m[2] * m[4]);
}
// pcl::umeyama from the sums (sum p, sum q, sum q p^T); Ti row-major float 4x4
__device__ inline bool lc_umeyama(const slo_dd::DD* a, int64_t cnt, float* Ti) {
    const double n = (double)cnt;
    double sm[3], dm[3], sig[9];
    for (int k = 0; k < 3; ++k) { sm[k] = (a[k].hi + a[k].lo) / n; dm[k] = (a[3 + k].hi + a[3 + k].lo) / n; }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) sig[i * 3 + j] = (a[6 + i * 3 + j].hi + a[6 + i * 3 + j].lo) / n - dm[i] * sm[j];
    double U[9], S[3], V[9];
    if (!lc_svd3(sig, U, S, V)) return false;
    double D[3] = {1.0, 1.0, 1.0};
    if (lc_det3(U) * lc_det3(V) < 0.0) D[2] = -1.0;
    double R[9], t[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = (U[i * 3 + 0] * D[0]) * V[j * 3 + 0] + (U[i * 3 + 1] * D[1]) * V[j * 3 + 1] +
                                              (U[i * 3 + 2] * D[2]) * V[j * 3 + 2];
    for (int i = 0; i < 3; ++i) t[i] = dm[i] - (R[i * 3 + 0] * sm[0] + R[i * 3 + 1] * sm[1] + R[i * 3 + 2] * sm[2]);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) Ti[i * 4 + j] = (float)R[i * 3 + j];
        Ti[i * 4 + 3] = (float)t[i];
    }
    Ti[12] = Ti[13] = Ti[14] = 0.0f; Ti[15] = 1.0f;
    return true;
}

// block-wide double-double sum of NV terms + a count; result in thread 0
template <int NV>
__device__ inline void lc_block_reduce(slo_dd::DD* acc, int& cnt) {
    __shared__ slo_dd::DD sh[16 * NV];
    __shared__ int shi[16];
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

__device__ inline void lc_identity(float* T) {
    for (int i = 0; i < 16; ++i) T[i] = (i % 5 == 0) ? 1.0f : 0.0f;
}
__device__ inline void lc_result_init(slo_loop_result& r, int id) {
    r.id = id; r.ran = 0; r.converged = 0; r.accepted = 0; r.iters = 0; r.n_src = 0; r.n_tgt = 0; r.pad = 0;
    r.fitness = 0.0;
    for (int i = 0; i < 16; ++i) r.T[i] = 0.0f;
    for (int i = 0; i < 6; ++i) r.xyzrpy[i] = 0.0f;
}

// ---------------------------------------------------------------- kernels
__global__ void __launch_bounds__(256) k_lc_archive(DevView v, LcView l, double t) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    if (!st.kf_saved) return;
    LcState& ls = l.st[s];
    const int kf = st.n_keyframes - 1;
    const int off = ls.used;
    const int nc = st.n_corner_ds, ns = st.n_surf_ds;
    const int room = max(0, l.A - off);
    const int kc = min(nc, room), ks = min(ns, room - kc);
    float4* dst = l.kfa + (size_t)s * l.A + off;
    const float4* c = v.cur_c_ds + (size_t)s * v.cap_less_sharp;
    const float4* sf = v.cur_s_ds + (size_t)s * v.H;
    for (int i = threadIdx.x; i < kc; i += blockDim.x) dst[i] = c[i];
    for (int i = threadIdx.x; i < ks; i += blockDim.x) dst[kc + i] = sf[i];
    __syncthreads();   // every thread has read ls.used
    if (threadIdx.x == 0) {
        int32_t* m = l.kmeta + ((size_t)s * v.KFMAX + kf) * 3;
        m[0] = off; m[1] = kc; m[2] = ks;
        l.ktime[(size_t)s * v.KFMAX + kf] = t;
        ls.used = off + kc + ks;
        if (kc < nc || ks < ns) st.err |= SLO_ERR_MAP_CAPACITY;
    }
}

// candidates of the keyframe saved this scan (one workgroup per stream)
__global__ void __launch_bounds__(256) k_lc_select(DevView v, LcView l) {
    const int s = blockIdx.x;
    const StreamState& st = v.st[s];
    LcState& ls = l.st[s];
    __shared__ int best;
    if (threadIdx.x == 0) best = INT_MAX;
    __syncthreads();
    const bool go = st.det_valid && st.kf_saved && st.n_keyframes > 0;
    const int latest = st.n_keyframes - 1;
    if (go) {
        // currentRobotPosPoint == previousRobotPosPoint after the save (MO:1532-1547)
        const float cx = st.prevPos[0], cy = st.prevPos[1], cz = st.prevPos[2];
        const double rr = (double)v.cfg.history_keyframe_search_radius;
        const float r2 = (float)(rr * rr);
        const double tnow = l.ktime[(size_t)s * v.KFMAX + latest];
        const float* kp = v.kf_pose + (size_t)s * v.KFMAX * 6;
        for (int i = threadIdx.x; i <= latest; i += blockDim.x) {
            if (!(lc_sqdist(cx, cy, cz, make_float4(kp[i * 6], kp[i * 6 + 1], kp[i * 6 + 2], 0.f)) < r2)) continue;
            if (fabs(l.ktime[(size_t)s * v.KFMAX + i] - tnow) > v.cfg.loop_time_gap) { atomicMin(&best, i); break; }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ls.rs_id = go && best != INT_MAX ? best : -1;
        ls.sc_id = go ? st.det_loop_id : -1;
        ls.latest = latest;
        slo_loop_result* r = l.res + (size_t)s * 2;
        lc_result_init(r[0], ls.rs_id);
        lc_result_init(r[1], ls.sc_id);
        if (ls.sc_id >= 0) atomicAdd(l.n_active, ls.rs_id >= 0 ? 2 : 1);
    }
}

// one thread per stream: job state and the submap's keyframe table
__global__ void k_lc_plan(DevView v, LcView l, int pass) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    LcState& ls = l.st[s];
    const int id = pass == 0 ? ls.rs_id : ls.sc_id;
    const bool active = ls.sc_id >= 0 && id >= 0;
    ls.pass = pass;
    ls.active = active ? 1 : 0;
    ls.iter = 0;
    ls.converged = 0;
    ls.prev_mse = DBL_MAX;
    lc_identity(ls.T);
    lc_identity(ls.Ti);
    ls.n_src_raw = 0; ls.n_src = 0; ls.n_raw = 0; ls.n_tgt = 0; ls.nseg = 0;
    if (!active) return;
    const int latest = ls.latest;
    const int* kmeta = l.kmeta + (size_t)s * v.KFMAX * 3;
    const float* kp = v.kf_pose + (size_t)s * v.KFMAX * 6;
    ls.src_off = kmeta[latest * 3];
    ls.n_src_raw = kmeta[latest * 3 + 1] + kmeta[latest * 3 + 2];
    lc_pose_trig(kp + (pass == 0 ? latest : id) * 6, ls.src_trig);
    const int N = v.cfg.history_keyframe_search_num;
    int k = 0, tot = 0;
    for (int j = -N; j <= N; ++j) {
        const int kk = id + j;
        if (kk < 0 || kk > latest) continue;
        ls.seg_off[k] = tot;
        ls.seg_src[k] = kmeta[kk * 3];
        lc_pose_trig(kp + kk * 6, ls.seg_trig[k]);
        tot += kmeta[kk * 3 + 1] + kmeta[kk * 3 + 2];
        ++k;
    }
    ls.seg_off[k] = tot;
    ls.nseg = k;
    ls.n_raw = min(tot, l.A);
    atomicAdd(l.n_active, 1);
}

// the source cloud: one workgroup per stream, order-preserving compaction
__global__ void __launch_bounds__(1024) k_lc_source(DevView v, LcView l) {
    const int s = blockIdx.x;
    LcState& ls = l.st[s];
    if (!ls.active) return;
    __shared__ int wsum[16];
    __shared__ int base;
    const int n = ls.n_src_raw;
    const float4* in = l.kfa + (size_t)s * l.A + ls.src_off;
    float4* out = l.src + (size_t)s * l.cap_src;
    float4* out_t = l.src_t + (size_t)s * l.cap_src;
    float tr[9];
    for (int k = 0; k < 9; ++k) tr[k] = ls.src_trig[k];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += blockDim.x) {
        const int i = c0 + threadIdx.x;
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
        bool keep = false;
        if (i < n) { p = lc_pose_apply(tr, in[i]); keep = lc_keep(p.w); }
        const unsigned long long m = __ballot(keep);
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int pre = base;
        for (int k = 0; k < w; ++k) pre += wsum[k];
        pre += __popcll(m & ((1ull << lane) - 1ull));
        if (keep && pre < l.cap_src) { out[pre] = p; out_t[pre] = p; }
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += wsum[k];
            base += t;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) ls.n_src = min(base, l.cap_src);
}

// the submap, chip-wide: output point i -> its keyframe segment (binary search)
__global__ void __launch_bounds__(256) k_lc_gather(DevView v, LcView l, int nb) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, nb, s, chunk);
    if (s >= v.S) return;
    const LcState& ls = l.st[s];
    if (!ls.active) return;
    const int n = ls.n_raw;
    const float4* arc = l.kfa + (size_t)s * l.A;
    float4* out = l.raw + (size_t)s * l.A;
    for (int i = chunk * blockDim.x + threadIdx.x; i < n; i += nb * blockDim.x) {
        int lo = 0, hi = ls.nseg;   // last k with seg_off[k] <= i
        while (hi - lo > 1) {
            const int m = (lo + hi) >> 1;
            if (ls.seg_off[m] <= i) lo = m; else hi = m;
        }
        out[i] = lc_pose_apply(ls.seg_trig[lo], arc[ls.seg_src[lo] + (i - ls.seg_off[lo])]);
    }
}

// correspondences of one ICP iteration (CorrespondenceEstimation, max distance)
__global__ void __launch_bounds__(256) k_lc_corr(DevView v, LcView l, int nb) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, nb, s, chunk);
    if (s >= v.S) return;
    const LcState& ls = l.st[s];
    if (!ls.active) return;
    const int i = chunk * blockDim.x + threadIdx.x;
    if (i >= ls.n_src) return;
    float4* pt = l.src_t + (size_t)s * l.cap_src + i;
    float4 p = *pt;
    if (ls.iter > 0 && lc_finite(p)) {   // transformCloud(input_transformed, .., transformation_) of the last iteration
        p = lc_T_apply(ls.Ti, p);
        *pt = p;
    }
    int j = -1;
    float d = FLT_MAX;
    if (lc_finite(p)) lc_nn(l.g, l.tgt + (size_t)s * l.A, ls.n_tgt, s, p.x, p.y, p.z, j, d);
    const double max_d2 = v.cfg.icp_max_corr_dist * v.cfg.icp_max_corr_dist;
    l.corr_j[(size_t)s * l.cap_src + i] = (j >= 0 && !((double)d > max_d2)) ? j : -1;
    l.corr_d[(size_t)s * l.cap_src + i] = d;
}

// Umeyama step + DefaultConvergenceCriteria (one workgroup per stream)
__global__ void __launch_bounds__(256) k_lc_solve(DevView v, LcView l) {
    const int s = blockIdx.x;
    LcState& ls = l.st[s];
    if (!ls.active) return;
    const int n = ls.n_src;
    const float4* P = l.src_t + (size_t)s * l.cap_src;
    const float4* Q = l.tgt + (size_t)s * l.A;
    const int32_t* J = l.corr_j + (size_t)s * l.cap_src;
    const float* D = l.corr_d + (size_t)s * l.cap_src;
    slo_dd::DD acc[16];
    for (int k = 0; k < 16; ++k) acc[k] = slo_dd::zero();
    int cnt = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int j = J[i];
        if (j < 0) continue;
        const float4 p = P[i], q = Q[j];
        const double pv[3] = {p.x, p.y, p.z}, qv[3] = {q.x, q.y, q.z};
        for (int k = 0; k < 3; ++k) { slo_dd::add(acc[k], pv[k]); slo_dd::add(acc[3 + k], qv[k]); }
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) slo_dd::add(acc[6 + a * 3 + b], qv[a] * pv[b]);
        slo_dd::add(acc[15], (double)D[i]);
        ++cnt;
    }
    lc_block_reduce<16>(acc, cnt);
    if (threadIdx.x != 0) return;
    bool done = false;
    float Ti[16];
    if (cnt < 3 || !lc_umeyama(acc, cnt, Ti)) {   // min_number_correspondences_ = 3
        ls.converged = 0;
        done = true;
    } else {
        float R[16];
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b)
                R[a * 4 + b] = ((Ti[a * 4 + 0] * ls.T[0 * 4 + b] + Ti[a * 4 + 1] * ls.T[1 * 4 + b]) + Ti[a * 4 + 2] * ls.T[2 * 4 + b]) +
                               Ti[a * 4 + 3] * ls.T[3 * 4 + b];
        for (int k = 0; k < 16; ++k) { ls.T[k] = R[k]; ls.Ti[k] = Ti[k]; }
        const int it = ++ls.iter;
        const double cos_angle = 0.5 * (double)(Ti[0] + Ti[5] + Ti[10] - 1.0f);
        const double tsq = (double)(Ti[3] * Ti[3] + Ti[7] * Ti[7] + Ti[11] * Ti[11]);
        const double mse = (acc[15].hi + acc[15].lo) / (double)cnt;
        if (it >= v.cfg.icp_max_iterations) done = true;
        else if (cos_angle >= 1.0 - v.cfg.icp_transformation_epsilon && tsq <= v.cfg.icp_transformation_epsilon) done = true;
        else if (fabs(mse - ls.prev_mse) < 1e-12) done = true;
        else if (fabs(mse - ls.prev_mse) / ls.prev_mse < v.cfg.icp_fitness_epsilon) done = true;
        else ls.prev_mse = mse;
        if (done) ls.converged = 1;
    }
    if (done) {
        ls.active = 0;
        atomicSub(l.n_active, 1);
    }
}

// getFitnessScore's nearest neighbours of input_ under the final transformation
__global__ void __launch_bounds__(256) k_lc_fit(DevView v, LcView l, int nb) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, nb, s, chunk);
    if (s >= v.S) return;
    const LcState& ls = l.st[s];
    if (ls.n_src <= 0 || ls.n_tgt <= 0) return;
    const slo_loop_result& r = l.res[(size_t)s * 2 + ls.pass];
    if (r.id < 0 || l.st[s].sc_id < 0) return;
    const int i = chunk * blockDim.x + threadIdx.x;
    if (i >= ls.n_src) return;
    const float4 p = lc_T_apply(ls.T, l.src[(size_t)s * l.cap_src + i]);
    int j = -1;
    float d = FLT_MAX;
    if (lc_finite(p)) lc_nn(l.g, l.tgt + (size_t)s * l.A, ls.n_tgt, s, p.x, p.y, p.z, j, d);
    l.corr_j[(size_t)s * l.cap_src + i] = j;
    l.corr_d[(size_t)s * l.cap_src + i] = d;
}

__global__ void __launch_bounds__(256) k_lc_finish(DevView v, LcView l) {
    const int s = blockIdx.x;
    const LcState& ls = l.st[s];
    slo_loop_result& r = l.res[(size_t)s * 2 + ls.pass];
    if (r.id < 0 || ls.sc_id < 0) return;
    const bool have = ls.n_src > 0 && ls.n_tgt > 0;
    slo_dd::DD acc[1] = {slo_dd::zero()};
    int cnt = 0;
    if (have)
        for (int i = threadIdx.x; i < ls.n_src; i += blockDim.x)
            if (l.corr_j[(size_t)s * l.cap_src + i] >= 0) {
                slo_dd::add(acc[0], (double)l.corr_d[(size_t)s * l.cap_src + i]);
                ++cnt;
            }
    lc_block_reduce<1>(acc, cnt);
    if (threadIdx.x != 0) return;
    r.ran = 1;
    r.n_src = ls.n_src;
    r.n_tgt = ls.n_tgt;
    r.iters = ls.iter;
    r.converged = have ? ls.converged : 0;
    for (int k = 0; k < 16; ++k) r.T[k] = ls.T[k];
    r.fitness = cnt > 0 ? (acc[0].hi + acc[0].lo) / (double)cnt : DBL_MAX;
    r.accepted = r.converged && !(r.fitness > (double)v.cfg.history_keyframe_fitness_score);
    r.xyzrpy[0] = ls.T[3]; r.xyzrpy[1] = ls.T[7]; r.xyzrpy[2] = ls.T[11];
    r.xyzrpy[3] = slo_libm::atan2f_(ls.T[9], ls.T[10]);
    r.xyzrpy[4] = slo_libm::asinf_(-ls.T[8]);
    r.xyzrpy[5] = slo_libm::atan2f_(ls.T[4], ls.T[0]);
}

// slo_icp_align_batch: given clouds -> the source / target buffers, one ICP job per stream
__global__ void __launch_bounds__(256) k_lc_load(DevView v, LcView l, const float4* src, size_t src_stride,
                                                 const int32_t* nsrc, const float4* tgt, size_t tgt_stride,
                                                 const int32_t* ntgt) {
    const int s = blockIdx.y;
    LcState& ls = l.st[s];
    const int ns = min(max(nsrc[s], 0), l.cap_src), nt = min(max(ntgt[s], 0), l.A);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gridDim.x * blockDim.x) {
        const float4 p = src[(size_t)s * src_stride + i];
        l.src[(size_t)s * l.cap_src + i] = p;
        l.src_t[(size_t)s * l.cap_src + i] = p;
    }
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nt; i += gridDim.x * blockDim.x)
        l.tgt[(size_t)s * l.A + i] = tgt[(size_t)s * tgt_stride + i];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ls.pass = 1;
        ls.rs_id = -1;
        ls.sc_id = 0;
        ls.n_src = ns;
        ls.n_tgt = nt;
        ls.iter = 0;
        ls.converged = 0;
        ls.prev_mse = DBL_MAX;
        lc_identity(ls.T);
        lc_identity(ls.Ti);
        ls.active = (ns > 0 && nt > 0) ? 1 : 0;
        lc_result_init(l.res[(size_t)s * 2 + 0], -1);
        lc_result_init(l.res[(size_t)s * 2 + 1], 0);
        if (ls.active) atomicAdd(l.n_active, 1);
    }
}

// ---------------------------------------------------------------- host
int lc_alloc(slo_ctx* ctx) {
    LcView& l = ctx->lc;
    const DevView& v = ctx->v;
    const size_t S = ctx->S;
    l.A = ctx->cfg.loop_archive_points;
    l.cap_src = std::min<long long>((long long)l.A, (long long)v.cap_less_sharp + v.H);
    SLO_CHECK(hipMalloc(&l.kfa, sizeof(float4) * S * l.A));
    SLO_CHECK(hipMalloc(&l.kmeta, sizeof(int32_t) * S * v.KFMAX * 3));
    SLO_CHECK(hipMalloc(&l.ktime, sizeof(double) * S * v.KFMAX));
    SLO_CHECK(hipMalloc(&l.src, sizeof(float4) * S * l.cap_src));
    SLO_CHECK(hipMalloc(&l.src_t, sizeof(float4) * S * l.cap_src));
    SLO_CHECK(hipMalloc(&l.corr_j, sizeof(int32_t) * S * l.cap_src));
    SLO_CHECK(hipMalloc(&l.corr_d, sizeof(float) * S * l.cap_src));
    SLO_CHECK(hipMalloc(&l.raw, sizeof(float4) * S * l.A));
    SLO_CHECK(hipMalloc(&l.tgt, sizeof(float4) * S * l.A));
    SLO_CHECK(hipMalloc(&l.st, sizeof(LcState) * S));
    SLO_CHECK(hipMalloc(&l.res, sizeof(slo_loop_result) * S * 2));
    SLO_CHECK(hipMalloc(&l.n_active, sizeof(int32_t)));
    SLO_CHECK(hipMemset(l.kmeta, 0, sizeof(int32_t) * S * v.KFMAX * 3));
    SLO_CHECK(hipMemset(l.ktime, 0, sizeof(double) * S * v.KFMAX));
    SLO_CHECK(hipMemset(l.st, 0, sizeof(LcState) * S));
    SLO_CHECK(hipMemset(l.res, 0xff, sizeof(slo_loop_result) * S * 2));
    SLO_CHECK(hipMemset(l.n_active, 0, sizeof(int32_t)));
    SLO_CHECK(hipHostMalloc((void**)&ctx->h_lc_active, sizeof(int32_t)));
    int T = 1 << 12;
    while (T < (1 << 22) && T < l.A / 4) T <<= 1;
    if (int r = grid_alloc(ctx, ctx->grid_lc, T, (size_t)l.A, SLO_LC_CELL)) return r;
    l.g = grid_view(ctx->grid_lc);
    return 0;
}

void lc_free(slo_ctx* ctx) {
    LcView& l = ctx->lc;
    void* ps[] = {l.kfa, l.kmeta, l.ktime, l.src, l.src_t, l.corr_j, l.corr_d, l.raw, l.tgt, l.st, l.res, l.n_active};
    for (void* p : ps) if (p) hipFree(p);
    if (ctx->h_lc_active) hipHostFree(ctx->h_lc_active);
    ctx->h_lc_active = nullptr;
    grid_free(ctx->grid_lc);
    l = LcView{};
}

int lc_archive_run(slo_ctx* ctx, double t_scan) {
    if (!ctx->cfg.loop_verify) return 0;
    SLO_LAUNCH(ctx, "lc_archive", k_lc_archive, dim3(ctx->S), dim3(256), 0, ctx->v, ctx->lc, t_scan);
    SLO_CHECK(hipGetLastError());
    return 0;
}

static int lc_active(slo_ctx* ctx, int& n) {
    SLO_CHECK(hipMemcpyAsync(ctx->h_lc_active, ctx->lc.n_active, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    n = *ctx->h_lc_active;
    return 0;
}

// ICP iterations on the jobs set up in LcState (n_active live jobs), then the
// fitness score
static int lc_icp_iterate(slo_ctx* ctx) {
    const DevView& v = ctx->v;
    const LcView& l = ctx->lc;
    const int S = ctx->S;
    const int nb = (l.cap_src + 255) / 256;
    const int LSS = (int)(sizeof(LcState) / sizeof(int32_t));
    if (int r = grid_build(ctx, ctx->grid_lc, l.tgt, (size_t)l.A, &l.st->n_tgt, LSS)) return r;
    for (int it = 0; it < ctx->cfg.icp_max_iterations; ++it) {
        SLO_LAUNCH(ctx, "lc_corr", k_lc_corr, dim3(xcd_grid(S, nb)), dim3(256), 0, v, l, nb);
        SLO_LAUNCH(ctx, "lc_solve", k_lc_solve, dim3(S), dim3(256), 0, v, l);
        if ((it & 3) == 3) {   // stop launching once every job has finished
            int n = 0;
            if (int r = lc_active(ctx, n)) return r;
            if (n <= 0) break;
        }
    }
    SLO_LAUNCH(ctx, "lc_fit", k_lc_fit, dim3(xcd_grid(S, nb)), dim3(256), 0, v, l, nb);
    SLO_LAUNCH(ctx, "lc_finish", k_lc_finish, dim3(S), dim3(256), 0, v, l);
    SLO_CHECK(hipGetLastError());
    return 0;
}

int lc_run(slo_ctx* ctx) {
    if (!ctx->cfg.loop_verify) return 0;
    const DevView& v = ctx->v;
    const LcView& l = ctx->lc;
    const int S = ctx->S;
    SLO_CHECK(hipMemsetAsync(l.n_active, 0, sizeof(int32_t), ctx->stream));
    SLO_LAUNCH(ctx, "lc_select", k_lc_select, dim3(S), dim3(256), 0, v, l);
    int jobs = 0;
    if (int r = lc_active(ctx, jobs)) return r;
    if (jobs <= 0) return 0;
    const int LSS = (int)(sizeof(LcState) / sizeof(int32_t));
    const int nbg = std::max(1, std::min(64, (l.A + 255) / 256));
    for (int pass = 0; pass < 2; ++pass) {
        SLO_CHECK(hipMemsetAsync(l.n_active, 0, sizeof(int32_t), ctx->stream));
        SLO_LAUNCH(ctx, "lc_plan", k_lc_plan, dim3((S + 63) / 64), dim3(64), 0, v, l, pass);
        SLO_LAUNCH(ctx, "lc_source", k_lc_source, dim3(S), dim3(1024), 0, v, l);
        SLO_LAUNCH(ctx, "lc_gather", k_lc_gather, dim3(xcd_grid(S, nbg)), dim3(256), 0, v, l, nbg);
        if (int r = vg_run(ctx, "lc_vg", l.raw, (size_t)l.A, &l.st->n_raw, LSS, ctx->cfg.leaf_history, l.tgt,
                           (size_t)l.A, &l.st->n_tgt, LSS, l.A))
            return r;
        if (int r = lc_icp_iterate(ctx)) return r;
    }
    return pcl_fold_err(ctx);
}

int lc_icp_run(slo_ctx* ctx, const float4* src, size_t src_stride, const int32_t* nsrc, const float4* tgt,
               size_t tgt_stride, const int32_t* ntgt) {
    const DevView& v = ctx->v;
    const LcView& l = ctx->lc;
    const int S = ctx->S;
    SLO_CHECK(hipMemsetAsync(l.n_active, 0, sizeof(int32_t), ctx->stream));
    const int gx = std::max(1, std::min(64, (int)((std::max(src_stride, tgt_stride) + 255) / 256)));
    SLO_LAUNCH(ctx, "lc_load", k_lc_load, dim3(gx, S), dim3(256), 0, v, l, src, src_stride, nsrc, tgt, tgt_stride, ntgt);
    return lc_icp_iterate(ctx);
}

}  // namespace slo
