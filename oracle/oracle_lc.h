// oracle_lc.h — TEST INFRASTRUCTURE ONLY: CPU restatement of SC-LeGO-LOAM's
// loop-closure verification:
//   detectLoopClosure    mapOptmization.cpp:841-962  (RS radius search over
//                        the keyframe positions, the RS / SC submaps)
//   performLoopClosure   mapOptmization.cpp:964-1110 (minus the GTSAM factors)
// and of the third-party code those lines call, restated from the published
// algorithms (PCL 1.8 / Eigen 3.3 are absent here: parity to them unpinned):
//   pcl::IterativeClosestPoint<PointXYZI, PointXYZI, float>::align
//       (icp.hpp computeTransformation: CorrespondenceEstimation 1-NN with
//       max distance, TransformationEstimationSVD -> pcl::umeyama,
//       DefaultConvergenceCriteria, IterativeClosestPoint::transformCloud),
//   Registration::getFitnessScore (max_range = DBL_MAX),
//   Eigen::umeyama + JacobiSVD<Matrix3> (two-sided Jacobi, 3.3 ordering),
//   pcl::getTranslationAndEulerAngles.
//
// Arithmetic contract (shared with the GPU path, DESIGN.md "Loop closure"):
// PCL runs Umeyama in float through Eigen's vectorised reductions, whose
// order is not reproducible here.  This restatement forms the correspondence
// sums — sum p, sum q, sum q p^T over float points, sum of the float squared
// distances — in double-double (every product of two floats is exact in
// double) and rounds each once to double, so a tree reduction on the GPU and
// the sequential loop here give the same doubles; the means, the 3x3
// correlation and its SVD are double; the increment is rounded to float
// (PCL's Matrix4 is float).  Point transforms, the composed final transform
// and the fitness distances are float in PCL's own expression order.
// Deterministic gating (replaces the reference's 1 Hz loop thread, Q13):
// verification runs right after each keyframe's SC detect, with
// timeLaserOdometry = the mapped scan's time.
#pragma once

#include "oracle_mo.h"

namespace oracle {

struct LoopResult {
    int32_t id = -1;         // candidate keyframe (-1: none)
    int32_t ran = 0;         // ICP ran (only when the SC candidate exists, MO:925-927)
    int32_t converged = 0;   // icp.hasConverged()
    int32_t accepted = 0;    // converged && fitness <= historyKeyframeFitnessScore (MO:1020 / 1071)
    int32_t iters = 0;       // ICP iterations done
    int32_t n_src = 0, n_tgt = 0;  // source cloud / downsampled submap sizes
    int32_t pad = 0;
    double fitness = 0;      // icp.getFitnessScore()
    float T[16] = {0};       // icp.getFinalTransformation(), row-major
    float xyzrpy[6] = {0};   // pcl::getTranslationAndEulerAngles(T)
};

// ---------------------------------------------------------------- Eigen JacobiSVD<Matrix3d>
struct JRot { double c, s; };

// JacobiRotation::makeJacobi(x, y, z) for real scalars (Jacobi.h)
inline void make_jacobi(double x, double y, double z, JRot& r) {
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

// rows p, q of the row-major 3x3 M: x' = c x + s y, y' = -s x + c y (applyOnTheLeft)
inline void rot_rows(double* M, int p, int q, const JRot& j) {
    for (int i = 0; i < 3; ++i) {
        const double x = M[p * 3 + i], y = M[q * 3 + i];
        M[p * 3 + i] = j.c * x + j.s * y;
        M[q * 3 + i] = -j.s * x + j.c * y;
    }
}
// columns p, q: applyOnTheRight(p, q, j) = the plane rotation by j^T = (c, -s)
inline void rot_cols(double* M, int p, int q, const JRot& j) {
    for (int i = 0; i < 3; ++i) {
        const double x = M[i * 3 + p], y = M[i * 3 + q];
        M[i * 3 + p] = j.c * x - j.s * y;
        M[i * 3 + q] = j.s * x + j.c * y;
    }
}

// JacobiSVD<Matrix3d>(A, ComputeFullU | ComputeFullV): A = U diag(S) V^T,
// S descending.  Returns false for a non-finite A (Eigen: InvalidInput).
inline bool jacobi_svd3(const double* A, double* U, double* S, double* V) {
    double scale = 0.0;
    for (int i = 0; i < 9; ++i) scale = std::max(scale, fabs(A[i]));
    if (!std::isfinite(scale)) return false;
    if (scale == 0.0) scale = 1.0;
    double W[9];
    for (int i = 0; i < 9; ++i) { W[i] = A[i] / scale; U[i] = V[i] = (i % 4 == 0) ? 1.0 : 0.0; }
    const double precision = 2.0 * DBL_EPSILON, considerAsZero = DBL_MIN;
    double maxDiag = std::max(fabs(W[0]), std::max(fabs(W[4]), fabs(W[8])));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 64; ++sweep) {   // Eigen: until no rotation applies (a few sweeps)
        finished = true;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const double threshold = std::max(considerAsZero, precision * maxDiag);
                if (fabs(W[p * 3 + q]) > threshold || fabs(W[q * 3 + p]) > threshold) {
                    finished = false;
                    // real_2x2_jacobi_svd (JacobiSVD.h)
                    double m00 = W[p * 3 + p], m01 = W[p * 3 + q], m10 = W[q * 3 + p], m11 = W[q * 3 + q];
                    JRot rot1;
                    const double t = m00 + m11, d = m10 - m01;
                    if (fabs(d) < DBL_MIN) { rot1.s = 0.0; rot1.c = 1.0; }
                    else {
                        const double u = t / d;
                        const double tmp = sqrt(1.0 + u * u);
                        rot1.s = 1.0 / tmp;
                        rot1.c = u / tmp;
                    }
                    {   // m.applyOnTheLeft(0, 1, rot1)
                        const double a0 = m00, a1 = m01, b0 = m10, b1 = m11;
                        m00 = rot1.c * a0 + rot1.s * b0; m01 = rot1.c * a1 + rot1.s * b1;
                        m10 = -rot1.s * a0 + rot1.c * b0; m11 = -rot1.s * a1 + rot1.c * b1;
                    }
                    JRot jr;
                    make_jacobi(m00, m01, m11, jr);
                    const JRot jrt{jr.c, -jr.s};   // j_right->transpose()
                    JRot jl;                        // rot1 * j_right^T
                    jl.c = rot1.c * jrt.c - rot1.s * jrt.s;
                    jl.s = rot1.c * jrt.s + rot1.s * jrt.c;
                    rot_rows(W, p, q, jl);
                    rot_cols(U, p, q, JRot{jl.c, -jl.s});   // applyOnTheRight(p, q, j_left.transpose())
                    rot_cols(W, p, q, jr);
                    rot_cols(V, p, q, jr);
                    maxDiag = std::max(maxDiag, std::max(fabs(W[p * 3 + p]), fabs(W[q * 3 + q])));
                }
            }
    }
    for (int i = 0; i < 3; ++i) {
        const double a = W[i * 3 + i];
        S[i] = fabs(a);
        if (a < 0.0) for (int r = 0; r < 3; ++r) U[r * 3 + i] = -U[r * 3 + i];
    }
    for (int i = 0; i < 3; ++i) S[i] *= scale;
    for (int i = 0; i < 3; ++i) {   // descending; maxCoeff takes the first maximum
        int pos = i;
        for (int k = i + 1; k < 3; ++k) if (S[k] > S[pos]) pos = k;
        if (S[pos] == 0.0) break;
        if (pos != i) {
            std::swap(S[i], S[pos]);
            for (int r = 0; r < 3; ++r) { std::swap(U[r * 3 + i], U[r * 3 + pos]); std::swap(V[r * 3 + i], V[r * 3 + pos]); }
        }
    }
    return true;
}

inline double det3(const double* m) {   // Eigen bruteforce_det3_helper order
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[3] * (m[1] * m[8] - m[2] * m[7]) + m[6] * (m[1] * m[5] - m[2] * m[4]);
}

// The correspondence sums of one ICP iteration (double-double, slo_ddsum.h).
struct IcpSums {
    slo_dd::DD s[16];   // sum p (3), sum q (3), sum q_i p_j (9, row i), sum d (1)
    int64_t n = 0;
    IcpSums() { for (auto& x : s) x = slo_dd::zero(); }
    void add(const Pt& p, const Pt& q, float d) {
        const double pv[3] = {p.x, p.y, p.z}, qv[3] = {q.x, q.y, q.z};
        for (int k = 0; k < 3; ++k) { slo_dd::add(s[k], pv[k]); slo_dd::add(s[3 + k], qv[k]); }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) slo_dd::add(s[6 + i * 3 + j], qv[i] * pv[j]);
        slo_dd::add(s[15], (double)d);
        ++n;
    }
};

// pcl::umeyama(src, dst, false) from the sums: increment T (row-major float 4x4)
inline bool umeyama_from_sums(const IcpSums& a, float* T) {
    const double n = (double)a.n;
    double sm[3], dm[3], sig[9];
    for (int k = 0; k < 3; ++k) { sm[k] = (a.s[k].hi + a.s[k].lo) / n; dm[k] = (a.s[3 + k].hi + a.s[3 + k].lo) / n; }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const slo_dd::DD& x = a.s[6 + i * 3 + j];
            sig[i * 3 + j] = (x.hi + x.lo) / n - dm[i] * sm[j];
        }
    double U[9], S[3], V[9];
    if (!jacobi_svd3(sig, U, S, V)) return false;
    double D[3] = {1.0, 1.0, 1.0};
    if (det3(U) * det3(V) < 0.0) D[2] = -1.0;
    double R[9], t[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = (U[i * 3 + 0] * D[0]) * V[j * 3 + 0] + (U[i * 3 + 1] * D[1]) * V[j * 3 + 1] +
                                              (U[i * 3 + 2] * D[2]) * V[j * 3 + 2];
    for (int i = 0; i < 3; ++i) t[i] = dm[i] - (R[i * 3 + 0] * sm[0] + R[i * 3 + 1] * sm[1] + R[i * 3 + 2] * sm[2]);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[i * 4 + j] = (float)R[i * 3 + j];
        T[i * 4 + 3] = (float)t[i];
    }
    T[12] = T[13] = T[14] = 0.0f; T[15] = 1.0f;
    return true;
}

// x' = ((r0 x + r1 y) + r2 z) + r3 in float (IterativeClosestPoint::transformCloud's
// tr * (x, y, z, 1) and pcl::transformPointCloud evaluate the same sums)
inline Pt apply_T(const float* T, const Pt& p) {
    Pt o;
    o.x = ((T[0] * p.x + T[1] * p.y) + T[2] * p.z) + T[3];
    o.y = ((T[4] * p.x + T[5] * p.y) + T[6] * p.z) + T[7];
    o.z = ((T[8] * p.x + T[9] * p.y) + T[10] * p.z) + T[11];
    o.intensity = p.intensity;
    return o;
}
inline void mul_T(const float* A, const float* B, float* C) {   // C = A * B (float 4x4, k order)
    float R[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            R[i * 4 + j] = ((A[i * 4 + 0] * B[0 * 4 + j] + A[i * 4 + 1] * B[1 * 4 + j]) + A[i * 4 + 2] * B[2 * 4 + j]) +
                           A[i * 4 + 3] * B[3 * 4 + j];
    memcpy(C, R, sizeof(R));
}

inline bool finite3(const Pt& p) { return std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z); }

// icp.align(); icp.getFitnessScore() (parameters MO:1006-1011)
inline void icp_align(const slo_config& cfg, const Cloud& src, const Cloud& tgt, LoopResult& r) {
    r.ran = 1;
    r.n_src = (int)src.size();
    r.n_tgt = (int)tgt.size();
    for (int i = 0; i < 16; ++i) r.T[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    r.converged = 0;
    r.iters = 0;
    r.fitness = DBL_MAX;
    const bool have = !src.empty() && !tgt.empty();   // else Registration::initCompute fails: nothing aligned
    KdTree tree;
    if (have) {
    tree.build(tgt);
    Cloud cur = src;   // input_transformed (guess = identity)
    const double max_d2 = cfg.icp_max_corr_dist * cfg.icp_max_corr_dist;
    const double rot_th = 1.0 - cfg.icp_transformation_epsilon, trans_th = cfg.icp_transformation_epsilon;
    double prev_mse = DBL_MAX;   // correspondences_prev_mse_
    for (;;) {
        IcpSums a;
        for (const Pt& p : cur) {   // CorrespondenceEstimation::determineCorrespondences
            if (!finite3(p)) continue;   // the kd-tree refuses non-finite queries
            int j; float d;
            if (tree.knn(p, 1, &j, &d) < 1) continue;
            if ((double)d > max_d2) continue;
            a.add(p, tgt[j], d);
        }
        if (a.n < 3) { r.converged = 0; break; }   // min_number_correspondences_
        float Ti[16];
        if (!umeyama_from_sums(a, Ti)) { r.converged = 0; break; }
        for (Pt& p : cur) if (finite3(p)) p = apply_T(Ti, p);
        mul_T(Ti, r.T, r.T);
        ++r.iters;
        // DefaultConvergenceCriteria::hasConverged
        if (r.iters >= cfg.icp_max_iterations) { r.converged = 1; break; }
        const double cos_angle = 0.5 * (double)(Ti[0] + Ti[5] + Ti[10] - 1.0f);
        const double tsq = (double)(Ti[3] * Ti[3] + Ti[7] * Ti[7] + Ti[11] * Ti[11]);
        if (cos_angle >= rot_th && tsq <= trans_th) { r.converged = 1; break; }
        const double mse = (a.s[15].hi + a.s[15].lo) / (double)a.n;
        if (fabs(mse - prev_mse) < 1e-12) { r.converged = 1; break; }                      // mse_threshold_absolute_
        if (fabs(mse - prev_mse) / prev_mse < cfg.icp_fitness_epsilon) { r.converged = 1; break; }   // relative
        prev_mse = mse;
    }
    }
    // getFitnessScore(): every transformed input point's nearest target
    slo_dd::DD fs = slo_dd::zero();
    int64_t nr = 0;
    if (have)
    for (const Pt& p0 : src) {
        const Pt p = apply_T(r.T, p0);
        if (!finite3(p)) continue;
        int j; float d;
        if (tree.knn(p, 1, &j, &d) < 1) continue;
        slo_dd::add(fs, (double)d);
        ++nr;
    }
    r.fitness = nr > 0 ? (fs.hi + fs.lo) / (double)nr : DBL_MAX;
    r.accepted = r.converged && !(r.fitness > (double)cfg.history_keyframe_fitness_score);
    r.xyzrpy[0] = r.T[3]; r.xyzrpy[1] = r.T[7]; r.xyzrpy[2] = r.T[11];
    r.xyzrpy[3] = oracle_libm::atan2f_(r.T[9], r.T[10]);   // roll = atan2(t(2,1), t(2,2))
    r.xyzrpy[4] = oracle_libm::asinf_(-r.T[8]);           // pitch = asin(-t(2,0))
    r.xyzrpy[5] = oracle_libm::atan2f_(r.T[4], r.T[0]);    // yaw = atan2(t(1,0), t(0,0))
}

// (int)intensity >= 0 (MO:884-889, 931-936) with x86's cvttss2si semantics
// (NaN / out of range -> INT_MIN, rejected)
inline bool keep_intensity(float v) { return v > -1.0f && v < 2147483648.0f; }

// detectLoopClosure + performLoopClosure for the newest keyframe; sc_id from
// detectLoopClosureID (MO:916).  out[0] = RS, out[1] = SC.
inline void perform_loop_closure(const slo_config& cfg, MapOptimization& mo, int sc_id, double t_now,
                                 LoopResult out[2], bool stable_voxel) {
    out[0] = LoopResult();
    out[1] = LoopResult();
    if (mo.keyPoses.empty()) return;
    const int latest = (int)mo.keyPoses.size() - 1;
    // 1. RS: radiusSearch over cloudKeyPoses3D (FLANN: d^2 < r^2), oldest id
    //    whose time differs by more than 30 s (MO:856-875)
    const Pt cur{mo.currentRobotPosPoint.x, mo.currentRobotPosPoint.y, mo.currentRobotPosPoint.z, 0};
    const float r2 = (float)((double)cfg.history_keyframe_search_radius * (double)cfg.history_keyframe_search_radius);
    int rs = -1;
    for (int i = 0; i <= latest && rs < 0; ++i) {
        const Pose6& k = mo.keyPoses[i];
        if (!(sqdist(cur, Pt{k.x, k.y, k.z, 0}) < r2)) continue;
        if (fabs(mo.keyTimes[i] - t_now) > cfg.loop_time_gap) rs = i;
    }
    out[0].id = rs;
    out[1].id = sc_id;
    if (sc_id < 0) return;   // MO:925-927: no SC candidate -> no ICP at all
    auto submap = [&](int id, int src_pose, Cloud& src, Cloud& tgt) {
        const Pose6& P = mo.keyPoses[src_pose];
        Cloud both = MapOptimization::transformPointCloud(mo.cornerCloudKeyFrames[latest], P);
        Cloud s2 = MapOptimization::transformPointCloud(mo.surfCloudKeyFrames[latest], P);
        both.insert(both.end(), s2.begin(), s2.end());
        src.clear();
        for (const Pt& p : both) if (keep_intensity(p.intensity)) src.push_back(p);
        Cloud raw;
        const int N = cfg.history_keyframe_search_num;
        for (int j = -N; j <= N; ++j) {
            const int k = id + j;
            if (k < 0 || k > latest) continue;
            Cloud c = MapOptimization::transformPointCloud(mo.cornerCloudKeyFrames[k], mo.keyPoses[k]);
            Cloud s = MapOptimization::transformPointCloud(mo.surfCloudKeyFrames[k], mo.keyPoses[k]);
            raw.insert(raw.end(), c.begin(), c.end());
            raw.insert(raw.end(), s.begin(), s.end());
        }
        voxel_grid(raw, cfg.leaf_history, tgt, stable_voxel);
    };
    Cloud src, tgt;
    if (rs >= 0) {   // RS: the newest keyframe in its own pose (MO:879-880)
        submap(rs, latest, src, tgt);
        icp_align(cfg, src, tgt, out[0]);
    }
    submap(sc_id, sc_id, src, tgt);   // SC: the newest keyframe in the candidate's pose (MO:924-925)
    icp_align(cfg, src, tgt, out[1]);
}

}  // namespace oracle
