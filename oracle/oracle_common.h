// oracle_common.h — TEST INFRASTRUCTURE ONLY (parity oracle).
//
// CPU restatement of the third-party arithmetic the SC-LeGO-LOAM hot path
// calls.  None of these libraries exist in this image,
// so each is restated from its published algorithm and the exact call sites:
//   * PCL 1.8 VoxelGrid<PointXYZI>::applyFilter + CentroidPoint
//     (featureAssociation.cpp:779-780, mapOptmization.cpp:1224-1262);
//   * PCL KdTreeFLANN exact k-NN, L2_Simple float distance over x,y,z
//     (featureAssociation.cpp:1054/1165, mapOptmization.cpp:1271/1353) —
//     ties resolved to the lowest index (FLANN's own tie order is
//     traversal-dependent);
//   * OpenCV 3.x cv::solve(DECOMP_QR) = hal::QR32f, cv::eigen = JacobiImpl_,
//     Mat::inv() = 3x3 cofactor in double / n>3 LUImpl, and GEMM with double
//     accumulation (featureAssociation.cpp:1324-1349, mapOptmization.cpp:1298,
//     1361, 1445-1470).
// Parity of these restatements against the real libraries is UNPINNED: the
// reference ships no fixtures and the libraries are absent.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
// anything under oracle/.
#pragma once

#include <stdint.h>
#include <math.h>
#include <float.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include <limits>
#include <atomic>
#include "../sc-lego-loam_amd/csrc/slo_ddsum.h"

namespace oracle {

struct Pt { float x, y, z, intensity; };
typedef std::vector<Pt> Cloud;

// ------------------------------------------------------------ VoxelGrid
// stable_order=false: std::sort on (idx, point) by idx only (PCL, exact
// reference behaviour, unstable within a voxel); true: ties kept in input
// order (what the GPU path does; DESIGN.md "VoxelGrid order").
struct VoxIdx { unsigned int idx; unsigned int cloud_point_index; };

inline void voxel_grid(const Cloud& in, float leaf, Cloud& out, bool stable_order) {
    out.clear();
    if (in.empty()) return;
    const float inv = 1.0f / leaf;  // Array4f::Ones() / leaf_size_
    float minx = FLT_MAX, miny = FLT_MAX, minz = FLT_MAX;
    float maxx = -FLT_MAX, maxy = -FLT_MAX, maxz = -FLT_MAX;
    for (const Pt& p : in) {  // getMinMax3D over the (dense) cloud
        minx = std::min(minx, p.x); miny = std::min(miny, p.y); minz = std::min(minz, p.z);
        maxx = std::max(maxx, p.x); maxy = std::max(maxy, p.y); maxz = std::max(maxz, p.z);
    }
    int64_t dx = (int64_t)((maxx - minx) * inv) + 1;
    int64_t dy = (int64_t)((maxy - miny) * inv) + 1;
    int64_t dz = (int64_t)((maxz - minz) * inv) + 1;
    if (dx * dy * dz > (int64_t)std::numeric_limits<int32_t>::max()) {  // PCL warns, returns input
        out = in;
        return;
    }
    int minbx = (int)floorf(minx * inv), minby = (int)floorf(miny * inv), minbz = (int)floorf(minz * inv);
    int maxbx = (int)floorf(maxx * inv), maxby = (int)floorf(maxy * inv);
    int divx = maxbx - minbx + 1, divy = maxby - minby + 1;
    int mul1 = divx, mul2 = divx * divy;
    std::vector<VoxIdx> iv;
    iv.reserve(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
        const Pt& p = in[i];
        int ijk0 = (int)(floorf(p.x * inv) - (float)minbx);
        int ijk1 = (int)(floorf(p.y * inv) - (float)minby);
        int ijk2 = (int)(floorf(p.z * inv) - (float)minbz);
        int idx = ijk0 * 1 + ijk1 * mul1 + ijk2 * mul2;
        iv.push_back({(unsigned int)idx, (unsigned int)i});
    }
    if (stable_order)
        std::stable_sort(iv.begin(), iv.end(), [](const VoxIdx& a, const VoxIdx& b) { return a.idx < b.idx; });
    else
        std::sort(iv.begin(), iv.end(), [](const VoxIdx& a, const VoxIdx& b) { return a.idx < b.idx; });
    size_t index = 0;
    while (index < iv.size()) {
        size_t i = index + 1;
        while (i < iv.size() && iv[i].idx == iv[index].idx) ++i;
        float sx = 0, sy = 0, sz = 0, si = 0;
        for (size_t li = index; li < i; ++li) {
            const Pt& p = in[iv[li].cloud_point_index];
            sx += p.x; sy += p.y; sz += p.z; si += p.intensity;
        }
        float n = (float)(i - index);
        out.push_back({sx / n, sy / n, sz / n, si / n});
        index = i;
    }
}

// ------------------------------------------------------------ exact kd-tree
// k-NN by (float distance, index); distance = ((dx*dx)+dy*dy)+dz*dz with
// d = query - point (FLANN L2_Simple accumulation order).
inline float sqdist(const Pt& q, const Pt& p) {
    float d0 = q.x - p.x, d1 = q.y - p.y, d2 = q.z - p.z;
    float r = 0.0f;
    r += d0 * d0;
    r += d1 * d1;
    r += d2 * d2;
    return r;
}

struct KdTree {
    struct Node { int lo, hi, axis, left, right; float split; float bmin[3], bmax[3]; };
    // setInputCloud copies the points (PCL converts the cloud into FLANN's
    // own matrix), so a tree that is not rebuilt keeps searching old points.
    Cloud own;
    const Cloud* pts = &own;
    std::vector<int> idx;
    std::vector<Node> nodes;
    static constexpr int kLeaf = 15;

    void build(const Cloud& c) {
        own = c;
        pts = &own;
        idx.resize(c.size());
        for (size_t i = 0; i < c.size(); ++i) idx[i] = (int)i;
        nodes.clear();
        if (!c.empty()) build_rec(0, (int)c.size());
    }
    KdTree() {}
    KdTree(const KdTree& o) : own(o.own), idx(o.idx), nodes(o.nodes) { pts = &own; }
    KdTree& operator=(const KdTree& o) {
        own = o.own; idx = o.idx; nodes = o.nodes; pts = &own;
        return *this;
    }
    float coord(int i, int a) const { const Pt& p = (*pts)[i]; return a == 0 ? p.x : a == 1 ? p.y : p.z; }
    int build_rec(int lo, int hi) {
        Node n; n.lo = lo; n.hi = hi; n.left = n.right = -1; n.axis = 0; n.split = 0;
        for (int a = 0; a < 3; ++a) { n.bmin[a] = FLT_MAX; n.bmax[a] = -FLT_MAX; }
        for (int i = lo; i < hi; ++i)
            for (int a = 0; a < 3; ++a) {
                float v = coord(idx[i], a);
                n.bmin[a] = std::min(n.bmin[a], v); n.bmax[a] = std::max(n.bmax[a], v);
            }
        int me = (int)nodes.size();
        nodes.push_back(n);
        if (hi - lo > kLeaf) {
            int ax = 0; float sp = -1;
            for (int a = 0; a < 3; ++a) if (n.bmax[a] - n.bmin[a] > sp) { sp = n.bmax[a] - n.bmin[a]; ax = a; }
            int mid = (lo + hi) / 2;
            std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi,
                             [&](int a, int b) { return coord(a, ax) < coord(b, ax); });
            nodes[me].axis = ax;
            nodes[me].split = coord(idx[mid], ax);
            int l = build_rec(lo, mid);
            int r = build_rec(mid, hi);
            nodes[me].left = l; nodes[me].right = r;
        }
        return me;
    }
    // box lower bound in double (conservative: never prunes a true candidate)
    static double box_d2(const Node& n, const Pt& q) {
        double d = 0, qc[3] = {q.x, q.y, q.z};
        for (int a = 0; a < 3; ++a) {
            double v = 0;
            if (qc[a] < n.bmin[a]) v = n.bmin[a] - qc[a];
            else if (qc[a] > n.bmax[a]) v = qc[a] - n.bmax[a];
            d += v * v;
        }
        return d;
    }
    // k nearest (sorted by (d, index)); returns count found (<= k).
    int knn(const Pt& q, int k, int* oi, float* od) const {
        int cnt = 0;
        if (nodes.empty()) return 0;
        knn_rec(0, q, k, oi, od, cnt);
        return cnt;
    }
    void knn_rec(int ni, const Pt& q, int k, int* oi, float* od, int& cnt) const {
        const Node& n = nodes[ni];
        if (cnt == k) {
            // prune with a small slack so float-vs-double boundary cases are kept
            if (box_d2(n, q) > (double)od[k - 1] * (1.0 + 1e-6) + 1e-12) return;
        }
        if (n.left < 0) {
            for (int i = n.lo; i < n.hi; ++i) {
                int pi = idx[i];
                float d = sqdist(q, (*pts)[pi]);
                if (cnt == k && (d > od[k - 1] || (d == od[k - 1] && pi > oi[k - 1]))) continue;
                int pos = cnt < k ? cnt : k - 1;
                while (pos > 0 && (od[pos - 1] > d || (od[pos - 1] == d && oi[pos - 1] > pi))) {
                    od[pos] = od[pos - 1]; oi[pos] = oi[pos - 1]; --pos;
                }
                od[pos] = d; oi[pos] = pi;
                if (cnt < k) ++cnt;
            }
            return;
        }
        double qa = n.axis == 0 ? q.x : n.axis == 1 ? q.y : q.z;
        int first = qa < n.split ? n.left : n.right;
        int second = first == n.left ? n.right : n.left;
        knn_rec(first, q, k, oi, od, cnt);
        knn_rec(second, q, k, oi, od, cnt);
    }
};

// ------------------------------------------------------------ OpenCV restatements
// matAtA = matAt * matA, matAtB = matAt * matB (cv::Mat GEMM on float Mats,
// FA:1324-1326 / 1425-1427, MO:1445-1447).  Two accumulation modes
// (t_gemm_mode, per calling thread, set per stream by oracle_step):
//   0 (default; what the GPU computes): products of floats are exact in
//     double; the sum is taken in double-double and rounded once
//     (slo_ddsum.h) — the correctly rounded float of the exact sum, which the
//     GPU's tree reductions reproduce;
//   1 OpenCV 3.x's own C++ GEMM as recalled (Q11; OpenCV is absent here, so
//     this too is unpinned): cv::gemm on a 6 x 6 / 3 x 3 result takes
//     GEMMSingleMul<float, double>.  matAtA (flags 0, d.width * 4 <= 1600):
//     one double accumulator per output, k in order, rounded to float once.
//     matAtB (a one-column result, so B is read as a transposed row, GEMM_2_T):
//     four double accumulators over k mod 4 (CV_ENABLE_UNROLLED), the tail
//     into the first, then s0 + s1 + s2 + s3 left to right, rounded once.
// tools/faithful_drift.py --gemm measures what the difference does to the
// poses.
inline thread_local int t_gemm_mode = 0;
// process-wide tallies (only while g_gemm_tally is on: both modes are then
// evaluated and the stream's mode picks the one used): entries computed,
// entries where the two modes give different floats
inline std::atomic<bool> g_gemm_tally{false};
inline std::atomic<long long> g_gemm_entries{0}, g_gemm_differ{0};
inline void gemm_AtA(const std::vector<float>& A, int n, int m, float* AtA) {
    const bool both = g_gemm_tally.load(std::memory_order_relaxed);
    long long differ = 0;
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
            double q = 0;
            slo_dd::DD s = slo_dd::zero();
            const bool dd = both || t_gemm_mode != 1, seq = both || t_gemm_mode == 1;
            for (int k = 0; k < n; ++k) {
                const double p = (double)A[k * m + i] * (double)A[k * m + j];
                if (seq) q += p;
                if (dd) slo_dd::add(s, p);
            }
            const float f0 = slo_dd::to_float(s), f1 = (float)q;
            differ += memcmp(&f0, &f1, 4) != 0;
            AtA[i * m + j] = t_gemm_mode == 1 ? f1 : f0;
        }
    if (both) {
        g_gemm_entries += (long long)m * m;
        g_gemm_differ += differ;
    }
}
inline void gemm_AtB(const std::vector<float>& A, const std::vector<float>& B, int n, int m, float* AtB) {
    const bool both = g_gemm_tally.load(std::memory_order_relaxed);
    long long differ = 0;
    for (int i = 0; i < m; ++i) {
        double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        int k = 0;
        for (; k <= n - 4; k += 4) {
            s0 += (double)A[k * m + i] * (double)B[k];
            s1 += (double)A[(k + 1) * m + i] * (double)B[k + 1];
            s2 += (double)A[(k + 2) * m + i] * (double)B[k + 2];
            s3 += (double)A[(k + 3) * m + i] * (double)B[k + 3];
        }
        for (; k < n; ++k) s0 += (double)A[k * m + i] * (double)B[k];
        slo_dd::DD s = slo_dd::zero();
        if (both || t_gemm_mode != 1)
            for (int k2 = 0; k2 < n; ++k2) slo_dd::add(s, (double)A[k2 * m + i] * (double)B[k2]);
        const float f0 = slo_dd::to_float(s), f1 = (float)(s0 + s1 + s2 + s3);
        differ += memcmp(&f0, &f1, 4) != 0;
        AtB[i] = t_gemm_mode == 1 ? f1 : f0;
    }
    if (both) {
        g_gemm_entries += m;
        g_gemm_differ += differ;
    }
}
// small dense C = A(r x k) * B(k x c), double accumulation
inline void gemm_small(const float* A, const float* B, int r, int kk, int c, float* C) {
    for (int i = 0; i < r; ++i)
        for (int j = 0; j < c; ++j) {
            double s = 0;
            for (int k = 0; k < kk; ++k) s += (double)A[i * kk + k] * (double)B[k * c + j];
            C[i * c + j] = (float)s;
        }
}

// hal::QR32f -> QRImpl<float>(A, m, n, k=1, b, eps = FLT_EPSILON*10).
// Solves min |A x - b| in place: b's first n entries become x.  Returns 0 on
// a (near-)singular R diagonal (cv::solve then zero-fills the result).
inline int qr_solve(float* A, int m, int n, float* b) {
    float vl[16];
    float hf[16];
    const float eps = FLT_EPSILON * 10;
    for (int l = 0; l < n; l++) {
        int vlSize = m - l;
        float vlNorm = 0.0f;
        for (int i = 0; i < vlSize; i++) {
            vl[i] = A[(l + i) * n + l];
            vlNorm += vl[i] * vl[i];
        }
        float tmpV = vl[0];
        vl[0] = vl[0] + (vl[0] >= 0 ? 1.0f : -1.0f) * sqrtf(vlNorm);
        vlNorm = sqrtf(vlNorm + vl[0] * vl[0] - tmpV * tmpV);
        for (int i = 0; i < vlSize; i++) vl[i] /= vlNorm;
        for (int j = l; j < n; j++) {
            float v_lA = 0.0f;
            for (int i = l; i < m; i++) v_lA += vl[i - l] * A[i * n + j];
            for (int i = l; i < m; i++) A[i * n + j] -= 2 * vl[i - l] * v_lA;
        }
        hf[l] = vl[0] * vl[0];
        for (int i = 1; i < vlSize; i++) A[(l + i) * n + l] = vl[i] / vl[0];
    }
    for (int l = 0; l < n; l++) {
        vl[0] = 1.0f;
        for (int j = 1; j < m - l; j++) vl[j] = A[(j + l) * n + l];
        float v_lB = 0.0f;
        for (int i = l; i < m; i++) v_lB += vl[i - l] * b[i];
        for (int i = l; i < m; i++) b[i] -= 2 * vl[i - l] * v_lB * hf[l];
    }
    for (int i = n - 1; i >= 0; i--) {
        for (int j = n - 1; j > i; j--) b[i] -= b[j] * A[i * n + j];
        if (fabsf(A[i * n + i]) < eps) return 0;
        b[i] /= A[i * n + i];
    }
    return 1;
}

// cv::solve(A(m x n), b(m x 1), x, DECOMP_QR) for float.
inline void cv_solve_qr(const float* A_in, const float* b_in, int m, int n, float* x) {
    float A[64], b[16];
    memcpy(A, A_in, sizeof(float) * m * n);
    memcpy(b, b_in, sizeof(float) * m);
    if (!qr_solve(A, m, n, b)) {
        for (int i = 0; i < n; ++i) x[i] = 0;
        return;
    }
    for (int i = 0; i < n; ++i) x[i] = b[i];
}

// cv::eigen for symmetric float: JacobiImpl_, eigenvalues descending,
// eigenvectors in rows.
inline void cv_eigen_sym(const float* S, int n, float* W, float* V) {
    float A[36];
    memcpy(A, S, sizeof(float) * n * n);
    const float eps = FLT_EPSILON;
    int indR[6], indC[6];
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) V[i * n + j] = 0.0f;
        V[i * n + i] = 1.0f;
    }
    int maxIters = n * n * 30;
    float mv = 0.0f;
    int k, m, i, l;
    for (k = 0; k < n; k++) {
        W[k] = A[(n + 1) * k];
        if (k < n - 1) {
            for (m = k + 1, mv = fabsf(A[n * k + m]), i = k + 2; i < n; i++) {
                float val = fabsf(A[n * k + i]);
                if (mv < val) mv = val, m = i;
            }
            indR[k] = m;
        }
        if (k > 0) {
            for (m = 0, mv = fabsf(A[k]), i = 1; i < k; i++) {
                float val = fabsf(A[n * i + k]);
                if (mv < val) mv = val, m = i;
            }
            indC[k] = m;
        }
    }
    if (n > 1)
        for (int iters = 0; iters < maxIters; iters++) {
            for (k = 0, mv = fabsf(A[indR[0]]), i = 1; i < n - 1; i++) {
                float val = fabsf(A[n * i + indR[i]]);
                if (mv < val) mv = val, k = i;
            }
            l = indR[k];
            for (i = 1; i < n; i++) {
                float val = fabsf(A[n * indC[i] + i]);
                if (mv < val) mv = val, k = indC[i], l = i;
            }
            float p = A[n * k + l];
            if (fabsf(p) <= eps) break;
            float y = (float)((W[l] - W[k]) * 0.5);
            float t = fabsf(y) + hypotf(p, y);
            float s = hypotf(p, t);
            float c = t / s;
            s = p / s;
            t = (p / t) * p;
            if (y < 0) s = -s, t = -t;
            A[n * k + l] = 0;
            W[k] -= t;
            W[l] += t;
            float a0, b0;
#define ORACLE_ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
            for (i = 0; i < k; i++) ORACLE_ROT(A[n * i + k], A[n * i + l]);
            for (i = k + 1; i < l; i++) ORACLE_ROT(A[n * k + i], A[n * i + l]);
            for (i = l + 1; i < n; i++) ORACLE_ROT(A[n * k + i], A[n * l + i]);
            for (i = 0; i < n; i++) ORACLE_ROT(V[n * k + i], V[n * l + i]);
#undef ORACLE_ROT
            for (int j = 0; j < 2; j++) {
                int idx = j == 0 ? k : l;
                if (idx < n - 1) {
                    for (m = idx + 1, mv = fabsf(A[n * idx + m]), i = idx + 2; i < n; i++) {
                        float val = fabsf(A[n * idx + i]);
                        if (mv < val) mv = val, m = i;
                    }
                    indR[idx] = m;
                }
                if (idx > 0) {
                    for (m = 0, mv = fabsf(A[idx]), i = 1; i < idx; i++) {
                        float val = fabsf(A[n * i + idx]);
                        if (mv < val) mv = val, m = i;
                    }
                    indC[idx] = m;
                }
            }
        }
    for (k = 0; k < n - 1; k++) {
        m = k;
        for (i = k + 1; i < n; i++)
            if (W[m] < W[i]) m = i;
        if (k != m) {
            std::swap(W[m], W[k]);
            for (i = 0; i < n; i++) std::swap(V[n * m + i], V[n * k + i]);
        }
    }
}

// Mat::inv() (DECOMP_LU) for float: n==3 cofactor formula in double,
// n>3 hal::LU32f on the identity.  Returns false (and zeros) when singular.
inline bool cv_inv(const float* S, int n, float* D) {
    if (n == 3) {
#define Sf(y, x) ((double)S[(y) * 3 + (x)])
        double d = Sf(0, 0) * (Sf(1, 1) * Sf(2, 2) - Sf(1, 2) * Sf(2, 1)) -
                   Sf(0, 1) * (Sf(1, 0) * Sf(2, 2) - Sf(1, 2) * Sf(2, 0)) +
                   Sf(0, 2) * (Sf(1, 0) * Sf(2, 1) - Sf(1, 1) * Sf(2, 0));
        if (d == 0.) { for (int i = 0; i < 9; ++i) D[i] = 0; return false; }
        d = 1. / d;
        double t[9];
        t[0] = (Sf(1, 1) * Sf(2, 2) - Sf(1, 2) * Sf(2, 1)) * d;
        t[1] = (Sf(0, 2) * Sf(2, 1) - Sf(0, 1) * Sf(2, 2)) * d;
        t[2] = (Sf(0, 1) * Sf(1, 2) - Sf(0, 2) * Sf(1, 1)) * d;
        t[3] = (Sf(1, 2) * Sf(2, 0) - Sf(1, 0) * Sf(2, 2)) * d;
        t[4] = (Sf(0, 0) * Sf(2, 2) - Sf(0, 2) * Sf(2, 0)) * d;
        t[5] = (Sf(0, 2) * Sf(1, 0) - Sf(0, 0) * Sf(1, 2)) * d;
        t[6] = (Sf(1, 0) * Sf(2, 1) - Sf(1, 1) * Sf(2, 0)) * d;
        t[7] = (Sf(0, 1) * Sf(2, 0) - Sf(0, 0) * Sf(2, 1)) * d;
        t[8] = (Sf(0, 0) * Sf(1, 1) - Sf(0, 1) * Sf(1, 0)) * d;
#undef Sf
        for (int i = 0; i < 9; ++i) D[i] = (float)t[i];
        return true;
    }
    float A[36], b[36];
    memcpy(A, S, sizeof(float) * n * n);
    for (int i = 0; i < n * n; ++i) b[i] = 0;
    for (int i = 0; i < n; ++i) b[i * n + i] = 1;
    const float eps = FLT_EPSILON * 10;
    int m = n;
    for (int i = 0; i < m; i++) {
        int k = i;
        for (int j = i + 1; j < m; j++)
            if (fabsf(A[j * n + i]) > fabsf(A[k * n + i])) k = j;
        if (fabsf(A[k * n + i]) < eps) { for (int q = 0; q < n * n; ++q) D[q] = 0; return false; }
        if (k != i) {
            for (int j = i; j < m; j++) std::swap(A[i * n + j], A[k * n + j]);
            for (int j = 0; j < n; j++) std::swap(b[i * n + j], b[k * n + j]);
        }
        float d = -1 / A[i * n + i];
        for (int j = i + 1; j < m; j++) {
            float alpha = A[j * n + i] * d;
            for (int kk = i + 1; kk < m; kk++) A[j * n + kk] += alpha * A[i * n + kk];
            for (int kk = 0; kk < n; kk++) b[j * n + kk] += alpha * b[i * n + kk];
        }
        A[i * n + i] = -d;
    }
    for (int i = m - 1; i >= 0; i--)
        for (int j = 0; j < n; j++) {
            float s = b[i * n + j];
            for (int k = i + 1; k < m; k++) s -= A[i * n + k] * b[k * n + j];
            b[i * n + j] = s * A[i * n + i];
        }
    memcpy(D, b, sizeof(float) * n * n);
    return true;
}

}  // namespace oracle
