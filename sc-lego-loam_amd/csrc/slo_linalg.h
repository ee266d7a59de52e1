// slo_linalg.h — OpenCV 3.x small dense routines as the reference calls them,
// written for one GPU lane (also compiles on the host).
//   qr_solve   : cv::solve(..., DECOMP_QR) -> hal::QR32f / QRImpl<float>
//                (FA:1327, 1428; MO:1361 (5x3 least squares), 1448)
//   eigen_sym  : cv::eigen -> JacobiImpl_<float>, eigenvalues descending,
//                eigenvectors in rows (FA:1334, 1435; MO:1298, 1455)
//   inv        : Mat::inv() (DECOMP_LU): 3x3 cofactors in double, n>3 LUImpl
//                (FA:1349, 1450; MO:1470)
//   mul        : float Mat product with double accumulation (GEMM 32F)
// The oracle (oracle/oracle_common.h) restates the same algorithms
// independently; the GPU parity tests compare the two.
#pragma once

#include <math.h>
#include <float.h>
#include "slo_libm.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SLO_LA_HD __host__ __device__ inline
#else
#define SLO_LA_HD inline
#endif

namespace slo_la {

// Householder QR least squares, A (m x n, row-major, m <= 8, n <= 6), b (m).
// On success b[0..n) holds x; returns 0 if a diagonal of R is below eps
// (the caller then zero-fills x, as cv::solve does).  Sizes are template
// parameters so every loop unrolls and the small arrays live in registers
// (on the GPU a runtime-sized local array goes to scratch memory).
template <int M, int N>
SLO_LA_HD int qr_solve_t(float* A, float* b) {
    constexpr int m = M, n = N;
    float vl[8], hf[8];
    const float eps = FLT_EPSILON * 10;
    for (int l = 0; l < n; l++) {
        const int vs = m - l;
        float nrm = 0.0f;
        for (int i = 0; i < vs; i++) {
            vl[i] = A[(l + i) * n + l];
            nrm += vl[i] * vl[i];
        }
        const float v0 = vl[0];
        vl[0] = vl[0] + (vl[0] >= 0 ? 1.0f : -1.0f) * sqrtf(nrm);
        nrm = sqrtf(nrm + vl[0] * vl[0] - v0 * v0);
        for (int i = 0; i < vs; i++) vl[i] /= nrm;
        for (int j = l; j < n; j++) {
            float d = 0.0f;
            for (int i = l; i < m; i++) d += vl[i - l] * A[i * n + j];
            for (int i = l; i < m; i++) A[i * n + j] -= 2 * vl[i - l] * d;
        }
        hf[l] = vl[0] * vl[0];
        for (int i = 1; i < vs; i++) A[(l + i) * n + l] = vl[i] / vl[0];
    }
    for (int l = 0; l < n; l++) {
        vl[0] = 1.0f;
        for (int j = 1; j < m - l; j++) vl[j] = A[(j + l) * n + l];
        float d = 0.0f;
        for (int i = l; i < m; i++) d += vl[i - l] * b[i];
        for (int i = l; i < m; i++) b[i] -= 2 * vl[i - l] * d * hf[l];
    }
    for (int i = n - 1; i >= 0; i--) {
        for (int j = n - 1; j > i; j--) b[i] -= b[j] * A[i * n + j];
        if (fabsf(A[i * n + i]) < eps) return 0;
        b[i] /= A[i * n + i];
    }
    return 1;
}

// x = solve(A, b) as cv::solve(DECOMP_QR) returns it (zeros on failure)
template <int M, int N>
SLO_LA_HD void solve_qr_t(const float* Ain, const float* bin, float* x) {
    float A[M * N], b[M];
#pragma unroll
    for (int i = 0; i < M * N; ++i) A[i] = Ain[i];
#pragma unroll
    for (int i = 0; i < M; ++i) b[i] = bin[i];
    if (!qr_solve_t<M, N>(A, b)) {
        for (int i = 0; i < N; ++i) x[i] = 0.0f;
        return;
    }
    for (int i = 0; i < N; ++i) x[i] = b[i];
}
// the shapes the path uses: 3x3 (FA), 5x3 (MO plane fit), 6x6 (MO)
SLO_LA_HD void solve_qr(const float* A, const float* b, int m, int n, float* x) {
    if (m == 3 && n == 3) solve_qr_t<3, 3>(A, b, x);
    else if (m == 5 && n == 3) solve_qr_t<5, 3>(A, b, x);
    else solve_qr_t<6, 6>(A, b, x);
}

// Jacobi eigen-decomposition of a symmetric n x n (n <= 6).  The rotation
// indices are data-dependent, so on the GPU the matrix, W, V and the row /
// column maxima live in memory: eigen_sym_ws takes them from the caller
// (LDS in the one-lane solves, where private arrays went to scratch memory).
template <int N>
SLO_LA_HD void eigen_sym_ws(const float* S, float* W, float* V, float* A, int* indR, int* indC) {
    constexpr int n = N;
#pragma unroll
    for (int i = 0; i < n * n; ++i) A[i] = S[i];
    const float eps = FLT_EPSILON;
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) V[i * n + j] = 0.0f;
        V[i * n + i] = 1.0f;
    }
    float mv;
    int k, m, i, l;
    for (k = 0; k < n; k++) {
        W[k] = A[(n + 1) * k];
        if (k < n - 1) {
            m = k + 1; mv = fabsf(A[n * k + m]);
            for (i = k + 2; i < n; i++) { float a = fabsf(A[n * k + i]); if (mv < a) { mv = a; m = i; } }
            indR[k] = m;
        }
        if (k > 0) {
            m = 0; mv = fabsf(A[k]);
            for (i = 1; i < k; i++) { float a = fabsf(A[n * i + k]); if (mv < a) { mv = a; m = i; } }
            indC[k] = m;
        }
    }
    const int maxIters = n * n * 30;
    if (n > 1)
        for (int it = 0; it < maxIters; it++) {
            k = 0; mv = fabsf(A[indR[0]]);
            for (i = 1; i < n - 1; i++) { float a = fabsf(A[n * i + indR[i]]); if (mv < a) { mv = a; k = i; } }
            l = indR[k];
            for (i = 1; i < n; i++) { float a = fabsf(A[n * indC[i] + i]); if (mv < a) { mv = a; k = indC[i]; l = i; } }
            float p = A[n * k + l];
            if (fabsf(p) <= eps) break;
            float y = (float)((W[l] - W[k]) * 0.5);
            float t = fabsf(y) + slo_libm::hypotf_(p, y);
            float s = slo_libm::hypotf_(p, t);
            float c = t / s;
            s = p / s;
            t = (p / t) * p;
            if (y < 0) { s = -s; t = -t; }
            A[n * k + l] = 0;
            W[k] -= t;
            W[l] += t;
            for (i = 0; i < k; i++) { float a0 = A[n * i + k], b0 = A[n * i + l]; A[n * i + k] = a0 * c - b0 * s; A[n * i + l] = a0 * s + b0 * c; }
            for (i = k + 1; i < l; i++) { float a0 = A[n * k + i], b0 = A[n * i + l]; A[n * k + i] = a0 * c - b0 * s; A[n * i + l] = a0 * s + b0 * c; }
            for (i = l + 1; i < n; i++) { float a0 = A[n * k + i], b0 = A[n * l + i]; A[n * k + i] = a0 * c - b0 * s; A[n * l + i] = a0 * s + b0 * c; }
            for (i = 0; i < n; i++) { float a0 = V[n * k + i], b0 = V[n * l + i]; V[n * k + i] = a0 * c - b0 * s; V[n * l + i] = a0 * s + b0 * c; }
            for (int jj = 0; jj < 2; jj++) {
                int idx = jj == 0 ? k : l;
                if (idx < n - 1) {
                    m = idx + 1; mv = fabsf(A[n * idx + m]);
                    for (i = idx + 2; i < n; i++) { float a = fabsf(A[n * idx + i]); if (mv < a) { mv = a; m = i; } }
                    indR[idx] = m;
                }
                if (idx > 0) {
                    m = 0; mv = fabsf(A[idx]);
                    for (i = 1; i < idx; i++) { float a = fabsf(A[n * i + idx]); if (mv < a) { mv = a; m = i; } }
                    indC[idx] = m;
                }
            }
        }
    for (k = 0; k < n - 1; k++) {
        m = k;
        for (i = k + 1; i < n; i++) if (W[m] < W[i]) m = i;
        if (k != m) {
            float t = W[m]; W[m] = W[k]; W[k] = t;
            for (i = 0; i < n; i++) { float a = V[n * m + i]; V[n * m + i] = V[n * k + i]; V[n * k + i] = a; }
        }
    }
}
template <int N>
SLO_LA_HD void eigen_sym_t(const float* S, float* W, float* V) {
    float A[N * N];
    int indR[6], indC[6];
    eigen_sym_ws<N>(S, W, V, A, indR, indC);
}
SLO_LA_HD void eigen_sym(const float* S, int n, float* W, float* V) {
    if (n == 3) eigen_sym_t<3>(S, W, V);
    else eigen_sym_t<6>(S, W, V);
}

SLO_LA_HD void inv_ws(const float* S, int n, float* D, float* A, float* b);
SLO_LA_HD void inv(const float* S, int n, float* D) {
    if (n == 3) {
        double s00 = S[0], s01 = S[1], s02 = S[2], s10 = S[3], s11 = S[4], s12 = S[5], s20 = S[6], s21 = S[7], s22 = S[8];
        double d = s00 * (s11 * s22 - s12 * s21) - s01 * (s10 * s22 - s12 * s20) + s02 * (s10 * s21 - s11 * s20);
        if (d == 0.) { for (int i = 0; i < 9; ++i) D[i] = 0; return; }
        d = 1. / d;
        D[0] = (float)((s11 * s22 - s12 * s21) * d);
        D[1] = (float)((s02 * s21 - s01 * s22) * d);
        D[2] = (float)((s01 * s12 - s02 * s11) * d);
        D[3] = (float)((s12 * s20 - s10 * s22) * d);
        D[4] = (float)((s00 * s22 - s02 * s20) * d);
        D[5] = (float)((s02 * s10 - s00 * s12) * d);
        D[6] = (float)((s10 * s21 - s11 * s20) * d);
        D[7] = (float)((s01 * s20 - s00 * s21) * d);
        D[8] = (float)((s00 * s11 - s01 * s10) * d);
        return;
    }
    float A[36], b[36];
    inv_ws(S, n, D, A, b);
}
// the n > 3 LU inverse with the caller's workspaces A, b (n * n each)
SLO_LA_HD void inv_ws(const float* S, int n, float* D, float* A, float* b) {
    for (int i = 0; i < n * n; ++i) { A[i] = S[i]; b[i] = 0; }
    for (int i = 0; i < n; ++i) b[i * n + i] = 1;
    const float eps = FLT_EPSILON * 10;
    for (int i = 0; i < n; i++) {
        int k = i;
        for (int j = i + 1; j < n; j++) if (fabsf(A[j * n + i]) > fabsf(A[k * n + i])) k = j;
        if (fabsf(A[k * n + i]) < eps) { for (int q = 0; q < n * n; ++q) D[q] = 0; return; }
        if (k != i) {
            for (int j = i; j < n; j++) { float t = A[i * n + j]; A[i * n + j] = A[k * n + j]; A[k * n + j] = t; }
            for (int j = 0; j < n; j++) { float t = b[i * n + j]; b[i * n + j] = b[k * n + j]; b[k * n + j] = t; }
        }
        float d = -1 / A[i * n + i];
        for (int j = i + 1; j < n; j++) {
            float alpha = A[j * n + i] * d;
            for (int q = i + 1; q < n; q++) A[j * n + q] += alpha * A[i * n + q];
            for (int q = 0; q < n; q++) b[j * n + q] += alpha * b[i * n + q];
        }
        A[i * n + i] = -d;
    }
    for (int i = n - 1; i >= 0; i--)
        for (int j = 0; j < n; j++) {
            float s = b[i * n + j];
            for (int q = i + 1; q < n; q++) s -= A[i * n + q] * b[q * n + j];
            b[i * n + j] = s * A[i * n + i];
        }
    for (int i = 0; i < n * n; ++i) D[i] = b[i];
}

// C (r x c) = A (r x k) * B (k x c), double accumulation, float result
SLO_LA_HD void mul(const float* A, const float* B, int r, int k, int c, float* C) {
    for (int i = 0; i < r; ++i)
        for (int j = 0; j < c; ++j) {
            double s = 0;
            for (int q = 0; q < k; ++q) s += (double)A[i * k + q] * (double)B[q * c + j];
            C[i * c + j] = (float)s;
        }
}

}  // namespace slo_la
