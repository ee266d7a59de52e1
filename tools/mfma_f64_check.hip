// mfma_f64_check.hip — what v_mfma_f64_16x16x4_f64 computes, bit for bit.
//
// For the Scan Context column cosines (Scancontext.cpp:69-90) to run on the
// matrix cores and still equal Eigen's SSE2 order (four lane accumulators,
// each a sequential double sum of exact float x float products), each
// accumulator must be a k-ordered chain of fused multiply-adds.  This program
// feeds random tiles (general doubles of mixed magnitudes, so that different
// summation orders round differently) and counts, per hypothesis, the output
// elements that differ:
//   H0  D = fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0, C))))   (k-ordered fma chain)
//   H1  the same chain in the order k = 3, 2, 1, 0
//   H2  products rounded, then added left to right: ((C + p0) + p1) + ...
//   H3  C + ((p0 + p1) + (p2 + p3)) with exact products (tree), one rounding per add
// Layout (cdna_hip_programming.md "f64 MFMA"): lane l holds A[l&15][l>>4] and
// B[l>>4][l&15]; D row (l>>4) + 4 r, column l&15, in register r.
//   hipcc --offload-arch=gfx950 -O2 -o mfma_f64_check tools/mfma_f64_check.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_mfma(const double* A, const double* B, const double* C, double* D, int tiles) {
    const int t = blockIdx.x, l = threadIdx.x;
    if (t >= tiles) return;
    const double* a = A + (size_t)t * 64;   // [16][4]
    const double* b = B + (size_t)t * 64;   // [4][16]
    const double* c = C + (size_t)t * 256;  // [16][16]
    const double av = a[(l & 15) * 4 + (l >> 4)], bv = b[(l >> 4) * 16 + (l & 15)];
    d4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = c[((l >> 4) + 4 * r) * 16 + (l & 15)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[(size_t)t * 256 + ((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

// throughput: every wave issues ITER x 4 independent 16x16x4 f64 MFMAs back to back
#define ITER 4096
__global__ void __launch_bounds__(256) k_rate(double* out, double seed) {
    const int l = threadIdx.x & 63;
    const double a = seed + l, b = seed - l;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < ITER; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
    const double s = (c0[0] + c1[1]) + (c2[2] + c3[3]);
    if (s == 12345.678) out[0] = s;   // keep the chains alive
}

int main(int argc, char** argv) {
    const int tiles = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-1.0, 1.0), e(-30.0, 30.0);
    auto rnd = [&]() { return u(g) * std::ldexp(1.0, (int)e(g)); };
    std::vector<double> A(64 * (size_t)tiles), B(64 * (size_t)tiles), C(256 * (size_t)tiles), D(256 * (size_t)tiles);
    for (auto& x : A) x = rnd();
    for (auto& x : B) x = rnd();
    for (size_t i = 0; i < C.size(); ++i) C[i] = (i % 5 == 0) ? 0.0 : rnd();
    double *dA, *dB, *dC, *dD;
    hipMalloc(&dA, 8 * A.size()); hipMalloc(&dB, 8 * B.size()); hipMalloc(&dC, 8 * C.size()); hipMalloc(&dD, 8 * D.size());
    hipMemcpy(dA, A.data(), 8 * A.size(), hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 8 * B.size(), hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), 8 * C.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma, dim3(tiles), dim3(64), 0, 0, dA, dB, dC, dD, tiles);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
    hipMemcpy(D.data(), dD, 8 * D.size(), hipMemcpyDeviceToHost);
    long long bad[4] = {0, 0, 0, 0}, n = 0;
    for (int t = 0; t < tiles; ++t)
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                const double* a = &A[(size_t)t * 64 + i * 4];
                double bk[4];
                for (int k = 0; k < 4; ++k) bk[k] = B[(size_t)t * 64 + k * 16 + j];
                const double c = C[(size_t)t * 256 + i * 16 + j], d = D[(size_t)t * 256 + i * 16 + j];
                double h0 = c, h1 = c, h2 = c;
                for (int k = 0; k < 4; ++k) h0 = std::fma(a[k], bk[k], h0);
                for (int k = 3; k >= 0; --k) h1 = std::fma(a[k], bk[k], h1);
                for (int k = 0; k < 4; ++k) { volatile double p = a[k] * bk[k]; h2 = h2 + p; }
                volatile double p0 = a[0] * bk[0], p1 = a[1] * bk[1], p2 = a[2] * bk[2], p3 = a[3] * bk[3];
                const double h3 = c + ((p0 + p1) + (p2 + p3));
                const double h[4] = {h0, h1, h2, h3};
                for (int q = 0; q < 4; ++q) bad[q] += std::memcmp(&h[q], &d, 8) != 0;
                ++n;
            }
    printf("elements %lld  mismatches: H0 k-ordered fma chain %lld, H1 reversed %lld, H2 rounded products %lld, "
           "H3 tree %lld\n", n, bad[0], bad[1], bad[2], bad[3]);
    printf(bad[0] == 0 ? "MFMA_F64_IS_K_ORDERED_FMA_CHAIN\n" : "MFMA_F64_NOT_H0\n");
    // f64 MFMA peak, measured: 8192 workgroups of four waves (every SIMD busy)
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int wg = 8192;
    hipLaunchKernelGGL(k_rate, dim3(wg), dim3(256), 0, 0, dD, 0.5);   // warm-up
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate, dim3(wg), dim3(256), 0, 0, dD, 0.25);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = (double)wg * 4 * ITER * 4 * 2048.0;
    printf("f64 MFMA 16x16x4: %.1f TFLOP/s over %.3f ms (%d waves x %d MFMAs)\n", flop / (ms * 1e-3) / 1e12, ms,
           wg * 4, ITER * 4);
    return 0;
}
