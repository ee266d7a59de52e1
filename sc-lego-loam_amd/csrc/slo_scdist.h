// slo_scdist.h — Scan Context arithmetic shared by the in-session detect
// (slo_sc.hip), the descriptor build (slo_map.hip) and the cross-session
// store (slo_xsc.hip), each in the reference's exact evaluation order:
//   eigen_sum   Eigen 3.3 SSE2 packet-order sum (Appendix A Q12d)
//   l2_nf       nanoflann's 4-unrolled float L2 (the ring-key tree, NF:383-408)
//   ESum        streaming form of eigen_sum for the column norms / dots
//   sc_pair_distance  SCManager::distanceBtnScanContext (SCc:116-148): the
//               sector-key alignment over all shifts (fastAlignUsingVkey,
//               SCc:93-113), the 7-shift window sorted ascending, the
//               column-cosine distance per shift (distDirectSC, SCc:69-90)
//               from the column Gram on the matrix cores (sc_gram_mfma),
//               first minimum — run by a whole workgroup.
#pragma once
#include "slo_internal.h"

namespace slo {

#define SC_K SLO_SC_MAX_K
#define SC_NS SLO_SC_MAX_SECTOR

__device__ inline double eigen_sum(const double* x, int n, int stride) {
    if (n < 2) return n ? x[0] : 0.0;
    const int a2 = (n / 4) * 4, a1 = (n / 2) * 2;
    double p0a = x[0], p0b = x[stride];
    if (a1 > 2) {
        double p1a = x[2 * stride], p1b = x[3 * stride];
        for (int i = 4; i < a2; i += 4) {
            p0a += x[i * stride]; p0b += x[(i + 1) * stride];
            p1a += x[(i + 2) * stride]; p1b += x[(i + 3) * stride];
        }
        p0a += p1a; p0b += p1b;
        if (a1 > a2) { p0a += x[a2 * stride]; p0b += x[(a2 + 1) * stride]; }
    }
    double r = p0a + p0b;
    for (int i = a1; i < n; ++i) r += x[i * stride];
    return r;
}

__device__ inline float l2_nf(const float* a, const float* b, int n) {
    float result = 0;
    int d = 0;
    for (; d + 3 < n; d += 4) {
        const float d0 = a[d] - b[d], d1 = a[d + 1] - b[d + 1], d2 = a[d + 2] - b[d + 2], d3 = a[d + 3] - b[d + 3];
        result += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
    for (; d < n; ++d) { const float d0 = a[d] - b[d]; result += d0 * d0; }
    return result;
}

// streaming Eigen SSE2 sum: 4 lane accumulators, combined (0+2)+(1+3)
struct ESum {
    double a0, a1, a2, a3;
    int n;
    __device__ ESum() : a0(0), a1(0), a2(0), a3(0), n(0) {}
    __device__ void add(double x) {
        switch (n & 3) { case 0: a0 = n < 4 ? x : a0 + x; break; case 1: a1 = n < 4 ? x : a1 + x; break;
                         case 2: a2 = n < 4 ? x : a2 + x; break; default: a3 = n < 4 ? x : a3 + x; }
        ++n;
    }
    __device__ double get() const { return (a0 + a2) + (a1 + a3); }  // valid for n % 4 == 0, n >= 4
};

__device__ inline unsigned long long wave_min_u64(unsigned long long x) {
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(x, o, 64);
        x = y < x ? y : x;
    }
    return x;
}

// workgroup scratch of sc_pair_distance
#define SC_GS (SC_NS + 1)   // Gram row stride (doubles): odd, so a column walk spreads over the banks
struct ScPairLds {
    double sim[7 * SC_NS];
    int simok[7 * SC_NS];
    double dist7[7];
    double shnorm[SC_NS];
    int shifts[7];
    double n1[SC_NS], n2[SC_NS];   // column norms of sc1 / sc2 (the MFMA form)
    double G[SC_NS * SC_GS];       // column Gram sc1^T sc2 (the MFMA form)
};

// ---- the column cosines of distDirectSC (SCc:69-90) on the matrix cores.
// Every shift's cosines are entries of ONE column Gram G = sc1^T sc2 (NS x NS,
// G[i][j] = sum over rings r of sc1[r][i] * sc2[r][j]): shift sh reads
// G[j][(j - sh) mod NS].  Eigen's SSE2 order for such a 20-term dot (ESum:
// four lane accumulators over r mod 4, each a sequential double sum of exact
// float x float products, combined (0 + 2) + (1 + 3)) maps onto
// v_mfma_f64_16x16x4_f64, which computes a k-ordered chain of fused
// multiply-adds bit for bit (tools/mfma_f64_check.hip: 0 of 5.1 M random
// outputs differ from the chain): accumulator u takes rings u, u + 4, u + 8,
// u + 12 as k = 0..3 of one MFMA and u + 16, ... in the next, from a zero C.
// A product of two floats is exact in double, so fma(a, b, acc) = acc + a*b,
// as Eigen adds it (a zero start turns a leading -0 product into +0, which
// no cosine, norm or mean can tell apart).  The workgroup's four waves take
// the four 16-row tile rows of the 64 x 64 padded Gram: per wave 4 tiles x
// 4 accumulators x ceil(NR / 16) MFMAs (32 at NR = 20).  Needs NR % 4 == 0
// (ESum's combine, as the VALU form) and 256 threads.
typedef double sc_d4 __attribute__((ext_vector_type(4)));
__device__ inline void sc_gram_mfma(const double* sc1, const double* sc2, int NR, int NS, double* G) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, kq = lane >> 4, c = lane & 15;
    const int nm = (NR + 15) >> 4;
    const int ia = 16 * w + c;
    for (int J = 0; J < 4; ++J) {
        const int jb = 16 * J + c;
        sc_d4 acc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = sc_d4{0.0, 0.0, 0.0, 0.0};
        for (int m = 0; m < nm; ++m) {
            double a[4], b[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {   // unconditional (clamped) loads, all in flight before the MFMAs
                const int r = u + 4 * kq + 16 * m, rr = min(r, NR - 1);
                a[u] = sc1[rr * NS + min(ia, NS - 1)];
                b[u] = sc2[rr * NS + min(jb, NS - 1)];
                a[u] = (r < NR && ia < NS) ? a[u] : 0.0;
                b[u] = (r < NR && jb < NS) ? b[u] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc[u], 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // D row (lane >> 4) + 4 q, column lane & 15
            const int i = 16 * w + kq + 4 * q;
            if (i < NS && jb < NS) G[i * SC_GS + jb] = (acc[0][q] + acc[2][q]) + (acc[1][q] + acc[3][q]);
        }
    }
}

// distanceBtnScanContext(sc1, sc2) -> (*dist, *align), valid in thread 0;
// every thread of the workgroup must call it (it synchronises).  With 256
// threads and NR % 4 == 0 (every preset: 20 rings) the column cosines come
// from the MFMA Gram (sc_gram_mfma), else from per-thread ESum dots; the two
// give the same doubles.
__device__ inline void sc_pair_distance(const double* sc1, const double* vk1, const double* sc2, const double* vk2,
                                        int NR, int NS, double search_ratio, ScPairLds& L, double* dist,
                                        int* align) {
    const int tid = threadIdx.x;
    const bool mfma = blockDim.x == 256 && NR >= 4 && (NR & 3) == 0;
    // fastAlignUsingVkey: 60 shifts on 60 lanes; the column norms beside it
    if (tid < NS) {
        ESum e;
        for (int j = 0; j < NS; ++j) {
            double d = vk1[j] - vk2[((j - tid) % NS + NS) % NS];
            e.add(d * d);
        }
        L.shnorm[tid] = sqrt(e.get());
    } else if (mfma && tid >= 64 && tid < 64 + 2 * NS && tid < 256) {
        const int j = (tid - 64) % NS;
        const double* d = tid < 64 + NS ? sc1 : sc2;
        ESum e;
        for (int r = 0; r < NR; ++r) {
            const double a = d[r * NS + j];
            e.add(a * a);
        }
        (tid < 64 + NS ? L.n1 : L.n2)[j] = sqrt(e.get());
    }
    if (mfma) sc_gram_mfma(sc1, sc2, NR, NS, L.G);
    __syncthreads();
    if (tid == 0) {
        int argmin = 0;
        double mn = 10000000;
        for (int sh = 0; sh < NS; ++sh)
            if (L.shnorm[sh] < mn) { argmin = sh; mn = L.shnorm[sh]; }
        const int R = (int)round(0.5 * search_ratio * NS);
        int sp[7], n = 0;
        sp[n++] = argmin;
        for (int ii = 1; ii < R + 1 && n < 7; ii++) {
            sp[n++] = (argmin + ii + NS) % NS;
            sp[n++] = (argmin - ii + NS) % NS;
        }
        for (int a = 1; a < n; ++a) {  // ascending (std::sort on 7 ints)
            int x = sp[a], b = a - 1;
            while (b >= 0 && sp[b] > x) { sp[b + 1] = sp[b]; --b; }
            sp[b + 1] = x;
        }
        for (int k = 0; k < 7; ++k) L.shifts[k] = k < n ? sp[k] : -1;
    }
    __syncthreads();
    // column cosines for the 7 shifts
    for (int t = tid; t < 7 * NS; t += blockDim.x) {
        const int k = t / NS, j = t - k * NS;
        const int sh = L.shifts[k];
        L.simok[t] = 0;
        if (sh < 0) continue;
        const int j2 = ((j - sh) % NS + NS) % NS;
        double nn1, nn2, dt;
        if (mfma) {
            nn1 = L.n1[j]; nn2 = L.n2[j2]; dt = L.G[j * SC_GS + j2];
        } else {
            ESum n1, n2, d;
            for (int r = 0; r < NR; ++r) {
                double a = sc1[r * NS + j], b = sc2[r * NS + j2];
                n1.add(a * a); n2.add(b * b); d.add(a * b);
            }
            nn1 = sqrt(n1.get()); nn2 = sqrt(n2.get()); dt = d.get();
        }
        if ((nn1 == 0) | (nn2 == 0)) continue;
        L.sim[t] = dt / (nn1 * nn2);
        L.simok[t] = 1;
    }
    __syncthreads();
    if (tid < 7) {
        double sum = 0;
        int ne = 0;
        for (int j = 0; j < NS; ++j)
            if (L.simok[tid * NS + j]) { sum = sum + L.sim[tid * NS + j]; ne = ne + 1; }
        L.dist7[tid] = L.shifts[tid] < 0 ? 10000000 : 1.0 - sum / ne;
    }
    __syncthreads();
    if (tid == 0) {
        int am = 0;
        double md = 10000000;
        for (int k = 0; k < 7; ++k)
            if (L.shifts[k] >= 0 && L.dist7[k] < md) { am = L.shifts[k]; md = L.dist7[k]; }
        *dist = md;
        *align = am;
    }
    __syncthreads();
}

}  // namespace slo
