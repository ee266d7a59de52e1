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
        float E[3], V[9], V2[9], Vi[9];
        slo_la::eigen_sym(AtA, 3, E, V);
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
//   k_fa_search<PH>  one thread per query, S x ceil(cap/256) workgroups: the
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
            st.iters_surf = st.iters_corner = 0;
            st.odo_phase = 3;
        }
        return;
    }
    if (tid == 0) {  // updateTransformation (FA:1666-1672)
        st.iters_surf = st.iters_corner = 0;
        st.odo_phase = (st.cornerLastNum < 10 || st.surfLastNum < 100) ? 2 : 0;
    }
}

// min of sq3_ref over a[j0..j1) visited upward / downward with the
// reference's strict '<' (so ties keep the first index met)
__device__ inline void walk_up(const float4* a, int j0, int j1, const P4& q, float& m, int& mi) {
#pragma unroll 4
    for (int j = j0; j < j1; ++j) {
        const float d = sq3_ref(a[j], q);
        if (d < m) { m = d; mi = j; }
    }
}
__device__ inline void walk_down(const float4* a, int j0, int j1, const P4& q, float& m, int& mi) {
#pragma unroll 4
    for (int j = j1 - 1; j >= j0; --j) {
        const float d = sq3_ref(a[j], q);
        if (d < m) { m = d; mi = j; }
    }
}

// findCorrespondingSurfFeatures (FA:1155-1268) / ...CornerFeatures
// (FA:1044-1153) for one query: exact 1-NN in the tree cloud, then the
// ring-ordered walk for the 2nd (and 3rd) points within +-2.5 rings.
//
// The *Last clouds are concatenated ring by ring, so the reference's walk —
// step away from `closest` until the ring leaves [cscan-2, cscan+2], sorting
// each point into "same/lower ring" or "other ring" by its ring — is exactly a
// min over four index ranges cut at the ring boundaries (roff_last), in the
// same visiting order: forward over [closest+1, ...) bounded by Q7's
// min(query count, cloud size), then backward from closest-1.
//
// 1-NN: surf (dense, ~10^4-10^5 points) through the 1 m hash grid; corner
// (sparse, <= 120 R points) by brute force, the cloud streamed through LDS in
// 256-point tiles shared by the workgroup's 256 queries (lowest index wins
// ties: strict '<' in index order).
template <int PH>
__global__ void __launch_bounds__(256) k_fa_search(DevView v, int nb) {
    int s, chunk;
    xcd_stream_chunk(blockIdx.x, nb, s, chunk);
    if (s >= v.S) return;
    const StreamState& st = v.st[s];
    if (st.odo_phase != PH) return;
    const int i = chunk * blockDim.x + threadIdx.x;
    const int nq = PH == 0 ? st.n_flat : st.n_sharp;
    if (chunk * (int)blockDim.x >= nq) return;   // whole workgroup idle (uniform)
    const bool active = i < nq;
    const float gate = v.cfg.nearest_feature_search_sq_dist;
    const int R = v.cfg.n_scan;
    float tc[6];
    for (int k = 0; k < 6; ++k) tc[k] = st.transformCur[k];
    const float4* qp = PH == 0 ? v.flat + (size_t)s * v.cap_flat : v.sharp + (size_t)s * v.cap_sharp;
    const P4 sel = slo_pose::transform_to_start(ld4(qp, active ? i : 0), tc);
    const int32_t* rf = v.roff_last + ((size_t)s * 2 + (PH == 0 ? 1 : 0)) * (R + 1);
    auto ring_first = [&](int r) { return rf[min(max(r, 0), R)]; };
    int ci; float cd;
    if (PH == 0) {
        nn1_grid(v.g_os, s, gate, sel, ci, cd);
    } else {
        __shared__ float4 tile[256];
        const float4* kd = v.kd_corner + (size_t)s * v.cap_less_sharp;
        const int n = st.kdCornerNum;
        ci = -1; cd = FLT_MAX;
        const bool fin = isfinite(sel.x) && isfinite(sel.y) && isfinite(sel.z);
        for (int t0 = 0; t0 < n; t0 += 256) {
            __syncthreads();
            if (t0 + (int)threadIdx.x < n) tile[threadIdx.x] = kd[t0 + threadIdx.x];
            __syncthreads();
            const int m = min(256, n - t0);
            if (active && fin)
                for (int k = 0; k < m; ++k) {
                    const float d = sqdist_flann(sel, tile[k]);
                    if (d < cd) { cd = d; ci = t0 + k; }
                }
        }
    }
    if (!active) return;
    if (PH == 0) {
        const float4* slast = v.surf_last + (size_t)s * v.cap_less_flat;
        const int surfLastNum = st.surfLastNum;
        int closest = -1, i2 = -1, i3 = -1;
        if (cd < gate && ci >= 0 && ci < surfLastNum) {
            closest = ci;
            const int cscan = (int)slast[closest].w;
            const int lim = min(nq, surfLastNum);                        // Q7: bounded by the flat count
            const int e0 = ring_first(cscan + 1), e2 = ring_first(cscan + 3);
            const int b0 = ring_first(cscan), b2 = ring_first(cscan - 2);
            float m2 = gate, m3 = gate;
            walk_up(slast, closest + 1, min(e0, lim), sel, m2, i2);         // ring == cscan
            walk_up(slast, max(closest + 1, e0), min(e2, lim), sel, m3, i3); // cscan < ring <= cscan+2
            walk_down(slast, b0, closest, sel, m2, i2);                      // ring == cscan
            walk_down(slast, b2, min(b0, closest), sel, m3, i3);             // cscan-2 <= ring < cscan
        }
        int32_t* ind = v.ind_surf + (size_t)s * v.cap_flat * 3;
        ind[3 * i] = closest; ind[3 * i + 1] = i2; ind[3 * i + 2] = i3;
    } else {
        const float4* clast = v.corner_last + (size_t)s * v.cap_less_sharp;
        const int cornerLastNum = st.cornerLastNum;
        int closest = -1, i2 = -1;
        if (cd < gate && ci >= 0 && ci < cornerLastNum) {
            closest = ci;
            const int cscan = (int)clast[closest].w;
            const int lim = min(nq, cornerLastNum);                      // Q7: bounded by the sharp count
            float m2 = gate;
            walk_up(clast, max(closest + 1, ring_first(cscan + 1)), min(ring_first(cscan + 3), lim), sel, m2, i2);
            walk_down(clast, ring_first(cscan - 2), min(ring_first(cscan), closest), sel, m2, i2);
        }
        int32_t* indc = v.ind_corner + (size_t)s * v.cap_sharp * 2;
        indc[2 * i] = closest; indc[2 * i + 1] = i2;
    }
}

// iterations iter0 .. iter0+4 of calculateTransformationSurf (FA:1270-1377)
// or ...Corner (FA:1379-1478) for one stream
template <int PH>
__global__ void __launch_bounds__(256) k_fa_iter(DevView v, int iter0) {
    const int s = blockIdx.x;
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
    if (threadIdx.x < 6) tc[threadIdx.x] = st.transformCur[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) slo_pose::tc_trig(tc, tct);
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
        const P4 q = slo_pose::transform_to_end(ld4(corner ? lsharp : lflat, k), tc, tct);
        const float4 o = make_float4(q.x, q.y, q.z, q.w);
        (corner ? cnext : snext)[k] = o;
        if (rebuild) (corner ? kdc : kds)[k] = o;
    }
}

// integrate (FA:1697-1725) and the *Last / tree bookkeeping, per stream
__global__ void __launch_bounds__(64) k_fa_odo_finish(DevView v) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    if (st.odo_phase == 3) return;
    copy_ring_offsets(v, s);
    if (threadIdx.x == 0) {
        float tc[6];
        for (int k = 0; k < 6; ++k) tc[k] = st.transformCur[k];
        slo_pose::integrate(st.transformSum, tc);
        const int nLS = st.n_less_sharp, nLF = st.n_less_flat;
        st.cornerLastNum = nLS;
        st.surfLastNum = nLF;
        if (nLS > 10 && nLF > 100) { st.kdCornerNum = nLS; st.kdSurfNum = nLF; }
    }
}

int fa_odometry_run(slo_ctx* ctx, bool first_scan) {
    DevView& v = ctx->v;
    const int S = ctx->S;
    SLO_LAUNCH(ctx, "fa_odo_begin", k_fa_odo_begin, dim3(S), dim3(256), 0, v, first_scan ? 1 : 0);
    if (!first_scan) {
        const int nbs = (v.cap_flat + 255) / 256, nbc = (v.cap_sharp + 255) / 256;
        for (int b = 0; b < 5; ++b) {
            SLO_LAUNCH(ctx, "fa_search_surf", k_fa_search<0>, dim3(xcd_grid(S, nbs)), dim3(256), 0, v, nbs);
            SLO_LAUNCH(ctx, "fa_iter_surf", k_fa_iter<0>, dim3(S), dim3(256), 0, v, 5 * b);
        }
        for (int b = 0; b < 5; ++b) {
            SLO_LAUNCH(ctx, "fa_search_corner", k_fa_search<1>, dim3(xcd_grid(S, nbc)), dim3(256), 0, v, nbc);
            SLO_LAUNCH(ctx, "fa_iter_corner", k_fa_iter<1>, dim3(S), dim3(256), 0, v, 5 * b);
        }
    }
    SLO_LAUNCH(ctx, "fa_to_end", k_fa_to_end, dim3(xcd_grid(S, SLO_TOEND_BLOCKS)), dim3(256), 0, v);
    SLO_LAUNCH(ctx, "fa_odo_finish", k_fa_odo_finish, dim3(S), dim3(64), 0, v);
    SLO_CHECK(hipGetLastError());
    // the clouds just written become *Last for the next scan
    std::swap(ctx->v.corner_last, ctx->v.corner_next);
    std::swap(ctx->v.surf_last, ctx->v.surf_next);
    // setInputCloud: hash grid over the (possibly unchanged) surf tree cloud
    // (the corner tree is searched by brute force, k_fa_search<1>)
    const int SS = (int)(sizeof(StreamState) / sizeof(int32_t));
    return grid_build(ctx, ctx->grid_os, v.kd_surf, v.cap_less_flat, &v.st->kdSurfNum, SS);
}

}  // namespace slo
