// slo_odom.hip — scan-to-scan odometry of featureAssociation.cpp for a batch
// of S streams: updateTransformation (FA:1666-1695) with the surf / corner
// correspondence searches (FA:1044-1268) and 3-DOF Gauss-Newton solvers
// (FA:1270-1478), integrateTransformation (FA:1697-1725) and
// publishCloudsLast (FA:1759-1788) / checkSystemInitialization (FA:1605-1637).
//
// One 256-thread workgroup owns one stream for the whole <=25+25 iteration
// loop (the iterations are sequential; the streams are independent), so no
// host round trip happens per iteration.  Per iteration every lane
// transforms its queries, (every 5th iteration) finds the exact nearest
// neighbour in a 1 m hash grid over the "kd-tree" cloud (rebuilt after every
// scan by fa_odometry_run, like setInputCloud), walks the ring-ordered target
// cloud for the 2nd/3rd points exactly as the reference (including Q7's
// bound), and accumulates its rows of A^T A / A^T b in double-double
// (slo_ddsum.h); a wave-shuffle + LDS tree reduces them and lane 0 rounds once
// to float and runs the 3x3 QR / Jacobi / degeneracy projection.
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

// exact 1-NN in the 1 m hash grid of the "tree" cloud: shells of cells at
// Chebyshev distance r = 0,1,..; every point outside shells <= r is more than
// r metres away, so once the best float distance is < r^2 nothing unseen can
// beat or tie it (fl(d) is monotone in the exact distance).  r stops at
// rmax = ceil(sqrt(nearestFeatureSearchSqDist)): anything further fails the
// gate anyway, as it would after the reference's exact FLANN search.
// Ties -> lowest index.
__device__ inline void nn1_grid(const float4* ent, const int32_t* off, const int32_t* cnt, int T, int s,
                                size_t es, int rmax, const P4& q, int& bi, float& bd) {
    bi = -1; bd = FLT_MAX;
    if (!(isfinite(q.x) && isfinite(q.y) && isfinite(q.z))) return;
    const int cx = (int)floorf(q.x), cy = (int)floorf(q.y), cz = (int)floorf(q.z);
    const int base = off[(size_t)s * T];
    const float4* E = ent + (size_t)s * es;
    for (int r = 0; r <= rmax; ++r) {
        for (int dz = -r; dz <= r; ++dz)
            for (int dy = -r; dy <= r; ++dy) {
                const bool edge = (dz == -r || dz == r || dy == -r || dy == r);
                for (int dx = -r; dx <= r; dx += (edge ? 1 : 2 * r > 0 ? 2 * r : 1)) {
                    const int tx = cx + dx, ty = cy + dy, tz = cz + dz;
                    const unsigned int b = grid_hash(tx, ty, tz, T);
                    const int st = off[(size_t)s * T + b] - base, m = cnt[(size_t)s * T + b];
                    for (int k = 0; k < m; ++k) {
                        const float4 p = E[st + k];
                        if ((int)floorf(p.x) != tx || (int)floorf(p.y) != ty || (int)floorf(p.z) != tz) continue;
                        const float d = sqdist_flann(q, p);
                        const int idx = __float_as_int(p.w);
                        if (d < bd || (d == bd && idx < bi)) { bd = d; bi = idx; }
                    }
                    if (r == 0) break;
                }
            }
        if (r >= 1 && bd < (float)(r * r)) break;
    }
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

__global__ void __launch_bounds__(256) k_fa_odometry(DevView v, int first_scan) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    const int tid = threadIdx.x, T = blockDim.x;
    const float4* sharp = v.sharp + (size_t)s * v.cap_sharp;
    const float4* flat = v.flat + (size_t)s * v.cap_flat;
    const float4* lsharp = v.less_sharp + (size_t)s * v.cap_less_sharp;
    const float4* lflat = v.less_flat + (size_t)s * v.cap_less_flat;
    float4* cnext = v.corner_next + (size_t)s * v.cap_less_sharp;
    float4* snext = v.surf_next + (size_t)s * v.cap_less_flat;
    float4* kdc = v.kd_corner + (size_t)s * v.cap_less_sharp;
    float4* kds = v.kd_surf + (size_t)s * v.cap_less_flat;
    const int nLS = st.n_less_sharp, nLF = st.n_less_flat;

    if (first_scan) {  // checkSystemInitialization: swap, build trees, no odometry
        for (int i = tid; i < nLS; i += T) { cnext[i] = lsharp[i]; kdc[i] = lsharp[i]; }
        for (int i = tid; i < nLF; i += T) { snext[i] = lflat[i]; kds[i] = lflat[i]; }
        if (tid == 0) {
            st.cornerLastNum = nLS; st.surfLastNum = nLF;
            st.kdCornerNum = nLS; st.kdSurfNum = nLF;
            st.iters_surf = st.iters_corner = 0;
        }
        return;
    }

    __shared__ float tc[6];
    __shared__ int s_ctl;      // 0 = go on, 1 = skip solve (continue), 2 = break
    __shared__ slo_dd::DD sh[4 * 9];
    __shared__ int shi[4];
    if (tid == 0) for (int k = 0; k < 6; ++k) tc[k] = st.transformCur[k];
    __syncthreads();
    const float4* clast = v.corner_last + (size_t)s * v.cap_less_sharp;
    const float4* slast = v.surf_last + (size_t)s * v.cap_less_flat;
    const int cornerLastNum = st.cornerLastNum, surfLastNum = st.surfLastNum;
    const float gate = v.cfg.nearest_feature_search_sq_dist;
    const int rmax = (int)ceilf(sqrtf(gate));
    int iters_surf = 0, iters_corner = 0;

    if (!(cornerLastNum < 10 || surfLastNum < 100)) {
        // ------------------------------------------------ surf phase
        const int nq = st.n_flat;
        int32_t* ind = v.ind_surf + (size_t)s * v.cap_flat * 3;
        for (int iterCount = 0; iterCount < 25; iterCount++) {
            slo_dd::DD acc[9];
            for (int k = 0; k < 9; ++k) acc[k] = slo_dd::zero();
            int cnt = 0;
            float srx = slo_libm::sinf_(tc[0]), crx = slo_libm::cosf_(tc[0]);
            float sry = slo_libm::sinf_(tc[1]), cry = slo_libm::cosf_(tc[1]);
            float srz = slo_libm::sinf_(tc[2]), crz = slo_libm::cosf_(tc[2]);
            float tx = tc[3], ty = tc[4], tz = tc[5];
            float a1 = crx * sry * srz; float a2 = crx * crz * sry; float a3 = srx * sry; float a4 = tx * a1 - ty * a2 - tz * a3;
            float a5 = srx * srz; float a6 = crz * srx; float a7 = ty * a6 - tz * crx - tx * a5;
            float a8 = crx * cry * srz; float a9 = crx * cry * crz; float a10 = cry * srx; float a11 = tz * a10 + ty * a9 - tx * a8;
            float b1 = -crz * sry - cry * srx * srz; float b2 = cry * crz * srx - sry * srz;
            float b5 = cry * crz - srx * sry * srz; float b6 = cry * srz + crz * srx * sry;
            float c1 = -b6; float c2 = b5; float c3 = tx * b6 - ty * b5; float c4 = -crx * crz; float c5 = crx * srz; float c6 = ty * c5 + tx * -c4;
            float c7 = b2; float c8 = -b1; float c9 = tx * -b2 - ty * -b1;
            const int rounds = (nq + T - 1) / T;
            for (int rd = 0; rd < rounds; ++rd) {
                const int i = rd * T + tid;
                const bool active = i < nq;
                P4 po = active ? ld4(flat, i) : P4{0, 0, 0, 0};
                P4 sel = slo_pose::transform_to_start(po, tc);
                if (iterCount % 5 == 0) {
                    int ci; float cd;
                    nn1_grid(v.gos_ent, v.gos_off, v.gos_cnt, v.Tos, s, v.cap_less_flat, rmax, sel, ci, cd);
                    int closest = -1, i2 = -1, i3 = -1;
                    if (active && cd < gate && ci >= 0 && ci < surfLastNum) {
                        closest = ci;
                        int cscan = (int)slast[closest].w;
                        float m2 = gate, m3 = gate;
                        for (int j = closest + 1; j < nq && j < surfLastNum; j++) {
                            if ((int)slast[j].w > cscan + 2.5) break;
                            float d = sq3_ref(slast[j], sel);
                            if ((int)slast[j].w <= cscan) { if (d < m2) { m2 = d; i2 = j; } }
                            else { if (d < m3) { m3 = d; i3 = j; } }
                        }
                        for (int j = closest - 1; j >= 0; j--) {
                            if ((int)slast[j].w < cscan - 2.5) break;
                            float d = sq3_ref(slast[j], sel);
                            if ((int)slast[j].w >= cscan) { if (d < m2) { m2 = d; i2 = j; } }
                            else { if (d < m3) { m3 = d; i3 = j; } }
                        }
                    }
                    if (active) { ind[3 * i] = closest; ind[3 * i + 1] = i2; ind[3 * i + 2] = i3; }
                }
                if (!active) continue;
                const int j1 = ind[3 * i], j2 = ind[3 * i + 1], j3 = ind[3 * i + 2];
                if (j2 >= 0 && j3 >= 0) {
                    float4 t1 = slast[j1], t2 = slast[j2], t3 = slast[j3];
                    float pa = (t2.y - t1.y) * (t3.z - t1.z) - (t3.y - t1.y) * (t2.z - t1.z);
                    float pb = (t2.z - t1.z) * (t3.x - t1.x) - (t3.z - t1.z) * (t2.x - t1.x);
                    float pc = (t2.x - t1.x) * (t3.y - t1.y) - (t3.x - t1.x) * (t2.y - t1.y);
                    float pd = -(pa * t1.x + pb * t1.y + pc * t1.z);
                    float ps = sqrtf(pa * pa + pb * pb + pc * pc);
                    pa /= ps; pb /= ps; pc /= ps; pd /= ps;
                    float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
                    float sw = 1;
                    if (iterCount >= 5)
                        sw = (float)(1 - 1.8 * fabsf(pd2) / sqrtf(sqrtf(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z)));
                    if (sw > 0.1 && pd2 != 0) {
                        float cx = sw * pa, cy = sw * pb, cz = sw * pc, cw = sw * pd2;
                        const P4& p = po;
                        float arx = (-a1 * p.x + a2 * p.y + a3 * p.z + a4) * cx + (a5 * p.x - a6 * p.y + crx * p.z + a7) * cy +
                                    (a8 * p.x - a9 * p.y - a10 * p.z + a11) * cz;
                        float arz = (c1 * p.x + c2 * p.y + c3) * cx + (c4 * p.x - c5 * p.y + c6) * cy + (c7 * p.x + c8 * p.y + c9) * cz;
                        float aty = -b6 * cx + c4 * cy + b2 * cz;
                        float bb = (float)(-0.05 * cw);
                        double A0 = arx, A1 = arz, A2 = aty, B = bb;
                        accumulate9(acc, A0, A1, A2, B);
                        cnt++;
                    }
                }
            }
            block_reduce<9>(acc, cnt, sh, shi);
            iters_surf = iterCount + 1;
            if (tid == 0) {
                s_ctl = 0;
                if (cnt < 10) s_ctl = 1;
                else {
                    float X[3];
                    solve_step(st, acc, iterCount, X);
                    tc[0] += X[0]; tc[2] += X[1]; tc[4] += X[2];
                    for (int k = 0; k < 6; k++) if (isnan(tc[k])) tc[k] = 0;
                    double r0 = X[0] * 180.0 / M_PI, r1 = X[1] * 180.0 / M_PI;
                    double t2 = (double)(X[2] * 100);
                    float deltaR = (float)sqrt(r0 * r0 + r1 * r1);
                    float deltaT = (float)sqrt(t2 * t2);
                    if (deltaR < 0.1 && deltaT < 0.1) s_ctl = 2;
                }
            }
            __syncthreads();
            if (s_ctl == 2) break;
        }
        // ------------------------------------------------ corner phase
        const int nc = st.n_sharp;
        int32_t* indc = v.ind_corner + (size_t)s * v.cap_sharp * 2;
        for (int iterCount = 0; iterCount < 25; iterCount++) {
            slo_dd::DD acc[9];
            for (int k = 0; k < 9; ++k) acc[k] = slo_dd::zero();
            int cnt = 0;
            float srx = slo_libm::sinf_(tc[0]), crx = slo_libm::cosf_(tc[0]);
            float sry = slo_libm::sinf_(tc[1]), cry = slo_libm::cosf_(tc[1]);
            float srz = slo_libm::sinf_(tc[2]), crz = slo_libm::cosf_(tc[2]);
            float tx = tc[3], ty = tc[4], tz = tc[5];
            float b1 = -crz * sry - cry * srx * srz; float b2 = cry * crz * srx - sry * srz; float b3 = crx * cry; float b4 = tx * -b1 + ty * -b2 + tz * b3;
            float b5 = cry * crz - srx * sry * srz; float b6 = cry * srz + crz * srx * sry; float b7 = crx * sry; float b8 = tz * b7 - ty * b6 - tx * b5;
            float c5 = crx * srz;
            const int rounds = (nc + T - 1) / T;
            for (int rd = 0; rd < rounds; ++rd) {
                const int i = rd * T + tid;
                const bool active = i < nc;
                P4 po = active ? ld4(sharp, i) : P4{0, 0, 0, 0};
                P4 sel = slo_pose::transform_to_start(po, tc);
                if (iterCount % 5 == 0) {
                    int ci; float cd;
                    nn1_grid(v.goc_ent, v.goc_off, v.goc_cnt, v.Toc, s, v.cap_less_sharp, rmax, sel, ci, cd);
                    int closest = -1, i2 = -1;
                    if (active && cd < gate && ci >= 0 && ci < cornerLastNum) {
                        closest = ci;
                        int cscan = (int)clast[closest].w;
                        float m2 = gate;
                        for (int j = closest + 1; j < nc && j < cornerLastNum; j++) {
                            if ((int)clast[j].w > cscan + 2.5) break;
                            float d = sq3_ref(clast[j], sel);
                            if ((int)clast[j].w > cscan) { if (d < m2) { m2 = d; i2 = j; } }
                        }
                        for (int j = closest - 1; j >= 0; j--) {
                            if ((int)clast[j].w < cscan - 2.5) break;
                            float d = sq3_ref(clast[j], sel);
                            if ((int)clast[j].w < cscan) { if (d < m2) { m2 = d; i2 = j; } }
                        }
                    }
                    if (active) { indc[2 * i] = closest; indc[2 * i + 1] = i2; }
                }
                if (!active) continue;
                const int j1 = indc[2 * i], j2 = indc[2 * i + 1];
                if (j2 >= 0) {
                    float4 t1 = clast[j1], t2 = clast[j2];
                    float x0 = sel.x, y0 = sel.y, z0 = sel.z;
                    float x1 = t1.x, y1 = t1.y, z1 = t1.z, x2 = t2.x, y2 = t2.y, z2 = t2.z;
                    float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
                    float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
                    float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
                    float a012 = sqrtf(m11 * m11 + m22 * m22 + m33 * m33);
                    float l12 = sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
                    float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
                    float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
                    float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
                    float ld2 = a012 / l12;
                    float sw = 1;
                    if (iterCount >= 5) sw = (float)(1 - 1.8 * fabsf(ld2));
                    if (sw > 0.1 && ld2 != 0) {
                        float cx = sw * la, cy = sw * lb, cz = sw * lc, cw = sw * ld2;
                        const P4& p = po;
                        float ary = (b1 * p.x + b2 * p.y - b3 * p.z + b4) * cx + (b5 * p.x + b6 * p.y - b7 * p.z + b8) * cz;
                        float atx = -b5 * cx + c5 * cy + b1 * cz;
                        float atz = b7 * cx - srx * cy - b3 * cz;
                        float bb = (float)(-0.05 * cw);
                        double A0 = ary, A1 = atx, A2 = atz, B = bb;
                        accumulate9(acc, A0, A1, A2, B);
                        cnt++;
                    }
                }
            }
            block_reduce<9>(acc, cnt, sh, shi);
            iters_corner = iterCount + 1;
            if (tid == 0) {
                s_ctl = 0;
                if (cnt < 10) s_ctl = 1;
                else {
                    float X[3];
                    solve_step(st, acc, iterCount, X);
                    tc[1] += X[0]; tc[3] += X[1]; tc[5] += X[2];
                    for (int k = 0; k < 6; k++) if (isnan(tc[k])) tc[k] = 0;
                    double r0 = X[0] * 180.0 / M_PI;
                    double t1 = (double)(X[1] * 100), t2 = (double)(X[2] * 100);
                    float deltaR = (float)sqrt(r0 * r0);
                    float deltaT = (float)sqrt(t1 * t1 + t2 * t2);
                    if (deltaR < 0.1 && deltaT < 0.1) s_ctl = 2;
                }
            }
            __syncthreads();
            if (s_ctl == 2) break;
        }
    }
    if (tid == 0) {
        for (int k = 0; k < 6; ++k) st.transformCur[k] = tc[k];
        slo_pose::integrate(st.transformSum, tc);
        st.iters_surf = iters_surf;
        st.iters_corner = iters_corner;
    }
    __syncthreads();
    // publishCloudsLast: TransformToEnd into the next *Last buffers
    for (int i = tid; i < nLS; i += T) {
        P4 q = slo_pose::transform_to_end(ld4(lsharp, i), tc);
        cnext[i] = make_float4(q.x, q.y, q.z, q.w);
    }
    for (int i = tid; i < nLF; i += T) {
        P4 q = slo_pose::transform_to_end(ld4(lflat, i), tc);
        snext[i] = make_float4(q.x, q.y, q.z, q.w);
    }
    __syncthreads();
    const bool rebuild = nLS > 10 && nLF > 100;
    if (rebuild) {
        for (int i = tid; i < nLS; i += T) kdc[i] = cnext[i];
        for (int i = tid; i < nLF; i += T) kds[i] = snext[i];
    }
    if (tid == 0) {
        st.cornerLastNum = nLS;
        st.surfLastNum = nLF;
        if (rebuild) { st.kdCornerNum = nLS; st.kdSurfNum = nLF; }
    }
}

int fa_odometry_run(slo_ctx* ctx, bool first_scan) {
    DevView& v = ctx->v;
    SLO_LAUNCH(ctx, "fa_odometry", k_fa_odometry, dim3(ctx->S), dim3(256), 0, v, first_scan ? 1 : 0);
    SLO_CHECK(hipGetLastError());
    // the clouds just written become *Last for the next scan
    std::swap(ctx->v.corner_last, ctx->v.corner_next);
    std::swap(ctx->v.surf_last, ctx->v.surf_next);
    // setInputCloud: hash grids over the (possibly unchanged) tree clouds
    const int SS = (int)(sizeof(StreamState) / sizeof(int32_t));
    int r = grid_build(ctx, ctx->grid_oc, v.kd_corner, v.cap_less_sharp, &v.st->kdCornerNum, SS);
    if (r) return r;
    return grid_build(ctx, ctx->grid_os, v.kd_surf, v.cap_less_flat, &v.st->kdSurfNum, SS);
}

}  // namespace slo
