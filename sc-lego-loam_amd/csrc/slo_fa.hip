// slo_fa.hip — feature extraction (featureAssociation.cpp:491-784) for a
// batch of S streams.
//
//   adjustDistortion (FA:491-619): the one-way halfPassed latch is a prefix
//     OR, so pass 1 finds the first point whose pre-half orientation passes
//     start+pi (wave-reduced atomicMin) and pass 2 deskews every point.
//   calculateSmoothness + markOccludedPoints (FA:621-678): one thread per
//     position in gather form — each position ORs in every occlusion mark
//     that covers it, so there is no write race and the reset-then-mark order
//     of the reference is kept.  Positions outside [5, S-5) keep the stale
//     values persisted from earlier scans (Appendix A Q5).
//   extractFeatures (FA:680-784): rings are independent except through the
//     stale cloudSmoothness[4] entry of ring 0 (Q5); when that entry points
//     outside ring 0, ring 0 runs first (k_fa_extract_stale), and the rings
//     run in parallel, staged in LDS (k_fa_sort: wave
//     bitonic sorts, with the exact libstdc++ introsort restatement for
//     sectors holding ties, Q4/Q6; k_fa_pick: the greedy picks, sequential
//     per ring as in the reference).
//   per-ring VoxelGrid(0.2) (FA:778-782): one block per ring, bitonic sort
//     of (voxel idx, position) keys in LDS, centroid of each voxel summed in
//     position order (DESIGN.md "VoxelGrid order").
#include "slo_internal.h"
#include "slo_pclsort.h"
#include "slo_libm.h"
#include "slo_introsort.h"
#include "slo_imu.h"
#include <float.h>

namespace slo {

__device__ inline int wave_min_fa(int x) {
    for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
    return x;
}

// orientation of point i under the "not yet half passed" branch (FA:504-512)
__device__ inline float ori_first_half(float ori, float start) {
    if (ori < start - M_PI / 2) ori = (float)(ori + 2 * M_PI);
    else if (ori > start + M_PI * 3 / 2) ori = (float)(ori - 2 * M_PI);
    return ori;
}

__global__ void k_fa_halfpass(DevView v) {
    const int s = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int S = v.st[s].seg_count;
    int hit = INT_MAX;
    if (i < S) {
        float4 q = v.seg[(size_t)s * v.H + i];
        const float start = v.orient[3 * s];
        float ori = ori_first_half(-slo_libm::atan2f_(q.y, q.x), start);
        if (ori - start > M_PI) hit = i;
    }
    hit = wave_min_fa(hit);
    if ((threadIdx.x & 63) == 0 && hit != INT_MAX) atomicMin(&v.st[s].first_half, hit);
}

// adjustDistortion's IMU state for the scan (FA:525-616), one lane per
// stream: the first point's IMU values become the scan's start (rpy,
// velocity; the angular rotation since the last scan), and the ring position
// the deskew starts from is latched before imuPointerLastIteration moves on
// (FA:616).  The other points are deskewed in k_fa_points.
__global__ void k_fa_imu_start(DevView v) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    ImuState& m = v.imu[s];
    m.iter_scan = m.last_iter;
    if (m.last >= 0 && v.st[s].seg_count > 0) {
        const float4 q = v.seg[(size_t)s * v.H];
        const float start = v.orient[3 * s], diff = v.orient[3 * s + 2];
        const float ori = ori_first_half(-slo_libm::atan2f_(q.y, q.x), start);   // point 0: first half
        const float relTime = (ori - start) / diff;
        const float pointTime = relTime * v.cfg.scan_period;
        const slo_imu::ImuAt c = slo_imu::imu_at(m, m.iter_scan, v.io->t_scan, pointTime);
        m.rollStart = m.rollCur = c.roll;
        m.pitchStart = m.pitchCur = c.pitch;
        m.yawStart = m.yawCur = c.yaw;
        for (int k = 0; k < 3; ++k) {
            m.veloStart[k] = c.velo[k];
            m.angFromStart[k] = c.ang[k] - m.angLast[k];
            m.angLast[k] = c.ang[k];
        }
    }
    m.last_iter = m.last;
}

// deskew + curvature + occlusion marks, one thread per position
__global__ void __launch_bounds__(256) k_fa_points(DevView v) {
    const int s = blockIdx.y;
    const int p0 = blockIdx.x * 256, p = p0 + threadIdx.x;
    const int S = v.st[s].seg_count;
    if (p0 >= S) return;
    const size_t base = (size_t)s * v.H;
    // the block's ranges and columns with a 6-point halo each side, staged in
    // LDS (coalesced): the smoothness and occlusion windows read them there
    __shared__ float lr[256 + 12];
    __shared__ uint32_t lcol[256 + 12];
    for (int k = threadIdx.x; k < 256 + 12; k += 256) {
        const int i = p0 - 6 + k;
        if (i >= 0 && i < S) { lr[k] = v.seg_range[base + i]; lcol[k] = v.seg_col[base + i]; }
    }
    __syncthreads();
    if (p >= S) return;
    // ---- adjustDistortion (non-IMU)
    {
        float4 q = v.seg[base + p];
        const float start = v.orient[3 * s], end = v.orient[3 * s + 1], diff = v.orient[3 * s + 2];
        float px = q.y, py = q.z, pz = q.x;
        float ori = -slo_libm::atan2f_(px, pz);
        if (p <= v.st[s].first_half) {
            ori = ori_first_half(ori, start);
        } else {
            ori = (float)(ori + 2 * M_PI);
            if (ori < end - M_PI * 3 / 2) ori = (float)(ori + 2 * M_PI);
            else if (ori > end + M_PI / 2) ori = (float)(ori - 2 * M_PI);
        }
        float relTime = (ori - start) / diff;
        const float intensity = (float)(int)q.w + v.cfg.scan_period * relTime;
        ImuState& m = v.imu[s];
        if (m.last >= 0 && p > 0) {   // VeloToStartIMU + TransformToStartIMU (FA:609-612)
            const float pointTime = relTime * v.cfg.scan_period;
            const slo_imu::ImuAt c = slo_imu::imu_at(m, m.iter_scan, v.io->t_scan, pointTime);
            const slo_imu::ImuStartTrig t = slo_imu::start_trig(m.rollStart, m.pitchStart, m.yawStart);
            if (p == S - 1) {   // the imu*Cur the scan leaves behind (updateInitialGuess reads them)
                slo_imu::imu_velo_to_start(c.velo, m.veloStart, t, m.veloFromStartCur);
                m.rollCur = c.roll;
                m.pitchCur = c.pitch;
                m.yawCur = c.yaw;
            }
            slo_imu::imu_to_start(px, py, pz, c, t);
        }
        v.fpts[base + p] = make_float4(px, py, pz, intensity);
    }
    auto r = [&](int i) { return lr[6 - p0 + i]; };      // seg_range[i], i in [p0 - 6, p0 + 262)
    auto col = [&](int i) { return lcol[6 - p0 + i]; };  // seg_col[i]
    // ---- calculateSmoothness
    const bool inner = p >= 5 && p < S - 5;
    if (inner) {
        float d = r(p - 5) + r(p - 4) + r(p - 3) + r(p - 2) + r(p - 1) - r(p) * 10 + r(p + 1) + r(p + 2) +
                  r(p + 3) + r(p + 4) + r(p + 5);
        float c = d * d;
        v.curv[base + p] = c;
        v.clabel[base + p] = 0;
        v.smooth[base + p] = Smooth{c, p};
    }
    // ---- markOccludedPoints (gather form); marks come from i in [5, S-7]
    int pk = inner ? 0 : v.picked[base + p];
    const int ilo = 5, ihi = S - 7;
    for (int i = max(ilo, p); i <= min(ihi, p + 5) && !pk; ++i) {  // case A marks [i-5, i]
        int cd = abs((int)(col(i + 1) - col(i)));
        if (cd < 10 && r(i) - r(i + 1) > 0.3) pk = 1;
    }
    for (int i = max(ilo, p - 6); i <= min(ihi, p - 1) && !pk; ++i) {  // case B marks [i+1, i+6]
        int cd = abs((int)(col(i + 1) - col(i)));
        if (cd < 10 && !(r(i) - r(i + 1) > 0.3) && r(i + 1) - r(i) > 0.3) pk = 1;
    }
    if (!pk && p >= ilo && p <= ihi) {
        float diff1 = fabsf((float)(r(p - 1) - r(p)));
        float diff2 = fabsf((float)(r(p + 1) - r(p)));
        if (diff1 > 0.02 * r(p) && diff2 > 0.02 * r(p)) pk = 1;
    }
    v.picked[base + p] = pk;
}

struct SmoothLess {
    __device__ bool operator()(const Smooth& a, const Smooth& b) const { return a.value < b.value; }
};

__device__ inline uint32_t col_at(const uint32_t* col, int k) { return k < 0 ? 0u : col[k]; }

__device__ inline void mark_neighbors(int32_t* picked, const uint32_t* col, int ind) {
    for (int l = 1; l <= 5; l++) {
        if (abs((int)(col_at(col, ind + l) - col_at(col, ind + l - 1))) > 10) break;
        picked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; l--) {
        if (abs((int)(col_at(col, ind + l) - col_at(col, ind + l + 1))) > 10) break;
        if (ind + l >= 0) picked[ind + l] = 1;
    }
}

// ---------------------------------------------------------------- extractFeatures (FA:680-784)
// Sector bounds of ring [rs, re] (FA:693-696).
__device__ inline int sec_sp(int rs, int re, int j) { return (rs * (6 - j) + re * j) / 6; }
__device__ inline int sec_ep(int rs, int re, int j) { return (rs * (5 - j) + re * (j + 1)) / 6 - 1; }

// The restatement on global memory, for ring 0 (its sector 0 starts at the
// stale cloudSmoothness[4] entry, whose index can point anywhere, Q5 — which is
// why ring 0 runs alone, first) and for rings too long to stage.  Lanes 0..5
// sort the six sectors with the libstdc++ introsort restatement (Q4/Q6), lane 0
// picks.  Every thread of the block must call it.
__device__ void extract_ring_global(const DevView& v, int s, int ring) {
    const int R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    const size_t base = (size_t)s * v.H;
    const int S = v.st[s].seg_count;
    const int* se = v.ring_se + (size_t)s * R * 2;
    const int rs = se[2 * ring], re = se[2 * ring + 1];
    Smooth* sm = v.smooth + base;
    const int tid = threadIdx.x;
    if (tid < 6) {
        const int sp = sec_sp(rs, re, tid), ep = sec_ep(rs, re, tid);
        if (sp < ep) slo_sort::std_sort_small(sm + sp, ep - sp, SmoothLess());
    }
    __syncthreads();
    if (tid != 0) return;
    int32_t* picked = v.picked + base;
    int32_t* lab = v.clabel + base;
    const float* curv = v.curv + base;
    const uint8_t* gflag = v.seg_ground + base;
    const uint32_t* col = v.seg_col + base;
    const float4* fp = v.fpts + base;
    const size_t rr = (size_t)s * R + ring;
    float4* o_sharp = v.r_sharp + rr * 12;
    float4* o_lsharp = v.r_less_sharp + rr * 120;
    float4* o_flat = v.r_flat + rr * 24;
    float4* o_lf = v.r_lf_scan + rr * C;
    int n_sharp = 0, n_lsharp = 0, n_flat = 0, n_lf = 0;
    for (int j = 0; j < 6; j++) {
        const int sp = sec_sp(rs, re, j), ep = sec_ep(rs, re, j);
        if (sp >= ep) continue;
        int largestPickedNum = 0;
        for (int k = ep; k >= sp; k--) {
            const int ind = sm[k].ind;
            if (ind >= S) continue;
            if (picked[ind] == 0 && curv[ind] > v.cfg.edge_threshold && gflag[ind] == 0) {
                largestPickedNum++;
                if (largestPickedNum <= 2) {
                    lab[ind] = 2;
                    o_sharp[n_sharp++] = fp[ind];
                    o_lsharp[n_lsharp++] = fp[ind];
                } else if (largestPickedNum <= 20) {
                    lab[ind] = 1;
                    o_lsharp[n_lsharp++] = fp[ind];
                } else {
                    break;
                }
                picked[ind] = 1;
                mark_neighbors(picked, col, ind);
            }
        }
        int smallestPickedNum = 0;
        for (int k = sp; k <= ep; k++) {
            const int ind = sm[k].ind;
            if (ind >= S) continue;
            if (picked[ind] == 0 && curv[ind] < v.cfg.surf_threshold && gflag[ind] == 1) {
                lab[ind] = -1;
                o_flat[n_flat++] = fp[ind];
                smallestPickedNum++;
                if (smallestPickedNum >= 4) break;
                picked[ind] = 1;
                mark_neighbors(picked, col, ind);
            }
        }
        for (int k = sp; k <= ep; k++)
            if (lab[k] <= 0 && n_lf < C) o_lf[n_lf++] = fp[k];
    }
    int* rc = v.ring_cnt + rr * 4;
    rc[0] = n_sharp; rc[1] = n_lsharp; rc[2] = n_flat;
    v.r_lf_n[rr] = n_lf;
}

#define SLO_RING_STAGE 2080
#ifndef SLO_SORT_LCV
#define SLO_SORT_LCV 0   // 1: k_fa_sort stages the window's curvature in LDS too (27 KB: five workgroups per CU against eight;
#endif                   // the kernel alone the same, C3 live +0.6 % and +1.8 % in two A/B pairs with 0, r05)

// A ring's sorts, picks and marks stay inside its window [rs-5, re+5) when
// every entry of its sectors is one of its own points.  That holds for every
// ring with rs >= 5 (entries at positions >= 5 are this scan's, ind =
// position), and for the ring holding the stale cloudSmoothness[4] entry (the
// first ring with points, rs = 4, Q5) when that entry's index is one of the
// ring's own points — the usual case: it was left there by the previous
// scan's sort of the same ring.  Such rings run in parallel in LDS (k_fa_sort,
// k_fa_pick) if the window fits SLO_RING_STAGE.
__device__ inline bool ring_window(const DevView& v, int s, int ring, int& rs, int& re, int& lo, int& hi) {
    const int* se = v.ring_se + (size_t)s * v.cfg.n_scan * 2;
    rs = se[2 * ring]; re = se[2 * ring + 1];
    lo = max(0, rs - 5); hi = min(v.H, re + 5);
    if (!(hi > lo && hi - lo <= SLO_RING_STAGE)) return false;
    if (rs >= 5) return true;
    // its marks (+-5) must stay in the window too; below position 0 they are
    // dropped (lo == 0 for the first ring).  The entry is usually {0, 0}: the
    // zero-initialised array's entry 4 sorts first forever (curvature 0).
    const int i4 = v.smooth[(size_t)s * v.H + 4].ind;
    return i4 >= 0 && (i4 - 5 >= lo || lo == 0) && i4 + 5 < hi && i4 < v.st[s].seg_count;
}

// The rings whose sectors may start at the stale entry 4 (rs < 5: the empty
// leading rings and the first ring with points), in ring order with the
// global-memory restatement — unless ring_window keeps the stale ring local,
// then k_fa_sort / k_fa_pick take it with the others.  Runs before them: a
// stale index can point into any ring.
__global__ void __launch_bounds__(256) k_fa_extract_stale(DevView v) {
    const int s = blockIdx.y, R = v.cfg.n_scan;
    const int* se = v.ring_se + (size_t)s * R * 2;
    for (int ring = 0; ring < R && se[2 * ring] < 5; ++ring) {
        int rs, re, lo, hi;
        if (ring_window(v, s, ring, rs, re, lo, hi)) break;
        extract_ring_global(v, s, ring);
        __syncthreads();
    }
}

// One wave sorts one sector of n <= 64*NE entries in registers (bitonic
// network over unique keys; padding keys are all-ones).
__device__ inline unsigned int f2ord_fa(float f) {
    const unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float ord2f_fa(unsigned int o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// Sorts a[0, n) of one sector by curvature in registers.  Keys are
// (curvature, not-a-candidate, index): equal curvatures are std::sort's only
// freedom, and their order is observable only through the pick lists, i.e.
// between two candidates of the same list (cand(ind): the point is in the
// sector's sharp or flat list — for one curvature value all candidates are in
// the same list).  So candidates come first inside a group of equal
// curvatures, and when a group holds two of them the sector is flagged for
// the exact introsort; otherwise the result is written back (its order of
// non-candidates inside a group is never read) — except the
// first entry of the sector that starts at position 4 (first_exact): it
// becomes the next scan's stale entry (Q5), so a tie for it falls back too.
template <int NE, class Cand>
__device__ inline void bitonic_sort_wave(Smooth* a, int n, int lane, int* tie_flag, Cand&& cand, bool first_exact) {
    unsigned long long k[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        const int i = e * 64 + lane;
        k[e] = ~0ull;
        if (i < n) {
            const Smooth x = a[i];
            k[e] = ((unsigned long long)f2ord_fa(x.value) << 32) | (cand(x.ind) ? 0u : 0x80000000u) |
                   (unsigned int)x.ind;
        }
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
                    const int p = e * 64 + lane;
                    const bool up = (p & size) == 0;
                    const unsigned long long x = k[e], y = k[e | es];
                    const bool sw = up ? (x > y) : (x < y);
                    k[e] = sw ? y : x;
                    k[e | es] = sw ? x : y;
                }
            } else {              // partner in lane ^ stride
#pragma unroll
                for (int e = 0; e < NE; ++e) {
                    const int p = e * 64 + lane;
                    const unsigned long long y = __shfl_xor(k[e], stride, 64);
                    const bool up = (p & size) == 0;
                    const bool lower = (lane & stride) == 0;
                    // the lower position keeps the min when ascending
                    const bool take_min = (up == lower);
                    k[e] = take_min ? (k[e] < y ? k[e] : y) : (k[e] > y ? k[e] : y);
                }
            }
        }
    }
    // ties that matter: two candidates of equal curvature, adjacent
    bool tie = false;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        const int p = e * 64 + lane;
        const unsigned long long up1 = __shfl_up(k[e], 1, 64);                      // lane - 1
        const unsigned long long wrap = e > 0 ? __shfl(k[e > 0 ? e - 1 : 0], 63, 64) : ~0ull;   // all lanes
        const unsigned long long prev = lane == 0 ? wrap : up1;
        if (p > 0 && p < n && (prev >> 32) == (k[e] >> 32) &&
            ((!(prev & 0x80000000ull) && !(k[e] & 0x80000000ull)) || (first_exact && p == 1)))
            tie = true;
    }
    const bool any_tie = __any(tie);
    if (!any_tie) {
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int p = e * 64 + lane;
            if (p < n) a[p] = Smooth{ord2f_fa((unsigned int)(k[e] >> 32)), (int)((unsigned int)k[e] & 0x7fffffffu)};
        }
    } else if (lane == 0) {
        *tie_flag = 1;
    }
}

// The rings ring_window keeps local (ring = blockIdx.x), in two launches.
// Both kernels stage the ring's window in LDS in compact form, work on it
// with plain LDS accesses and write it back; concurrent rings never share a
// word.  The other rings are the stale ones k_fa_extract_stale has done and
// rings whose window exceeds SLO_RING_STAGE, which take the global-memory
// restatement (extract_ring_global) inside k_fa_pick.
//
// k_fa_sort (256 threads): the six sector sorts (std::sort on [sp, ep),
// Q4/Q6).  Without equal curvatures a sort's result is unique, so a wave
// bitonic-sorts each sector in registers; only a sector holding a tie is
// sorted by a wave with the exact libstdc++ introsort restatement
// (slo_pclsort.h wave_sort), whose order of equal keys is the reference's.  Then the
// pick eligibility that picks cannot change (curvature, ground flag) is
// evaluated by all lanes and compacted into per-sector candidate lists in
// visiting order (sharp ep..sp, flat sp..ep), stored for k_fa_pick.
//
// k_fa_pick (one wave): the greedy picks (FA:701-766) walk only those lists,
// 64 candidates per round, one pick per round (see the loop) — a small LDS
// footprint so many rings share each CU — then all lanes gather the
// points and collect the less-flat points (label <= 0, FA:768-776) with a
// wave ballot: a sector's picks only label that sector's own points, so
// collecting after all six sectors equals the reference's interleaving.

// A tie sector is sorted by a whole wave with slo_pclsort.h's exact std::sort
// restatement (wave_sort: the same introsort steps, partitions taken
// lane-parallel) on (curvature order key << 32 | index) items in place of the
// sector's entries — SmoothLess compares the curvature alone, as the PCL
// sort's items compare their high words.  (Round 6: one lane ran
// slo_sort::std_sort_small on it while the workgroup waited — 193 us per
// launch on one stream, 62 with the wave; C3's fa_sort 10.5 -> 6.5 ms per
// instrumented pass at 29.5 KB of LDS against 18.7.)
__global__ void __launch_bounds__(256) k_fa_sort(DevView v) {
    const int s = blockIdx.y;
    const int ring = blockIdx.x;
    const int R = v.cfg.n_scan;
    int rs, re, lo, hi;
    const bool local = ring_window(v, s, ring, rs, re, lo, hi);
    // the decision for k_fa_pick (which must not re-evaluate it: this kernel
    // rewrites the stale entry 4)
    int* cnt = v.ex_cnt + ((size_t)s * R + ring) * SLO_EX_CNT;
    if (threadIdx.x == 0) cnt[12] = local;
    if (!local) return;   // uniform
    const size_t base = (size_t)s * v.H;
    const int S = v.st[s].seg_count;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    Smooth* sm = v.smooth + base;
    __shared__ Smooth lsm[SLO_RING_STAGE];   // (alignas(8): also the wave tie sort's u64 items)
#if SLO_SORT_LCV
    __shared__ float lcv[SLO_RING_STAGE];
#define SORT_CV(ind) lcv[(ind) - lo]
#else
    const float* gcv = v.curv + base;   // the list predicates read curvature from L2: 27 -> 19 KB of LDS
#define SORT_CV(ind) gcv[ind]
#endif
    __shared__ uint8_t lgf[SLO_RING_STAGE];
    __shared__ int s_tie[6];
#if SLO_DIAG
    unsigned long long t_d = clock64();
#define SORT_STAMP(k) if (tid == 0) { const unsigned long long t_n = clock64(); atomicAdd(&v.st[s].dbg[k], t_n - t_d); t_d = t_n; }
#else
#define SORT_STAMP(k)
#endif
    for (int k = tid; k < hi - lo; k += blockDim.x) {
        lsm[k] = sm[lo + k];
#if SLO_SORT_LCV
        lcv[k] = v.curv[base + lo + k];
#endif
        lgf[k] = v.seg_ground[base + lo + k];
    }
    if (tid < 6) s_tie[tid] = 0;
    __syncthreads();
    SORT_STAMP(0)
    // ---- sector sorts: two rounds of (up to) four sectors, one wave each
    for (int r0 = 0; r0 < 6; r0 += 4) {
        const int j = r0 + wave;
        if (j < 6) {
            const int sp = sec_sp(rs, re, j), n = sec_ep(rs, re, j) - sp;
            Smooth* a = &lsm[sp - lo];
            // the list predicates of the candidate pass below (FA:704-705, 737-738)
            auto cand = [&](int ind) __attribute__((always_inline)) {
                const float c = SORT_CV(ind);
                const int g = lgf[ind - lo];
                return ind < S && ((c > v.cfg.edge_threshold && g == 0) || (c < v.cfg.surf_threshold && g == 1));
            };
            switch ((n + 63) >> 6) {
                case 0: break;
                case 1: if (n > 1) bitonic_sort_wave<1>(a, n, lane, &s_tie[j], cand, sp < 5); break;
                case 2: bitonic_sort_wave<2>(a, n, lane, &s_tie[j], cand, sp < 5); break;
                case 3: case 4: bitonic_sort_wave<4>(a, n, lane, &s_tie[j], cand, sp < 5); break;
                case 5: case 6: case 7: case 8: bitonic_sort_wave<8>(a, n, lane, &s_tie[j], cand, sp < 5); break;
                default: if (lane == 0) s_tie[j] = 1; break;
            }
        }
    }
    __syncthreads();
    SORT_STAMP(1)
    {   // ties (or a long sector): the exact sort, a wave each
        constexpr int kTieMax = 2048;   // the wave path's longest sector
        __shared__ unsigned short ttbl[4][kTieMax / 2 + 1];
        __shared__ slo_pcl::WaveSmem tws[4];
        __shared__ int s_terr;
        if (tid == 0) s_terr = 0;
        __syncthreads();
        for (int j = wave; j < 6; j += 4) {
            if (!s_tie[j]) continue;   // (uniform in the wave)
            const int sp = sec_sp(rs, re, j), n = sec_ep(rs, re, j) - sp;
            if (n > kTieMax) {
                if (lane == 0) slo_sort::std_sort_small(&lsm[sp - lo], n, SmoothLess());
                continue;
            }
            // each lane turns its own entries into items and back: no entry moves between the two
            slo_pcl::u64* it = reinterpret_cast<slo_pcl::u64*>(&lsm[sp - lo]);
            for (int k = lane; k < n; k += 64) {
                const Smooth x = lsm[sp - lo + k];
                it[k] = ((slo_pcl::u64)f2ord_fa(x.value) << 32) | (unsigned int)x.ind;
            }
            slo_pcl::wave_fence();
            slo_pcl::wave_sort<64>(it, n, 2 * slo_pcl::lg2(n), ttbl[wave], tws[wave], &s_terr);
            slo_pcl::wave_fence();
            for (int k = lane; k < n; k += 64) {
                const slo_pcl::u64 q = it[k];
                lsm[sp - lo + k] = Smooth{ord2f_fa((unsigned int)(q >> 32)), (int)(unsigned int)q};
            }
        }
        __syncthreads();
        if (tid == 0 && s_terr) atomicOr(&v.st[s].err, SLO_ERR_SORT);
    }
    SORT_STAMP(2)
    // ---- candidate lists: point indices as window offsets, in visiting order
    int16_t* l_sh = v.ex_list + (size_t)s * v.H * 2;
    int16_t* l_fl = l_sh + v.H;
    for (int r0 = 0; r0 < 6; r0 += 4) {
        const int j = r0 + wave;
        if (j >= 6) continue;
        const int sp = sec_sp(rs, re, j), ep = sec_ep(rs, re, j);
        int ns = 0, nf = 0;
        if (sp < ep)
            for (int kb = 0; kb <= ep - sp; kb += 64) {
                const int ks = ep - kb - lane, kf = sp + kb + lane;
                bool es = false, ef = false;
                int is = 0, iff = 0;
                if (ks >= sp) {
                    is = lsm[ks - lo].ind;
                    es = is < S && SORT_CV(is) > v.cfg.edge_threshold && lgf[is - lo] == 0;
                }
                if (kf <= ep) {
                    iff = lsm[kf - lo].ind;
                    ef = iff < S && SORT_CV(iff) < v.cfg.surf_threshold && lgf[iff - lo] == 1;
                }
                const unsigned long long ms = __ballot(es), mf = __ballot(ef);
                const unsigned long long below = (1ull << lane) - 1;
                if (es) l_sh[sp + ns + __popcll(ms & below)] = (int16_t)(is - lo);
                if (ef) l_fl[sp + nf + __popcll(mf & below)] = (int16_t)(iff - lo);
                ns += __popcll(ms);
                nf += __popcll(mf);
            }
        if (lane == 0) { cnt[2 * j] = ns; cnt[2 * j + 1] = nf; }
    }
    SORT_STAMP(3)
    for (int k = tid; k < hi - lo; k += blockDim.x) sm[lo + k] = lsm[k];
#if SLO_DIAG
    if (tid < 6 && s_tie[tid]) atomicAdd(&v.st[s].dbg[5], 1ull);
#endif
    SORT_STAMP(4)
#undef SORT_STAMP
#undef SORT_CV
}

__global__ void __launch_bounds__(64) k_fa_pick(DevView v) {
    const int s = blockIdx.y;
    const int ring = blockIdx.x;
    const int R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    const int* cnt = v.ex_cnt + ((size_t)s * R + ring) * SLO_EX_CNT;
    int rs, re, lo, hi;
    ring_window(v, s, ring, rs, re, lo, hi);   // bounds only; the decision is k_fa_sort's
    if (!cnt[12]) {   // uniform per block
        if (rs >= 5) extract_ring_global(v, s, ring);   // too long to stage (rs < 5: done, k_fa_extract_stale)
        return;
    }
    const size_t base = (size_t)s * v.H;
    const int lane = threadIdx.x;
    int32_t* picked = v.picked + base;
    int32_t* lab = v.clabel + base;
    const float4* fp = v.fpts + base;
    __shared__ uint16_t lcol[SLO_RING_STAGE];
    __shared__ int8_t lpk[SLO_RING_STAGE], llab[SLO_RING_STAGE];
    __shared__ int p_sh[12], p_ls[120], p_fl[24];
    const int16_t* g_sh = v.ex_list + (size_t)s * v.H * 2;
    const int16_t* g_fl = g_sh + v.H;
    const int nw = hi - lo;
    for (int k0 = 0; k0 < nw; k0 += 8 * 64) {   // eight points per lane loaded before they are staged
        int a[8], b[8];
        uint32_t c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int k = min(k0 + u * 64 + lane, nw - 1);
            a[u] = picked[lo + k];
            b[u] = lab[lo + k];
            c[u] = v.seg_col[base + lo + k];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int k = k0 + u * 64 + lane;
            if (k < nw) { lpk[k] = (int8_t)a[u]; llab[k] = (int8_t)b[u]; lcol[k] = (uint16_t)c[u]; }
        }
    }
    __syncthreads();
    // FA:719-731 / 752-764 on lanes 1..10: lanes 1..5 test the column gaps
    // forward, 6..10 backward; a neighbour is marked when every gap up to it
    // passes (the reference's walk breaks at the first failing gap).
    // colInd[-1] reads 0 (Q5).
    auto mark = [&](int ind) __attribute__((always_inline)) {
        auto col = [&](int i) __attribute__((always_inline)) { return i < 0 ? 0 : (int)lcol[max(i, lo) - lo]; };
        const int l = lane <= 5 ? lane : lane - 5;
        const bool fwd = lane >= 1 && lane <= 5, bwd = lane >= 6 && lane <= 10;
        const int tgt = fwd ? ind + l : ind - l;
        bool ok = false;
        if (fwd) ok = abs(col(ind + l) - col(ind + l - 1)) <= 10;
        else if (bwd) ok = abs(col(ind - l) - col(ind - l + 1)) <= 10;
        const unsigned long long m = __ballot(ok);
        const unsigned int need = (1u << l) - 1;
        if (fwd && (((unsigned int)(m >> 1) & need) == need)) lpk[tgt - lo] = 1;
        if (bwd && (((unsigned int)(m >> 6) & need) == need) && tgt >= 0) lpk[tgt - lo] = 1;
    };
    // Greedy picks (FA:701-766), one wave per ring.  The candidates of a list
    // are taken 64 at a time; each round the first one still unpicked is the
    // one the serial walk picks next (every earlier one is already marked, and
    // marks only accumulate), so the rounds = picks, not candidates.
    int n_sharp = 0, n_lsharp = 0, n_flat = 0;
    for (int j = 0; j < 6; j++) {
        const int sp = sec_sp(rs, re, j), ep = sec_ep(rs, re, j);
        if (sp >= ep) continue;
        for (int phase = 0; phase < 2; ++phase) {   // sharp, then flat
            const int n = cnt[2 * j + phase];
            const int16_t* list = (phase == 0 ? g_sh : g_fl) + sp;
            int npk = 0;
            bool done = false;
            for (int c0 = 0; c0 < n && !done; c0 += 64) {
                const int myind = c0 + lane < n ? lo + list[c0 + lane] : -1;
                int cur = 0;
                while (true) {
                    const bool ok = lane >= cur && myind >= 0 && lpk[myind - lo] == 0;
                    const unsigned long long m = __ballot(ok);
                    if (!m) break;
                    const int f = __ffsll((long long)m) - 1;
                    const int ind = __shfl(myind, f, 64);
                    cur = f + 1;
                    ++npk;
                    if (phase == 0) {
                        if (npk > 20) { done = true; break; }
                        if (lane == 0) {
                            llab[ind - lo] = npk <= 2 ? 2 : 1;
                            if (npk <= 2) p_sh[n_sharp] = ind;
                            p_ls[n_lsharp] = ind;
                        }
                        n_sharp += npk <= 2;
                        ++n_lsharp;
                    } else {
                        if (lane == 0) { llab[ind - lo] = -1; p_fl[n_flat] = ind; }
                        ++n_flat;
                        if (npk >= 4) { done = true; break; }
                    }
                    if (lane == 0) lpk[ind - lo] = 1;
                    mark(ind);
                    __syncthreads();   // one wave: orders this round's LDS writes before the next reads
                }
            }
        }
    }
    __syncthreads();
    const int s_cnt[3] = {n_sharp, n_lsharp, n_flat};
    const size_t rr = (size_t)s * R + ring;
    for (int t = lane; t < s_cnt[0]; t += 64) v.r_sharp[rr * 12 + t] = fp[p_sh[t]];
    for (int t = lane; t < s_cnt[1]; t += 64) v.r_less_sharp[rr * 120 + t] = fp[p_ls[t]];
    for (int t = lane; t < s_cnt[2]; t += 64) v.r_flat[rr * 24 + t] = fp[p_fl[t]];
    // ---- surfPointsLessFlatScan; sectors with sp >= ep are skipped, as the
    // reference's `continue`
    float4* o_lf = v.r_lf_scan + rr * C;
    int n_lf = 0;
    for (int kb0 = rs; kb0 < re; kb0 += 4 * 64) {
        // four points per lane loaded before any is written (named, so they stay in registers)
        const float4 q0 = fp[min(kb0 + lane, re - 1)], q1 = fp[min(kb0 + 64 + lane, re - 1)];
        const float4 q2 = fp[min(kb0 + 128 + lane, re - 1)], q3 = fp[min(kb0 + 192 + lane, re - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float4 qu = u == 0 ? q0 : u == 1 ? q1 : u == 2 ? q2 : q3;
            const int k = kb0 + u * 64 + lane;
            bool take = false;
            if (k < re) {
                for (int j = 0; j < 6; ++j) {
                    const int sp = sec_sp(rs, re, j), ep = sec_ep(rs, re, j);
                    if (k >= sp && k <= ep) { take = sp < ep; break; }
                }
                take = take && llab[k - lo] <= 0;
            }
            const unsigned long long m = __ballot(take);
            const int pos = n_lf + __popcll(m & ((1ull << lane) - 1));
            if (take && pos < C) o_lf[pos] = qu;
            n_lf += __popcll(m);
        }
    }
    if (lane == 0) {
        int* rc = v.ring_cnt + rr * 4;
        rc[0] = s_cnt[0]; rc[1] = s_cnt[1]; rc[2] = s_cnt[2];
        v.r_lf_n[rr] = min(n_lf, C);
    }
    for (int k = lane; k < hi - lo; k += 64) {
        picked[lo + k] = lpk[k];
        lab[lo + k] = llab[k];
    }
}

// ---------------------------------------------------------------- per-ring VoxelGrid(0.2)
// PCL VoxelGrid<PointXYZI>::applyFilter: bounds -> idx = floor(p/leaf) -
// min_b linearised x-fastest -> order by idx -> centroid of x,y,z,intensity.
// One 256-thread block per (ring, stream); keys (idx<<32 | pos) are sorted by
// a bitonic network in LDS, so points of a voxel are summed in position order.
#define SLO_DS_MAX 4096

__device__ inline void block_minmax(float& v0, float& v1, float& v2, float& w0, float& w1, float& w2, float* sh) {
    // min of v*, max of w* over the block (256 threads)
    for (int o = 32; o > 0; o >>= 1) {
        v0 = fminf(v0, __shfl_xor(v0, o, 64)); v1 = fminf(v1, __shfl_xor(v1, o, 64)); v2 = fminf(v2, __shfl_xor(v2, o, 64));
        w0 = fmaxf(w0, __shfl_xor(w0, o, 64)); w1 = fmaxf(w1, __shfl_xor(w1, o, 64)); w2 = fmaxf(w2, __shfl_xor(w2, o, 64));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh[w * 6 + 0] = v0; sh[w * 6 + 1] = v1; sh[w * 6 + 2] = v2;
        sh[w * 6 + 3] = w0; sh[w * 6 + 4] = w1; sh[w * 6 + 5] = w2;
    }
    __syncthreads();
    const int nw = blockDim.x >> 6;
    v0 = sh[0]; v1 = sh[1]; v2 = sh[2]; w0 = sh[3]; w1 = sh[4]; w2 = sh[5];
    for (int k = 1; k < nw; ++k) {
        v0 = fminf(v0, sh[k * 6 + 0]); v1 = fminf(v1, sh[k * 6 + 1]); v2 = fminf(v2, sh[k * 6 + 2]);
        w0 = fmaxf(w0, sh[k * 6 + 3]); w1 = fmaxf(w1, sh[k * 6 + 4]); w2 = fmaxf(w2, sh[k * 6 + 5]);
    }
    __syncthreads();
}

// Bitonic sort of the 256 * NE keys key_of(0 .. 256 NE) (padding ~0) by a
// 256-thread workgroup, result ascending in lds[0 ..): element g = w * 64 NE
// + e * 64 + lane lives in register e of lane `lane` of wave w, so every
// stage with a stride below 64 NE runs in registers (in-lane exchanges,
// cross-lane shuffles) and only the strides spanning waves (at most
// log2(4) per merge size) go through LDS with barriers.  The network is
// fully unrolled (constant register indices).
template <int NE, class KF>
__device__ inline void ring_sort_regs(unsigned long long* lds, KF&& key_of) {
    constexpr int WN = 64 * NE, N = 256 * NE;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned long long k[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) k[e] = key_of(w * WN + e * 64 + lane);
#pragma unroll
    for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= WN) {          // partner in another wave
#pragma unroll
                for (int e = 0; e < NE; ++e) lds[w * WN + e * 64 + lane] = k[e];
                __syncthreads();
#pragma unroll
                for (int e = 0; e < NE; ++e) {
                    const int g = w * WN + e * 64 + lane;
                    const unsigned long long y = lds[g ^ stride];
                    const bool take_min = ((g & size) == 0) == ((g & stride) == 0);
                    k[e] = take_min ? (k[e] < y ? k[e] : y) : (k[e] > y ? k[e] : y);
                }
                __syncthreads();
            } else if (stride >= 64) {   // partner in the same lane
                const int es = stride >> 6;
#pragma unroll
                for (int e = 0; e < NE; ++e) {
                    if (e & es) continue;
                    const bool up = ((w * WN + e * 64 + lane) & size) == 0;
                    const unsigned long long x = k[e], y = k[e | es];
                    const bool sw = up ? (x > y) : (x < y);
                    k[e] = sw ? y : x;
                    k[e | es] = sw ? x : y;
                }
            } else {                     // partner in lane ^ stride
#pragma unroll
                for (int e = 0; e < NE; ++e) {
                    const unsigned long long y = __shfl_xor(k[e], stride, 64);
                    const bool take_min = (((w * WN + e * 64 + lane) & size) == 0) == ((lane & stride) == 0);
                    k[e] = take_min ? (k[e] < y ? k[e] : y) : (k[e] > y ? k[e] : y);
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) lds[w * WN + e * 64 + lane] = k[e];
    __syncthreads();
}

// the stable in-voxel order (cfg.voxel_order == SLO_VOXEL_STABLE): one
// workgroup per ring, a bitonic sort of (voxel, index) keys
__global__ void __launch_bounds__(256) k_fa_ring_ds(DevView v) {
    const int s = blockIdx.y, ring = blockIdx.x;
    const int R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    const size_t rr = (size_t)s * R + ring;
    const int n = v.r_lf_n[rr];
    const float4* in = v.r_lf_scan + rr * C;
    float4* out = v.r_lf_ds + rr * C;
    extern __shared__ unsigned long long keys[];   // max(256, pow2 >= horizon_scan) keys (launch)
    __shared__ float sh[64];
    __shared__ int scan[256];
    const float leaf = v.cfg.leaf_less_flat;
    const float inv = 1.0f / leaf;
    float mnx = FLT_MAX, mny = FLT_MAX, mnz = FLT_MAX, mxx = -FLT_MAX, mxy = -FLT_MAX, mxz = -FLT_MAX;
    for (int b = 0; b < n; b += 8 * 256) {   // eight loads in flight per thread
        float4 pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = b + u * 256 + threadIdx.x;
            pp[u] = in[i < n ? i : n - 1];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float4 p = pp[u];
            mnx = fminf(mnx, p.x); mny = fminf(mny, p.y); mnz = fminf(mnz, p.z);
            mxx = fmaxf(mxx, p.x); mxy = fmaxf(mxy, p.y); mxz = fmaxf(mxz, p.z);
        }
    }
    block_minmax(mnx, mny, mnz, mxx, mxy, mxz, sh);
    if (n == 0) {
        if (threadIdx.x == 0) v.ring_cnt[rr * 4 + 3] = 0;
        return;
    }
    long long dx = (long long)((mxx - mnx) * inv) + 1, dy = (long long)((mxy - mny) * inv) + 1,
              dz = (long long)((mxz - mnz) * inv) + 1;
    if (dx * dy * dz > 2147483647LL) {  // PCL: integer indices would overflow -> output = input
        for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = in[i];
        if (threadIdx.x == 0) v.ring_cnt[rr * 4 + 3] = n;
        return;
    }
    const int minbx = (int)floorf(mnx * inv), minby = (int)floorf(mny * inv), minbz = (int)floorf(mnz * inv);
    const int maxbx = (int)floorf(mxx * inv), maxby = (int)floorf(mxy * inv);
    const int divx = maxbx - minbx + 1, divy = maxby - minby + 1;
    const int mul1 = divx, mul2 = divx * divy;
    auto key_of = [&](int i) -> unsigned long long {   // branch-free (n >= 1): the sort's loads all in flight
        const float4 p = in[min(i, n - 1)];
        const int ijk0 = (int)(floorf(p.x * inv) - (float)minbx);
        const int ijk1 = (int)(floorf(p.y * inv) - (float)minby);
        const int ijk2 = (int)(floorf(p.z * inv) - (float)minbz);
        const unsigned int idx = (unsigned int)(ijk0 + ijk1 * mul1 + ijk2 * mul2);
        return (((unsigned long long)idx << 32) | (unsigned int)i) | (0ull - (unsigned long long)(i >= n));
    };
    if (n <= 256) ring_sort_regs<1>(keys, key_of);
    else if (n <= 512) ring_sort_regs<2>(keys, key_of);
    else if (n <= 1024) ring_sort_regs<4>(keys, key_of);
    else if (n <= 2048) ring_sort_regs<8>(keys, key_of);
    else {   // rings longer than 2048 points (horizon_scan > 2048): bitonic in LDS
        int npow = 1;
        while (npow < n) npow <<= 1;
        for (int i = threadIdx.x; i < npow; i += blockDim.x) keys[i] = key_of(i);
        __syncthreads();
        for (int size = 2; size <= npow; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int t = threadIdx.x; t < npow / 2; t += blockDim.x) {
                    int lo = 2 * t - (t & (stride - 1));
                    int hi = lo + stride;
                    bool up = (lo & size) == 0;
                    unsigned long long a = keys[lo], b = keys[hi];
                    if ((a > b) == up) { keys[lo] = b; keys[hi] = a; }
                }
                __syncthreads();
            }
        }
    }
    // voxel heads -> rank via block scan over contiguous chunks
    const int T = blockDim.x;
    const int chunk = (n + T - 1) / T;
    const int i0 = threadIdx.x * chunk, i1 = min(n, i0 + chunk);
    int heads = 0;
    for (int i = i0; i < i1; ++i) heads += (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32));
    scan[threadIdx.x] = heads;
    __syncthreads();
    for (int d = 1; d < T; d <<= 1) {
        int a = threadIdx.x >= d ? scan[threadIdx.x - d] : 0;
        __syncthreads();
        scan[threadIdx.x] += a;
        __syncthreads();
    }
    int rank = scan[threadIdx.x] - heads;
    if (chunk <= 8) {   // rings of <= 2048 points: the chunk's points gathered at once, voxels summed in order
        float4 pp[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int i = i0 + c;
            pp[c] = i < i1 ? in[(unsigned int)keys[i]] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        bool have = false;   // a voxel started in this chunk is open
        unsigned int vid = 0;
        int cv = 0;
        float sx = 0, sy = 0, sz = 0, si = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int i = i0 + c;
            if (i < i1) {
                const unsigned int kv = (unsigned int)(keys[i] >> 32);
                if (i == 0 || kv != (unsigned int)(keys[i - 1] >> 32)) {
                    if (have) {
                        const float cnt = (float)cv;
                        out[rank++] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
                    }
                    have = true; vid = kv; cv = 0;
                    sx = 0; sy = 0; sz = 0; si = 0;
                }
                if (have) { sx += pp[c].x; sy += pp[c].y; sz += pp[c].z; si += pp[c].w; ++cv; }
            }
        }
        if (have) {   // the last voxel runs on past the chunk
            for (int e = i1; e < n && (unsigned int)(keys[e] >> 32) == vid; ++e) {
                const float4 p = in[(unsigned int)keys[e]];
                sx += p.x; sy += p.y; sz += p.z; si += p.w;
                ++cv;
            }
            const float cnt = (float)cv;
            out[rank++] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
        }
        if (threadIdx.x == T - 1) v.ring_cnt[rr * 4 + 3] = scan[T - 1];
        return;
    }
    for (int i = i0; i < i1; ++i) {
        if (!(i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32))) continue;
        unsigned int vid = (unsigned int)(keys[i] >> 32);
        float sx = 0, sy = 0, sz = 0, si = 0;
        int e = i;
        while (e < n && (unsigned int)(keys[e] >> 32) == vid) {
            float4 p = in[(unsigned int)keys[e]];
            sx += p.x; sy += p.y; sz += p.z; si += p.w;
            ++e;
        }
        float cnt = (float)(e - i);
        out[rank++] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
    }
    if (threadIdx.x == T - 1) v.ring_cnt[rr * 4 + 3] = scan[T - 1];
}

// PCL's own in-voxel order (cfg.voxel_order == SLO_VOXEL_PCL, the default):
// one workgroup of RW waves per ring (FA:779-780).  The bounds, the (voxel,
// index) keys in LDS, std::sort's order by slo_pcl::block_sort, then the
// voxel heads and the centroids summed in that order.  PMAX: the longest
// ring (the horizon_scan bound).
#ifndef RING_TLANE
#define RING_TLANE 64
#endif
#ifndef RING_OCC
#define RING_OCC 7          // waves per SIMD of the 4-wave ring VoxelGrid (23 KB of LDS: seven workgroups per CU)
#endif
#ifndef SLO_DIAG_RING
#define SLO_DIAG_RING 0     // 1: k_fa_ring_ds_pcl's sort counters in StreamState::dbg (tools/ring_diag.py; not with SLO_DIAG)
#endif
#ifndef RING_W
#define RING_W 4            // waves per ring (170 streams: 1.13 ms per launch against 1.53 with one wave,
#endif                      // since block_sort's pool); RING_FEW_W when the context has a few streams
#ifndef RING_FEW_W
#define RING_FEW_W 8        // one stream: 182 us per launch against 199 with 16 waves and 180 with 4 (r05)
#endif
// the ring VoxelGrid after its bounds (k_fa_ring_ds_pcl): the items into
// LDS, std::sort's order (slo_pcl::block_sort), the voxel heads and the
// centroids.  It: 64-bit (voxel << 32 | point) or 32-bit (voxel << 12 |
// point) items.  Returns the voxel count.
struct RingVg {
    const float4* in;
    float4* out;
    int n;
    float inv;
    int minbx, minby, minbz, mul1, mul2, tid, lane, wv;
};
__device__ inline unsigned long long ring_item(unsigned long long, unsigned int idx, int i) {
    return ((unsigned long long)idx << 32) | (unsigned int)i;
}
__device__ inline unsigned int ring_item(unsigned int, unsigned int idx, int i) {
    return (idx << slo_pcl::kPosBits) | (unsigned int)i;
}
__device__ inline unsigned int ring_point(unsigned long long it) { return (unsigned int)it; }
__device__ inline unsigned int ring_point(unsigned int it) { return it & ((1u << slo_pcl::kPosBits) - 1u); }
template <int PMAX, int RW, class It>
__device__ __forceinline__ int ring_vg_tail(const RingVg& g, It* keys, unsigned short* tbl, slo_pcl::WaveSmem* ws,
                                            slo_pcl::BlockQ<RW>& bq, int* serr, long long* rp, int* wsum) {
    constexpr int NT = 64 * RW;
    const int n = g.n, tid = g.tid, lane = g.lane, wv = g.wv;
    const float4* in = g.in;
    float4* out = g.out;
    const float inv = g.inv;
    for (int b = 0; b < n; b += 8 * NT) {
        float4 pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pp[u] = in[min(b + u * NT + tid, n - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = b + u * NT + tid;
            const int ijk0 = (int)(floorf(pp[u].x * inv) - (float)g.minbx);
            const int ijk1 = (int)(floorf(pp[u].y * inv) - (float)g.minby);
            const int ijk2 = (int)(floorf(pp[u].z * inv) - (float)g.minbz);
            const unsigned int idx = (unsigned int)(ijk0 + ijk1 * g.mul1 + ijk2 * g.mul2);
            if (i < n) keys[i] = ring_item(It(0), idx, i);
        }
    }
    __syncthreads();
    slo_pcl::block_sort<RING_TLANE, RW>(keys, n, 2 * slo_pcl::lg2(n), tbl, ws, bq, serr, rp);
    // voxel heads: a thread per contiguous chunk, ranks by a workgroup scan;
    // the chunk's points are gathered into registers first, every load in
    // flight at once (only a voxel running past the chunk's end loads more)
    constexpr int CHM = (PMAX + NT - 1) / NT;   // the longest chunk
    const int chunk = (n + NT - 1) / NT;
    const int i0 = min(n, tid * chunk), i1 = min(n, i0 + chunk);
    auto key = [&](int i) { return slo_pcl::vkey(keys[i]); };
    float4 q[CHM];
#pragma unroll
    for (int u = 0; u < CHM; ++u) q[u] = in[ring_point(keys[min(i0 + u, n - 1)])];
    int heads = 0;
#pragma unroll
    for (int u = 0; u < CHM; ++u) {
        const int i = i0 + u;
        heads += i < i1 && (i == 0 || key(i) != key(i - 1));
    }
    int incl = heads;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < RW; ++w) {
        if (w < wv) before += wsum[w];
        total += wsum[w];
    }
    int rank = before + incl - heads;
    // each voxel that starts in the chunk, summed in the sorted order (PCL's
    // in-order float chains); items before the chunk's first head belong to
    // the previous chunk's last voxel
    float sx = 0, sy = 0, sz = 0, si = 0;
    int cnt = 0;
    bool open = false;
#pragma unroll
    for (int u = 0; u < CHM; ++u) {
        const int i = i0 + u;
        if (i < i1) {
            if (i == 0 || key(i) != key(i - 1)) {
                if (open) out[rank++] = make_float4(sx / (float)cnt, sy / (float)cnt, sz / (float)cnt, si / (float)cnt);
                sx = sy = sz = si = 0;
                cnt = 0;
                open = true;
            }
            if (open) { sx += q[u].x; sy += q[u].y; sz += q[u].z; si += q[u].w; ++cnt; }
        }
    }
    if (open) {   // the chunk's last voxel, possibly running on past it
        const unsigned int vid = key(i1 - 1);
        for (int e = i1; e < n && key(e) == vid; ++e) {
            const float4 p = in[ring_point(keys[e])];
            sx += p.x; sy += p.y; sz += p.z; si += p.w;
            ++cnt;
        }
        out[rank++] = make_float4(sx / (float)cnt, sy / (float)cnt, sz / (float)cnt, si / (float)cnt);
    }
    return total;
}

template <int PMAX, int RW>
__global__ void __launch_bounds__(64 * RW) __attribute__((amdgpu_waves_per_eu(RW == 4 ? RING_OCC : 1))) k_fa_ring_ds_pcl(DevView v) {
    constexpr int NT = 64 * RW;
    const int s = blockIdx.y, ring = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    const size_t rr = (size_t)s * R + ring;
    const int n = v.r_lf_n[rr];
    const float4* in = v.r_lf_scan + rr * C;
    float4* out = v.r_lf_ds + rr * C;
    __shared__ unsigned long long keys[PMAX];
    __shared__ unsigned short tbl[PMAX / 2 + 1];
    __shared__ slo_pcl::WaveSmem ws[RW];
    __shared__ slo_pcl::BlockQ<RW> bq;
    __shared__ float mm[RW][6];
    __shared__ int wsum[RW];
    __shared__ int serr;
    if (n == 0) {
        if (tid == 0) v.ring_cnt[rr * 4 + 3] = 0;
        return;
    }
#if SLO_DIAG_RING
    // dbg[0] sort cycles, [1] the slowest sort, [2..5] block_sort's phases (thread 0): group levels, wave level,
    // bookkeeping, queue; [6] / [7] the slowest sort's cycles with its ring's size / ring
    unsigned long long t_r = clock64();
#define RING_STAMP(k) if (tid == 0) { const unsigned long long t_n = clock64(); atomicAdd(&v.st[s].dbg[k], t_n - t_r); t_r = t_n; }
    long long rprof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, *rp = rprof;
#else
#define RING_STAMP(k)
    long long* rp = nullptr;
#endif
    const float inv = 1.0f / v.cfg.leaf_less_flat;
    float mnx = FLT_MAX, mny = FLT_MAX, mnz = FLT_MAX, mxx = -FLT_MAX, mxy = -FLT_MAX, mxz = -FLT_MAX;
    for (int b = 0; b < n; b += 8 * NT) {   // eight loads in flight per thread
        float4 pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pp[u] = in[min(b + u * NT + tid, n - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            mnx = fminf(mnx, pp[u].x); mny = fminf(mny, pp[u].y); mnz = fminf(mnz, pp[u].z);
            mxx = fmaxf(mxx, pp[u].x); mxy = fmaxf(mxy, pp[u].y); mxz = fmaxf(mxz, pp[u].z);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mnx = fminf(mnx, __shfl_xor(mnx, o, 64)); mny = fminf(mny, __shfl_xor(mny, o, 64));
        mnz = fminf(mnz, __shfl_xor(mnz, o, 64)); mxx = fmaxf(mxx, __shfl_xor(mxx, o, 64));
        mxy = fmaxf(mxy, __shfl_xor(mxy, o, 64)); mxz = fmaxf(mxz, __shfl_xor(mxz, o, 64));
    }
    if (lane == 0) {
        mm[wv][0] = mnx; mm[wv][1] = mny; mm[wv][2] = mnz; mm[wv][3] = mxx; mm[wv][4] = mxy; mm[wv][5] = mxz;
    }
    if (tid == 0) serr = 0;
    __syncthreads();
    for (int w = 0; w < RW; ++w) {   // min / max are exact: any order gives the same bounds
        mnx = fminf(mnx, mm[w][0]); mny = fminf(mny, mm[w][1]); mnz = fminf(mnz, mm[w][2]);
        mxx = fmaxf(mxx, mm[w][3]); mxy = fmaxf(mxy, mm[w][4]); mxz = fmaxf(mxz, mm[w][5]);
    }
    const long long dx = (long long)((mxx - mnx) * inv) + 1, dy = (long long)((mxy - mny) * inv) + 1,
                    dz = (long long)((mxz - mnz) * inv) + 1;
    if (dx * dy * dz > 2147483647LL) {  // PCL: integer indices would overflow -> output = input
        for (int i = tid; i < n; i += NT) out[i] = in[i];
        if (tid == 0) v.ring_cnt[rr * 4 + 3] = n;
        return;
    }
    const int minbx = (int)floorf(mnx * inv), minby = (int)floorf(mny * inv), minbz = (int)floorf(mnz * inv);
    const int maxbx = (int)floorf(mxx * inv), maxby = (int)floorf(mxy * inv), maxbz = (int)floorf(mxz * inv);
    const int divx = maxbx - minbx + 1, divy = maxby - minby + 1;
    const int mul1 = divx, mul2 = divx * divy;
    // 32-bit items (voxel << 12 | point) when every voxel index of the ring's
    // box fits 20 bits (the near rings; the sort's LDS traffic and registers
    // halve), else 64-bit (voxel << 32 | point): the same comparisons, so the
    // same std::sort order
    const RingVg g{in, out, n, inv, minbx, minby, minbz, mul1, mul2, tid, lane, wv};
    int total;
    if ((long long)divx * divy * ((long long)maxbz - minbz + 1) <= (1LL << 20))
        total = ring_vg_tail<PMAX, RW>(g, reinterpret_cast<unsigned int*>(keys), tbl, ws, bq, &serr, rp, wsum);
    else
        total = ring_vg_tail<PMAX, RW>(g, keys, tbl, ws, bq, &serr, rp, wsum);
#if SLO_DIAG_RING
    if (tid == 0) {   // thread 0's phases of block_sort
        for (int k = 4; k < 8; ++k) atomicAdd(&v.st[s].dbg[k - 2], (unsigned long long)rprof[k]);
    }
#endif
    if (tid == 0 && serr) atomicOr(&v.st[s].err, SLO_ERR_SORT);
    if (tid == 0) v.ring_cnt[rr * 4 + 3] = total;
#undef RING_STAMP
}

// concatenate per-ring outputs in ring order: one block per (ring, stream),
// each summing the counts of the rings before its own.  `part`: 0 all four
// clouds; 1 sharp, less sharp and flat (fa_pick's); 2 less flat alone
// (fa_ring_ds's) — the two halves of a forked step (fa_features_run), which
// read and write disjoint counts
__global__ void __launch_bounds__(256) k_fa_gather(DevView v, int part) {
    const int r = blockIdx.x, s = blockIdx.y;
    const int R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    __shared__ int off[4], tot[4];
    const int* rc = v.ring_cnt + (size_t)s * R * 4;
    const bool pk = part != 2, ds = part != 1;
    if (threadIdx.x < 4 && (threadIdx.x == 3 ? ds : pk)) {
        const int c = threadIdx.x;
        int a = 0, b = 0;
        for (int q = 0; q < R; ++q) {
            const int x = rc[4 * q + c];
            if (q < r) a += x;
            b += x;
        }
        off[c] = a;
        tot[c] = b;
    }
    __syncthreads();
    // ring boundaries of less_sharp / less_flat (the odometry's ring windows)
    if (threadIdx.x == 0) {
        StreamState& st = v.st[s];
        if (pk) {
            v.roff_cur[((size_t)s * 2 + 0) * (R + 1) + r] = off[1];
            if (r == R - 1) {
                v.roff_cur[((size_t)s * 2 + 0) * (R + 1) + R] = tot[1];
                st.n_sharp = tot[0]; st.n_less_sharp = tot[1]; st.n_flat = tot[2];
            }
        }
        if (ds) {
            v.roff_cur[((size_t)s * 2 + 1) * (R + 1) + r] = min(off[3], v.cap_less_flat);
            if (r == R - 1) {
                v.roff_cur[((size_t)s * 2 + 1) * (R + 1) + R] = min(tot[3], v.cap_less_flat);
                st.n_less_flat = min(tot[3], v.cap_less_flat);
            }
        }
    }
    const size_t rr = (size_t)s * R + r;
    if (pk) {
        for (int i = threadIdx.x; i < rc[4 * r + 0]; i += blockDim.x)
            v.sharp[(size_t)s * v.cap_sharp + off[0] + i] = v.r_sharp[rr * 12 + i];
        for (int i = threadIdx.x; i < rc[4 * r + 1]; i += blockDim.x)
            v.less_sharp[(size_t)s * v.cap_less_sharp + off[1] + i] = v.r_less_sharp[rr * 120 + i];
        for (int i = threadIdx.x; i < rc[4 * r + 2]; i += blockDim.x)
            v.flat[(size_t)s * v.cap_flat + off[2] + i] = v.r_flat[rr * 24 + i];
    }
    if (ds)
        for (int i = threadIdx.x; i < rc[4 * r + 3]; i += blockDim.x)
            if (off[3] + i < v.cap_less_flat) v.less_flat[(size_t)s * v.cap_less_flat + off[3] + i] = v.r_lf_ds[rr * C + i];
}

// the less-flat VoxelGrids and their gather (fa_features_run)
static int fa_ring_ds_launch(slo_ctx* ctx, int part) {
    DevView& v = ctx->v;
    const int S = ctx->S, R = v.cfg.n_scan;
    if (v.cfg.voxel_order == SLO_VOXEL_PCL) {   // RING_W waves per ring; slo_create refuses rings over 4096 points
        const bool few = S <= 8;
        if (v.cfg.horizon_scan <= 2048) {
            if (few) SLO_LAUNCH(ctx, "fa_ring_ds", (k_fa_ring_ds_pcl<2048, RING_FEW_W>), dim3(R, S), dim3(64 * RING_FEW_W), 0, v);
            else SLO_LAUNCH(ctx, "fa_ring_ds", (k_fa_ring_ds_pcl<2048, RING_W>), dim3(R, S), dim3(64 * RING_W), 0, v);
        } else {
            if (few) SLO_LAUNCH(ctx, "fa_ring_ds", (k_fa_ring_ds_pcl<4096, RING_FEW_W>), dim3(R, S), dim3(64 * RING_FEW_W), 0, v);
            else SLO_LAUNCH(ctx, "fa_ring_ds", (k_fa_ring_ds_pcl<4096, RING_W>), dim3(R, S), dim3(64 * RING_W), 0, v);
        }
    } else {
        int ds_keys = 256;   // LDS keys of k_fa_ring_ds: a ring holds <= horizon_scan points
        while (ds_keys < v.cfg.horizon_scan) ds_keys <<= 1;
        SLO_LAUNCH(ctx, "fa_ring_ds", k_fa_ring_ds, dim3(R, S), dim3(256), ds_keys * sizeof(unsigned long long), v);
    }
    SLO_LAUNCH(ctx, "fa_gather", k_fa_gather, dim3(R, S), dim3(256), 0, v, part);
    SLO_CHECK(hipGetLastError());
    return 0;
}

// fork: the less-flat VoxelGrids (the reference's surfPointsLessFlatScan
// downsampling, FA:779-780) on ring_stream beside the odometry, which reads
// none of their output before its end (k_fa_to_end): fa_odometry_run joins
// there (fa_ring_join).  Contexts of at most SLO_PREP_DEFER_STREAMS streams,
// whose step the latency of these sorts would otherwise lengthen.
int fa_features_run(slo_ctx* ctx, bool fork) {
    DevView& v = ctx->v;
    const int S = ctx->S, R = v.cfg.n_scan;
    const int T = 256;
    dim3 gh((v.H + T - 1) / T, S);
    SLO_LAUNCH(ctx, "fa_halfpass", k_fa_halfpass, gh, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "fa_imu_start", k_fa_imu_start, dim3((S + 63) / 64), dim3(64), 0, v);
    SLO_LAUNCH(ctx, "fa_points", k_fa_points, gh, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "fa_extract_stale", k_fa_extract_stale, dim3(1, S), dim3(256), 0, v);
    SLO_LAUNCH(ctx, "fa_sort", k_fa_sort, dim3(R, S), dim3(256), 0, v);
    SLO_LAUNCH(ctx, "fa_pick", k_fa_pick, dim3(R, S), dim3(64), 0, v);
    if (!fork || !ctx->ring_stream) return fa_ring_ds_launch(ctx, 0);
    SLO_CHECK(hipEventRecord(ctx->ev_rfork, ctx->stream));
    SLO_CHECK(hipStreamWaitEvent(ctx->ring_stream, ctx->ev_rfork, 0));
    std::swap(ctx->stream, ctx->ring_stream);
    int r = fa_ring_ds_launch(ctx, 2);
    std::swap(ctx->stream, ctx->ring_stream);
    if (r) return r;
    SLO_CHECK(hipEventRecord(ctx->ev_rjoin, ctx->ring_stream));
    ctx->ring_pending = true;
    SLO_LAUNCH(ctx, "fa_gather", k_fa_gather, dim3(R, S), dim3(256), 0, v, 1);
    SLO_CHECK(hipGetLastError());
    return 0;
}

int fa_ring_join(slo_ctx* ctx) {
    if (!ctx->ring_pending) return 0;
    ctx->ring_pending = false;
    SLO_CHECK(hipStreamWaitEvent(ctx->stream, ctx->ev_rjoin, 0));
    return 0;
}

}  // namespace slo
