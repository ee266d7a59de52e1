// slo_ip.hip — image projection + ground + segmentation (imageProjection.cpp
// :181-460) for a batch of S streams, one scan each.
//
// Data-parallel recast of the reference's serial loops, with identical
// results:
//   projectPointCloud (IP:211-257): one thread per point; "last point wins"
//     (Q2) is atomicMax of the point index into a per-pixel owner word; the
//     first/last finite index (findStartEndAngle, IP:199) is a wave-reduced
//     atomicMin/Max.
//   groundRemoval (IP:260-310): one thread per pixel, reading the pair tests
//     (i-1,i) and (i,i+1) and applying the reference's overwrite order (Q15).
//   labelComponents BFS (IP:370-460): connected components of the symmetric
//     60-degree edge predicate over label-0 pixels (Q3) by lock-free
//     union-find that always links the larger root under the smaller, so
//     every root is its component's row-major-first pixel = the BFS seed;
//     size and row set (excluding the seed) feed the same feasibility rule.
//   cloudSegmentation compaction (IP:319-355): per-row counts, then a block
//     scan per row writes segmentedCloud / cloud_info in row-major order.
// All float math matches the host bit for bit (slo_libm, -ffp-contract=off,
// correctly rounded sqrtf/division).
#include "slo_internal.h"
#include "slo_fastatan.h"
#include "slo_libm.h"
#include <float.h>

namespace slo {

__device__ inline int wave_min(int x) {
    for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
    return x;
}
__device__ inline int wave_max(int x) {
    for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
    return x;
}

// atan2f value -> degrees as the reference writes it: atan2(..) * 180 / M_PI
// (float product, double quotient, narrowed to float)
__device__ inline float ip_deg(float a) { return (float)((double)(a * 180) / M_PI); }
// the row (IP:231-233, Q1: truncation, (-1,0) -> 0) and the unwrapped column
// (IP:235-238) of an elevation / azimuth atan2f value; both monotone in it
__device__ inline long long ip_row_of(const slo_config& c, float a) {
    const float rowf = (ip_deg(a) + c.ang_bottom) / c.ang_res_y;
    return (long long)rowf;
}
__device__ inline long long ip_col_of(const slo_config& c, float a) {
    const double colD = -round(((double)ip_deg(a) - 90.0) / (double)c.ang_res_x) + (double)(c.horizon_scan / 2);
    return (long long)colD;
}

// row / column of a finite point (IP:229-246); returns false if rejected.
// The bins are taken at both ends of the atan2f bracket (slo_fastatan.h);
// only when they differ is glibc's atan2f itself evaluated.
// ring >= 0: the row is the point's ring field (useCloudRing, IP:225-226).
__device__ inline bool project_point(const slo_config& c, float4 p, int ring, int& row, int& col, float& range) {
    float lo, hi;
    long long r;
    if (ring >= 0) {
        r = ring;
    } else {
        const float h = sqrtf(p.x * p.x + p.y * p.y);
        if (!slo_fast::atan2_bracket(p.z, h, lo, hi) || (r = ip_row_of(c, lo)) != ip_row_of(c, hi))
            r = ip_row_of(c, slo_libm::atan2f_(p.z, h));
    }
    if (r < 0 || r >= c.n_scan) return false;
    long long cc;
    if (!slo_fast::atan2_bracket(p.x, p.y, lo, hi) || (cc = ip_col_of(c, lo)) != ip_col_of(c, hi))
        cc = ip_col_of(c, slo_libm::atan2f_(p.x, p.y));
    if (cc >= c.horizon_scan) cc -= c.horizon_scan;
    if (cc < 0 || cc >= c.horizon_scan) return false;
    float rg = sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);
    if (rg < c.sensor_minimum_range) return false;
    row = (int)r; col = (int)cc; range = rg;
    return true;
}

// the owner image back to -1 (no point) and the first/last finite indices
// reset; a kernel rather than a memset, so a captured step graph holds
// plain kernel nodes only
__global__ void __launch_bounds__(256) k_ip_init(DevView v) {
    const size_t n4 = (size_t)v.S * v.H / 4, i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    int4* o = reinterpret_cast<int4*>(v.owner);
    for (size_t i = i0; i < n4; i += (size_t)gridDim.x * blockDim.x) o[i] = make_int4(-1, -1, -1, -1);
    for (size_t i = 4 * n4 + i0; i < (size_t)v.S * v.H; i += (size_t)gridDim.x * blockDim.x) v.owner[i] = -1;
    if (i0 < (size_t)v.S) {
        v.fl[2 * i0] = INT_MAX;
        v.fl[2 * i0 + 1] = -1;
    }
}

// A workgroup takes IP_PTS_PER_WG consecutive points (thread t: points t,
// t+256, ...).  The owner image is column-major ([S][C][R]): points arrive in
// firing order — all rings of one azimuth, then the next — so a wave's 64
// owner atomics land in one or two 128-byte lines of one column.  Device-scope
// atomics are executed beyond the XCD's L2 (they must be coherent across
// XCDs), so what they cost is the number of line requests, not of lanes.
#define IP_PTS_PER_WG 2048
__global__ void k_ip_project(DevView v) {
    const int s = blockIdx.y;
    const int n = v.io->npts[s];
    const int R = v.cfg.n_scan;
    int fmin = INT_MAX, fmax = -1;
    if ((int)blockIdx.x * IP_PTS_PER_WG >= n) return;   // no point of this stream here
    // every point of the thread loaded before the first is projected
    const float4* P = v.io->pts + (size_t)s * v.P;
    float4 pp[IP_PTS_PER_WG / 256];
#pragma unroll
    for (int k = 0; k < IP_PTS_PER_WG / 256; ++k)
        pp[k] = P[min((int)blockIdx.x * IP_PTS_PER_WG + k * 256 + (int)threadIdx.x, n - 1)];
#pragma unroll
    for (int k = 0; k < IP_PTS_PER_WG / 256; ++k) {
        const int i = blockIdx.x * IP_PTS_PER_WG + k * 256 + threadIdx.x;
        if (i >= n) break;
        const float4 p = pp[k];
        if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
            fmin = min(fmin, i); fmax = max(fmax, i);
            int row, col; float rg;
            const int ring = v.cfg.use_cloud_ring ? (int)v.rings[(size_t)s * v.P + i] : -1;
            if (project_point(v.cfg, p, ring, row, col, rg))
                atomicMax(&v.owner[(size_t)s * v.H + (size_t)col * R + row], i);
        }
    }
    fmin = wave_min(fmin); fmax = wave_max(fmax);
    if ((threadIdx.x & 63) == 0) {
        if (fmin != INT_MAX) atomicMin(&v.fl[2 * s], fmin);
        if (fmax >= 0) atomicMax(&v.fl[2 * s + 1], fmax);
    }
}

// ---------------------------------------------------------------- image tiles
// k_ip_tile, k_cc_stats: one workgroup per tile of all R rows x TC columns
// (IP_TILE_PX pixels, local index l = i * TC + jj, row-major like the global
// pixel index p = i * C + j, so local and global orders agree).
#ifndef IP_TILE_PX
#define IP_TILE_PX 2048   // 2048: 42 KB -> 22 KB of LDS, seven workgroups per CU instead of three; C3 ip_tile 10.5 -> 7.6 ms
#endif                    // per 24 launches (k_cc_merge +0.5 ms), 20.04 k -> 20.20 k and 19.95 k -> 20.43 k scans/s (r05)
#define IP_TILE_MAXC 256
#define IP_LROOT (1 << 30)   // csize flag: the pixel is a tile-local root (k_ip_tile)
__host__ __device__ inline int ip_tile_cols(int R) { return min(IP_TILE_MAXC, max(1, IP_TILE_PX / R)); }

// edge predicate of labelComponents (IP:411-423): atan2f(..) > segmentTheta,
// decided at both ends of the atan2f bracket (slo_fastatan.h) when it can be
__device__ inline bool seg_edge(const slo_config& c, float r1, float r2, bool horizontal) {
    float d1 = fmaxf(r1, r2), d2 = fminf(r1, r2);
    float sa = horizontal ? c.sin_alpha_x : c.sin_alpha_y;
    float ca = horizontal ? c.cos_alpha_x : c.cos_alpha_y;
    const float y = d2 * sa, x = d1 - d2 * ca;
    float lo, hi;
    if (slo_fast::atan2_bracket(y, x, lo, hi) && (lo > c.segment_theta) == (hi > c.segment_theta))
        return lo > c.segment_theta;
    return slo_libm::atan2f_(y, x) > c.segment_theta;
}

// Union-find that always links the larger root under the smaller, so a root
// is its component's smallest index.  In LDS (one tile) and in HBM (global
// pixel indices; device-scope atomics).
__device__ inline int lds_find(int* par, int x) {
    int y = __hip_atomic_load(&par[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (y != x) { x = y; y = __hip_atomic_load(&par[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
    return x;
}
__device__ inline void lds_unite(int* par, int a, int b) {
    while (true) {
        a = lds_find(par, a);
        b = lds_find(par, b);
        if (a == b) return;
        if (a < b) { int t = a; a = b; b = t; }
        int old = atomicCAS(&par[a], a, b);
        if (old == a) return;
        a = old;
    }
}
__device__ inline int ld_parent(int* a, int x) {
    return __hip_atomic_load(&a[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline int find_root(int* par, int x) {
    int y = ld_parent(par, x);
    while (y != x) { x = y; y = ld_parent(par, x); }
    return x;
}
// find_root with path halving above the first hop: every node passed on the
// way up is relinked to its grandparent, so the next find over the same chain
// is half as long.  A component spanning many tiles otherwise leaves a chain
// of tile-local roots, one per tile (k_cc_merge links each tile's root under
// its neighbour's), that every find walks in full: 64 dependent loads on a
// 2048-column scan.  Only roots and tile-local roots are relinked — a
// pixel's own parent stays its tile-local root (k_cc_stats relies on it) —
// and only ever to an ancestor, by a CAS from the parent it read, so
// concurrent finds, the CAS links of unite and k_cc_stats' final stores of
// the root (which a stale relink must not overwrite: k_ip_rowcount reads a
// pixel's root two hops up) stay correct; the roots (smallest index of each
// component) are the same as without it.
__device__ inline void st_parent(int* a, int x, int expect, int v) { atomicCAS(&a[x], expect, v); }
__device__ inline int find_root_h(int* par, int x) {
    int y = ld_parent(par, x);
    if (y == x) return x;
    x = y;   // the tile-local root (or a root): halving starts here
    for (;;) {
        y = ld_parent(par, x);
        if (y == x) return x;
        const int z = ld_parent(par, y);
        if (z == y) return y;
        st_parent(par, x, y, z);
        x = z;
    }
}
__device__ inline void unite(int* par, int a, int b) {
    while (true) {
        a = find_root_h(par, a);
        b = find_root_h(par, b);
        if (a == b) return;
        if (a < b) { int t = a; a = b; b = t; }
        int old = atomicCAS(&par[a], a, b);
        if (old == a) return;
        a = old;
    }
}

// Per tile: the owner columns are transposed through LDS; then per pixel the
// range, the full-cloud point, the final groundMat value (Q15; each row pair
// (i, i+1) is tested once, IP:268-300) and the label seed; then the
// components inside the tile by LDS union-find over the edges of
// labelComponents (IP:396-423) whose both ends are in the tile.  parent[]
// gets the global index of each pixel's tile-local root; the edges across
// tile boundaries (and the column wrap, IP:403-406) are k_cc_merge's.
__global__ void __launch_bounds__(256) k_ip_tile(DevView v) {
    const int s = blockIdx.y, R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    const int TC = ip_tile_cols(R), c0 = blockIdx.x * TC, nc = min(TC, C - c0), npx = R * TC;
    const size_t base = (size_t)s * v.H;
    const float4* pts = v.io->pts + (size_t)s * v.P;
    const int gsi = v.cfg.ground_scan_ind, tid = threadIdx.x;
    __shared__ int l_a[IP_TILE_PX];   // owner, then the union-find parents
    __shared__ float l_rg[IP_TILE_PX];
    __shared__ int8_t l_lab[IP_TILE_PX], l_pair[IP_TILE_PX];
    __shared__ double l_q[IP_TILE_MAXC];
    for (int k = tid; k < R * nc; k += 256) {
        const int jj = k / R, i = k - jj * R;
        l_a[i * TC + jj] = v.owner[base + (size_t)(c0 + jj) * R + i];
    }
    for (int jj = tid; jj < nc; jj += 256) l_q[jj] = (double)(float)(c0 + jj) / 10000.0;
    __syncthreads();
    const int npair = min(gsi, R - 1) * nc;
    for (int k = tid; k < npair; k += 256) {
        const int i = k / nc, jj = k - i * nc;
        const int lo = l_a[i * TC + jj], up = l_a[(i + 1) * TC + jj];
        int g = -1;
        if (lo >= 0 && up >= 0) {
            const float4 a = pts[lo], b = pts[up];
            const float dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
            const float h = sqrtf(dx * dx + dy * dy);
            // fabsf(angle - sensorMountAngle) <= 10 (IP:291) as its two
            // monotone halves, decided at the atan2f bracket's ends if they agree
            const float mount = v.cfg.sensor_mount_angle;
            float lo, hi;
            bool ok = slo_fast::atan2_bracket(dz, h, lo, hi);
            const float ul = ip_deg(lo) - mount, uh = ip_deg(hi) - mount;
            if (ok && (ul >= -10) == (uh >= -10) && (ul <= 10) == (uh <= 10)) {
                g = (ul >= -10 && ul <= 10) ? 1 : 0;
            } else {
                const float angle = ip_deg(slo_libm::atan2f_(dz, h));
                g = fabsf(angle - mount) <= 10 ? 1 : 0;
            }
        }
        l_pair[i * TC + jj] = (int8_t)g;
    }
    __syncthreads();
    for (int l = tid; l < npx; l += 256) {
        const int i = l / TC, jj = l - i * TC;
        if (jj >= nc) { l_lab[l] = -1; continue; }
        const size_t o = base + (size_t)i * C + c0 + jj;
        const int own = l_a[l];
        float rg = FLT_MAX;
        float4 f;
        if (own >= 0) {
            const float4 q = pts[own];
            rg = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z);
            f = make_float4(q.x, q.y, q.z, (float)((double)(float)i + l_q[jj]));
        } else {
            const float qn = __builtin_nanf("");
            f = make_float4(qn, qn, qn, -1.0f);
        }
        v.range[o] = rg;
        v.full[o] = f;
        int g = 0;   // Q15: final groundMat value of row i
        if (i <= gsi) {
            const int pi_ = (i < gsi && i + 1 < R) ? l_pair[l] : 0;
            const int pm = (i >= 1 && i - 1 < gsi) ? l_pair[l - TC] : 0;
            if (i < gsi && pi_ == -1) g = -1;
            else if (pi_ == 1 || pm == 1) g = 1;
        }
        v.ground[o] = (int8_t)g;
        const int lab = (g == 1 || rg == FLT_MAX) ? -1 : 0;
        v.label[o] = lab;
        l_lab[l] = (int8_t)lab;
        l_rg[l] = rg;
    }
    __syncthreads();
    for (int l = tid; l < npx; l += 256) l_a[l] = l_lab[l] == 0 ? l : -1;
    __syncthreads();
    for (int l = tid; l < npx; l += 256) {
        if (l_lab[l] != 0) continue;
        const int i = l / TC, jj = l - i * TC;
        if (jj + 1 < nc && l_lab[l + 1] == 0 && seg_edge(v.cfg, l_rg[l], l_rg[l + 1], true)) lds_unite(l_a, l, l + 1);
        if (i + 1 < R && l_lab[l + TC] == 0 && seg_edge(v.cfg, l_rg[l], l_rg[l + TC], false))
            lds_unite(l_a, l, l + TC);
    }
    __syncthreads();
    for (int l = tid; l < npx; l += 256) {
        const int i = l / TC, jj = l - i * TC;
        if (jj >= nc) continue;
        const int p = i * C + c0 + jj;
        int g = -1;
        if (l_lab[l] == 0) {
            const int r = lds_find(l_a, l), ri = r / TC;
            g = ri * C + c0 + (r - ri * TC);
        }
        v.parent[base + p] = g;
        v.csize[base + p] = g == p ? IP_LROOT : 0;   // sizes and row sets are only kept at roots
        if (g == p) { v.crows[2 * (base + p)] = 0ull; v.crows[2 * (base + p) + 1] = 0ull; }
    }
}

// the horizontal edges between tiles (and the wrap C-1 -> 0), one thread per
// (tile, row)
__global__ void k_cc_merge(DevView v, int ntiles) {
    const int s = blockIdx.y, R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ntiles * R) return;
    const int TC = ip_tile_cols(R), t = k / R, i = k - t * R;
    const int j = min(C, (t + 1) * TC) - 1, jn = j + 1 == C ? 0 : j + 1;
    const size_t base = (size_t)s * v.H;
    const int p = i * C + j, q = i * C + jn;
    if (v.label[base + p] == 0 && v.label[base + q] == 0 &&
        seg_edge(v.cfg, v.range[base + p], v.range[base + q], true))
        unite(v.parent + base, p, q);
}

// Component size and row set (seed excluded, Q3), per tile: the pixels are
// counted per tile-local root in LDS, and each local root then adds its
// totals to its component root with one set of atomics; it also stores that
// root as its own parent, so every pixel's root is parent[parent[p]].
// (k_cc_merge only relinks roots, so a non-root pixel's parent is still its
// tile-local root; local roots are flagged in csize.)
// Slots (tile-local roots counted in LDS) per workgroup: a dense scan's tile
// holds many small components — 1 200 local roots per 128 x 32 tile on C5's
// 128 x 2048 scans, up to ~950 per 64 x 64 tile on C2 / C3 — and a tile past
// its slots takes the slow path, per-pixel device atomics; so 768 slots for
// up to 64 rows, 1536 beyond (24 B each, 26 / 44 KB of LDS per workgroup).
#define IP_NOT_CAND 0xfffd
#define IP_NOT_ROOT 0xfffe
#define IP_OVERFLOW 0xffff
template <int SLOTS>
__global__ void __launch_bounds__(256) k_cc_stats(DevView v) {
    const int s = blockIdx.y, R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    const int TC = ip_tile_cols(R), c0 = blockIdx.x * TC, nc = min(TC, C - c0), npx = R * TC;
    const size_t base = (size_t)s * v.H;
    int* par = v.parent + base;
    const int tid = threadIdx.x;
    __shared__ uint16_t l_slot[IP_TILE_PX];
    __shared__ int l_cnt[SLOTS], l_fr[SLOTS];
    __shared__ unsigned long long l_rows[SLOTS][2];
    __shared__ int n_slots;
    if (tid == 0) n_slots = 0;
    for (int k = tid; k < SLOTS; k += 256) { l_cnt[k] = 0; l_rows[k][0] = 0ull; l_rows[k][1] = 0ull; }
    __syncthreads();
    for (int l = tid; l < npx; l += 256) {
        const int i = l / TC, jj = l - i * TC;
        if (jj >= nc) continue;
        const int p = i * C + c0 + jj;
        uint16_t code = IP_NOT_CAND;
        if (par[p] >= 0) {
            code = IP_NOT_ROOT;
            if (v.csize[base + p] & IP_LROOT) {
                const int fr = find_root_h(par, p);
                const int k = atomicAdd(&n_slots, 1);
                code = IP_OVERFLOW;
                if (k < SLOTS) { code = (uint16_t)k; l_fr[k] = fr; }
            }
        }
        l_slot[l] = code;
    }
    __syncthreads();
    for (int l = tid; l < npx; l += 256) {
        const int i = l / TC, jj = l - i * TC;
        if (jj >= nc) continue;
        const int code = l_slot[l];
        if (code == IP_NOT_CAND) continue;
        const int p = i * C + c0 + jj;
        int lr = l;
        if (code == IP_NOT_ROOT) {
            const int g = par[p], gi = g / C;
            lr = gi * TC + (g - gi * C - c0);
        }
        const int k = l_slot[lr];
        const unsigned long long bit = 1ull << (i & 63);
        if (k != IP_OVERFLOW) {
            atomicAdd(&l_cnt[k], 1);
            if (p != l_fr[k]) atomicOr(&l_rows[k][i >> 6], bit);
        } else {
            const int fr = find_root_h(par, lr == l ? p : par[p]);
            atomicAdd(&v.csize[base + fr], 1);
            if (p != fr) atomicOr(&v.crows[2 * (base + fr) + (i >> 6)], bit);
        }
    }
    __syncthreads();
    const int ns = min(n_slots, SLOTS);
    for (int k = tid; k < ns; k += 256) {
        const int fr = l_fr[k];
        atomicAdd(&v.csize[base + fr], l_cnt[k]);
        if (l_rows[k][0]) atomicOr(&v.crows[2 * (base + fr)], l_rows[k][0]);
        if (l_rows[k][1]) atomicOr(&v.crows[2 * (base + fr) + 1], l_rows[k][1]);
    }
    // compress: the local roots point at their component roots (every find
    // of this workgroup has finished; other workgroups only follow parent
    // links, which this keeps valid)
    for (int l = tid; l < npx; l += 256) {
        const int i = l / TC, jj = l - i * TC;
        if (jj >= nc) continue;
        const int code = l_slot[l];
        if (code == IP_NOT_CAND || code == IP_NOT_ROOT) continue;
        const int p = i * C + c0 + jj;
        par[p] = code == IP_OVERFLOW ? find_root(par, p) : l_fr[code];
    }
}

// final label of a label-0 pixel (IP:425-460): feasible segments keep a
// positive label (the reference numbers them by seed order; the number is
// only used by the visualisation cloud IP:363), the rest 999999
__device__ inline int final_label(const DevView& v, size_t base, size_t o) {
    const int r = v.parent[base + v.parent[o]];
    const int size = v.csize[base + r] & (IP_LROOT - 1);
    bool feasible = false;
    if (size >= 30) feasible = true;
    else if (size >= v.cfg.segment_valid_point_num) {
        const int lines = __popcll(v.crows[2 * (base + r)]) + __popcll(v.crows[2 * (base + r) + 1]);
        if (lines >= v.cfg.segment_valid_line_num) feasible = true;
    }
    return feasible ? r + 1 : 999999;
}

__device__ inline void pixel_kind(const DevView& v, size_t base, int i, int j, bool& kept, bool& outl) {
    const int C = v.cfg.horizon_scan;
    int lab = v.label[base + i * C + j];
    bool gnd = v.ground[base + i * C + j] == 1;
    kept = false; outl = false;
    if (lab > 0 || gnd) {
        if (lab == 999999) {
            outl = (i > v.cfg.ground_scan_ind && j % 5 == 0);
            return;
        }
        if (gnd && (j % 5 != 0 && j > 5 && j < C - 5)) return;
        kept = true;
    }
}

// block = 256 threads per (row, stream): final labels, then per-row kept /
// outlier counts
__global__ void k_ip_rowcount(DevView v) {
    const int s = blockIdx.y, i = blockIdx.x;
    const int C = v.cfg.horizon_scan;
    const size_t base = (size_t)s * v.H;
    int kc = 0, oc = 0;
    for (int j = threadIdx.x; j < C; j += blockDim.x) {
        const size_t o = base + (size_t)i * C + j;
        if (v.label[o] == 0) v.label[o] = final_label(v, base, o);
        bool k, ou;
        pixel_kind(v, base, i, j, k, ou);
        kc += k; oc += ou;
    }
    for (int o = 32; o > 0; o >>= 1) { kc += __shfl_xor(kc, o, 64); oc += __shfl_xor(oc, o, 64); }
    __shared__ int sk[16], so[16];
    if ((threadIdx.x & 63) == 0) { sk[threadIdx.x >> 6] = kc; so[threadIdx.x >> 6] = oc; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int a = 0, b = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { a += sk[w]; b += so[w]; }
        v.rowcnt[(size_t)s * v.cfg.n_scan * 2 + 2 * i] = a;
        v.rowcnt[(size_t)s * v.cfg.n_scan * 2 + 2 * i + 1] = b;
    }
}

// block = 256 threads per (row, stream): the row's kept and outlier pixels
// are appended in row-major order (cloudSegmentation, IP:319-355) after the
// rows before it.
__global__ void __launch_bounds__(256) k_ip_compact(DevView v) {
    const int s = blockIdx.y, i = blockIdx.x;
    const int C = v.cfg.horizon_scan, R = v.cfg.n_scan;
    const size_t base = (size_t)s * v.H;
    const int* rc = v.rowcnt + (size_t)s * R * 2;
    __shared__ int s_off[2], s_tot[2];
    __shared__ int s_red[4][4];
    {   // rows before i and all rows, kept / outlier
        int a = 0, b = 0, ta = 0, tb = 0;
        for (int r = threadIdx.x; r < R; r += blockDim.x) {
            const int x = rc[2 * r], y = rc[2 * r + 1];
            ta += x; tb += y;
            if (r < i) { a += x; b += y; }
        }
        for (int o = 32; o > 0; o >>= 1) {
            a += __shfl_xor(a, o, 64); b += __shfl_xor(b, o, 64);
            ta += __shfl_xor(ta, o, 64); tb += __shfl_xor(tb, o, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            const int w = threadIdx.x >> 6;
            s_red[w][0] = a; s_red[w][1] = b; s_red[w][2] = ta; s_red[w][3] = tb;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
                for (int c = 0; c < 4; ++c) s_red[0][c] += s_red[w][c];
            s_off[0] = s_red[0][0]; s_off[1] = s_red[0][1]; s_tot[0] = s_red[0][2]; s_tot[1] = s_red[0][3];
        }
    }
    // one pixel per thread per pass, in row order; positions by wave ballots
    // and a 4-wave scan
    __shared__ int s_wt[2][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long below = (1ull << lane) - 1;
    __syncthreads();
    int wk = s_off[0], wo = s_off[1];
    for (int j0 = 0; j0 < C; j0 += 256) {
        const int j = j0 + (int)threadIdx.x;
        bool k = false, o = false;
        if (j < C) pixel_kind(v, base, i, j, k, o);
        const unsigned long long mk = __ballot(k), mo = __ballot(o);
        if (lane == 0) { s_wt[0][w] = __popcll(mk); s_wt[1][w] = __popcll(mo); }
        __syncthreads();
        int pk = 0, po = 0, tk = 0, to = 0;
        for (int ww = 0; ww < 4; ++ww) {
            if (ww < w) { pk += s_wt[0][ww]; po += s_wt[1][ww]; }
            tk += s_wt[0][ww]; to += s_wt[1][ww];
        }
        const size_t px = base + (size_t)i * C + j;
        if (k) {
            const size_t d = base + wk + pk + __popcll(mk & below);
            v.seg[d] = v.full[px];
            v.seg_ground[d] = v.ground[px] == 1;
            v.seg_col[d] = (uint32_t)j;
            v.seg_range[d] = v.range[px];
        } else if (o) {
            v.outlier[base + wo + po + __popcll(mo & below)] = v.full[px];
        }
        wk += tk; wo += to;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        int* se = v.ring_se + (size_t)s * R * 2;
        se[2 * i] = s_off[0] - 1 + 5;
        se[2 * i + 1] = s_off[0] + rc[2 * i] - 1 - 5;
        if (i == 0) {
            StreamState& st = v.st[s];
            st.seg_count = s_tot[0];
            st.outlier_count = s_tot[1];
            st.first_half = INT_MAX;
            // findStartEndAngle (IP:199-209) on the first / last finite point
            int f0 = v.fl[2 * s], f1 = v.fl[2 * s + 1];
            float* orr = v.orient + 3 * s;
            if (f1 >= 0) {
                const float4* ip = v.io->pts + (size_t)s * v.P;
                float4 a = ip[f0], b = ip[f1];
                float so = -slo_libm::atan2f_(a.y, a.x);
                float eo = (float)(-slo_libm::atan2f_(b.y, b.x) + 2 * M_PI);
                if (eo - so > 3 * M_PI) eo = (float)(eo - 2 * M_PI);
                else if (eo - so < M_PI) eo = (float)(eo + 2 * M_PI);
                orr[0] = so; orr[1] = eo; orr[2] = eo - so;
            }
        }
    }
}

int ip_run(slo_ctx* ctx) {
    DevView& v = ctx->v;
    const int S = ctx->S;
    const int gi = (int)std::max<size_t>((S + 255) / 256, std::min<size_t>(4096, ((size_t)S * v.H / 4 + 255) / 256));
    SLO_LAUNCH(ctx, "ip_init", k_ip_init, dim3(gi), dim3(256), 0, v);
    const int T = 256;
    dim3 gp((v.P + IP_PTS_PER_WG - 1) / IP_PTS_PER_WG, S), gr(v.cfg.n_scan, S);
    SLO_LAUNCH(ctx, "ip_project", k_ip_project, gp, dim3(T), 0, v);
    const int ntiles = (v.cfg.horizon_scan + ip_tile_cols(v.cfg.n_scan) - 1) / ip_tile_cols(v.cfg.n_scan);
    SLO_LAUNCH(ctx, "ip_tile", k_ip_tile, dim3(ntiles, S), dim3(T), 0, v);
    SLO_LAUNCH(ctx, "ip_cc_merge", k_cc_merge, dim3((ntiles * v.cfg.n_scan + T - 1) / T, S), dim3(T), 0, v, ntiles);
    // slots for a tile's local roots (more go through device atomics): C5's
    // 128-row tiles hold ~1 200 at 4 096 pixels, ~600 at 2 048
    constexpr int kWide = IP_TILE_PX <= 2048 ? 768 : 1536;
    if (v.cfg.n_scan <= 64) SLO_LAUNCH(ctx, "ip_cc_stats", k_cc_stats<768>, dim3(ntiles, S), dim3(T), 0, v);
    else SLO_LAUNCH(ctx, "ip_cc_stats", k_cc_stats<kWide>, dim3(ntiles, S), dim3(T), 0, v);
    SLO_LAUNCH(ctx, "ip_rowcount", k_ip_rowcount, gr, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "ip_compact", k_ip_compact, gr, dim3(T), 0, v);
    SLO_CHECK(hipGetLastError());
    return 0;
}

}  // namespace slo
