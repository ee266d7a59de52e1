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

// row / column of a finite point (IP:229-246); returns false if rejected
__device__ inline bool project_point(const slo_config& c, float4 p, int& row, int& col, float& range) {
    float verticalAngle = (float)((double)(slo_libm::atan2f_(p.z, sqrtf(p.x * p.x + p.y * p.y)) * 180) / M_PI);
    float rowf = (verticalAngle + c.ang_bottom) / c.ang_res_y;
    long long r = (long long)rowf;  // Q1: truncation; (-1,0) -> 0
    if (r < 0 || r >= c.n_scan) return false;
    float horizonAngle = (float)((double)(slo_libm::atan2f_(p.x, p.y) * 180) / M_PI);
    double colD = -round(((double)horizonAngle - 90.0) / (double)c.ang_res_x) + (double)(c.horizon_scan / 2);
    long long cc = (long long)colD;
    if (cc >= c.horizon_scan) cc -= c.horizon_scan;
    if (cc < 0 || cc >= c.horizon_scan) return false;
    float rg = sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);
    if (rg < c.sensor_minimum_range) return false;
    row = (int)r; col = (int)cc; range = rg;
    return true;
}

__global__ void k_ip_init(DevView v) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    v.fl[2 * s] = INT_MAX;
    v.fl[2 * s + 1] = -1;
}

// A workgroup takes IP_PTS_PER_WG consecutive points (thread t: points t,
// t+256, ...).  Points arrive in firing order — all rings of one azimuth, then
// the next — so the workgroup's owner atomics keep hitting the same few
// cache lines (one per ring over ~IP_PTS_PER_WG/R columns) while they are
// resident in L2, instead of touching every line once per point.
#define IP_PTS_PER_WG 2048
__global__ void k_ip_project(DevView v) {
    const int s = blockIdx.y;
    const int n = v.npts[s];
    int fmin = INT_MAX, fmax = -1;
    for (int k = 0; k < IP_PTS_PER_WG / 256; ++k) {
        const int i = blockIdx.x * IP_PTS_PER_WG + k * 256 + threadIdx.x;
        if (i >= n) break;
        float4 p = v.pts[(size_t)s * v.P + i];
        if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
            fmin = min(fmin, i); fmax = max(fmax, i);
            int row, col; float rg;
            if (project_point(v.cfg, p, row, col, rg))
                atomicMax(&v.owner[(size_t)s * v.H + row * v.cfg.horizon_scan + col], i);
        }
    }
    fmin = wave_min(fmin); fmax = wave_max(fmax);
    if ((threadIdx.x & 63) == 0) {
        if (fmin != INT_MAX) atomicMin(&v.fl[2 * s], fmin);
        if (fmax >= 0) atomicMax(&v.fl[2 * s + 1], fmax);
    }
}

// pair test of rows (i, i+1) at column j: -1 invalid, 1 ground, 0 not ground
__device__ inline int ground_pair(const DevView& v, int s, int i, int j) {
    const int C = v.cfg.horizon_scan;
    int lo = v.owner[(size_t)s * v.H + i * C + j];
    int up = v.owner[(size_t)s * v.H + (i + 1) * C + j];
    if (lo < 0 || up < 0) return -1;
    float4 a = v.pts[(size_t)s * v.P + lo], b = v.pts[(size_t)s * v.P + up];
    float dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
    float angle = (float)((double)(slo_libm::atan2f_(dz, sqrtf(dx * dx + dy * dy)) * 180) / M_PI);
    return fabsf(angle - v.cfg.sensor_mount_angle) <= 10 ? 1 : 0;
}

__global__ void k_ip_image(DevView v) {
    const int s = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= v.H) return;
    const int C = v.cfg.horizon_scan;
    const int i = p / C, j = p - i * C;
    const size_t o = (size_t)s * v.H + p;
    int own = v.owner[o];
    float rg = FLT_MAX;
    float4 f;
    if (own >= 0) {
        float4 q = v.pts[(size_t)s * v.P + own];
        rg = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z);
        f = make_float4(q.x, q.y, q.z, (float)((double)(float)i + (double)(float)j / 10000.0));
    } else {
        float qn = __builtin_nanf("");
        f = make_float4(qn, qn, qn, -1.0f);
    }
    v.range[o] = rg;
    v.full[o] = f;
    // Q15: final groundMat value of row i
    int g = 0;
    const int gsi = v.cfg.ground_scan_ind;
    if (i <= gsi) {
        int pi_ = (i < gsi) ? ground_pair(v, s, i, j) : 0;
        int pm = (i >= 1 && i - 1 < gsi) ? ground_pair(v, s, i - 1, j) : 0;
        if (i < gsi && pi_ == -1) g = -1;
        else if (pi_ == 1 || pm == 1) g = 1;
    }
    v.ground[o] = (int8_t)g;
    int lab = (g == 1 || rg == FLT_MAX) ? -1 : 0;
    v.label[o] = lab;
    v.parent[o] = lab == 0 ? p : -1;
    v.csize[o] = 0;
    v.crows[2 * o] = 0ull;
    v.crows[2 * o + 1] = 0ull;
}

__device__ inline int ld_parent(int* a, int x) {
    return __hip_atomic_load(&a[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline int find_root(int* par, int x) {
    int y = ld_parent(par, x);
    while (y != x) { x = y; y = ld_parent(par, x); }
    return x;
}
__device__ inline void unite(int* par, int a, int b) {
    while (true) {
        a = find_root(par, a);
        b = find_root(par, b);
        if (a == b) return;
        if (a < b) { int t = a; a = b; b = t; }
        int old = atomicCAS(&par[a], a, b);
        if (old == a) return;
        a = old;
    }
}

// edge predicate of labelComponents (IP:411-423)
__device__ inline bool seg_edge(const slo_config& c, float r1, float r2, bool horizontal) {
    float d1 = fmaxf(r1, r2), d2 = fminf(r1, r2);
    float sa = horizontal ? c.sin_alpha_x : c.sin_alpha_y;
    float ca = horizontal ? c.cos_alpha_x : c.cos_alpha_y;
    float angle = slo_libm::atan2f_(d2 * sa, (d1 - d2 * ca));
    return angle > c.segment_theta;
}

__global__ void k_cc_union(DevView v) {
    const int s = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= v.H) return;
    const int C = v.cfg.horizon_scan, R = v.cfg.n_scan;
    const size_t base = (size_t)s * v.H;
    if (v.label[base + p] != 0) return;
    const int i = p / C, j = p - i * C;
    int* par = v.parent + base;
    const float rp = v.range[base + p];
    int q = i * C + (j + 1 == C ? 0 : j + 1);  // right neighbour (column wrap, IP:403-406)
    if (v.label[base + q] == 0 && seg_edge(v.cfg, rp, v.range[base + q], true)) unite(par, p, q);
    if (i + 1 < R) {
        q = p + C;                              // next row
        if (v.label[base + q] == 0 && seg_edge(v.cfg, rp, v.range[base + q], false)) unite(par, p, q);
    }
}

// Component size and row set (seed excluded, Q3).  Large components put
// thousands of pixels on one root, so the lanes of a wave that share a root
// are combined first (one atomic per distinct root per wave).
__global__ void k_cc_stats(DevView v) {
    const int s = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t base = (size_t)s * v.H;
    int* par = v.parent + base;
    int r = -1;
    unsigned long long rows0 = 0, rows1 = 0;
    if (p < v.H && par[p] >= 0) {
        r = p;
        int y = par[r];
        while (y != r) { r = y; y = par[r]; }
        par[p] = r;
        if (p != r) {
            const int row = p / v.cfg.horizon_scan;
            (row >> 6 ? rows1 : rows0) = 1ull << (row & 63);
        }
    }
    unsigned long long pending = __ballot(r >= 0);
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const int lr = __shfl(r, leader, 64);
        const bool mine = r == lr;
        const unsigned long long grp = __ballot(mine);
        unsigned long long a = mine ? rows0 : 0ull, b = mine ? rows1 : 0ull;
        for (int o = 32; o > 0; o >>= 1) { a |= __shfl_xor(a, o, 64); b |= __shfl_xor(b, o, 64); }
        if ((int)(threadIdx.x & 63) == leader) {
            atomicAdd(&v.csize[base + lr], __popcll(grp));
            if (a) atomicOr(&v.crows[2 * (base + lr)], a);
            if (b) atomicOr(&v.crows[2 * (base + lr) + 1], b);
        }
        pending &= ~grp;
    }
}

__global__ void k_cc_label(DevView v) {
    const int s = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= v.H) return;
    const size_t base = (size_t)s * v.H;
    int r = v.parent[base + p];
    if (r < 0) return;
    int size = v.csize[base + r];
    bool feasible = false;
    if (size >= 30) feasible = true;
    else if (size >= v.cfg.segment_valid_point_num) {
        int lines = __popcll(v.crows[2 * (base + r)]) + __popcll(v.crows[2 * (base + r) + 1]);
        if (lines >= v.cfg.segment_valid_line_num) feasible = true;
    }
    // feasible segments keep a positive label (the reference numbers them by
    // seed order; the number is only used by the visualisation cloud IP:363)
    v.label[base + p] = feasible ? r + 1 : 999999;
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

// block = 256 threads per (row, stream): per-row kept / outlier counts
__global__ void k_ip_rowcount(DevView v) {
    const int s = blockIdx.y, i = blockIdx.x;
    const int C = v.cfg.horizon_scan;
    const size_t base = (size_t)s * v.H;
    int kc = 0, oc = 0;
    for (int j = threadIdx.x; j < C; j += blockDim.x) {
        bool k, o;
        pixel_kind(v, base, i, j, k, o);
        kc += k; oc += o;
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

// block = 256 threads per (row, stream); thread t owns a contiguous chunk of
// the row so a block scan keeps row-major order.
__global__ void k_ip_compact(DevView v) {
    const int s = blockIdx.y, i = blockIdx.x;
    const int C = v.cfg.horizon_scan, R = v.cfg.n_scan;
    const size_t base = (size_t)s * v.H;
    const int* rc = v.rowcnt + (size_t)s * R * 2;
    __shared__ int s_off[2], s_tot[2];
    __shared__ int sc_k[256], sc_o[256];
    if (threadIdx.x == 0) {
        int a = 0, b = 0, ta = 0, tb = 0;
        for (int r = 0; r < R; ++r) {
            if (r < i) { a += rc[2 * r]; b += rc[2 * r + 1]; }
            ta += rc[2 * r]; tb += rc[2 * r + 1];
        }
        s_off[0] = a; s_off[1] = b; s_tot[0] = ta; s_tot[1] = tb;
    }
    const int T = blockDim.x;
    const int chunk = (C + T - 1) / T;
    const int j0 = threadIdx.x * chunk, j1 = min(C, j0 + chunk);
    int kc = 0, oc = 0;
    for (int j = j0; j < j1; ++j) { bool k, o; pixel_kind(v, base, i, j, k, o); kc += k; oc += o; }
    sc_k[threadIdx.x] = kc; sc_o[threadIdx.x] = oc;
    __syncthreads();
    // inclusive scan (Hillis-Steele) over 256 entries
    for (int d = 1; d < T; d <<= 1) {
        int a = threadIdx.x >= d ? sc_k[threadIdx.x - d] : 0;
        int b = threadIdx.x >= d ? sc_o[threadIdx.x - d] : 0;
        __syncthreads();
        sc_k[threadIdx.x] += a; sc_o[threadIdx.x] += b;
        __syncthreads();
    }
    int wk = s_off[0] + sc_k[threadIdx.x] - kc;
    int wo = s_off[1] + sc_o[threadIdx.x] - oc;
    for (int j = j0; j < j1; ++j) {
        bool k, o;
        pixel_kind(v, base, i, j, k, o);
        const size_t px = base + i * C + j;
        if (k) {
            const size_t d = base + wk;
            v.seg[d] = v.full[px];
            v.seg_ground[d] = v.ground[px] == 1;
            v.seg_col[d] = (uint32_t)j;
            v.seg_range[d] = v.range[px];
            ++wk;
        } else if (o) {
            v.outlier[base + wo] = v.full[px];
            ++wo;
        }
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
                float4 a = v.pts[(size_t)s * v.P + f0], b = v.pts[(size_t)s * v.P + f1];
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
    SLO_CHECK(hipMemsetAsync(v.owner, 0xff, sizeof(int32_t) * (size_t)S * v.H, ctx->stream));
    SLO_LAUNCH(ctx, "ip_init", k_ip_init, dim3((S + 63) / 64), dim3(64), 0, v);
    const int T = 256;
    dim3 gp((v.P + IP_PTS_PER_WG - 1) / IP_PTS_PER_WG, S), gh((v.H + T - 1) / T, S), gr(v.cfg.n_scan, S);
    SLO_LAUNCH(ctx, "ip_project", k_ip_project, gp, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "ip_image", k_ip_image, gh, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "ip_cc_union", k_cc_union, gh, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "ip_cc_stats", k_cc_stats, gh, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "ip_cc_label", k_cc_label, gh, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "ip_rowcount", k_ip_rowcount, gr, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "ip_compact", k_ip_compact, gr, dim3(T), 0, v);
    SLO_CHECK(hipGetLastError());
    return 0;
}

}  // namespace slo
