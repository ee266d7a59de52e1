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
//     stale cloudSmoothness[4] entry of ring 0 (Q5), so ring 0 runs first and
//     rings 1..R-1 then run in parallel, one wavefront each.  The six sector
//     sorts of a ring run in six lanes with an exact restatement of
//     libstdc++'s introsort (slo_introsort.h, Q4/Q6); the greedy picks are
//     sequential per ring as in the reference.
//   per-ring VoxelGrid(0.2) (FA:778-782): one block per ring, bitonic sort
//     of (voxel idx, position) keys in LDS, centroid of each voxel summed in
//     position order (DESIGN.md "VoxelGrid order").
#include "slo_internal.h"
#include "slo_libm.h"
#include "slo_introsort.h"
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

// deskew + curvature + occlusion marks, one thread per position
__global__ void k_fa_points(DevView v) {
    const int s = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int S = v.st[s].seg_count;
    if (p >= S) return;
    const size_t base = (size_t)s * v.H;
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
        v.fpts[base + p] = make_float4(px, py, pz, (float)(int)q.w + v.cfg.scan_period * relTime);
    }
    const float* r = v.seg_range + base;
    const uint32_t* col = v.seg_col + base;
    // ---- calculateSmoothness
    const bool inner = p >= 5 && p < S - 5;
    if (inner) {
        float d = r[p - 5] + r[p - 4] + r[p - 3] + r[p - 2] + r[p - 1] - r[p] * 10 + r[p + 1] + r[p + 2] +
                  r[p + 3] + r[p + 4] + r[p + 5];
        float c = d * d;
        v.curv[base + p] = c;
        v.clabel[base + p] = 0;
        v.smooth[base + p] = Smooth{c, p};
    }
    // ---- markOccludedPoints (gather form); marks come from i in [5, S-7]
    int pk = inner ? 0 : v.picked[base + p];
    const int ilo = 5, ihi = S - 7;
    for (int i = max(ilo, p); i <= min(ihi, p + 5) && !pk; ++i) {  // case A marks [i-5, i]
        int cd = abs((int)(col[i + 1] - col[i]));
        if (cd < 10 && r[i] - r[i + 1] > 0.3) pk = 1;
    }
    for (int i = max(ilo, p - 6); i <= min(ihi, p - 1) && !pk; ++i) {  // case B marks [i+1, i+6]
        int cd = abs((int)(col[i + 1] - col[i]));
        if (cd < 10 && !(r[i] - r[i + 1] > 0.3) && r[i + 1] - r[i] > 0.3) pk = 1;
    }
    if (!pk && p >= ilo && p <= ihi) {
        float diff1 = fabsf((float)(r[p - 1] - r[p]));
        float diff2 = fabsf((float)(r[p + 1] - r[p]));
        if (diff1 > 0.02 * r[p] && diff2 > 0.02 * r[p]) pk = 1;
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

// one 64-lane block per (ring, stream); ring = ring0 + blockIdx.x
__global__ void __launch_bounds__(64) k_fa_extract(DevView v, int ring0) {
    const int s = blockIdx.y;
    const int ring = ring0 + blockIdx.x;
    const int R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    const size_t base = (size_t)s * v.H;
    const int S = v.st[s].seg_count;
    const int* se = v.ring_se + (size_t)s * R * 2;
    const int rs = se[2 * ring], re = se[2 * ring + 1];
    Smooth* sm = v.smooth + base;
    const int lane = threadIdx.x;
    // sector sorts (FA:693-699), lanes 0..5
    if (lane < 6) {
        int j = lane;
        int sp = (rs * (6 - j) + re * j) / 6;
        int ep = (rs * (5 - j) + re * (j + 1)) / 6 - 1;
        if (sp < ep) slo_sort::std_sort(sm + sp, ep - sp, SmoothLess());
    }
    __syncthreads();
    if (lane != 0) return;
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
        int sp = (rs * (6 - j) + re * j) / 6;
        int ep = (rs * (5 - j) + re * (j + 1)) / 6 - 1;
        if (sp >= ep) continue;
        int largestPickedNum = 0;
        for (int k = ep; k >= sp; k--) {
            int ind = sm[k].ind;
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
            int ind = sm[k].ind;
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

__global__ void __launch_bounds__(256) k_fa_ring_ds(DevView v) {
    const int s = blockIdx.y, ring = blockIdx.x;
    const int R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    const size_t rr = (size_t)s * R + ring;
    const int n = v.r_lf_n[rr];
    const float4* in = v.r_lf_scan + rr * C;
    float4* out = v.r_lf_ds + rr * C;
    __shared__ unsigned long long keys[SLO_DS_MAX];
    __shared__ float sh[64];
    __shared__ int scan[256];
    const float leaf = v.cfg.leaf_less_flat;
    const float inv = 1.0f / leaf;
    float mnx = FLT_MAX, mny = FLT_MAX, mnz = FLT_MAX, mxx = -FLT_MAX, mxy = -FLT_MAX, mxz = -FLT_MAX;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        float4 p = in[i];
        mnx = fminf(mnx, p.x); mny = fminf(mny, p.y); mnz = fminf(mnz, p.z);
        mxx = fmaxf(mxx, p.x); mxy = fmaxf(mxy, p.y); mxz = fmaxf(mxz, p.z);
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
    int npow = 1;
    while (npow < n) npow <<= 1;
    for (int i = threadIdx.x; i < npow; i += blockDim.x) {
        unsigned long long k = ~0ull;
        if (i < n) {
            float4 p = in[i];
            int ijk0 = (int)(floorf(p.x * inv) - (float)minbx);
            int ijk1 = (int)(floorf(p.y * inv) - (float)minby);
            int ijk2 = (int)(floorf(p.z * inv) - (float)minbz);
            unsigned int idx = (unsigned int)(ijk0 + ijk1 * mul1 + ijk2 * mul2);
            k = ((unsigned long long)idx << 32) | (unsigned int)i;
        }
        keys[i] = k;
    }
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

// concatenate per-ring outputs in ring order (one block per stream)
__global__ void k_fa_gather(DevView v) {
    const int s = blockIdx.x;
    const int R = v.cfg.n_scan, C = v.cfg.horizon_scan;
    __shared__ int off[4][129];
    const int* rc = v.ring_cnt + (size_t)s * R * 4;
    if (threadIdx.x < 4) {
        int a = 0;
        for (int r = 0; r < R; ++r) { off[threadIdx.x][r] = a; a += rc[4 * r + threadIdx.x]; }
        off[threadIdx.x][R] = a;
    }
    __syncthreads();
    // ring boundaries of less_sharp / less_flat (the odometry's ring windows)
    for (int r = threadIdx.x; r <= R; r += blockDim.x) {
        v.roff_cur[((size_t)s * 2 + 0) * (R + 1) + r] = off[1][r];
        v.roff_cur[((size_t)s * 2 + 1) * (R + 1) + r] = min(off[3][r], v.cap_less_flat);
    }
    StreamState& st = v.st[s];
    if (threadIdx.x == 0) {
        st.n_sharp = off[0][R]; st.n_less_sharp = off[1][R]; st.n_flat = off[2][R];
        st.n_less_flat = min(off[3][R], v.cap_less_flat);
    }
    for (int r = 0; r < R; ++r) {
        const size_t rr = (size_t)s * R + r;
        for (int i = threadIdx.x; i < rc[4 * r + 0]; i += blockDim.x)
            v.sharp[(size_t)s * v.cap_sharp + off[0][r] + i] = v.r_sharp[rr * 12 + i];
        for (int i = threadIdx.x; i < rc[4 * r + 1]; i += blockDim.x)
            v.less_sharp[(size_t)s * v.cap_less_sharp + off[1][r] + i] = v.r_less_sharp[rr * 120 + i];
        for (int i = threadIdx.x; i < rc[4 * r + 2]; i += blockDim.x)
            v.flat[(size_t)s * v.cap_flat + off[2][r] + i] = v.r_flat[rr * 24 + i];
        for (int i = threadIdx.x; i < rc[4 * r + 3]; i += blockDim.x)
            if (off[3][r] + i < v.cap_less_flat)
                v.less_flat[(size_t)s * v.cap_less_flat + off[3][r] + i] = v.r_lf_ds[rr * C + i];
    }
}

int fa_features_run(slo_ctx* ctx) {
    DevView& v = ctx->v;
    const int S = ctx->S, R = v.cfg.n_scan;
    const int T = 256;
    dim3 gh((v.H + T - 1) / T, S);
    SLO_LAUNCH(ctx, "fa_halfpass", k_fa_halfpass, gh, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "fa_points", k_fa_points, gh, dim3(T), 0, v);
    SLO_LAUNCH(ctx, "fa_extract_ring0", k_fa_extract, dim3(1, S), dim3(64), 0, v, 0);
    if (R > 1) SLO_LAUNCH(ctx, "fa_extract", k_fa_extract, dim3(R - 1, S), dim3(64), 0, v, 1);
    SLO_LAUNCH(ctx, "fa_ring_ds", k_fa_ring_ds, dim3(R, S), dim3(256), 0, v);
    SLO_LAUNCH(ctx, "fa_gather", k_fa_gather, dim3(S), dim3(256), 0, v);
    SLO_CHECK(hipGetLastError());
    return 0;
}

}  // namespace slo
