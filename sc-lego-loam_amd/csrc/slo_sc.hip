// slo_sc.hip — SCManager::detectLoopClosureID (Scancontext.cpp:247-338) for
// every stream that saved a keyframe this scan.
//
// One workgroup per stream.  The ring-key "tree" is a snapshot of the first
// N-50 ring keys refreshed every 10th query (Scancontext.cpp:264-276, Q12c);
// the 10-NN over it is exact: every lane keeps a sorted top-10 of its strided
// share by (float L2 in nanoflann's 4-unrolled order, index), and the lists
// are merged pairwise in log2(256) rounds.  Unfilled slots stay 0 as in the
// reference.  For each candidate the 60 sector-key shifts run on 60 lanes,
// the 7 window shifts x 60 column cosines on the whole workgroup, and the
// per-shift sums run in column order, so every f64 value is the reference's
// (Eigen SSE2 reduction order, Q12d).
#include "slo_internal.h"
#include <float.h>

namespace slo {

struct Cand { float d; int i; };

__device__ inline bool cand_less(const Cand& a, const Cand& b) { return a.d < b.d || (a.d == b.d && a.i < b.i); }

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

#define SC_K SLO_SC_MAX_K
#define SC_NS SLO_SC_MAX_SECTOR

__device__ inline unsigned long long wave_min_u64(unsigned long long x) {
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(x, o, 64);
        x = y < x ? y : x;
    }
    return x;
}

__global__ void __launch_bounds__(256) k_sc_detect(DevView v) {
    const int s = blockIdx.x;
    StreamState& st = v.st[s];
    const int tid = threadIdx.x;
    if (!st.kf_saved) {
        if (tid == 0) st.det_valid = 0;
        return;
    }
    const int NR = v.cfg.sc_num_ring, NS = v.cfg.sc_num_sector, K = v.cfg.sc_num_candidates;
    const int N = st.sc_count;
    __shared__ int s_treen, s_skip;
    __shared__ unsigned long long keys[SLO_KFMAX];   // (f32 L2 bits << 32 | index) of the snapshot
    __shared__ unsigned long long wmin[4];
    __shared__ int cands[SC_K];
    __shared__ double sim[7 * SC_NS];
    __shared__ int simok[7 * SC_NS];
    __shared__ double dist7[7];
    __shared__ double shnorm[SC_NS];
    __shared__ int shifts[7];
    __shared__ double cdist[SC_K];
    __shared__ int calign[SC_K];
    if (tid == 0) {
        st.det_valid = 1;
        s_skip = 0;
        if (N < v.cfg.sc_num_exclude_recent + 1) {
            st.det_loop_id = -1; st.det_yaw = 0; st.det_min_dist = 10000000; st.det_nn_idx = 0;
            s_skip = 1;
        } else {
            if (st.sc_counter % v.cfg.sc_tree_making_period == 0) st.sc_tree_n = N - v.cfg.sc_num_exclude_recent;
            st.sc_counter = st.sc_counter + 1;
            s_treen = st.sc_tree_n;
        }
    }
    __syncthreads();
    if (s_skip) return;
    const size_t hb = (size_t)s * v.KFMAX;
    const float* q = v.sc_ring + (hb + N - 1) * NR;
    // ---- exact K-NN over the snapshot: distances once into LDS as
    // order-preserving (distance, index) keys (L2 >= 0, so the float bits sort
    // like the values), then K rounds of block-wide "smallest key above the
    // previous pick".  Ties resolve to the lower index; slots beyond the
    // snapshot size stay 0, as with the reference's zero-initialised
    // candidate_indexes (SCc:282).
    const int n = s_treen;
    for (int j = tid; j < n; j += blockDim.x)
        keys[j] = ((unsigned long long)__float_as_uint(l2_nf(q, v.sc_ring + (hb + j) * NR, NR)) << 32) |
                  (unsigned int)j;
    __syncthreads();
    unsigned long long prev = 0;
    for (int k = 0; k < K; ++k) {
        unsigned long long best = ~0ull;
        for (int j = tid; j < n; j += blockDim.x) {
            const unsigned long long x = keys[j];
            if ((k == 0 || x > prev) && x < best) best = x;
        }
        best = wave_min_u64(best);
        if ((tid & 63) == 0) wmin[tid >> 6] = best;
        __syncthreads();
        best = wmin[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) best = wmin[w] < best ? wmin[w] : best;
        if (tid == 0) cands[k] = best == ~0ull ? 0 : (int)(best & 0xffffffffu);
        prev = best;
        __syncthreads();
    }
    const double* sc1 = v.sc_desc + (hb + N - 1) * NR * NS;
    const double* vk1 = v.sc_sect + (hb + N - 1) * NS;
    for (int c = 0; c < K; ++c) {
        const int ci = cands[c];
        const double* sc2 = v.sc_desc + (hb + ci) * NR * NS;
        const double* vk2 = v.sc_sect + (hb + ci) * NS;
        // fastAlignUsingVkey: 60 shifts on 60 lanes
        if (tid < NS) {
            ESum e;
            for (int j = 0; j < NS; ++j) {
                double d = vk1[j] - vk2[((j - tid) % NS + NS) % NS];
                e.add(d * d);
            }
            shnorm[tid] = sqrt(e.get());
        }
        __syncthreads();
        if (tid == 0) {
            int argmin = 0;
            double mn = 10000000;
            for (int sh = 0; sh < NS; ++sh)
                if (shnorm[sh] < mn) { argmin = sh; mn = shnorm[sh]; }
            const int R = (int)round(0.5 * v.cfg.sc_search_ratio * NS);
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
            for (int k = 0; k < 7; ++k) shifts[k] = k < n ? sp[k] : -1;
        }
        __syncthreads();
        // column cosines for the 7 shifts
        for (int t = tid; t < 7 * NS; t += blockDim.x) {
            const int k = t / NS, j = t - k * NS;
            const int sh = shifts[k];
            simok[t] = 0;
            if (sh < 0) continue;
            const int j2 = ((j - sh) % NS + NS) % NS;
            ESum n1, n2, dt;
            for (int r = 0; r < NR; ++r) {
                double a = sc1[r * NS + j], b = sc2[r * NS + j2];
                n1.add(a * a); n2.add(b * b); dt.add(a * b);
            }
            double nn1 = sqrt(n1.get()), nn2 = sqrt(n2.get());
            if ((nn1 == 0) | (nn2 == 0)) continue;
            sim[t] = dt.get() / (nn1 * nn2);
            simok[t] = 1;
        }
        __syncthreads();
        if (tid < 7) {
            double sum = 0;
            int ne = 0;
            for (int j = 0; j < NS; ++j)
                if (simok[tid * NS + j]) { sum = sum + sim[tid * NS + j]; ne = ne + 1; }
            dist7[tid] = shifts[tid] < 0 ? 10000000 : 1.0 - sum / ne;
        }
        __syncthreads();
        if (tid == 0) {
            int am = 0;
            double md = 10000000;
            for (int k = 0; k < 7; ++k)
                if (shifts[k] >= 0 && dist7[k] < md) { am = shifts[k]; md = dist7[k]; }
            cdist[c] = md;
            calign[c] = am;
        }
        __syncthreads();
    }
    if (tid == 0) {
        double min_dist = 10000000;
        int nn_align = 0, nn_idx = 0;
        for (int c = 0; c < K; ++c)
            if (cdist[c] < min_dist) { min_dist = cdist[c]; nn_align = calign[c]; nn_idx = cands[c]; }
        st.det_loop_id = min_dist < v.cfg.sc_dist_thres ? nn_idx : -1;
        float deg = (float)(nn_align * (360.0 / (double)NS));
        st.det_yaw = (float)(deg * M_PI / 180.0);
        st.det_min_dist = min_dist;
        st.det_nn_idx = nn_idx;
        for (int c = 0; c < K; ++c) st.det_cand[c] = cands[c];
    }
}

int sc_detect_run(slo_ctx* ctx) {
    SLO_LAUNCH(ctx, "sc_detect", k_sc_detect, dim3(ctx->S), dim3(256), 0, ctx->v);
    SLO_CHECK(hipGetLastError());
    return 0;
}

__global__ void k_sc_force(DevView v) { v.st[0].kf_saved = 1; }

// detectLoopClosureID on stream 0 only (single-scan API)
int sc_detect_run_one(slo_ctx* ctx) {
    SLO_LAUNCH(ctx, "sc_force", k_sc_force, dim3(1), dim3(1), 0, ctx->v);
    SLO_LAUNCH(ctx, "sc_detect", k_sc_detect, dim3(1), dim3(256), 0, ctx->v);
    SLO_CHECK(hipGetLastError());
    return 0;
}

// Per-stream record shared across ranks by the RCCL all-gather (SURVEY §8(e)
// mode M): odometry pose, mapped pose, keyframe count, loop result and the
// newest ring key.  40 floats = 160 B per stream.
__global__ void k_pack_records(DevView v, float* out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    const StreamState& st = v.st[s];
    float* o = out + (size_t)s * SLO_RECORD_FLOATS;
    for (int k = 0; k < 6; ++k) { o[k] = st.transformSum[k]; o[6 + k] = st.transformAftMapped[k]; }
    o[12] = (float)st.n_keyframes;
    o[13] = (float)st.kf_saved;
    o[14] = st.det_valid ? (float)st.det_loop_id : -2.0f;
    o[15] = st.det_valid ? (float)st.det_min_dist : 0.0f;
    const int NR = v.cfg.sc_num_ring;
    const float* rk = st.sc_count > 0 ? v.sc_ring + ((size_t)s * v.KFMAX + st.sc_count - 1) * NR : nullptr;
    for (int k = 0; k < 20; ++k) o[16 + k] = (rk && k < NR) ? rk[k] : 0.0f;
    o[36] = (float)st.sc_count; o[37] = (float)st.err; o[38] = 0; o[39] = 0;
}

int pack_records_run(slo_ctx* ctx, float* d_out) {
    SLO_LAUNCH(ctx, "pack_records", k_pack_records, dim3((ctx->S + 63) / 64), dim3(64), 0, ctx->v, d_out);
    SLO_CHECK(hipGetLastError());
    return 0;
}

}  // namespace slo
