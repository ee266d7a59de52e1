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
#include "slo_scdist.h"
#include <float.h>

namespace slo {

// SPLIT (a context of a few streams, where one workgroup's ten candidate
// distances in a row are the detect's latency): the K-NN here, then
// k_sc_pairs (a workgroup per candidate) and k_sc_pick (the first minimum)
template <bool SPLIT>
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
    __shared__ ScPairLds pl;
    __shared__ double cdist[SC_K];
    __shared__ int calign[SC_K];
    if (tid == 0) {
        st.det_valid = 1;
        s_skip = 0;
        if (N < v.cfg.sc_num_exclude_recent + 1) {
            st.det_loop_id = -1; st.det_yaw = 0; st.det_min_dist = 10000000; st.det_nn_idx = 0;
            s_skip = 1;
        } else {
            atomicAdd(&v.wctr[0], (unsigned long long)K);   // K candidate distances follow
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
    if (SPLIT) {
        if (tid < K) st.det_cand[tid] = cands[tid];
        if (tid == 0) st.det_pending = 1;
        return;
    }
    const double* sc1 = v.sc_desc + (hb + N - 1) * NR * NS;
    const double* vk1 = v.sc_sect + (hb + N - 1) * NS;
    for (int c = 0; c < K; ++c) {
        const int ci = cands[c];
        sc_pair_distance(sc1, vk1, v.sc_desc + (hb + ci) * NR * NS, v.sc_sect + (hb + ci) * NS, NR, NS,
                         v.cfg.sc_search_ratio, pl, &cdist[c], &calign[c]);
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

// candidate c of stream s (grid K x S): distanceBtnScanContext into det_cdist / det_calign
__global__ void __launch_bounds__(256) k_sc_pairs(DevView v) {
    const int c = blockIdx.x, s = blockIdx.y;
    StreamState& st = v.st[s];
    if (!(st.kf_saved && st.det_pending)) return;
    __shared__ ScPairLds pl;
    const int NR = v.cfg.sc_num_ring, NS = v.cfg.sc_num_sector;
    const size_t hb = (size_t)s * v.KFMAX;
    const int N = st.sc_count, ci = st.det_cand[c];
    sc_pair_distance(v.sc_desc + (hb + N - 1) * NR * NS, v.sc_sect + (hb + N - 1) * NS, v.sc_desc + (hb + ci) * NR * NS,
                     v.sc_sect + (hb + ci) * NS, NR, NS, v.cfg.sc_search_ratio, pl, &st.det_cdist[c], &st.det_calign[c]);
}

// the first minimum over the K distances, in candidate order (as k_sc_detect)
__global__ void k_sc_pick(DevView v) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    StreamState& st = v.st[s];
    if (!(st.kf_saved && st.det_pending)) return;
    st.det_pending = 0;
    const int K = v.cfg.sc_num_candidates, NS = v.cfg.sc_num_sector;
    double min_dist = 10000000;
    int nn_align = 0, nn_idx = 0;
    for (int c = 0; c < K; ++c)
        if (st.det_cdist[c] < min_dist) { min_dist = st.det_cdist[c]; nn_align = st.det_calign[c]; nn_idx = st.det_cand[c]; }
    st.det_loop_id = min_dist < v.cfg.sc_dist_thres ? nn_idx : -1;
    float deg = (float)(nn_align * (360.0 / (double)NS));
    st.det_yaw = (float)(deg * M_PI / 180.0);
    st.det_min_dist = min_dist;
    st.det_nn_idx = nn_idx;
}

#ifndef SLO_SC_SPLIT_STREAMS
#define SLO_SC_SPLIT_STREAMS 8
#endif
int sc_detect_run(slo_ctx* ctx) {
    const int S = ctx->S, K = ctx->cfg.sc_num_candidates;
    if (S <= SLO_SC_SPLIT_STREAMS && K > 0) {
        SLO_LAUNCH(ctx, "sc_detect", k_sc_detect<true>, dim3(S), dim3(256), 0, ctx->v);
        SLO_LAUNCH(ctx, "sc_pairs", k_sc_pairs, dim3(K, S), dim3(256), 0, ctx->v);
        SLO_LAUNCH(ctx, "sc_pick", k_sc_pick, dim3((S + 63) / 64), dim3(64), 0, ctx->v);
    } else {
        SLO_LAUNCH(ctx, "sc_detect", k_sc_detect<false>, dim3(S), dim3(256), 0, ctx->v);
    }
    SLO_CHECK(hipGetLastError());
    return 0;
}

__global__ void k_sc_force(DevView v) { v.st[0].kf_saved = 1; }

// detectLoopClosureID on stream 0 only (single-scan API)
int sc_detect_run_one(slo_ctx* ctx) {
    SLO_LAUNCH(ctx, "sc_force", k_sc_force, dim3(1), dim3(1), 0, ctx->v);
    SLO_LAUNCH(ctx, "sc_detect", k_sc_detect<false>, dim3(1), dim3(256), 0, ctx->v);
    SLO_CHECK(hipGetLastError());
    return 0;
}

// Per-stream record shared across ranks by the RCCL all-gather (SURVEY §8(e)
// mode M; layout SLO_REC_* in include/slo_abi.h): poses, ids, this step's
// loop result, the newest ring key and, when a keyframe was saved, its
// descriptor as exact floats.  One workgroup per stream.
__global__ void __launch_bounds__(256) k_pack_records(DevView v, float* out) {
    const int s = blockIdx.x;
    const StreamState& st = v.st[s];
    float* o = out + (size_t)s * SLO_RECORD_FLOATS;
    const int NR = v.cfg.sc_num_ring, NS = v.cfg.sc_num_sector;
    const int kf = st.sc_count - 1;
    // a keyframe whose descriptor did not fit the history sends none (the
    // newest stored one is an older keyframe's)
    const bool saved = st.kf_saved && st.sc_wrote && kf >= 0;
    const double* d = saved ? v.sc_desc + ((size_t)s * v.KFMAX + kf) * NR * NS : nullptr;
    for (int i = threadIdx.x; i < SLO_SC_MAX_CELLS; i += blockDim.x)
        o[SLO_REC_DESC + i] = (saved && i < NR * NS) ? (float)d[i] : 0.0f;
    if (threadIdx.x != 0) return;
    for (int k = 0; k < 6; ++k) { o[SLO_REC_POSE + k] = st.transformSum[k]; o[SLO_REC_MAPPED + k] = st.transformAftMapped[k]; }
    o[SLO_REC_N_KEYFRAMES] = (float)st.n_keyframes;
    o[SLO_REC_KF_SAVED] = saved ? 1.0f : 0.0f;
    o[SLO_REC_LOOP_ID] = st.det_valid ? (float)st.det_loop_id : -2.0f;
    o[SLO_REC_MIN_DIST] = st.det_valid ? (float)st.det_min_dist : 0.0f;
    const float* rk = st.sc_count > 0 ? v.sc_ring + ((size_t)s * v.KFMAX + st.sc_count - 1) * NR : nullptr;
    for (int k = 0; k < 20; ++k) o[SLO_REC_RING_KEY + k] = (rk && k < NR) ? rk[k] : 0.0f;
    o[SLO_REC_SC_COUNT] = (float)st.sc_count;
    o[SLO_REC_ERR] = (float)st.err;
    o[SLO_REC_KF_INDEX] = saved ? (float)kf : -1.0f;
    o[SLO_REC_YAW] = st.det_valid ? st.det_yaw : 0.0f;
}

int pack_records_run(slo_ctx* ctx, float* d_out) {
    SLO_LAUNCH(ctx, "pack_records", k_pack_records, dim3(ctx->S), dim3(256), 0, ctx->v, d_out);
    SLO_CHECK(hipGetLastError());
    return 0;
}

}  // namespace slo
