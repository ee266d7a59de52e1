// slo_xsc.hip — cross-stream (multi-session) Scan Context candidates over the
// all-gathered per-stream records.
//
// Every rank all-gathers one record per stream per step (slo_pack_records:
// poses, ids and — when the stream saved a keyframe — its 20 x 60 Scan
// Context descriptor as exact floats), so every rank can hold every stream's
// descriptor history.  slo_xsc_ingest appends the new descriptors to a
// per-stream ring of `cap` entries and derives their ring / sector keys
// (SCc:198-227, Eigen reduction order); slo_xsc_query answers, for each of
// the caller's own records that carries a new keyframe, detectLoopClosureID
// (SCc:247-338) against the OTHER streams' histories: the K nearest ring keys
// (float L2 in nanoflann's order, exact; ties to the lower entry code
// stream * cap + slot), distanceBtnScanContext for each, the first minimum,
// accepted below SC_DIST_THRES.  The reference is single-session; this is the
// multi-session use of its own detector that the record exchange serves.
//
// Device layout per store: desc f64 [N][cap][NR*NS], sector keys f64
// [N][cap][NS], ring keys f32 [N][cap][NR], keyframe index [N][cap], count
// [N].  One workgroup per record in both kernels.
#include "slo_internal.h"
#include "slo_scdist.h"
#include "../../include/slo_abi.h"
#include <float.h>
#include <new>

struct slo_xsc {
    slo_config cfg;
    int dev = 0, N = 0, cap = 0, NR = 0, NS = 0;
    double* desc = nullptr;
    double* sect = nullptr;
    float* ring = nullptr;
    int32_t* kfi = nullptr;
    int32_t* cnt = nullptr;
};

namespace slo {

#define XSC_KMAX 16   // candidates per query (NUM_CANDIDATES_FROM_TREE = 10)

struct XscView {
    int N, cap, NR, NS, K;
    double thres, ratio;
    double* desc;
    double* sect;
    float* ring;
    int32_t* kfi;
    int32_t* cnt;
};

// the descriptor of a record (floats, exact) and its ring / sector keys
__device__ inline void xsc_keys(const XscView& x, const float* rec, double* desc, double* sect, float* ringf) {
    const int NR = x.NR, NS = x.NS;
    for (int i = threadIdx.x; i < NR * NS; i += blockDim.x) desc[i] = (double)rec[SLO_REC_DESC + i];
    __syncthreads();
    if (threadIdx.x < NR) {
        ringf[threadIdx.x] = (float)(eigen_sum(desc + threadIdx.x * NS, NS, 1) / (double)NS);
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + NS) {
        const int c = threadIdx.x - 64;
        sect[c] = eigen_sum(desc + c, NR, NS) / (double)NR;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(256) k_xsc_ingest(XscView x, const float* recs, int n) {
    const int r = blockIdx.x;
    const float* rec = recs + (size_t)r * SLO_RECORD_FLOATS;
    if (rec[SLO_REC_KF_SAVED] == 0.0f || rec[SLO_REC_KF_INDEX] < 0.0f) return;
    const size_t slot = (size_t)r * x.cap + (size_t)(x.cnt[r] % x.cap);
    const int NR = x.NR, NS = x.NS;
    double* d = x.desc + slot * NR * NS;
    __shared__ float ringf[64];
    xsc_keys(x, rec, d, x.sect + slot * NS, ringf);
    if (threadIdx.x < NR) x.ring[slot * NR + threadIdx.x] = ringf[threadIdx.x];
    if (threadIdx.x == 0) {
        x.kfi[slot] = (int32_t)rec[SLO_REC_KF_INDEX];
        x.cnt[r] = x.cnt[r] + 1;
    }
}

// sorted insert of (d, code) into a register-resident top-K list
__device__ inline void topk_insert(unsigned long long key, unsigned long long (&L)[XSC_KMAX], int K) {
    if (key >= L[K - 1]) return;
    bool placed = false;
#pragma unroll
    for (int k = XSC_KMAX - 1; k >= 1; --k) {
        if (k < K && !placed) {
            if (key < L[k - 1]) L[k] = L[k - 1];
            else { L[k] = key; placed = true; }
        }
    }
    if (!placed) L[0] = key;
}

__global__ void __launch_bounds__(256) k_xsc_query(XscView x, const float* recs, int nq, int global0,
                                                   slo_xsc_match* out) {
    const int q = blockIdx.x, tid = threadIdx.x;
    const float* rec = recs + (size_t)q * SLO_RECORD_FLOATS;
    slo_xsc_match* o = out + q;
    if (rec[SLO_REC_KF_SAVED] == 0.0f || rec[SLO_REC_KF_INDEX] < 0.0f) {
        if (tid == 0) { *o = slo_xsc_match{}; o->nn_stream = -1; o->nn_keyframe = -1; }
        return;
    }
    const int self = global0 + q, NR = x.NR, NS = x.NS, K = x.K;
    __shared__ double qdesc[SLO_SC_MAX_CELLS];
    __shared__ double qsect[SC_NS];
    __shared__ float qring[64];
    __shared__ unsigned long long wmin[4];
    __shared__ unsigned long long cand[XSC_KMAX];
    __shared__ ScPairLds pl;
    __shared__ double cdist[XSC_KMAX];
    __shared__ int calign[XSC_KMAX];
    xsc_keys(x, rec, qdesc, qsect, qring);
    // ---- exact K-NN over every other stream's history
    unsigned long long L[XSC_KMAX];
#pragma unroll
    for (int k = 0; k < XSC_KMAX; ++k) L[k] = ~0ull;
    const long long total = (long long)x.N * x.cap;
    for (long long e = tid; e < total; e += blockDim.x) {
        const int t = (int)(e / x.cap), j = (int)(e - (long long)t * x.cap);
        if (t == self || j >= min(x.cnt[t], x.cap)) continue;
        const float d = l2_nf(qring, x.ring + (size_t)e * NR, NR);
        topk_insert(((unsigned long long)__float_as_uint(d) << 32) | (unsigned int)e, L, K);
    }
    // K rounds of block-wide minimum over the lists' heads
    int head = 0;
    for (int k = 0; k < K; ++k) {
        unsigned long long b = head < K ? L[0] : ~0ull;
        const unsigned long long mine = b;
        b = wave_min_u64(b);
        if ((tid & 63) == 0) wmin[tid >> 6] = b;
        __syncthreads();
        b = wmin[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) b = wmin[w] < b ? wmin[w] : b;
        if (tid == 0) cand[k] = b;
        if (mine == b && b != ~0ull) {   // the winner pops its head (codes are unique)
#pragma unroll
            for (int i = 0; i < XSC_KMAX - 1; ++i) L[i] = L[i + 1];
            L[XSC_KMAX - 1] = ~0ull;
            ++head;
        }
        __syncthreads();
    }
    int nc = 0;
    for (int k = 0; k < K; ++k) nc += cand[k] != ~0ull;
    for (int c = 0; c < nc; ++c) {
        const size_t e = (size_t)(cand[c] & 0xffffffffu);
        sc_pair_distance(qdesc, qsect, x.desc + e * NR * NS, x.sect + e * NS, NR, NS, x.ratio, pl, &cdist[c],
                         &calign[c]);
    }
    if (tid == 0) {
        double md = 10000000;
        int am = 0, bc = -1;
        for (int c = 0; c < nc; ++c)
            if (cdist[c] < md) { md = cdist[c]; am = calign[c]; bc = c; }
        slo_xsc_match m{};
        m.n_cand = nc;
        m.nn_stream = -1;
        m.nn_keyframe = -1;
        m.min_dist = md;
        if (bc >= 0) {
            const size_t e = (size_t)(cand[bc] & 0xffffffffu);
            m.nn_stream = (int32_t)(e / x.cap);
            m.nn_keyframe = x.kfi[e];
            m.loop = md < x.thres ? 1 : 0;
            m.yaw = (float)((float)(am * (360.0 / (double)NS)) * M_PI / 180.0);
        }
        m.valid = 1;
        *o = m;
    }
}

XscView xsc_view(const slo_xsc* g) {
    XscView x;
    x.N = g->N; x.cap = g->cap; x.NR = g->NR; x.NS = g->NS; x.K = g->cfg.sc_num_candidates;
    x.thres = g->cfg.sc_dist_thres; x.ratio = g->cfg.sc_search_ratio;
    x.desc = g->desc; x.sect = g->sect; x.ring = g->ring; x.kfi = g->kfi; x.cnt = g->cnt;
    return x;
}

}  // namespace slo

extern "C" {

int slo_xsc_create(const slo_config* cfg, int hip_device, int n_streams, int cap, slo_xsc** out) {
    if (!cfg || !out || n_streams <= 0 || cap <= 0 || cfg->sc_num_ring < 1 || cfg->sc_num_ring > 64 ||
        cfg->sc_num_sector < 1 || cfg->sc_num_sector > SLO_SC_MAX_SECTOR ||
        cfg->sc_num_ring * cfg->sc_num_sector > SLO_SC_MAX_CELLS || cfg->sc_num_candidates < 1 ||
        cfg->sc_num_candidates > XSC_KMAX || (long long)n_streams * cap >= (1LL << 32))
        return SLO_E_ARG;
    *out = nullptr;
    slo_xsc* g = new (std::nothrow) slo_xsc();
    if (!g) return SLO_E_CAPACITY;
    g->cfg = *cfg;
    g->dev = hip_device;
    g->N = n_streams;
    g->cap = cap;
    g->NR = cfg->sc_num_ring;
    g->NS = cfg->sc_num_sector;
    const size_t E = (size_t)n_streams * cap;
    if (hipSetDevice(hip_device) != hipSuccess || hipMalloc(&g->desc, E * g->NR * g->NS * 8) != hipSuccess ||
        hipMalloc(&g->sect, E * g->NS * 8) != hipSuccess || hipMalloc(&g->ring, E * g->NR * 4) != hipSuccess ||
        hipMalloc(&g->kfi, E * 4) != hipSuccess || hipMalloc(&g->cnt, (size_t)n_streams * 4) != hipSuccess ||
        hipMemset(g->cnt, 0, (size_t)n_streams * 4) != hipSuccess) {
        slo_xsc_destroy(g);
        return SLO_E_HIP;
    }
    *out = g;
    return SLO_OK;
}

void slo_xsc_destroy(slo_xsc* g) {
    if (!g) return;
    hipSetDevice(g->dev);
    hipFree(g->desc);
    hipFree(g->sect);
    hipFree(g->ring);
    hipFree(g->kfi);
    hipFree(g->cnt);
    delete g;
}

int slo_xsc_ingest(slo_xsc* g, const void* d_records, int n_records, void* hip_stream) {
    if (!g || !d_records || n_records != g->N) return SLO_E_ARG;
    if (hipSetDevice(g->dev) != hipSuccess) return SLO_E_HIP;
    hipLaunchKernelGGL(slo::k_xsc_ingest, dim3(n_records), dim3(256), 0, (hipStream_t)hip_stream, slo::xsc_view(g),
                       (const float*)d_records, n_records);
    return hipGetLastError() == hipSuccess ? SLO_OK : SLO_E_HIP;
}

int slo_xsc_query(slo_xsc* g, const void* d_records, int n_query, int global0, void* d_out, void* hip_stream) {
    if (!g || !d_records || !d_out || n_query <= 0 || global0 < 0 || global0 + n_query > g->N) return SLO_E_ARG;
    if (hipSetDevice(g->dev) != hipSuccess) return SLO_E_HIP;
    hipLaunchKernelGGL(slo::k_xsc_query, dim3(n_query), dim3(256), 0, (hipStream_t)hip_stream, slo::xsc_view(g),
                       (const float*)d_records, n_query, global0, (slo_xsc_match*)d_out);
    return hipGetLastError() == hipSuccess ? SLO_OK : SLO_E_HIP;
}

}  // extern "C"
