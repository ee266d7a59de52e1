// slo_ctx.hip — context lifetime, HBM arena, batched pipeline driver and the
// C ABI of include/slo_abi.h.
#include "slo_internal.h"
#include "../../include/slo_abi.h"
#include "slo_gen.h"
#include "slo_libm.h"
#include "slo_pose.h"
#include <string.h>
#include <algorithm>
#include <atomic>
#include <thread>

using slo::DevView;
using slo::StreamState;

namespace slo {

// the filter's names (slo_timing_filter: one name or a comma-separated list)
static int stamp_id(const slo_ctx* ctx, const char* name) {
    for (size_t k = 0; k < ctx->stamp_names.size(); ++k)
        if (ctx->stamp_names[k] == name) return (int)k;
    return -1;
}
bool timing_on(const slo_ctx* ctx, const char* name) {
    return ctx->timing_only.empty() || stamp_id(ctx, name) >= 0;
}
// one timestamp of the device's constant-rate clock and the name it belongs to
__global__ void k_stamp(unsigned long long* st, int id) {
    const unsigned int i = atomicAdd((unsigned int*)(st + 2 * SLO_STAMP_CAP), 1u) % SLO_STAMP_CAP;
    st[2 * i] = wall_clock64();
    st[2 * i + 1] = (unsigned long long)id;
}
static bool stamping(const slo_ctx* ctx) { return !ctx->timing_only.empty() && ctx->d_stamp; }
void timing_begin(slo_ctx* ctx, const char* name, hipEvent_t* a) {
    if (stamping(ctx)) {
        *a = nullptr;
        hipLaunchKernelGGL(k_stamp, dim3(1), dim3(1), 0, ctx->stream, ctx->d_stamp, stamp_id(ctx, name));
        return;
    }
    hipEventCreate(a);
    hipEventRecord(*a, ctx->stream);
}
void timing_end(slo_ctx* ctx, const char* name, hipEvent_t a) {
    if (stamping(ctx)) {
        hipLaunchKernelGGL(k_stamp, dim3(1), dim3(1), 0, ctx->stream, ctx->d_stamp, stamp_id(ctx, name));
        return;
    }
    hipEvent_t b;
    hipEventCreate(&b);
    hipEventRecord(b, ctx->stream);
    ctx->pending.push_back({name, {a, b}});
}
static void timing_flush(slo_ctx* ctx) {
    if (stamping(ctx)) {   // consecutive (begin, end) stamps of each filtered launch, in stream order
        std::vector<unsigned long long> h(2 * SLO_STAMP_CAP + 1);
        hipStreamSynchronize(ctx->stream);
        hipMemcpy(h.data(), ctx->d_stamp, sizeof(unsigned long long) * (2 * SLO_STAMP_CAP + 1), hipMemcpyDeviceToHost);
        const unsigned int n = std::min((unsigned int)h[2 * SLO_STAMP_CAP], (unsigned int)SLO_STAMP_CAP);
        if (h[2 * SLO_STAMP_CAP] > SLO_STAMP_CAP)   // the ring wrapped since the last flush: stamps were lost
            ctx->ktimes["!stamps_lost"].n += (long long)(h[2 * SLO_STAMP_CAP] - SLO_STAMP_CAP);
        for (unsigned int i = 0; i + 1 < n; i += 2) {
            const int id = (int)h[2 * i + 1];
            if (id < 0 || id >= (int)ctx->stamp_names.size() || (int)h[2 * i + 3] != id) continue;
            auto& k = ctx->ktimes[ctx->stamp_names[id]];
            k.total_ms += (double)(h[2 * i + 2] - h[2 * i]) / ctx->stamp_khz;
            k.n += 1;
        }
        hipMemsetAsync(ctx->d_stamp + 2 * SLO_STAMP_CAP, 0, sizeof(unsigned long long), ctx->stream);
        hipStreamSynchronize(ctx->stream);
    }
    if (ctx->pending.empty()) return;
    hipStreamSynchronize(ctx->stream);
    for (auto& p : ctx->pending) {
        float ms = 0;
        hipEventElapsedTime(&ms, p.second.first, p.second.second);
        auto& k = ctx->ktimes[p.first];
        k.total_ms += ms;
        k.n += 1;
        hipEventDestroy(p.second.first);
        hipEventDestroy(p.second.second);
    }
    ctx->pending.clear();
}

// what = 1: the scan's points, 2: its stamp, 3: both
__global__ void k_set_io(SloIo* io, const float4* pts, const int32_t* npts, double t_scan, int what) {
    if (what & 1) {
        io->pts = pts;
        io->npts = npts;
    }
    if (what & 2) io->t_scan = t_scan;
}

// the scan the following launches read (DevView::io), in stream order
static int set_io(slo_ctx* ctx, const void* pts, const int32_t* npts) {
    hipLaunchKernelGGL(k_set_io, dim3(1), dim3(1), 0, ctx->stream, ctx->d_io, (const float4*)pts, npts, 0.0, 1);
    SLO_CHECK(hipGetLastError());
    return 0;
}
static int set_io_time(slo_ctx* ctx, const void* pts, const int32_t* npts, double t_scan, int what) {
    hipLaunchKernelGGL(k_set_io, dim3(1), dim3(1), 0, ctx->stream, ctx->d_io, (const float4*)pts, npts, t_scan,
                       what);
    SLO_CHECK(hipGetLastError());
    return 0;
}

void graphs_drop(slo_ctx* ctx) {
    for (int k = 0; k < 4; ++k) {
        if (ctx->graph_exec[k]) hipGraphExecDestroy(ctx->graph_exec[k]);
        ctx->graph_exec[k] = nullptr;
    }
}

}  // namespace slo

namespace {

struct Carver {
    size_t off = 0;
    std::vector<std::pair<void**, size_t>> items;
    template <class T>
    void add(T** p, size_t count) {
        items.push_back({(void**)p, sizeof(T) * count});
        off += (sizeof(T) * count + 255) & ~(size_t)255;
    }
    void assign(char* base) {
        size_t o = 0;
        for (auto& it : items) {
            *it.first = base + o;
            o += (it.second + 255) & ~(size_t)255;
        }
    }
};

}  // namespace

extern "C" {

int slo_config_preset(int preset, slo_config* out) {
    if (!out) return SLO_E_ARG;
    return slo_config_preset_impl(preset, out) == 0 ? SLO_OK : SLO_E_ARG;
}

const char* slo_last_error(const slo_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }
void* slo_stream(slo_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int slo_create(const slo_config* cfg, int hip_device, int n_streams, slo_ctx** out) {
    if (!cfg || !out || n_streams <= 0 || cfg->n_scan <= 0 || cfg->n_scan > 128 || cfg->horizon_scan <= 0 ||
        cfg->horizon_scan > 4096 || cfg->max_points <= 0 || cfg->keyframe_cloud_cap < 0 ||
        (cfg->loop_verify && (cfg->loop_archive_points <= 0 || cfg->history_keyframe_search_num < 0 ||
                              cfg->history_keyframe_search_num > SLO_LC_MAX_N || cfg->icp_max_iterations < 1 ||
                              !(cfg->leaf_history > 0) || !(cfg->icp_max_corr_dist >= 0))) || cfg->sc_num_candidates < 1 ||
        cfg->sc_num_candidates > SLO_SC_MAX_K || cfg->sc_num_ring < 1 || cfg->sc_num_ring > 64 ||
        cfg->sc_num_sector < 1 || cfg->sc_num_sector > SLO_SC_MAX_SECTOR ||
        cfg->sc_num_ring * cfg->sc_num_sector > SLO_SC_MAX_CELLS || cfg->surrounding_keyframe_search_num < 1 ||
        cfg->surrounding_keyframe_search_num + 2 > 64 || cfg->sc_tree_making_period < 1 ||
        cfg->map_keyframes < 0 || cfg->map_keyframes > SLO_MAPK_MAX || cfg->keyframe_ring < 0 ||
        (cfg->loop_closure_enable && cfg->keyframe_ring && cfg->keyframe_ring < cfg->surrounding_keyframe_search_num + 2) ||
        (!cfg->loop_closure_enable && !(cfg->leaf_surrounding_key_poses > 0)) ||
        !(cfg->nearest_feature_search_sq_dist >= 0.0f) ||
        std::ceil(std::sqrt(cfg->nearest_feature_search_sq_dist) / SLO_ODO_SURF_CELL) > SLO_ODO_SURF_R)
        return SLO_E_ARG;   // the odometry surf search box (SLO_ODO_SURF_R cells) must cover the gate
    slo_ctx* ctx = new slo_ctx();
    if (const char* e = getenv("SLO_VG_ONESWEEP")) ctx->vg_onesweep = e[0] == '1';   // experiment switch (slo_vg.hip)
    ctx->cfg = *cfg;
    ctx->dev = hip_device;
    ctx->S = n_streams;
    *out = nullptr;
    if (hipSetDevice(hip_device) != hipSuccess) { delete ctx; return SLO_E_HIP; }
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) { delete ctx; return SLO_E_HIP; }
    DevView& v = ctx->v;
    memset(&v, 0, sizeof(v));
    v.cfg = *cfg;
    v.S = n_streams;
    v.P = cfg->max_points;
    const int R = cfg->n_scan, C = cfg->horizon_scan;
    v.H = R * C;
    v.cap_sharp = 12 * R;
    v.cap_less_sharp = 120 * R;
    v.cap_flat = 24 * R;
    v.cap_less_flat = v.H;
    const size_t S = n_streams, H = v.H;
    Carver c;
    c.add(&ctx->d_in, S * v.P);
    c.add(&ctx->d_ring_in, S * v.P);
    c.add(&ctx->d_cnt, S);
    c.add(&v.owner, S * H);
    c.add(&v.fl, 2 * S);
    c.add(&v.range, S * H);
    c.add(&v.full, S * H);
    c.add(&v.ground, S * H);
    c.add(&v.label, S * H);
    c.add(&v.parent, S * H);
    c.add(&v.csize, S * H);
    c.add(&v.crows, 2 * S * H);
    c.add(&v.rowcnt, 2 * S * R);
    c.add(&v.seg, S * H);
    c.add(&v.seg_ground, S * H);
    c.add(&v.seg_col, S * H);
    c.add(&v.seg_range, S * H);
    c.add(&v.ring_se, 2 * S * R);
    c.add(&v.orient, 3 * S);
    c.add(&v.outlier, S * H);
    c.add(&v.fpts, S * H);
    c.add(&v.curv, S * H);
    c.add(&v.picked, S * H);
    c.add(&v.clabel, S * H);
    c.add(&v.smooth, S * H);
    c.add(&v.ex_list, 2 * S * H);
    c.add(&v.ex_cnt, SLO_EX_CNT * S * R);
    c.add(&v.ring_cnt, 4 * S * R);
    c.add(&v.r_sharp, S * R * 12);
    c.add(&v.r_less_sharp, S * R * 120);
    c.add(&v.r_flat, S * R * 24);
    c.add(&v.r_lf_scan, S * R * C);
    c.add(&v.r_lf_n, S * R);
    c.add(&v.r_lf_ds, S * R * C);
    c.add(&v.sharp, S * v.cap_sharp);
    c.add(&v.less_sharp, S * v.cap_less_sharp);
    c.add(&v.flat, S * v.cap_flat);
    c.add(&v.less_flat, S * v.cap_less_flat);
    c.add(&v.corner_last, S * v.cap_less_sharp);
    c.add(&v.surf_last, S * v.cap_less_flat);
    c.add(&v.corner_next, S * v.cap_less_sharp);
    c.add(&v.surf_next, S * v.cap_less_flat);
    c.add(&v.kd_corner, S * v.cap_less_sharp);
    c.add(&v.kd_surf, S * v.cap_less_flat);
    c.add(&v.roff_cur, S * 2 * (R + 1));
    c.add(&v.roff_last, S * 2 * (R + 1));
    c.add(&v.sx_surf_last, S * v.cap_less_flat);
    c.add(&v.sx_surf_next, S * v.cap_less_flat);
    c.add(&v.sx_kd_corner, S * v.cap_less_sharp);
    c.add(&v.sharp_perm, S * v.cap_sharp);
    c.add(&v.ind_surf, S * v.cap_flat * 3);
    c.add(&v.ind_corner, S * v.cap_sharp * 2);
    c.add(&v.st, S);
    c.add(&ctx->d_io, 1);
    c.add(&v.imu, S);
    c.add(&v.wctr, 8);
    // ---- mapping + Scan Context history
    // Capacities are worst-case bounds, so no cloud is ever clipped: a
    // VoxelGrid output is no larger than its input, the surf DS of a scan is
    // a subset-DS of <= H points, the outlier cloud keeps every 5th column
    // (IP:341-345) of at most R rows.
    const int NKF = cfg->surrounding_keyframe_search_num;
    const bool radius = !cfg->loop_closure_enable;   // MO:1167-1222 branch
    // keyframe cloud slots: the recent-NKF deque + the one being added; the
    // radius branch may bring back any keyframe (the reference keeps all)
    v.KFR = cfg->keyframe_ring > 0 ? cfg->keyframe_ring : (radius ? 1024 : NKF + 2);
    v.KFMAX = SLO_KFMAX;
    v.MAPK = cfg->map_keyframes > 0 ? cfg->map_keyframes : (radius ? 128 : NKF);
    v.cap_kc = v.cap_less_sharp;
    v.cap_ks = (int)H;
    v.cap_ko = R * ((C + 4) / 5);
    v.cap_mc = v.MAPK * v.cap_kc;
    const int kcap = cfg->keyframe_cloud_cap;
    v.cap_kfs = kcap > 0 ? std::min(v.cap_ks, kcap) : v.cap_ks;
    v.cap_kfo = kcap > 0 ? std::min(v.cap_ko, kcap) : v.cap_ko;
    v.cap_ms = v.MAPK * (v.cap_kfs + v.cap_kfo);
    v.cap_st = (int)H + v.cap_ko;
    const size_t NRS = (size_t)cfg->sc_num_ring * cfg->sc_num_sector;
    c.add(&v.outl_cam, S * H);
    c.add(&v.kf_corner, S * v.KFR * v.cap_kc);
    c.add(&v.kf_surf, S * v.KFR * v.cap_kfs);
    c.add(&v.kf_outl, S * v.KFR * v.cap_kfo);
    c.add(&v.kf_n, S * v.KFR * 3);
    c.add(&v.kf_pose, S * v.KFMAX * 6);
    c.add(&v.map_ids, S * v.MAPK);
    c.add(&v.map_c, S * v.cap_mc);
    c.add(&v.map_s, S * v.cap_ms);
    c.add(&v.map_c_ds, S * v.cap_mc);
    c.add(&v.map_s_ds, S * v.cap_ms);
    c.add(&v.cur_raw_ds, S * v.P);
    c.add(&v.cur_c_ds, S * v.cap_less_sharp);
    c.add(&v.cur_s_ds, S * H);
    c.add(&v.cur_o_ds, S * v.cap_ko);
    c.add(&v.cur_st, S * v.cap_st);
    c.add(&v.cur_st_ds, S * v.cap_st);
    c.add(&v.mo_part, S * SLO_MO_BLOCKS * SLO_MO_PART);
    c.add(&v.tick, S);
    v.cap_q = v.cap_less_sharp + v.cap_st;
    c.add(&v.mo_nn, S * (size_t)v.cap_q * 5);
    c.add(&v.mo_perm, S * (size_t)v.cap_q);
    c.add(&v.sc_desc, S * v.KFMAX * NRS);
    c.add(&v.sc_ring, S * v.KFMAX * cfg->sc_num_ring);
    c.add(&v.sc_ringd, S * v.KFMAX * cfg->sc_num_ring);
    c.add(&v.sc_sect, S * v.KFMAX * cfg->sc_num_sector);
    ctx->arena_bytes = c.off;
    if (hipMalloc(&ctx->arena, ctx->arena_bytes) != hipSuccess) {
        ctx->err = "hipMalloc arena failed";
        hipStreamDestroy(ctx->stream);
        delete ctx;
        return SLO_E_HIP;
    }
    c.assign((char*)ctx->arena);
    v.io = ctx->d_io;
    // zero everything: persistent FA arrays start as the zero pages new[] gives
    if (hipMemsetAsync(ctx->arena, 0, ctx->arena_bytes, ctx->stream) != hipSuccess ||
        hipHostMalloc((void**)&ctx->h_st, sizeof(StreamState) * S) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
        slo_destroy(ctx);
        return SLO_E_HIP;
    }
    memset(ctx->h_st, 0, sizeof(StreamState) * S);
    // Grid cells (powers of two, GridView): the map grids answer 5-NN within
    // 1 m (MO:1281/1364) in 0.5 m cells (rings <= 2, usually done after 1)
    // hashed into 2^19 buckets per stream (2^17 measured 1.3x slower in
    // mo_knn: a row's bucket run then holds other cells' points);
    // the odometry surf grid answers 1-NN within 5 m (nearestFeatureSearchSqDist)
    // in 1 m cells (2^15 buckets: built in LDS by one workgroup per stream,
    // slo_vg.hip); the sparse corner cloud is searched by brute force.
    if (slo::vg_alloc(ctx) || slo::grid_alloc(ctx, ctx->grid_c, 1 << SLO_MAP_TLOG2, v.cap_mc, SLO_MAP_CELL) ||
        slo::grid_alloc(ctx, ctx->grid_s, 1 << SLO_MAP_TLOG2, v.cap_ms, SLO_MAP_CELL) ||
        slo::grid_alloc(ctx, ctx->grid_os, 1 << 15, v.cap_less_flat, SLO_ODO_SURF_CELL) ||
        (S <= SLO_PREP_DEFER_STREAMS && slo::fa_prep_init(ctx))) {
        slo_destroy(ctx);
        return SLO_E_HIP;
    }
    if (cfg->pose_graph && slo::pg_alloc(ctx)) {
        slo_destroy(ctx);
        return SLO_E_CAPACITY;
    }
    if (cfg->loop_verify && slo::lc_alloc(ctx)) {
        slo_destroy(ctx);
        return SLO_E_HIP;
    }
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, hip_device) != hipSuccess || khz <= 0 ||
        hipMalloc(&ctx->d_stamp, sizeof(unsigned long long) * (2 * SLO_STAMP_CAP + 1)) != hipSuccess ||
        hipMemset(ctx->d_stamp, 0, sizeof(unsigned long long) * (2 * SLO_STAMP_CAP + 1)) != hipSuccess) {
        slo_destroy(ctx);
        return SLO_E_HIP;
    }
    ctx->stamp_khz = khz;
    ctx->pp_corner0 = v.corner_last;
    if (slo::imu_init(ctx) || hipStreamSynchronize(ctx->stream) != hipSuccess) {
        slo_destroy(ctx);
        return SLO_E_HIP;
    }
    v.g_os = slo::grid_view(ctx->grid_os);
    v.g_mc = slo::grid_view(ctx->grid_c);
    v.g_ms = slo::grid_view(ctx->grid_s);
    *out = ctx;
    return SLO_OK;
}

void slo_destroy(slo_ctx* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->dev);
    slo::pipe_free(ctx);   // slo_pipeline's stage contexts and rings
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    for (auto& p : ctx->pending) { hipEventDestroy(p.second.first); hipEventDestroy(p.second.second); }
    slo::graphs_drop(ctx);
    slo::vg_side_free(ctx);
    slo::fa_prep_free(ctx);
    slo::vg_free(ctx);
    slo::pcl_free(ctx);
    slo::grid_free(ctx->grid_c);
    slo::grid_free(ctx->grid_s);
    slo::grid_free(ctx->grid_oc);
    slo::grid_free(ctx->grid_os);
    slo::lc_free(ctx);
    slo::pg_free(ctx);
    if (ctx->arena) hipFree(ctx->arena);
    if (ctx->h_st) hipHostFree(ctx->h_st);
    if (ctx->h_stage) hipHostFree(ctx->h_stage);
    if (ctx->d_stamp) hipFree(ctx->d_stamp);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
}

int slo_prepare_mapping(slo_ctx* ctx) {
    if (!ctx) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    if (int r = slo::map_ws_ensure(ctx)) return r;
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    return SLO_OK;
}

int slo_synchronize(slo_ctx* ctx) {
    if (!ctx) return SLO_E_ARG;
    hipSetDevice(ctx->dev);
    if (ctx->pipe)   // slo_pipeline: the front and odometry stages too
        for (slo_ctx* c : slo::pipe_stages(ctx)) SLO_CHECK(hipStreamSynchronize(c->stream));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    return SLO_OK;
}

int slo_batch_set_rings(slo_ctx* ctx, const uint16_t* d_rings) {
    if (!ctx) return SLO_E_ARG;
    if (ctx->v.rings != d_rings) slo::graphs_drop(ctx);   // the captured launches carry the old pointer
    ctx->v.rings = d_rings;
    return SLO_OK;
}

int slo_batch_scan_time(slo_ctx* ctx, double t_scan) {
    if (!ctx) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    return slo::set_io_time(ctx, nullptr, nullptr, t_scan, 2);
}

int slo_graph_mode(slo_ctx* ctx, int on) {
    if (!ctx) return SLO_E_ARG;
    if (!on) slo::graphs_drop(ctx);
    ctx->graphs = on != 0;
    return SLO_OK;
}

int slo_batch_image_projection(slo_ctx* ctx, const void* d_points, const int32_t* d_counts) {
    if (!ctx || !d_points || !d_counts) return SLO_E_ARG;
    if (ctx->cfg.use_cloud_ring && !ctx->v.rings) {
        ctx->err = "cfg.use_cloud_ring needs slo_batch_set_rings";
        return SLO_E_STATE;
    }
    SLO_CHECK(hipSetDevice(ctx->dev));
    if (int r = slo::set_io(ctx, d_points, d_counts)) return r;
    return slo::ip_run(ctx);
}

}  // extern "C"

namespace slo {
// FA frameCount / publish gate (FA:1790-1792); the init scan never publishes
static void fa_advance(slo_ctx* ctx, bool first) {
    ctx->fa_published = false;
    if (first) {
        ctx->fa_inited = true;
        ctx->fa_frame_count = ctx->cfg.skip_frame_num;
    } else {
        ctx->fa_frame_count++;
        if (ctx->fa_frame_count >= ctx->cfg.skip_frame_num + 1) {
            ctx->fa_frame_count = 0;
            ctx->fa_published = true;
        }
    }
    ctx->scan_index++;
}

// MO's gate (MO:1685): this scan reached mapping (FA published it) and the
// mapping interval has elapsed
static bool map_gate(slo_ctx* ctx, double t_scan) {
    ctx->mapped_now = false;
    if (!ctx->fa_published) return false;
    if (!(t_scan - ctx->t_last_processing >= ctx->cfg.mapping_process_interval)) return false;
    ctx->t_last_processing = t_scan;
    return true;
}
}  // namespace slo

extern "C" {

int slo_batch_feature_association(slo_ctx* ctx) {
    if (!ctx) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    int r = slo::fa_features_run(ctx);
    if (r) return r;
    const bool first = !ctx->fa_inited;
    r = slo::fa_odometry_run(ctx, first);
    if (r) return r;
    slo::fa_advance(ctx, first);
    return SLO_OK;
}

}  // extern "C"

namespace slo {
__global__ void k_clear_flags(DevView v) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    v.st[s].mo_ran = 0;
    v.st[s].kf_saved = 0;
    v.st[s].det_valid = 0;
}
}  // namespace slo

extern "C" {

// Runs the mapping step if this scan reached mapping (FA published it,
// FA:1790-1814) and the mapping interval has elapsed (MO:1685).
int slo_batch_map_optimization(slo_ctx* ctx, const void* d_points, const int32_t* d_counts, double t_scan) {
    if (!ctx || !d_points || !d_counts) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    if (int r = slo::set_io(ctx, d_points, d_counts)) return r;
    SLO_LAUNCH(ctx, "clear_flags", slo::k_clear_flags, dim3((ctx->S + 63) / 64), dim3(64), 0, ctx->v);
    if (!slo::map_gate(ctx, t_scan)) return SLO_OK;
    int r = slo::map_ws_ensure(ctx);
    if (!r) r = slo::map_run(ctx);
    if (r) return r;
    ctx->mapped_now = true;
    // the graph half of saveKeyFramesAndFactor, then correctPoses (MO:1697-1699)
    if (ctx->cfg.pose_graph && (r = slo::pg_after_mapping(ctx))) return r;
    return slo::lc_archive_run(ctx, t_scan);   // keyframe archive for loop verification (cfg.loop_verify)
}

int slo_batch_sc_detect(slo_ctx* ctx) {
    if (!ctx) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    return slo::sc_detect_run(ctx);
}

}  // extern "C"

namespace slo {
// One step of the batched pipeline after the first scan, without the host
// round trips of loop verification and the pose graph: projection,
// features, odometry, the mapping step when `map`, Scan Context detect.
// Launches only (the host state is advanced by the caller), so the same
// calls can be captured into a graph.
// With at most SLO_PREP_DEFER_STREAMS streams the odometry's preparation of
// the next scan's searches (fa_prep_*, slo_odom.hip) is left to the next step,
// forked beside its projection and features: it leaves a scan's critical path.
static int step_launches(slo_ctx* ctx, bool map) {
    // (not with a kernel-name timing filter: its in-stream stamps pair up per stream, as map_run's fork)
    const bool defer = ctx->S <= SLO_PREP_DEFER_STREAMS && !(ctx->timing && !ctx->timing_only.empty());
    const bool forked = ctx->prep_pending && defer;
    ctx->map_forked = false;
    int r = map && defer && ctx->map_fork_ready ? map_side_fork(ctx) : 0;
    if (!r && forked) r = fa_prep_fork(ctx);
    if (!r) r = ip_run(ctx);
    if (!r) r = fa_features_run(ctx, defer);   // its less-flat VoxelGrids beside the odometry
    if (!r && forked) r = fa_prep_join(ctx);
    if (!r) r = fa_odometry_run(ctx, false, true, defer);
    if (r) return r;
    SLO_LAUNCH(ctx, "clear_flags", k_clear_flags, dim3((ctx->S + 63) / 64), dim3(64), 0, ctx->v);
    if (map && (r = map_run(ctx))) return r;
    if (ctx->cfg.loop_closure_enable) r = sc_detect_run(ctx);
    return r;
}

// slo_batch_process as one HIP graph launch per scan.  A step's launch
// sequence depends only on host state (FA's publish counter, the mapping
// interval) and the kernels' arguments only on which half of the odometry
// ping-pong buffers is current (fa_swap_last), so a step is one of four
// graphs: with or without the mapping stage, times the two layouts.  Each
// is captured once — after the step kind has run eagerly, so every workspace
// has been sized — and then replayed.  The scan itself is read through the io
// slot set before each launch.  Returns 1 when the step is not eligible
// (eager path).
static int step_graph(slo_ctx* ctx, const void* d_points, const int32_t* d_counts, double t_scan) {
    if (!ctx->graphs || (ctx->timing && ctx->timing_only.empty()) || !ctx->fa_inited || ctx->cfg.loop_verify ||
        ctx->cfg.pose_graph)
        return 1;   // per-kernel event timing and the host round trips need the eager path
    SLO_CHECK(hipSetDevice(ctx->dev));
    fa_advance(ctx, false);
    const bool map = map_gate(ctx, t_scan);
    const int kind = map ? 1 : 0, key = 2 * kind + (ctx->v.corner_last == ctx->pp_corner0 ? 0 : 1);
    if (int r = set_io_time(ctx, d_points, d_counts, t_scan, 3)) return r;
    if (ctx->graph_exec[key] && (ctx->graph_ws[key] != ctx->ws_gen ||
                                 memcmp(&ctx->graph_v[key], &ctx->v, sizeof(DevView)) != 0)) {
        hipGraphExecDestroy(ctx->graph_exec[key]);   // its arguments are stale: capture again
        ctx->graph_exec[key] = nullptr;
    }
    if (!ctx->graph_exec[key]) {
        if (!ctx->graph_seen[kind]) {   // first occurrence of the kind: eager
            ctx->graph_seen[kind] = 1;
            int r = step_launches(ctx, map);
            if (!r && map) ctx->mapped_now = true;
            return r;
        }
        memcpy(&ctx->graph_v[key], &ctx->v, sizeof(DevView));
        const unsigned int ws0 = ctx->ws_gen;
        // a capture that cannot become a graph: undo what the captured launches
        // did to the host state (the ping-pong swap) and run this step eagerly,
        // with graphs off from now on, so the stream stays in step
        auto eager_instead = [&](const std::string& why) {
            memcpy(&ctx->v, &ctx->graph_v[key], sizeof(DevView));
            ctx->graphs = false;
            ctx->err = why;
            const int r2 = step_launches(ctx, map);
            if (!r2 && map) ctx->mapped_now = true;
            return r2;
        };
        SLO_CHECK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
        const int r = step_launches(ctx, map);   // swaps the ping-pong halves, as a replay does below
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(ctx->stream, &g);
        if (r || e != hipSuccess) {
            if (g) hipGraphDestroy(g);
            if (r) return r;   // a launch failed: a real error
            return eager_instead(std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
        }
        if (ctx->ws_gen != ws0) {   // a workspace moved while capturing (not expected): no graph
            hipGraphDestroy(g);
            // the stream-ordered initialisations of the new workspaces went into
            // the discarded graph: run them now, before the eager step
            if (int r = vg_ws_reinit(ctx)) return r;
            return eager_instead("a workspace was reallocated during graph capture");
        }
        ctx->graph_ws[key] = ws0;
        const hipError_t ei = hipGraphInstantiate(&ctx->graph_exec[key], g, nullptr, nullptr, 0);
        hipGraphDestroy(g);
        if (ei != hipSuccess) {
            ctx->graph_exec[key] = nullptr;
            return eager_instead(std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
        }
    } else {
        fa_swap_last(ctx);   // what the captured fa_odometry_run did on the host
    }
    SLO_CHECK(hipGraphLaunch(ctx->graph_exec[key], ctx->stream));
    if (map) ctx->mapped_now = true;
    return 0;
}
}  // namespace slo

extern "C" {

int slo_batch_process(slo_ctx* ctx, const void* d_points, const int32_t* d_counts, double t_scan) {
    if (!ctx || !d_points || !d_counts) return SLO_E_ARG;
    if (ctx->pipe) return slo::pipe_step(ctx, d_points, d_counts, t_scan);   // slo_pipeline
    if (ctx->cfg.use_cloud_ring && !ctx->v.rings) {
        ctx->err = "cfg.use_cloud_ring needs slo_batch_set_rings";
        return SLO_E_STATE;
    }
    SLO_CHECK(hipSetDevice(ctx->dev));
    if (int r = slo::map_ws_ensure(ctx)) return r;   // before step_graph may capture
    if (ctx->S <= SLO_PREP_DEFER_STREAMS) {   // the few-stream step's forks (step_launches)
        if (int r = slo::fa_ring_init(ctx)) return r;
        if (int r = slo::map_fork_prepare(ctx)) return r;
    }
    int r = slo::step_graph(ctx, d_points, d_counts, t_scan);
    if (r <= 0) return r;
    if ((r = slo_batch_scan_time(ctx, t_scan))) return r;
    r = slo_batch_image_projection(ctx, d_points, d_counts);
    if (r) return r;
    r = slo_batch_feature_association(ctx);
    if (r) return r;
    r = slo_batch_map_optimization(ctx, d_points, d_counts, t_scan);
    if (r) return r;
    // without loop closure the loop thread returns at once (MO:831-832): the
    // keyframes still get descriptors (MO:1630), nothing queries them
    if (!ctx->cfg.loop_closure_enable) return SLO_OK;
    r = slo_batch_sc_detect(ctx);
    if (r || !ctx->cfg.loop_verify) return r;
    r = slo_batch_loop_closure(ctx);
    if (r || !ctx->cfg.pose_graph || !ctx->mapped_now) return r;
    return slo::pg_after_loops(ctx);   // the loop factors (MO:1038-1046, 1083-1091)
}

// ---------------------------------------------------------------- Mode S
// The slabs that travel between the contexts of one stream split over
// several (include/slo_abi.h "Mode S"): each a [S][...] array of the arena,
// copied whole.  carry: featureAssociation's persistent arrays (Q5), the
// cloud_info arrays (their tails past a scan's points are read, FA:730-745)
// and the orientations an empty scan keeps; features: what odometry and
// mapping read of a scan's front end.
}  // extern "C"
namespace slo {
struct ModesSlab { void* p; size_t bytes; };
static std::vector<ModesSlab> modes_carry(slo_ctx* ctx) {
    const DevView& v = ctx->v;
    const size_t S = ctx->S, H = v.H;
    return {{v.smooth, S * H * sizeof(Smooth)}, {v.curv, S * H * 4}, {v.picked, S * H * 4}, {v.clabel, S * H * 4},
            {v.seg_col, S * H * 4}, {v.seg_ground, S * H}, {v.seg_range, S * H * 4}, {v.orient, S * 3 * 4}};
}
#define MODES_NCOUNT 8   // per stream: n_sharp, n_less_sharp, n_flat, n_less_flat, seg_count, outlier_count, err, first_half
static std::vector<ModesSlab> modes_features(slo_ctx* ctx, int32_t** counts) {
    const DevView& v = ctx->v;
    const size_t S = ctx->S, H = v.H, R = v.cfg.n_scan;
    *counts = nullptr;   // (a slab of its own, packed by k_modes_counts)
    return {{v.sharp, S * v.cap_sharp * 16}, {v.less_sharp, S * v.cap_less_sharp * 16}, {v.flat, S * v.cap_flat * 16},
            {v.less_flat, S * v.cap_less_flat * 16}, {v.outlier, S * H * 16}, {v.roff_cur, S * 2 * (R + 1) * 4},
            {nullptr, S * MODES_NCOUNT * 4}};
}
static size_t modes_bytes(const std::vector<ModesSlab>& sl) {
    size_t o = 0;
    for (const auto& x : sl) o += (x.bytes + 255) & ~(size_t)255;
    return o;
}
// copy every slab with a pointer between the arena and the buffer (out: arena -> buffer)
static int modes_copy(slo_ctx* ctx, const std::vector<ModesSlab>& sl, char* buf, bool out, int first, int last) {
    size_t o = 0;
    for (int k = 0; k < (int)sl.size(); ++k) {
        if (k >= first && k < last && sl[k].p)
            SLO_CHECK(hipMemcpyAsync(out ? (void*)(buf + o) : sl[k].p, out ? sl[k].p : (const void*)(buf + o),
                                     sl[k].bytes, hipMemcpyDeviceToDevice, ctx->stream));
        o += (sl[k].bytes + 255) & ~(size_t)255;
    }
    return 0;
}
// Mode S carries no IMU ring (the deskew of a front context and the
// initial guess of the odometry context would read rings fed elsewhere), so a
// context that ingested IMU messages refuses the Mode S entry points, and
// slo_batch_imu / slo_imu_handler refuse a context Mode S ran on
int modes_enter(slo_ctx* ctx) {
    if (ctx->imu_fed) {
        ctx->err = "Mode S entry point on a context fed IMU messages (Mode S carries no IMU ring)";
        return SLO_E_STATE;
    }
    ctx->modes_used = true;
    return 0;
}
// after imageProjection: the cloud_info tails past this scan's points and, for
// a scan without a finite point, the orientations come from the carry
__global__ void k_modes_merge(DevView v, const uint32_t* col, const uint8_t* gnd, const float* rng, const float* orient) {
    const int s = blockIdx.y;
    const size_t b = (size_t)s * v.H;
    const int n = v.st[s].seg_count;
    for (int i = n + blockIdx.x * blockDim.x + threadIdx.x; i < v.H; i += gridDim.x * blockDim.x) {
        v.seg_col[b + i] = col[b + i];
        v.seg_ground[b + i] = gnd[b + i];
        v.seg_range[b + i] = rng[b + i];
    }
    if (blockIdx.x == 0 && threadIdx.x < 3 && v.fl[2 * s + 1] < 0) v.orient[3 * s + threadIdx.x] = orient[3 * s + threadIdx.x];
}
__global__ void k_modes_counts(DevView v, int32_t* c, int out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    StreamState& st = v.st[s];
    int32_t* q = c + (size_t)s * MODES_NCOUNT;
    if (out) {
        q[0] = st.n_sharp; q[1] = st.n_less_sharp; q[2] = st.n_flat; q[3] = st.n_less_flat;
        q[4] = st.seg_count; q[5] = st.outlier_count; q[6] = st.err; q[7] = st.first_half;
    } else {
        st.n_sharp = q[0]; st.n_less_sharp = q[1]; st.n_flat = q[2]; st.n_less_flat = q[3];
        st.seg_count = q[4]; st.outlier_count = q[5]; st.err |= q[6]; st.first_half = q[7];
    }
}
}  // namespace slo
extern "C" {

size_t slo_modes_carry_bytes(slo_ctx* ctx) { return ctx ? slo::modes_bytes(slo::modes_carry(ctx)) : 0; }
size_t slo_modes_features_bytes(slo_ctx* ctx) {
    int32_t* c;
    return ctx ? slo::modes_bytes(slo::modes_features(ctx, &c)) : 0;
}

int slo_front_process(slo_ctx* ctx, const void* d_points, const int32_t* d_counts, double t_scan,
                      const void* d_carry_in, void* d_carry_out, void* d_features_out) {
    if (!ctx || !d_points || !d_counts || !d_features_out) return SLO_E_ARG;
    if (ctx->cfg.use_cloud_ring && !ctx->v.rings) { ctx->err = "cfg.use_cloud_ring needs slo_batch_set_rings"; return SLO_E_STATE; }
    if (int r = slo::modes_enter(ctx)) return r;
    SLO_CHECK(hipSetDevice(ctx->dev));
    if (int r = slo::set_io_time(ctx, d_points, d_counts, t_scan, 3)) return r;
    if (int r = slo::ip_run(ctx)) return r;
    const auto carry = slo::modes_carry(ctx);
    if (d_carry_in) {   // the previous scan's stale state (that scan's front end ran elsewhere)
        char* ci = (char*)d_carry_in;
        if (int r = slo::modes_copy(ctx, carry, ci, false, 0, 4)) return r;   // FA's persistent arrays, whole
        size_t o[8], x = 0;
        for (int k = 0; k < 8; ++k) { o[k] = x; x += (carry[k].bytes + 255) & ~(size_t)255; }
        const DevView& v = ctx->v;
        SLO_LAUNCH(ctx, "modes_merge", slo::k_modes_merge, dim3(std::max(1, std::min(64, (v.H + 255) / 256)), ctx->S),
                   dim3(256), 0, v, (const uint32_t*)(ci + o[4]), (const uint8_t*)(ci + o[5]), (const float*)(ci + o[6]),
                   (const float*)(ci + o[7]));
    }
    if (int r = slo::fa_features_run(ctx)) return r;
    if (d_carry_out)   // (NULL: the next scan's front end runs on this context, whose arrays hold it already)
        if (int r = slo::modes_copy(ctx, carry, (char*)d_carry_out, true, 0, 8)) return r;
    int32_t* cnt;
    const auto feat = slo::modes_features(ctx, &cnt);
    if (int r = slo::modes_copy(ctx, feat, (char*)d_features_out, true, 0, 6)) return r;
    const size_t oc = slo::modes_bytes(feat) - ((feat[6].bytes + 255) & ~(size_t)255);
    SLO_LAUNCH(ctx, "modes_counts", slo::k_modes_counts, dim3((ctx->S + 255) / 256), dim3(256), 0, ctx->v,
               (int32_t*)((char*)d_features_out + oc), 1);
    SLO_CHECK(hipGetLastError());
    return SLO_OK;
}

int slo_back_process(slo_ctx* ctx, const void* d_features, const void* d_points, const int32_t* d_counts,
                     double t_scan) {
    if (!ctx || !d_features || !d_points || !d_counts) return SLO_E_ARG;
    if (int r = slo::modes_enter(ctx)) return r;
    SLO_CHECK(hipSetDevice(ctx->dev));
    if (int r = slo::set_io_time(ctx, d_points, d_counts, t_scan, 3)) return r;
    int32_t* cnt;
    const auto feat = slo::modes_features(ctx, &cnt);
    if (int r = slo::modes_copy(ctx, feat, (char*)d_features, false, 0, 6)) return r;
    const size_t oc = slo::modes_bytes(feat) - ((feat[6].bytes + 255) & ~(size_t)255);
    SLO_LAUNCH(ctx, "modes_counts", slo::k_modes_counts, dim3((ctx->S + 255) / 256), dim3(256), 0, ctx->v,
               (int32_t*)((char*)d_features + oc), 0);
    const bool first = !ctx->fa_inited;
    if (int r = slo::fa_odometry_run(ctx, first)) return r;
    slo::fa_advance(ctx, first);
    int r = slo_batch_map_optimization(ctx, d_points, d_counts, t_scan);
    if (r || !ctx->cfg.loop_closure_enable) return r;
    return slo_batch_sc_detect(ctx);
}

}  // extern "C"
namespace slo {
// the back end split once more (three stages): the odometry context hands
// the mapping context what mapOptimization reads of featureAssociation — the
// clouds it publishes (laserCloudCornerLast / SurfLast after TransformToEnd,
// the outliers, FA:1790-1814) and the odometry pose transformSum (FA:1808)
#define MODES_NODOM 12   // per stream: cornerLastNum, surfLastNum, outlier_count, err, valid, -, transformSum[6]
static std::vector<ModesSlab> modes_odom(slo_ctx* ctx) {
    const DevView& v = ctx->v;
    const size_t S = ctx->S;
    return {{v.corner_last, S * v.cap_less_sharp * 16}, {v.surf_last, S * v.cap_less_flat * 16},
            {v.outlier, S * (size_t)v.H * 16}, {nullptr, S * MODES_NODOM * 4}};
}
__global__ void k_modes_odom(DevView v, int32_t* c, int out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    StreamState& st = v.st[s];
    int32_t* q = c + (size_t)s * MODES_NODOM;
    if (out) {
        q[0] = st.cornerLastNum; q[1] = st.surfLastNum; q[2] = st.outlier_count; q[3] = st.err;
        q[4] = st.odo_phase != 3; q[5] = 0;
        for (int k = 0; k < 6; ++k) q[6 + k] = __float_as_int(st.transformSum[k]);
        return;
    }
    st.cornerLastNum = q[0]; st.surfLastNum = q[1]; st.outlier_count = q[2]; st.err |= q[3];
    for (int k = 0; k < 6; ++k) st.transformSum[k] = __int_as_float(q[6 + k]);
    if (!q[4]) return;   // the initialisation scan: no odometry, nothing for transformFusion
    // TransformFusion::laserOdometryHandler (TF:186-219) as k_fa_odo_finish
    // does it, here in scan order after the previous scan's mapping step, so
    // with the mapping result that was current when this scan's odometry came
    float sum[6], incre[6];
    slo_pose::odom_handoff(st.transformSum, sum);
    slo_pose::associate_to_map(sum, st.tf_bef, st.tf_aft, incre, st.integrated);
}
}  // namespace slo
extern "C" {

size_t slo_modes_odom_bytes(slo_ctx* ctx) { return ctx ? slo::modes_bytes(slo::modes_odom(ctx)) : 0; }

int slo_odom_process(slo_ctx* ctx, const void* d_features, const void* d_points, const int32_t* d_counts,
                     double t_scan, void* d_odom_out) {
    if (!ctx || !d_features || !d_points || !d_counts || !d_odom_out) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    if (int r = slo::modes_enter(ctx)) return r;
    if (int r = slo::set_io_time(ctx, d_points, d_counts, t_scan, 3)) return r;
    int32_t* cnt;
    const auto feat = slo::modes_features(ctx, &cnt);
    if (int r = slo::modes_copy(ctx, feat, (char*)d_features, false, 0, 6)) return r;
    const size_t oc = slo::modes_bytes(feat) - ((feat[6].bytes + 255) & ~(size_t)255);
    SLO_LAUNCH(ctx, "modes_counts", slo::k_modes_counts, dim3((ctx->S + 255) / 256), dim3(256), 0, ctx->v,
               (int32_t*)((char*)d_features + oc), 0);
    const bool first = !ctx->fa_inited;
    // transformFusion is the mapping context's (k_modes_odom), in scan order after its mapping step
    if (int r = slo::fa_odometry_run(ctx, first, false)) return r;
    slo::fa_advance(ctx, first);
    const auto od = slo::modes_odom(ctx);   // after the swap: the clouds just published
    if (int r = slo::modes_copy(ctx, od, (char*)d_odom_out, true, 0, 3)) return r;
    const size_t oq = slo::modes_bytes(od) - ((od[3].bytes + 255) & ~(size_t)255);
    SLO_LAUNCH(ctx, "modes_odom", slo::k_modes_odom, dim3((ctx->S + 255) / 256), dim3(256), 0, ctx->v,
               (int32_t*)((char*)d_odom_out + oq), 1);
    SLO_CHECK(hipGetLastError());
    return SLO_OK;
}

int slo_map_process(slo_ctx* ctx, const void* d_odom, const void* d_points, const int32_t* d_counts, double t_scan) {
    if (!ctx || !d_odom || !d_points || !d_counts) return SLO_E_ARG;
    if (int r = slo::modes_enter(ctx)) return r;
    SLO_CHECK(hipSetDevice(ctx->dev));
    if (int r = slo::set_io_time(ctx, d_points, d_counts, t_scan, 3)) return r;
    const auto od = slo::modes_odom(ctx);
    if (int r = slo::modes_copy(ctx, od, (char*)d_odom, false, 0, 3)) return r;
    const size_t oq = slo::modes_bytes(od) - ((od[3].bytes + 255) & ~(size_t)255);
    SLO_LAUNCH(ctx, "modes_odom", slo::k_modes_odom, dim3((ctx->S + 255) / 256), dim3(256), 0, ctx->v,
               (int32_t*)((char*)d_odom + oq), 0);
    slo::fa_advance(ctx, !ctx->fa_inited);   // the publish gate, kept in step with the odometry context's
    int r = slo_batch_map_optimization(ctx, d_points, d_counts, t_scan);
    if (r || !ctx->cfg.loop_closure_enable) return r;
    return slo_batch_sc_detect(ctx);
}

}  // extern "C"
namespace slo {
// slo_pipeline: the Mode S three-stage split (front end | odometry |
// mapping) inside one context.  Per scan k, slot = k mod D of the rings:
//   front stream:    [wait evM[slot] of scan k - D] copy the input -> raw / cnt[slot],
//                    slo_front_process -> feat[slot], record evF[slot]
//   odometry stream: wait evF[slot], slo_odom_process(feat[slot]) -> odom[slot], record evO[slot]
//   mapping stream:  wait evO[slot], slo_map_process(odom[slot]), record evM[slot]
// Scan k - D's mapping step has read raw / cnt / odom[slot], and before it
// (evO) its odometry read feat[slot], so waiting on evM[slot] before the
// copy protects every buffer of the slot; each stage's own state is ordered
// by its stream.  The host never waits.
struct SloPipe {
    slo_ctx* front = nullptr;
    slo_ctx* odo = nullptr;
    int D = 0;
    long long k = 0;
    size_t fbytes = 0, obytes = 0, rbytes = 0;
    std::vector<void*> feat, odom, raw, cnt;
    std::vector<hipEvent_t> evF, evO, evM;
};
void pipe_free(slo_ctx* ctx) {
    SloPipe* p = ctx->pipe;
    if (!p) return;
    for (slo_ctx* c : {p->front, p->odo})
        if (c) hipStreamSynchronize(c->stream);
    hipStreamSynchronize(ctx->stream);
    for (auto* v : {&p->feat, &p->odom, &p->raw, &p->cnt})
        for (void* q : *v)
            if (q) hipFree(q);
    for (auto* v : {&p->evF, &p->evO, &p->evM})
        for (hipEvent_t e : *v)
            if (e) hipEventDestroy(e);
    slo_destroy(p->front);
    slo_destroy(p->odo);
    delete p;
    ctx->pipe = nullptr;
}
// the stage whose context computes slo_get's field `name` (the mapping stage,
// ctx itself, for everything mapOptimization, transformFusion and Scan
// Context write, and for the fields the odometry buffer hands it)
slo_ctx* pipe_stage_of(slo_ctx* ctx, const std::string& name) {
    static const char* front[] = {"range", "label", "ground", "full_cloud", "seg_pts", "seg_ground", "seg_col",
                                  "seg_range", "ring_start", "ring_end", "orient", "fa_seg_pts", "curvature",
                                  "picked", "cloud_label", "smooth_ind", "sharp", "less_sharp", "flat", "less_flat"};
    static const char* odom[] = {"transform_cur", "fa_iters", "imu"};
    for (const char* f : front)
        if (name == f) return ctx->pipe->front;
    for (const char* f : odom)
        if (name == f) return ctx->pipe->odo;
    return ctx;
}
static int pipe_fail(slo_ctx* ctx, slo_ctx* stage, int r) {
    if (stage != ctx) ctx->err = stage->err;
    return r;
}
std::vector<slo_ctx*> pipe_stages(slo_ctx* ctx) { return {ctx->pipe->front, ctx->pipe->odo}; }
int pipe_step(slo_ctx* ctx, const void* d_points, const int32_t* d_counts, double t_scan) {
    SloPipe& p = *ctx->pipe;
    SLO_CHECK(hipSetDevice(ctx->dev));
    const int slot = (int)(p.k % p.D);
    slo_ctx* F = p.front;
    slo_ctx* O = p.odo;
    if (p.k >= p.D) SLO_CHECK(hipStreamWaitEvent(F->stream, p.evM[slot], 0));
    SLO_CHECK(hipMemcpyAsync(p.raw[slot], d_points, p.rbytes, hipMemcpyDeviceToDevice, F->stream));
    SLO_CHECK(hipMemcpyAsync(p.cnt[slot], d_counts, sizeof(int32_t) * ctx->S, hipMemcpyDeviceToDevice, F->stream));
    const int32_t* cnt = (const int32_t*)p.cnt[slot];
    int r = slo_front_process(F, p.raw[slot], cnt, t_scan, nullptr, nullptr, p.feat[slot]);
    if (r) return pipe_fail(ctx, F, r);
    SLO_CHECK(hipEventRecord(p.evF[slot], F->stream));
    SLO_CHECK(hipStreamWaitEvent(O->stream, p.evF[slot], 0));
    r = slo_odom_process(O, p.feat[slot], p.raw[slot], cnt, t_scan, p.odom[slot]);
    if (r) return pipe_fail(ctx, O, r);
    SLO_CHECK(hipEventRecord(p.evO[slot], O->stream));
    SLO_CHECK(hipStreamWaitEvent(ctx->stream, p.evO[slot], 0));
    r = slo_map_process(ctx, p.odom[slot], p.raw[slot], cnt, t_scan);
    if (r) return r;
    SLO_CHECK(hipEventRecord(p.evM[slot], ctx->stream));
    ++p.k;
    return SLO_OK;
}
}  // namespace slo
extern "C" {

int slo_pipeline(slo_ctx* ctx, int depth) {
    if (!ctx || depth < 0 || depth == 1 || depth > 64) return SLO_E_ARG;
    if (ctx->fa_inited || ctx->modes_used || (ctx->pipe && ctx->pipe->k > 0)) {
        ctx->err = "slo_pipeline: only on a context that has not processed a scan";
        return SLO_E_STATE;
    }
    if (ctx->imu_fed || ctx->cfg.loop_verify || ctx->cfg.pose_graph || ctx->cfg.use_cloud_ring) {
        ctx->err = "slo_pipeline: not with IMU input, loop verification, the pose graph or useCloudRing";
        return SLO_E_STATE;
    }
    SLO_CHECK(hipSetDevice(ctx->dev));
    slo::pipe_free(ctx);
    if (depth == 0) return SLO_OK;
    slo::SloPipe* p = new (std::nothrow) slo::SloPipe();
    if (!p) return SLO_E_CAPACITY;
    ctx->pipe = p;
    int r = slo_create(&ctx->cfg, ctx->dev, ctx->S, &p->front);
    if (!r) r = slo_create(&ctx->cfg, ctx->dev, ctx->S, &p->odo);
    if (!r) r = slo::map_ws_ensure(ctx);
    if (r) {
        slo::pipe_free(ctx);
        return r;
    }
    p->D = depth;
    p->fbytes = slo_modes_features_bytes(ctx);
    p->obytes = slo_modes_odom_bytes(ctx);
    p->rbytes = (size_t)ctx->S * ctx->v.P * sizeof(float4);
    bool ok = true;
    for (int i = 0; i < depth && ok; ++i) {
        void *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
        hipEvent_t e[3] = {nullptr, nullptr, nullptr};
        ok = hipMalloc(&a, p->fbytes) == hipSuccess && hipMalloc(&b, p->obytes) == hipSuccess &&
             hipMalloc(&c, p->rbytes) == hipSuccess && hipMalloc(&d, sizeof(int32_t) * ctx->S) == hipSuccess;
        for (int j = 0; j < 3 && ok; ++j) ok = hipEventCreateWithFlags(&e[j], hipEventDisableTiming) == hipSuccess;
        p->feat.push_back(a); p->odom.push_back(b); p->raw.push_back(c); p->cnt.push_back(d);
        p->evF.push_back(e[0]); p->evO.push_back(e[1]); p->evM.push_back(e[2]);
    }
    if (!ok) {
        slo::pipe_free(ctx);
        ctx->err = "slo_pipeline: out of device memory for the stage rings";
        return SLO_E_HIP;
    }
    return SLO_OK;
}

int slo_batch_loop_closure(slo_ctx* ctx) {
    if (!ctx) return SLO_E_ARG;
    if (!ctx->cfg.loop_verify) { ctx->err = "loop verification needs cfg.loop_verify"; return SLO_E_STATE; }
    SLO_CHECK(hipSetDevice(ctx->dev));
    return slo::lc_run(ctx);
}

int slo_loop_closure(slo_ctx* ctx, slo_loop_result* out) {
    if (!ctx || !out) return SLO_E_ARG;
    int r = slo_batch_loop_closure(ctx);
    if (r) return r;
    SLO_CHECK(hipMemcpyAsync(out, ctx->lc.res, 2 * sizeof(slo_loop_result), hipMemcpyDeviceToHost, ctx->stream));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    return SLO_OK;
}

int slo_icp_align_batch(slo_ctx* ctx, const void* d_src, size_t src_stride, const int32_t* d_nsrc, const void* d_tgt,
                        size_t tgt_stride, const int32_t* d_ntgt, slo_loop_result* h_out) {
    if (!ctx || !d_src || !d_nsrc || !d_tgt || !d_ntgt || !h_out) return SLO_E_ARG;
    if (!ctx->cfg.loop_verify) { ctx->err = "ICP needs cfg.loop_verify (its buffers)"; return SLO_E_STATE; }
    SLO_CHECK(hipSetDevice(ctx->dev));
    int r = slo::lc_icp_run(ctx, (const float4*)d_src, src_stride, d_nsrc, (const float4*)d_tgt, tgt_stride, d_ntgt);
    if (r) return r;
    SLO_CHECK(hipMemcpy2DAsync(h_out, sizeof(slo_loop_result), ctx->lc.res + 1, 2 * sizeof(slo_loop_result),
                               sizeof(slo_loop_result), ctx->S, hipMemcpyDeviceToHost, ctx->stream));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    return SLO_OK;
}

// ---------------------------------------------------------------- readback
int slo_get(slo_ctx* ctx, int stream, const char* name_c, void* dst, size_t cap_bytes) {
    if (!ctx || !name_c || stream < 0 || stream >= ctx->S) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    if (ctx->pipe) {   // slo_pipeline: the field from the stage that computes it
        slo_ctx* st = slo::pipe_stage_of(ctx, std::string(name_c));
        if (st != ctx) return slo_get(st, stream, name_c, dst, cap_bytes);
    }
    slo::timing_flush(ctx);
    const DevView& v = ctx->v;
    StreamState st;
    SLO_CHECK(hipMemcpy(&st, v.st + stream, sizeof(st), hipMemcpyDeviceToHost));
    const std::string name(name_c);
    const size_t s = stream, H = v.H, R = v.cfg.n_scan;
    const void* src = nullptr;
    size_t count = 0, esz = 0;
    std::vector<char> tmp;
    auto dev = [&](const void* p, size_t n, size_t e) { src = p; count = n; esz = e; };
    if (name == "range") dev(v.range + s * H, H, 4);
    else if (name == "label") dev(v.label + s * H, H, 4);
    else if (name == "ground") dev(v.ground + s * H, H, 1);
    else if (name == "full_cloud") dev(v.full + s * H, H, 16);
    else if (name == "seg_pts") dev(v.seg + s * H, st.seg_count, 16);
    else if (name == "seg_ground") dev(v.seg_ground + s * H, st.seg_count, 1);
    else if (name == "seg_col") dev(v.seg_col + s * H, st.seg_count, 4);
    else if (name == "seg_range") dev(v.seg_range + s * H, st.seg_count, 4);
    else if (name == "ring_start" || name == "ring_end") {
        std::vector<int32_t> se(2 * R);
        SLO_CHECK(hipMemcpy(se.data(), v.ring_se + s * 2 * R, sizeof(int32_t) * 2 * R, hipMemcpyDeviceToHost));
        tmp.resize(4 * R);
        for (size_t i = 0; i < R; ++i) ((int32_t*)tmp.data())[i] = se[2 * i + (name == "ring_end")];
        count = R; esz = 4;
    } else if (name == "orient") dev(v.orient + 3 * s, 3, 4);
    else if (name == "outlier") dev(v.outlier + s * H, st.outlier_count, 16);
    else if (name == "fa_seg_pts") dev(v.fpts + s * H, st.seg_count, 16);
    else if (name == "curvature") dev(v.curv + s * H, H, 4);
    else if (name == "picked") dev(v.picked + s * H, H, 4);
    else if (name == "cloud_label") dev(v.clabel + s * H, H, 4);
    else if (name == "smooth_ind") {
        std::vector<slo::Smooth> sm(H);
        SLO_CHECK(hipMemcpy(sm.data(), v.smooth + s * H, sizeof(slo::Smooth) * H, hipMemcpyDeviceToHost));
        tmp.resize(4 * H);
        for (size_t i = 0; i < H; ++i) ((int32_t*)tmp.data())[i] = sm[i].ind;
        count = H; esz = 4;
    } else if (name == "sharp") dev(v.sharp + s * v.cap_sharp, st.n_sharp, 16);
    else if (name == "less_sharp") dev(v.less_sharp + s * v.cap_less_sharp, st.n_less_sharp, 16);
    else if (name == "flat") dev(v.flat + s * v.cap_flat, st.n_flat, 16);
    else if (name == "less_flat") dev(v.less_flat + s * v.cap_less_flat, st.n_less_flat, 16);
    else if (name == "corner_last") dev(v.corner_last + s * v.cap_less_sharp, st.cornerLastNum, 16);
    else if (name == "surf_last") dev(v.surf_last + s * v.cap_less_flat, st.surfLastNum, 16);
    else if (name == "transform_sum") { tmp.resize(24); memcpy(tmp.data(), st.transformSum, 24); count = 6; esz = 4; }
    else if (name == "integrated") { tmp.resize(24); memcpy(tmp.data(), st.integrated, 24); count = 6; esz = 4; }
    else if (name == "transform_cur") { tmp.resize(24); memcpy(tmp.data(), st.transformCur, 24); count = 6; esz = 4; }
    else if (name == "fa_iters") { int32_t a[2] = {st.iters_surf, st.iters_corner}; tmp.resize(8); memcpy(tmp.data(), a, 8); count = 2; esz = 4; }
    else if (name == "mapped") { tmp.resize(24); memcpy(tmp.data(), st.transformAftMapped, 24); count = 6; esz = 4; }
    else if (name == "n_keyframes") { tmp.resize(4); memcpy(tmp.data(), &st.n_keyframes, 4); count = 1; esz = 4; }
    else if (name == "flags") {
        int32_t f = (st.mo_ran ? 2 : 0) | (st.kf_saved ? 4 : 0) | (st.det_valid ? 8 : 0);
        tmp.resize(4); memcpy(tmp.data(), &f, 4); count = 1; esz = 4;
    }
    else if (name == "tobe_mapped") { tmp.resize(24); memcpy(tmp.data(), st.transformTobeMapped, 24); count = 6; esz = 4; }
    else if (name == "mo_iters") { tmp.resize(4); memcpy(tmp.data(), &st.mo_iters, 4); count = 1; esz = 4; }
    else if (name == "err") {   // the stream's sticky bits, with the VoxelGrid sorts' own per-stream flags
        int32_t e = st.err;
        for (const slo::PclWs* pw : {&ctx->pws, &ctx->pws2}) {
            int32_t x = 0;
            for (int g = 0; pw->serr && g < VG_MAXG; ++g) {   // every filter's virtual stream (vg_run_groups)
                SLO_CHECK(hipMemcpy(&x, pw->serr + (size_t)g * ctx->S + stream, 4, hipMemcpyDeviceToHost));
                e |= x;
            }
        }
        tmp.resize(4); memcpy(tmp.data(), &e, 4); count = 1; esz = 4;
    }
    else if (name == "vg_stats") {   // PCL-order sort (slo_vgpcl.hip): [0] ranges the one-lane fallback took,
                                     // [2] inconsistent wave-sort steps, [3] / [4] inconsistent tail cuts /
                                     // partners (2-4 must stay 0); [1] clipped outputs
        int32_t a[5] = {0, 0, 0, 0, 0};
        for (const slo::PclWs* pw : {&ctx->pws, &ctx->pws2}) {   // the side stream's sorts count in pws2
            int32_t c[4] = {0, 0, 0, 0};
            if (pw->cstat) SLO_CHECK(hipMemcpy(c, pw->cstat, 16, hipMemcpyDeviceToHost));
            a[0] += c[0]; a[2] += c[1]; a[3] += c[2]; a[4] += c[3];
        }
        for (const slo::MapWs* mw : {&ctx->mws, &ctx->mws2}) {
            int32_t e = 0;
            if (mw->errflag) SLO_CHECK(hipMemcpy(&e, mw->errflag, 4, hipMemcpyDeviceToHost));
            a[1] |= e;
        }
        tmp.resize(20); memcpy(tmp.data(), a, 20); count = 5; esz = 4;
    }
    else if (name == "pcl_work") {   // PCL-order sort work counters, cumulative (slo_vgpcl.hip PW_*)
        unsigned long long a[32] = {0};
        for (const slo::PclWs* pw : {&ctx->pws, &ctx->pws2}) {   // the side stream's sorts count in pws2
            unsigned long long b[32] = {0};
            if (pw->pstat) SLO_CHECK(hipMemcpy(b, pw->pstat, sizeof(b), hipMemcpyDeviceToHost));
            for (int i = 0; i < 32; ++i) a[i] += b[i];
        }
        tmp.resize(sizeof(a)); memcpy(tmp.data(), a, sizeof(a)); count = 32; esz = 8;
    }
    else if (name == "dbg") { tmp.resize(64); memcpy(tmp.data(), st.dbg, 64); count = 8; esz = 8; }
    else if (name == "work") dev(v.wctr, 8, 8);   // context-wide work counters (DevView::wctr)
    else if (name == "imu") {   // FA's IMU scalars (slo::ImuState), as float64
        slo::ImuState m;
        SLO_CHECK(hipMemcpy(&m, v.imu + stream, sizeof(m), hipMemcpyDeviceToHost));
        const double a[23] = {(double)m.last, (double)m.last_iter, m.rollStart, m.pitchStart, m.yawStart,
                              m.veloStart[0], m.veloStart[1], m.veloStart[2], m.rollCur, m.pitchCur, m.yawCur,
                              m.veloFromStartCur[0], m.veloFromStartCur[1], m.veloFromStartCur[2], m.angLast[0],
                              m.angLast[1], m.angLast[2], m.angFromStart[0], m.angFromStart[1], m.angFromStart[2],
                              m.rollLast, m.pitchLast, m.yawLast};
        tmp.resize(sizeof(a)); memcpy(tmp.data(), a, sizeof(a)); count = 23; esz = 8;
    }
    else if (name == "keyposes") dev(v.kf_pose + s * v.KFMAX * 6, (size_t)st.n_keyframes * 6, 4);
    else if (name == "vg_in") {   // the items of the last mapping step's seven batched VoxelGrids (map_run order)
        slo::SloIo io;
        SLO_CHECK(hipMemcpy(&io, ctx->d_io, sizeof(io), hipMemcpyDeviceToHost));
        int32_t raw = 0;
        if (io.npts) SLO_CHECK(hipMemcpy(&raw, io.npts + stream, 4, hipMemcpyDeviceToHost));
        const int32_t a[7] = {st.n_corner_map, st.n_surf_map, raw, st.cornerLastNum, st.surfLastNum,
                              st.outlier_count, st.n_st};
        tmp.resize(sizeof(a)); memcpy(tmp.data(), a, sizeof(a)); count = 7; esz = 4;
    }
    else if (name == "counts") {   // the stream's cloud sizes in one read (bench.py's algorithmic-byte models):
        // [0] segmented, [1] outliers, [2] sharp, [3] less sharp, [4] flat, [5] less flat (after the ring
        // VoxelGrid), [6] less-flat ring points before it (FA:779 input), [7] cornerLast, [8] surfLast,
        // [9] kd corner, [10] kd surf, [11] corner DS, [12] surf-total DS, [13] map corner DS, [14] map surf
        // DS, [15] raw DS, [16..16+R] the less-flat ring offsets of the current scan (x-sorts' segments)
        std::vector<int32_t> lf(R);
        SLO_CHECK(hipMemcpy(lf.data(), v.r_lf_n + s * R, 4 * R, hipMemcpyDeviceToHost));
        int32_t lfn = 0;
        for (size_t i = 0; i < R; ++i) lfn += lf[i];
        std::vector<int32_t> a{st.seg_count, st.outlier_count, st.n_sharp, st.n_less_sharp, st.n_flat, st.n_less_flat,
                               lfn, st.cornerLastNum, st.surfLastNum, st.kdCornerNum, st.kdSurfNum, st.n_corner_ds,
                               st.n_surf_total_ds, st.n_cmap_ds, st.n_smap_ds, st.n_raw_ds};
        a.resize(16 + R + 1);
        SLO_CHECK(hipMemcpy(a.data() + 16, v.roff_cur + (s * 2 + 1) * (R + 1), 4 * (R + 1), hipMemcpyDeviceToHost));
        tmp.resize(4 * a.size()); memcpy(tmp.data(), a.data(), tmp.size()); count = a.size(); esz = 4;
    }
    else if (name == "map_raw_n") {   // laserCloudCornerFromMap / laserCloudSurfFromMap sizes before their VoxelGrids
        int32_t a[2] = {st.n_corner_map, st.n_surf_map}; tmp.resize(8); memcpy(tmp.data(), a, 8); count = 2; esz = 4;
    }
    else if (name == "map_ids") {   // keyframes of the last local map, in concatenation order
        if (v.cfg.loop_closure_enable) { tmp.resize(4 * st.recent_n); memcpy(tmp.data(), st.recent_ids, 4 * st.recent_n); count = st.recent_n; esz = 4; }
        else dev(v.map_ids + s * v.MAPK, st.recent_n, 4);
    }
    else if (name == "raw_ds") dev(v.cur_raw_ds + s * v.P, st.n_raw_ds, 16);
    else if (name == "corner_ds") dev(v.cur_c_ds + s * v.cap_less_sharp, st.n_corner_ds, 16);
    else if (name == "surf_total_ds") dev(v.cur_st_ds + s * v.cap_st, st.n_surf_total_ds, 16);
    else if (name == "map_corner_ds") dev(v.map_c_ds + s * v.cap_mc, st.n_cmap_ds, 16);
    else if (name == "map_surf_ds") dev(v.map_s_ds + s * v.cap_ms, st.n_smap_ds, 16);
    else if (name == "sc_desc" || name == "ring_key" || name == "sector_key") {
        if (st.sc_count == 0) { count = 0; esz = 8; }
        else {
            const size_t NR = v.cfg.sc_num_ring, NSc = v.cfg.sc_num_sector, k = st.sc_count - 1;
            if (name == "sc_desc") dev(v.sc_desc + (s * v.KFMAX + k) * NR * NSc, NR * NSc, 8);
            else if (name == "ring_key") dev(v.sc_ringd + (s * v.KFMAX + k) * NR, NR, 8);
            else dev(v.sc_sect + (s * v.KFMAX + k) * NSc, NSc, 8);
        }
    } else if (name == "detect") {
        if (!st.det_valid) { count = 0; esz = 4; }
        else {
            std::vector<int32_t> d{st.det_loop_id, st.det_nn_idx, st.sc_count >= v.cfg.sc_num_exclude_recent + 1 ? v.cfg.sc_num_candidates : 0};
            for (int i = 0; i < d[2]; ++i) d.push_back(st.det_cand[i]);
            tmp.resize(4 * d.size()); memcpy(tmp.data(), d.data(), 4 * d.size()); count = d.size(); esz = 4;
        }
    } else if (name == "detect_f") {
        if (!st.det_valid) { count = 0; esz = 8; }
        else { double d[2] = {(double)st.det_yaw, st.det_min_dist}; tmp.resize(16); memcpy(tmp.data(), d, 16); count = 2; esz = 8; }
    } else if (name == "loop") {   // RS, SC verification of this scan's detect
        if (ctx->cfg.loop_verify && st.det_valid) dev(ctx->lc.res + 2 * s, 2, sizeof(slo_loop_result));
        else { count = 0; esz = sizeof(slo_loop_result); }
    } else if (name == "key_times") {
        if (ctx->cfg.loop_verify) dev(ctx->lc.ktime + s * v.KFMAX, std::min(st.n_keyframes, v.KFMAX), 8);
        else { count = 0; esz = 8; }
    }
    else return SLO_E_ARG;
    const size_t bytes = std::min(cap_bytes, count * esz);
    if (dst && bytes) {
        if (src) SLO_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
        else memcpy(dst, tmp.data(), bytes);
    }
    return (int)count;
}

int slo_timing_enable(slo_ctx* ctx, int enable) {
    if (!ctx) return SLO_E_ARG;
    if (ctx->timing != (enable != 0)) slo::graphs_drop(ctx);   // captured graphs carry the timing launches
    ctx->timing = enable != 0;
    return SLO_OK;
}
int slo_timing_filter(slo_ctx* ctx, const char* name) {
    if (!ctx) return SLO_E_ARG;
    slo::timing_flush(ctx);   // stamps of the previous filter
    slo::graphs_drop(ctx);
    ctx->timing_only = name ? name : "";
    ctx->stamp_names.clear();
    for (size_t a = 0; a < ctx->timing_only.size();) {
        size_t b = ctx->timing_only.find(',', a);
        if (b == std::string::npos) b = ctx->timing_only.size();
        if (b > a) ctx->stamp_names.push_back(ctx->timing_only.substr(a, b - a));
        a = b + 1;
    }
    return SLO_OK;
}
int slo_timing_reset(slo_ctx* ctx) {
    if (!ctx) return SLO_E_ARG;
    slo::timing_flush(ctx);
    ctx->ktimes.clear();
    return SLO_OK;
}
int slo_timing_read(slo_ctx* ctx, char* names_buf, size_t buf_bytes, double* total_ms, int64_t* launches, int cap) {
    if (!ctx) return SLO_E_ARG;
    slo::timing_flush(ctx);
    int i = 0;
    size_t off = 0;
    for (auto& kv : ctx->ktimes) {
        if (i >= cap) break;
        size_t L = kv.first.size() + 1;
        if (names_buf && off + L <= buf_bytes) { memcpy(names_buf + off, kv.first.c_str(), L); off += L; }
        if (total_ms) total_ms[i] = kv.second.total_ms;
        if (launches) launches[i] = kv.second.n;
        ++i;
    }
    return i;
}

int slo_gen_scan(int preset, int config_id, int stream_id, int scan_index, float* out_xyzi) {
    slo_config cfg;
    if (slo_config_preset_impl(preset, &cfg) || !out_xyzi) return SLO_E_ARG;
    slo_gen::Stream s = slo_gen::make_stream(cfg, config_id, stream_id);
    return slo_gen::stream_scan(s, scan_index, out_xyzi);
}

// ---------------------------------------------------------------- single scan (stream 0)
static int stage_points(slo_ctx* ctx, const void* pts, size_t n, size_t stride, size_t off_xyz, size_t off_i) {
    if (n > (size_t)ctx->cfg.max_points) { ctx->err = "too many points"; return SLO_E_CAPACITY; }
    const size_t need = n * 16 + 16;
    if (ctx->h_stage_bytes < need) {
        if (ctx->h_stage) hipHostFree(ctx->h_stage);
        ctx->h_stage = nullptr;
        SLO_CHECK(hipHostMalloc(&ctx->h_stage, need));
        ctx->h_stage_bytes = need;
    }
    float* h = (float*)ctx->h_stage;
    const char* b = (const char*)pts;
    for (size_t i = 0; i < n; ++i) {
        memcpy(h + 4 * i, b + i * stride + off_xyz, 12);
        memcpy(h + 4 * i + 3, b + i * stride + off_i, 4);
    }
    int32_t cnt = (int32_t)n;
    memcpy(h + 4 * n, &cnt, 4);
    SLO_CHECK(hipMemcpyAsync(ctx->d_in, h, n * 16, hipMemcpyHostToDevice, ctx->stream));
    SLO_CHECK(hipMemcpyAsync(ctx->d_cnt, h + 4 * n, 4, hipMemcpyHostToDevice, ctx->stream));
    return SLO_OK;
}

// copy `bytes` of device memory into view slot `slot`; returns the host pointer
static const void* view_copy(slo_ctx* ctx, int slot, const void* dsrc, size_t bytes, int* rc) {
    auto& b = ctx->h_view[slot];
    b.resize(std::max<size_t>(bytes, 16));
    if (bytes) {
        hipError_t e = hipMemcpy(b.data(), dsrc, bytes, hipMemcpyDeviceToHost);
        if (e != hipSuccess) { ctx->err = hipGetErrorString(e); *rc = SLO_E_HIP; }
    }
    return b.data();
}

// The three node-level entry points drive a one-stream context exactly like
// the reference callbacks; a batched context must use slo_batch_*.
static int single_stream(slo_ctx* ctx) {
    if (ctx->S != 1) { ctx->err = "single-scan entry points need a context with n_streams == 1"; return SLO_E_STATE; }
    return SLO_OK;
}

// ImageProjection::cloudHandler (IP:181-196): copyPointCloud .. cloudSegmentation;
// *out mirrors /segmented_cloud, /segmented_cloud_info and /outlier_cloud.
int slo_image_projection_ring(slo_ctx* ctx, const void* pts, size_t n, size_t stride_bytes, size_t off_xyz,
                              size_t off_i, const uint16_t* rings, slo_seg_view* out) {
    if (!ctx || (!pts && n) || !out) return SLO_E_ARG;
    if (ctx->cfg.use_cloud_ring && !rings && n) { ctx->err = "cfg.use_cloud_ring needs rings"; return SLO_E_ARG; }
    int r = single_stream(ctx);
    if (r) return r;
    SLO_CHECK(hipSetDevice(ctx->dev));
    r = stage_points(ctx, pts, n, stride_bytes, off_xyz, off_i);
    if (r) return r;
    if (ctx->cfg.use_cloud_ring) {
        if (n) SLO_CHECK(hipMemcpyAsync(ctx->d_ring_in, rings, 2 * n, hipMemcpyHostToDevice, ctx->stream));
        ctx->v.rings = ctx->d_ring_in;
    }
    if ((r = slo::set_io(ctx, ctx->d_in, ctx->d_cnt))) return r;
    r = slo::ip_run(ctx);
    if (r) return r;
    memset(out, 0, sizeof(*out));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    const DevView& v = ctx->v;
    StreamState st;
    SLO_CHECK(hipMemcpy(&st, v.st, sizeof(st), hipMemcpyDeviceToHost));
    const int R = v.cfg.n_scan;
    int rc = SLO_OK;
    out->n_segmented = st.seg_count;
    out->segmented = (const float*)view_copy(ctx, 0, v.seg, 16 * (size_t)st.seg_count, &rc);
    out->ground_flag = (const uint8_t*)view_copy(ctx, 1, v.seg_ground, (size_t)st.seg_count, &rc);
    out->col_ind = (const uint32_t*)view_copy(ctx, 2, v.seg_col, 4 * (size_t)st.seg_count, &rc);
    out->range = (const float*)view_copy(ctx, 3, v.seg_range, 4 * (size_t)st.seg_count, &rc);
    const int32_t* se = (const int32_t*)view_copy(ctx, 4, v.ring_se, 8 * (size_t)R, &rc);
    for (int i = 0; i < R; ++i) { ctx->h_ring[0][i] = se[2 * i]; ctx->h_ring[1][i] = se[2 * i + 1]; }
    out->start_ring_index = ctx->h_ring[0];
    out->end_ring_index = ctx->h_ring[1];
    const float* o = (const float*)view_copy(ctx, 5, v.orient, 12, &rc);
    out->start_orientation = o[0]; out->end_orientation = o[1]; out->orientation_diff = o[2];
    out->n_outlier = st.outlier_count;
    out->outlier = (const float*)view_copy(ctx, 6, v.outlier, 16 * (size_t)st.outlier_count, &rc);
    return rc;
}

int slo_image_projection(slo_ctx* ctx, const void* pts, size_t n, size_t stride_bytes, size_t off_xyz, size_t off_i,
                         slo_seg_view* out) {
    return slo_image_projection_ring(ctx, pts, n, stride_bytes, off_xyz, off_i, nullptr, out);
}

// FeatureAssociation::runFeatureAssociation (FA:1817-1859) on the result of
// the previous slo_image_projection.  sharp/flat are this scan's features
// (start of sweep); less_sharp/less_flat are laserCloudCornerLast /
// laserCloudSurfLast after TransformToEnd (what FA publishes, FA:1790-1814).
int slo_feature_association(slo_ctx* ctx, double t_scan, slo_fa_view* out) {
    if (!ctx || !out) return SLO_E_ARG;
    int r = single_stream(ctx);
    if (r) return r;
    if ((r = slo_batch_scan_time(ctx, t_scan))) return r;   // cloudHeader.stamp: read by the IMU path only (Q13)
    r = slo_batch_feature_association(ctx);
    if (r) return r;
    memset(out, 0, sizeof(*out));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    const DevView& v = ctx->v;
    StreamState st;
    SLO_CHECK(hipMemcpy(&st, v.st, sizeof(st), hipMemcpyDeviceToHost));
    int rc = SLO_OK;
    memcpy(out->transform_sum, st.transformSum, 24);
    out->n_sharp = st.n_sharp; out->n_flat = st.n_flat;
    out->n_less_sharp = st.cornerLastNum; out->n_less_flat = st.surfLastNum;
    out->sharp = (const float*)view_copy(ctx, 7, v.sharp, 16 * (size_t)st.n_sharp, &rc);
    out->flat = (const float*)view_copy(ctx, 8, v.flat, 16 * (size_t)st.n_flat, &rc);
    out->less_sharp = (const float*)view_copy(ctx, 9, v.corner_last, 16 * (size_t)st.cornerLastNum, &rc);
    out->less_flat = (const float*)view_copy(ctx, 10, v.surf_last, 16 * (size_t)st.surfLastNum, &rc);
    out->published = ctx->fa_published;
    return rc;
}

// mapOptimization::run (MO:1673-1706) minus GTSAM / publishing: gating on the
// FA publish and mappingProcessInterval, then transformAssociateToMap ..
// saveKeyFramesAndFactor incl. makeAndSaveScancontextAndKeys on the raw scan.
int slo_map_optimization(slo_ctx* ctx, const void* raw_pts, size_t n, size_t stride_bytes, size_t off_xyz,
                         size_t off_i, double t_scan, slo_map_view* out) {
    if (!ctx || (!raw_pts && n) || !out) return SLO_E_ARG;
    int r = single_stream(ctx);
    if (r) return r;
    SLO_CHECK(hipSetDevice(ctx->dev));
    r = stage_points(ctx, raw_pts, n, stride_bytes, off_xyz, off_i);
    if (r) return r;
    r = slo_batch_map_optimization(ctx, ctx->d_in, ctx->d_cnt, t_scan);
    if (r) return r;
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    StreamState st;
    SLO_CHECK(hipMemcpy(&st, ctx->v.st, sizeof(st), hipMemcpyDeviceToHost));
    memset(out, 0, sizeof(*out));
    out->ran = st.mo_ran;
    out->keyframe_saved = st.kf_saved;
    out->n_keyframes = st.n_keyframes;
    memcpy(out->transform_aft_mapped, st.transformAftMapped, 24);
    return SLO_OK;
}

int slo_sc_make_and_save(slo_ctx* ctx, const void* pts, size_t n, size_t stride_bytes, size_t off_xyz,
                         size_t off_i) {
    if (!ctx || (!pts && n)) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    int r = stage_points(ctx, pts, n, stride_bytes, off_xyz, off_i);
    if (r) return r;
    // one workgroup = stream 0
    r = slo::sc_make_run(ctx, ctx->d_in, (size_t)ctx->cfg.max_points, ctx->d_cnt, 1, 1);
    if (r) return r;
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    return SLO_OK;
}

int slo_sc_detect(slo_ctx* ctx, int32_t* loop_id, float* yaw_rad, double* min_dist) {
    if (!ctx || !loop_id || !yaw_rad || !min_dist) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    int r = slo::sc_detect_run_one(ctx);
    if (r) return r;
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    StreamState st;
    SLO_CHECK(hipMemcpy(&st, ctx->v.st, sizeof(st), hipMemcpyDeviceToHost));
    *loop_id = st.det_loop_id;
    *yaw_rad = st.det_yaw;
    *min_dist = st.det_min_dist;
    return SLO_OK;
}

int slo_batch_sc_make(slo_ctx* ctx, const void* d_points, const int32_t* d_counts) {
    if (!ctx || !d_points || !d_counts) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    DevView& v = ctx->v;
    const int SS = (int)(sizeof(StreamState) / sizeof(int32_t));
    int r = slo::vg_run(ctx, "raw", (const float4*)d_points, v.P, d_counts, 1, v.cfg.leaf_sc, v.cur_raw_ds, v.P,
                        &v.st->n_raw_ds, SS, v.P);
    if (!r) r = slo::pcl_fold_err(ctx);
    if (r) return r;
    return slo::sc_make_run(ctx, v.cur_raw_ds, v.P, &v.st->n_raw_ds, SS, ctx->S);
}

// the SCManager helpers on host data: stage the inputs, one launch, read back
static int sc_api_host(slo_ctx* ctx, int op, const void* a, size_t na, const void* b, size_t nb, const int32_t* n,
                       size_t stride, void* o1, size_t no1, void* o2, size_t no2, void* o3, size_t no3) {
    SLO_CHECK(hipSetDevice(ctx->dev));
    const size_t al = 256, sz[6] = {na, nb, (size_t)(n ? 4 : 0), no1, no2, no3};
    size_t off[7] = {0};
    for (int i = 0; i < 6; ++i) off[i + 1] = off[i] + (sz[i] + al - 1) / al * al;
    char* d = nullptr;
    SLO_CHECK(hipMalloc(&d, std::max<size_t>(off[6], al)));
    auto dp = [&](int i) -> void* { return sz[i] ? d + off[i] : nullptr; };
    hipError_t e = hipSuccess;
    if (na) e = hipMemcpyAsync(dp(0), a, na, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess && nb) e = hipMemcpyAsync(dp(1), b, nb, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess && n) e = hipMemcpyAsync(dp(2), n, 4, hipMemcpyHostToDevice, ctx->stream);
    int r = e == hipSuccess ? slo::sc_api_run(ctx, op, 1, dp(0), dp(1), stride, (const int32_t*)dp(2), dp(3), dp(4),
                                               dp(5))
                            : SLO_E_HIP;
    void* outs[3] = {o1, o2, o3};
    for (int i = 0; i < 3 && !r; ++i)
        if (sz[3 + i] && outs[i] && hipMemcpyAsync(outs[i], dp(3 + i), sz[3 + i], hipMemcpyDeviceToHost, ctx->stream))
            r = SLO_E_HIP;
    if (hipStreamSynchronize(ctx->stream) != hipSuccess && !r) r = SLO_E_HIP;
    hipFree(d);
    if (r == SLO_E_HIP) ctx->err = "SCManager helper: HIP copy / launch failed";
    return r;
}

int slo_sc_make_scancontext(slo_ctx* ctx, const void* pts, size_t n, size_t stride_bytes, size_t off_xyz,
                            double* desc) {
    if (!ctx || (!pts && n) || !desc || (n && stride_bytes < off_xyz + 12)) return SLO_E_ARG;
    const int NR = ctx->cfg.sc_num_ring, NS = ctx->cfg.sc_num_sector;
    std::vector<float> p4(4 * std::max<size_t>(n, 1), 0.0f);
    for (size_t i = 0; i < n; ++i) memcpy(&p4[4 * i], (const char*)pts + i * stride_bytes + off_xyz, 12);
    const int32_t cnt = (int32_t)n;
    return sc_api_host(ctx, 0, p4.data(), p4.size() * 4, nullptr, 0, &cnt, std::max<size_t>(n, 1), desc,
                       sizeof(double) * NR * NS, nullptr, sizeof(double) * NR, nullptr, sizeof(double) * NS);
}

int slo_sc_ring_key(slo_ctx* ctx, const double* desc, double* ring_key) {
    if (!ctx || !desc || !ring_key) return SLO_E_ARG;
    const int NR = ctx->cfg.sc_num_ring, NS = ctx->cfg.sc_num_sector;
    return sc_api_host(ctx, 1, desc, sizeof(double) * NR * NS, nullptr, 0, nullptr, 0, ring_key, sizeof(double) * NR,
                       nullptr, sizeof(double) * NS, nullptr, 0);
}

int slo_sc_sector_key(slo_ctx* ctx, const double* desc, double* sector_key) {
    if (!ctx || !desc || !sector_key) return SLO_E_ARG;
    const int NR = ctx->cfg.sc_num_ring, NS = ctx->cfg.sc_num_sector;
    return sc_api_host(ctx, 1, desc, sizeof(double) * NR * NS, nullptr, 0, nullptr, 0, nullptr, sizeof(double) * NR,
                       sector_key, sizeof(double) * NS, nullptr, 0);
}

int slo_sc_fast_align(slo_ctx* ctx, const double* vkey1, const double* vkey2, int32_t* shift) {
    if (!ctx || !vkey1 || !vkey2 || !shift) return SLO_E_ARG;
    const int NS = ctx->cfg.sc_num_sector;
    return sc_api_host(ctx, 2, vkey1, sizeof(double) * NS, vkey2, sizeof(double) * NS, nullptr, 0, shift, 4, nullptr,
                       0, nullptr, 0);
}

int slo_sc_dist_direct(slo_ctx* ctx, const double* sc1, const double* sc2, double* dist) {
    if (!ctx || !sc1 || !sc2 || !dist) return SLO_E_ARG;
    const size_t nb = sizeof(double) * ctx->cfg.sc_num_ring * ctx->cfg.sc_num_sector;
    return sc_api_host(ctx, 3, sc1, nb, sc2, nb, nullptr, 0, dist, 8, nullptr, 0, nullptr, 0);
}

int slo_sc_distance(slo_ctx* ctx, const double* sc1, const double* sc2, double* dist, int32_t* shift) {
    if (!ctx || !sc1 || !sc2 || !dist || !shift) return SLO_E_ARG;
    const size_t nb = sizeof(double) * ctx->cfg.sc_num_ring * ctx->cfg.sc_num_sector;
    return sc_api_host(ctx, 4, sc1, nb, sc2, nb, nullptr, 0, dist, 8, shift, 4, nullptr, 0);
}

int slo_batch_sc_distance(slo_ctx* ctx, const double* d_sc1, const double* d_sc2, int n, double* d_dist,
                          int32_t* d_shift) {
    if (!ctx || !d_sc1 || !d_sc2 || !d_dist || !d_shift || n < 0) return SLO_E_ARG;
    if (n == 0) return SLO_OK;
    SLO_CHECK(hipSetDevice(ctx->dev));
    return slo::sc_api_run(ctx, 4, n, d_sc1, d_sc2, 0, nullptr, d_dist, d_shift, nullptr);
}

int slo_batch_voxel_grid(slo_ctx* ctx, const void* d_in, size_t in_stride, const int32_t* d_n, float leaf,
                         void* d_out, size_t out_stride, int32_t* d_nout, int out_cap) {
    if (!ctx || !d_in || !d_n || !d_out || !d_nout || in_stride == 0 || out_cap < 0 || !(leaf > 0.0f))
        return SLO_E_ARG;
    if ((size_t)out_cap > out_stride) {   // stream s writes out[s * out_stride + r] for r < out_cap
        ctx->err = "slo_batch_voxel_grid: out_cap exceeds out_stride (output rows would overlap)";
        return SLO_E_ARG;
    }
    SLO_CHECK(hipSetDevice(ctx->dev));
    return slo::vg_run(ctx, "user", (const float4*)d_in, in_stride, d_n, 1, leaf, (float4*)d_out, out_stride, d_nout,
                       1, out_cap);
}

int slo_pack_records(slo_ctx* ctx, void* d_out) {
    if (!ctx || !d_out) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    return slo::pack_records_run(ctx, (float*)d_out);
}

int slo_record_floats(void) { return SLO_RECORD_FLOATS; }

int slo_gen_batch(int preset, int config_id, int stream0, int n_streams, int scan0, int n_scans, float* out,
                  int n_threads) {
    slo_config cfg;
    if (slo_config_preset_impl(preset, &cfg) || !out || n_streams <= 0 || n_scans <= 0) return SLO_E_ARG;
    const size_t P = (size_t)cfg.max_points;
    std::vector<slo_gen::Stream> st;
    for (int s = 0; s < n_streams; ++s) st.push_back(slo_gen::make_stream(cfg, config_id, stream0 + s));
    std::atomic<int> next{0};
    auto work = [&]() {
        while (true) {
            int j = next++;
            if (j >= n_streams * n_scans) break;
            int s = j / n_scans, k = j % n_scans;
            // layout [scan][stream][P][4]
            slo_gen::stream_scan(st[s], scan0 + k, out + ((size_t)k * n_streams + s) * P * 4);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < std::max(1, n_threads); ++t) th.emplace_back(work);
    for (auto& t : th) t.join();
    return SLO_OK;
}

}  // extern "C"
