// oracle_api.cpp — TEST INFRASTRUCTURE ONLY: C ABI over the CPU restatement,
// loaded by tests/ (ctypes), __graft_entry__.smoke() and bench.py's
// cpu_baseline leg.  Never linked into the product library.
//
// oracle_step() runs one scan through the reference's three nodes with the
// deterministic gating of SURVEY §8(d) replacing ROS timing (Appendix A Q13):
//   imageProjection every scan -> featureAssociation every scan ->
//   mapOptimization when FA publishes (every skipFrameNum+1 = 2nd scan) and
//   t - t_last >= mappingProcessInterval -> SC detect once per new keyframe.
// The raw cloud handed to mapping is the scan being mapped (Q16).
#include "oracle_fa.h"
#include "oracle_mo.h"
#include "oracle_lc.h"
#include <thread>
#include <chrono>
#include <atomic>
#include <string>
#include "../sc-lego-loam_amd/csrc/slo_gen.h"
#include "../include/slo_abi.h"   // the record layout (SLO_REC_*) of the interface the oracle checks

using namespace oracle;

struct OracleStream {
    slo_config cfg;
    ImageProjection ip;
    FeatureAssociation fa;
    MapOptimization mo;
    SCManager::DetectResult det{};
    bool det_valid = false;
    LoopResult loop[2];      // RS, SC verification of the last detect (cfg.loop_verify)
    int scan_index = 0;
    float integrated[6] = {0};   // /integrated_to_init (transformFusion's transformMapped)
    int gemm_mode = 0;           // oracle_common.h gemm_AtA / gemm_AtB (0 double-double, 1 OpenCV's order)
    explicit OracleStream(const slo_config& c) : cfg(c), ip(c), fa(c), mo(c) {}

    // returns bit flags: 1 = FA odometry ran, 2 = mapping ran, 4 = keyframe, 8 = detect ran
    int step(const float* pts, int n, double t) {
        const int f = step_map(pts, n, t);
        return f | step_loop(f, t);
    }
    // the nodes up to mapOptimization::run (flags 1, 2, 4)
    int step_map(const float* pts, int n, double t) {
        t_gemm_mode = gemm_mode;   // this thread runs this stream now
        det_valid = false;
        ip.cloudHandler(pts, n);
        fa.run(ip.segmentedCloud, ip.segMsg, ip.outlierCloud, t);
        return after_fa(pts, n, t);
    }

    // ---- Mode S: one stream's scans split between objects.
    // front(): imageProjection + featureAssociation's feature extraction
    // (adjustDistortion .. extractFeatures, FA:1833-1841) of one scan on one
    // object; back(): the odometry (FA:1843-1858), mapping and Scan Context
    // of that scan on the owner object, from the front's feature clouds.
    // What a scan's front end inherits from the previous scan's — the
    // carry — is the stale state of Appendix A Q5: featureAssociation's
    // persistent arrays (cloudSmoothness, cloudCurvature,
    // cloudNeighborPicked, cloudLabel: read at positions this scan does not
    // rewrite), the cloud_info arrays' tails past this scan's points
    // (segmentedCloudColInd[ind + 5] reads past the end, FA:730-745) and the
    // orientations an empty scan keeps.  front() runs imageProjection first
    // (it needs nothing from the previous scan) and merges the carry after it.
    // IMU input is not part of Mode S (the IMU ring would have to travel too).
    struct Carry {
        SegInfo seg;
        std::vector<Smooth> smooth;
        std::vector<float> curv;
        std::vector<int> picked, label;
    };
    struct Features { Cloud sharp, less_sharp, flat, less_flat, outlier; };
    void front(const float* pts, int n, double t, const Carry* in, Carry* out, Features* f) {
        t_gemm_mode = gemm_mode;
        ip.cloudHandler(pts, n);
        if (in) {
            const size_t S = ip.segmentedCloud.size(), H = ip.segMsg.segmentedCloudColInd.size();
            for (size_t i = S; i < H; ++i) {
                ip.segMsg.segmentedCloudColInd[i] = in->seg.segmentedCloudColInd[i];
                ip.segMsg.segmentedCloudGroundFlag[i] = in->seg.segmentedCloudGroundFlag[i];
                ip.segMsg.segmentedCloudRange[i] = in->seg.segmentedCloudRange[i];
            }
            if (ip.laserCloudIn.empty()) {
                ip.segMsg.startOrientation = in->seg.startOrientation;
                ip.segMsg.endOrientation = in->seg.endOrientation;
                ip.segMsg.orientationDiff = in->seg.orientationDiff;
            }
            fa.cloudSmoothness = in->smooth;
            fa.cloudCurvature = in->curv;
            fa.cloudNeighborPicked = in->picked;
            fa.cloudLabel = in->label;
        }
        fa.timeScanCur = t;
        fa.segmentedCloud = ip.segmentedCloud;
        fa.segInfo = ip.segMsg;
        fa.outlierCloud = ip.outlierCloud;
        fa.published_to_mapping = false;
        fa.adjustDistortion();
        fa.calculateSmoothness();
        fa.markOccludedPoints();
        fa.extractFeatures();
        *out = Carry{ip.segMsg, fa.cloudSmoothness, fa.cloudCurvature, fa.cloudNeighborPicked, fa.cloudLabel};
        *f = Features{fa.cornerPointsSharp, fa.cornerPointsLessSharp, fa.surfPointsFlat, fa.surfPointsLessFlat,
                      fa.outlierCloud};
    }
    // flags as step()
    int back(const Features& f, const float* pts, int n, double t) {
        t_gemm_mode = gemm_mode;
        det_valid = false;
        fa.timeScanCur = t;
        fa.cornerPointsSharp = f.sharp;
        fa.cornerPointsLessSharp = f.less_sharp;
        fa.surfPointsFlat = f.flat;
        fa.surfPointsLessFlat = f.less_flat;
        fa.outlierCloud = f.outlier;
        fa.published_to_mapping = false;
        if (!fa.systemInitedLM) {
            fa.checkSystemInitialization();
        } else {
            fa.updateInitialGuess();
            fa.updateTransformation();
            fa.integrateTransformation();
            fa.publishCloudsLast();
        }
        const int fl = after_fa(pts, n, t);
        return fl | step_loop(fl, t);
    }
    // back() in two stages on two objects, the reference's featureAssociation
    // | mapOptimization process boundary (launch/run.launch:15-16): odom()
    // runs the odometry and hands on what featureAssociation publishes to
    // mapping (FA:1790-1814) — the *Last clouds, the outliers, transformSum,
    // whether this scan was published — and whether the odometry ran (for
    // transformFusion); mapstage() runs transformFusion's
    // laserOdometryHandler, mapOptimization and Scan Context.
    struct Odom {
        Cloud corner_last, surf_last, outlier;
        float sum[6];
        int ran, published;
    };
    void odom(const Features& f, double t, Odom* o) {
        t_gemm_mode = gemm_mode;
        fa.timeScanCur = t;
        fa.cornerPointsSharp = f.sharp;
        fa.cornerPointsLessSharp = f.less_sharp;
        fa.surfPointsFlat = f.flat;
        fa.surfPointsLessFlat = f.less_flat;
        fa.outlierCloud = f.outlier;
        fa.published_to_mapping = false;
        if (!fa.systemInitedLM) {
            fa.checkSystemInitialization();
        } else {
            fa.updateInitialGuess();
            fa.updateTransformation();
            fa.integrateTransformation();
            fa.publishCloudsLast();
        }
        o->ran = fa.systemInitedLM && scan_index > 0;
        o->published = fa.published_to_mapping;
        o->corner_last = fa.laserCloudCornerLast;
        o->surf_last = fa.laserCloudSurfLast;
        o->outlier = fa.outlierCloud;
        memcpy(o->sum, fa.transformSum, sizeof o->sum);
        scan_index++;
    }
    int mapstage(const Odom& o, const float* pts, int n, double t) {
        t_gemm_mode = gemm_mode;
        det_valid = false;
        memcpy(fa.transformSum, o.sum, sizeof o.sum);   // what get("transform_sum") reads on this object
        int flags = o.ran ? 1 : 0;
        if (flags & 1) {   // as after_fa
            float sum[6], incre[6];
            odom_handoff(o.sum, sum);
            MapOptimization::associate_to_map(sum, mo.tfBef, mo.tfAft, incre, integrated);
        }
        if (o.published) {
            const bool ran = mo.run(o.corner_last, o.surf_last, o.outlier, o.sum, pts, n, t);
            if (ran) flags |= 2;
            if (ran && mo.saved_keyframe) flags |= 4;
        }
        scan_index++;
        return flags | step_loop(flags, t);
    }

    // featureAssociation has run on this scan: the hand-offs and mapping
    int after_fa(const float* pts, int n, double t) {
        int flags = 0;
        if (fa.systemInitedLM && scan_index > 0) flags |= 1;
        if (flags & 1) {
            // TransformFusion::laserOdometryHandler (TF:186-219) on this scan's
            // /laser_odom_to_init, with the /aft_mapped_to_init of the last
            // mapping run (the mapping of this scan publishes after it)
            float sum[6], incre[6];
            odom_handoff(fa.transformSum, sum);
            MapOptimization::associate_to_map(sum, mo.tfBef, mo.tfAft, incre, integrated);
        }
        if (fa.published_to_mapping) {
            bool ran = mo.run(fa.laserCloudCornerLast, fa.laserCloudSurfLast, fa.outlierCloud, fa.transformSum, pts, n, t);
            if (ran) flags |= 2;
            if (ran && mo.saved_keyframe) flags |= 4;
        }
        scan_index++;
        return flags;
    }
    // the loop thread after a keyframe (flags 8, 16): detect + verification
    int step_loop(int map_flags, double t) {
        int flags = 0;
        // loopClosureThread returns at once without loop closure (MO:831-832)
        if ((map_flags & 4) && cfg.loop_closure_enable) {
            det = mo.sc.detectLoopClosureID();
            det_valid = true;
            flags |= 8;
            if (cfg.loop_verify) {
                perform_loop_closure(cfg, mo, det.loop_id, t, loop, mo.stable_voxel);
                if (loop[1].ran) flags |= 16;
            }
        }
        return flags;
    }
};

// ---- Mode S (OracleStream::front / back) over byte blobs, so that ranks can
// exchange them: a carry is the stale state a scan's front end leaves for the
// next one, features are what the front end hands the owner
static size_t blob_put(std::vector<char>& b, const void* p, size_t n) {
    const size_t o = b.size();
    b.resize(o + n);
    if (n) memcpy(b.data() + o, p, n);
    return o;
}
template <class T> static void vec_put(std::vector<char>& b, const std::vector<T>& v) {
    const int64_t n = (int64_t)v.size();
    blob_put(b, &n, 8);
    blob_put(b, v.data(), sizeof(T) * v.size());
}
template <class T> static const char* vec_get(const char* p, std::vector<T>& v) {
    int64_t n;
    memcpy(&n, p, 8);
    v.resize((size_t)n);
    if (n) memcpy(v.data(), p + 8, sizeof(T) * (size_t)n);
    return p + 8 + sizeof(T) * (size_t)n;
}

extern "C" {

int oracle_config_preset(int preset, slo_config* out) { return slo_config_preset_impl(preset, out); }

void* oracle_create(const slo_config* cfg, int stable_voxel) {
    OracleStream* s = new OracleStream(*cfg);
    s->fa.stable_voxel = stable_voxel != 0;
    s->mo.stable_voxel = stable_voxel != 0;
    return s;
}
void oracle_destroy(void* h) { delete (OracleStream*)h; }

static std::vector<char> g_blob[2];   // the last front call's carry and features (per process; tests only)
// front end of one scan; carry_in = NULL for the first scan.  Returns the
// byte sizes of the carry and the features, fetched with oracle_front_blob.
int oracle_front(void* h, const float* pts, int n, double t, const void* carry_in, int64_t* sizes) {
    OracleStream* s = (OracleStream*)h;
    OracleStream::Carry in, out;
    if (carry_in) {
        const char* p = (const char*)carry_in;
        float o[3];
        memcpy(o, p, 12);
        p += 12;
        in.seg.startOrientation = o[0]; in.seg.endOrientation = o[1]; in.seg.orientationDiff = o[2];
        p = vec_get(p, in.seg.segmentedCloudColInd);
        p = vec_get(p, in.seg.segmentedCloudGroundFlag);
        p = vec_get(p, in.seg.segmentedCloudRange);
        p = vec_get(p, in.smooth);
        p = vec_get(p, in.curv);
        p = vec_get(p, in.picked);
        p = vec_get(p, in.label);
    }
    OracleStream::Features f;
    s->front(pts, n, t, carry_in ? &in : nullptr, &out, &f);
    std::vector<char>& c = g_blob[0];
    c.clear();
    const float o[3] = {out.seg.startOrientation, out.seg.endOrientation, out.seg.orientationDiff};
    blob_put(c, o, 12);
    vec_put(c, out.seg.segmentedCloudColInd);
    vec_put(c, out.seg.segmentedCloudGroundFlag);
    vec_put(c, out.seg.segmentedCloudRange);
    vec_put(c, out.smooth);
    vec_put(c, out.curv);
    vec_put(c, out.picked);
    vec_put(c, out.label);
    std::vector<char>& b = g_blob[1];
    b.clear();
    for (const Cloud* cl : {&f.sharp, &f.less_sharp, &f.flat, &f.less_flat, &f.outlier}) vec_put(b, *cl);
    sizes[0] = (int64_t)c.size();
    sizes[1] = (int64_t)b.size();
    return 0;
}
void oracle_front_blob(int which, void* out) { memcpy(out, g_blob[which].data(), g_blob[which].size()); }
int oracle_back(void* h, const void* features, const float* pts, int n, double t) {
    OracleStream::Features f;
    const char* p = (const char*)features;
    for (Cloud* cl : {&f.sharp, &f.less_sharp, &f.flat, &f.less_flat, &f.outlier}) p = vec_get(p, *cl);
    return ((OracleStream*)h)->back(f, pts, n, t);
}
// the back end's two stages over a blob (OracleStream::odom / mapstage):
// odom returns the blob's size, fetched with oracle_front_blob(2, ...)
static std::vector<char> g_odom;
int64_t oracle_odom(void* h, const void* features, double t) {
    OracleStream::Features f;
    const char* p = (const char*)features;
    for (Cloud* cl : {&f.sharp, &f.less_sharp, &f.flat, &f.less_flat, &f.outlier}) p = vec_get(p, *cl);
    OracleStream::Odom o;
    ((OracleStream*)h)->odom(f, t, &o);
    g_odom.clear();
    for (const Cloud* cl : {&o.corner_last, &o.surf_last, &o.outlier}) vec_put(g_odom, *cl);
    blob_put(g_odom, o.sum, sizeof o.sum);
    blob_put(g_odom, &o.ran, 4);
    blob_put(g_odom, &o.published, 4);
    return (int64_t)g_odom.size();
}
void oracle_odom_blob(void* out) { memcpy(out, g_odom.data(), g_odom.size()); }
int oracle_mapstage(void* h, const void* odom, const float* pts, int n, double t) {
    OracleStream::Odom o;
    const char* p = (const char*)odom;
    for (Cloud* cl : {&o.corner_last, &o.surf_last, &o.outlier}) p = vec_get(p, *cl);
    memcpy(o.sum, p, sizeof o.sum);
    memcpy(&o.ran, p + 24, 4);
    memcpy(&o.published, p + 28, 4);
    return ((OracleStream*)h)->mapstage(o, pts, n, t);
}
// the normal equations' accumulation order (oracle_common.h gemm_AtA): 0 double-double (default), 1 OpenCV 3.x
void oracle_set_gemm_mode(void* h, int mode) { ((OracleStream*)h)->gemm_mode = mode; }

int oracle_step(void* h, const float* pts, int n, double t) { return ((OracleStream*)h)->step(pts, n, t); }
int oracle_step_map(void* h, const float* pts, int n, double t) { return ((OracleStream*)h)->step_map(pts, n, t); }
int oracle_step_loop(void* h, int map_flags, double t) { return ((OracleStream*)h)->step_loop(map_flags, t); }
void oracle_set_key_poses(void* h, const float* poses6, int n, const float* transform6) {
    ((OracleStream*)h)->mo.set_key_poses(poses6, n, transform6);
}
// the RS loop factor's poseFrom (MO:1027-1037) as RzRyRx / Point3 arguments:
// pcl::getTransformation of the lidar-axes correction times that of the
// newest key pose, read back by pcl::getTranslationAndEulerAngles; float
// products row by column left to right (Eigen's order unpinned)
void oracle_rs_loop_from(const float* corr, const float* latest, float* out) {
    auto gt = [](float x, float y, float z, float roll, float pitch, float yaw, float* T) {
        const float A = cosf(yaw), B = sinf(yaw), C = cosf(pitch), D = sinf(pitch), E = cosf(roll), F = sinf(roll);
        const float DE = D * E, DF = D * F;
        const float m[16] = {A * C, A * DF - B * E, B * F + A * DE, x, B * C, A * E + B * DF, B * DE - A * F, y,
                             -D,    C * F,          C * E,          z, 0,     0,              0,              1};
        memcpy(T, m, sizeof m);
    };
    float L[16], W[16], M[16];
    gt(corr[2], corr[0], corr[1], corr[5], corr[3], corr[4], L);         // correctionLidarFrame
    gt(latest[2], latest[0], latest[1], latest[5], latest[3], latest[4], W);   // tWrong
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) M[4 * r + c] = (L[4 * r] * W[c] + L[4 * r + 1] * W[4 + c]) + L[4 * r + 2] * W[8 + c];
        M[4 * r + 3] = ((L[4 * r] * W[3] + L[4 * r + 1] * W[7]) + L[4 * r + 2] * W[11]) + L[4 * r + 3];
    }
    out[0] = atan2f(M[9], M[10]); out[1] = asinf(-M[8]); out[2] = atan2f(M[4], M[0]);
    out[3] = M[3]; out[4] = M[7]; out[5] = M[11];
}

// useCloudRing input for the next scans (the message's ring field, unfiltered order)
// imuHandler on n messages (slo_imu_msg layout), in order
void oracle_imu(void* h, const double* msgs, int n) {
    for (int k = 0; k < n; ++k) {
        const double* m = msgs + 11 * k;
        ((OracleStream*)h)->fa.imuHandler(ImuMsg{m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[9], m[10]});
    }
}
void oracle_set_rings(void* h, const uint16_t* rings, int n) { ((OracleStream*)h)->ip.rings.assign(rings, rings + n); }

// image projection only (for front-end parity of a single scan)
void oracle_image_projection(void* h, const float* pts, int n) { ((OracleStream*)h)->ip.cloudHandler(pts, n); }

static int copy_cloud(const Cloud& c, float* out, int cap) {
    int n = (int)c.size();
    if (out) for (int i = 0; i < n && i < cap; ++i) memcpy(out + 4 * i, &c[i], 16);
    return n;
}

// Named accessor: copies up to cap elements into out, returns the full count.
int oracle_get(void* h, const char* name_c, void* out, int cap) {
    OracleStream* s = (OracleStream*)h;
    std::string name(name_c);
    const int H = s->cfg.n_scan * s->cfg.horizon_scan;
    auto cp = [&](const void* src, int count, int esz) {
        if (out) memcpy(out, src, (size_t)std::min(count, cap) * esz);
        return count;
    };
    if (name == "range") return cp(s->ip.rangeMat.data(), H, 4);
    if (name == "label") return cp(s->ip.labelMat.data(), H, 4);
    if (name == "ground") return cp(s->ip.groundMat.data(), H, 1);
    if (name == "full_cloud") return copy_cloud(s->ip.fullCloud, (float*)out, cap);
    if (name == "seg_pts") return copy_cloud(s->ip.segmentedCloud, (float*)out, cap);
    int S = (int)s->ip.segmentedCloud.size();
    if (name == "seg_ground") return cp(s->ip.segMsg.segmentedCloudGroundFlag.data(), S, 1);
    if (name == "seg_col") return cp(s->ip.segMsg.segmentedCloudColInd.data(), S, 4);
    if (name == "seg_range") return cp(s->ip.segMsg.segmentedCloudRange.data(), S, 4);
    if (name == "ring_start") return cp(s->ip.segMsg.startRingIndex.data(), s->cfg.n_scan, 4);
    if (name == "ring_end") return cp(s->ip.segMsg.endRingIndex.data(), s->cfg.n_scan, 4);
    if (name == "orient") {
        float o[3] = {s->ip.segMsg.startOrientation, s->ip.segMsg.endOrientation, s->ip.segMsg.orientationDiff};
        return cp(o, 3, 4);
    }
    if (name == "outlier") return copy_cloud(s->ip.outlierCloud, (float*)out, cap);
    if (name == "fa_seg_pts") return copy_cloud(s->fa.segmentedCloud, (float*)out, cap);
    if (name == "curvature") return cp(s->fa.cloudCurvature.data(), H, 4);
    if (name == "picked") return cp(s->fa.cloudNeighborPicked.data(), H, 4);
    if (name == "cloud_label") return cp(s->fa.cloudLabel.data(), H, 4);
    if (name == "smooth_ind") {
        std::vector<int32_t> v(H);
        for (int i = 0; i < H; ++i) v[i] = (int32_t)s->fa.cloudSmoothness[i].ind;
        return cp(v.data(), H, 4);
    }
    if (name == "sharp") return copy_cloud(s->fa.cornerPointsSharp, (float*)out, cap);
    if (name == "flat") return copy_cloud(s->fa.surfPointsFlat, (float*)out, cap);
    if (name == "less_sharp") return copy_cloud(s->fa.cornerPointsLessSharp, (float*)out, cap);
    if (name == "less_flat") return copy_cloud(s->fa.surfPointsLessFlat, (float*)out, cap);
    if (name == "corner_last") return copy_cloud(s->fa.laserCloudCornerLast, (float*)out, cap);
    if (name == "surf_last") return copy_cloud(s->fa.laserCloudSurfLast, (float*)out, cap);
    if (name == "transform_sum") return cp(s->fa.transformSum, 6, 4);
    if (name == "imu") {   // the IMU scalars in slo_get("imu")'s order
        const FeatureAssociation& f = s->fa;
        const double a[23] = {(double)f.imuPointerLast, (double)f.imuPointerLastIteration, f.imuRollStart,
                              f.imuPitchStart, f.imuYawStart, f.imuVeloXStart, f.imuVeloYStart, f.imuVeloZStart,
                              f.imuRollCur, f.imuPitchCur, f.imuYawCur, f.imuVeloFromStartXCur, f.imuVeloFromStartYCur,
                              f.imuVeloFromStartZCur, f.imuAngularRotationXLast, f.imuAngularRotationYLast,
                              f.imuAngularRotationZLast, f.imuAngularFromStartX, f.imuAngularFromStartY,
                              f.imuAngularFromStartZ, f.imuRollLast, f.imuPitchLast, f.imuYawLast};
        return cp(a, 23, 8);
    }
    if (name == "integrated") return cp(s->integrated, 6, 4);
    if (name == "transform_cur") return cp(s->fa.transformCur, 6, 4);
    if (name == "fa_iters") { int v[2] = {s->fa.iters_surf, s->fa.iters_corner}; return cp(v, 2, 4); }
    if (name == "mapped") return cp(s->mo.transformAftMapped, 6, 4);
    if (name == "tobe_mapped") return cp(s->mo.transformTobeMapped, 6, 4);
    if (name == "mo_iters") return cp(&s->mo.lm_iters, 1, 4);
    if (name == "n_keyframes") { int v = (int)s->mo.keyPoses.size(); return cp(&v, 1, 4); }
    if (name == "keyposes") return cp(s->mo.keyPoses.data(), (int)s->mo.keyPoses.size() * 6, 4);
    if (name == "raw_ds") return copy_cloud(s->mo.laserCloudRawDS, (float*)out, cap);
    if (name == "corner_ds") return copy_cloud(s->mo.laserCloudCornerLastDS, (float*)out, cap);
    if (name == "surf_total_ds") return copy_cloud(s->mo.laserCloudSurfTotalLastDS, (float*)out, cap);
    if (name == "map_corner_ds") return copy_cloud(s->mo.lastCornerMapDS, (float*)out, cap);
    if (name == "map_surf_ds") return copy_cloud(s->mo.lastSurfMapDS, (float*)out, cap);
    // the local maps before their VoxelGrid (MO:1224-1230), as last assembled
    if (name == "map_corner_raw") return copy_cloud(s->mo.lastCornerMapRaw, (float*)out, cap);
    if (name == "map_surf_raw") return copy_cloud(s->mo.lastSurfMapRaw, (float*)out, cap);
    if (name == "sc_desc") {
        if (s->mo.sc.polarcontexts_.empty()) return 0;
        auto& d = s->mo.sc.polarcontexts_.back();
        return cp(d.data(), (int)d.size(), 8);
    }
    if (name == "ring_key") {
        if (s->mo.sc.invkeys_.empty()) return 0;
        auto& d = s->mo.sc.invkeys_.back();
        return cp(d.data(), (int)d.size(), 8);
    }
    if (name == "sector_key") {
        if (s->mo.sc.vkeys_.empty()) return 0;
        auto& d = s->mo.sc.vkeys_.back();
        return cp(d.data(), (int)d.size(), 8);
    }
    if (name == "detect") {  // loop_id, nn_idx, n_cand, cand[K] as int32; then yaw, min_dist via detect_f
        if (!s->det_valid) return 0;
        std::vector<int32_t> v{s->det.loop_id, s->det.nn_idx, s->det.n_cand};
        for (int i = 0; i < s->det.n_cand; ++i) v.push_back(s->det.cand[i]);
        return cp(v.data(), (int)v.size(), 4);
    }
    if (name == "loop") {   // 2 x LoopResult (RS, SC) of the last detect
        if (!s->det_valid || !s->cfg.loop_verify) return 0;
        return cp(s->loop, 2, (int)sizeof(LoopResult));
    }
    if (name == "key_times") return cp(s->mo.keyTimes.data(), (int)s->mo.keyTimes.size(), 8);
    if (name == "kf_pre") return cp(s->mo.kfPre, 6, 4);
    if (name == "sc_count") { int v = (int)s->mo.sc.polarcontexts_.size(); return cp(&v, 1, 4); }
    if (name == "map_ids") {   // surroundingExistingKeyPosesID (loop closure disabled only)
        if (s->cfg.loop_closure_enable) return -1;
        return cp(s->mo.surroundingExistingKeyPosesID.data(), (int)s->mo.surroundingExistingKeyPosesID.size(), 4);
    }
    if (name == "detect_f") {
        if (!s->det_valid) return 0;
        double v[2] = {(double)s->det.yaw, s->det.min_dist};
        return cp(v, 2, 8);
    }
    return -1;
}

// ---- loop-closure unit entry points (oracle_lc.h)
// icp.align + getFitnessScore of src (n x XYZI) onto tgt (m x XYZI)
void oracle_icp_align(const slo_config* cfg, const float* src, int n, const float* tgt, int m, LoopResult* out) {
    Cloud a(n), b(m);
    if (n) memcpy(a.data(), src, 16 * (size_t)n);
    if (m) memcpy(b.data(), tgt, 16 * (size_t)m);
    *out = LoopResult();
    out->id = 0;
    icp_align(*cfg, a, b, *out);
}
// pcl::umeyama of the pairs (src[i], dst[i]) (one ICP increment); returns 0 on success
int oracle_umeyama(const float* src, const float* dst, int n, float* T) {
    IcpSums a;
    for (int i = 0; i < n; ++i) {
        Pt p{src[4 * i], src[4 * i + 1], src[4 * i + 2], 0}, q{dst[4 * i], dst[4 * i + 1], dst[4 * i + 2], 0};
        a.add(p, q, 0.0f);
    }
    return umeyama_from_sums(a, T) ? 0 : -1;
}
// JacobiSVD<Matrix3d> of a row-major 3x3
int oracle_svd3(const double* A, double* U, double* S, double* V) { return jacobi_svd3(A, U, S, V) ? 0 : -1; }
// the mapping node's angle round trips (oracle_tf.h): which = 0 tf hand-off, 1 keyframe estimate
void oracle_pose_roundtrip(int which, const float* in, float* out) {
    if (which == 0) odom_handoff(in, out);
    else keyframe_estimate(in, out);
}

// ---- SC unit entry points (pure functions over given descriptors)
double oracle_sc_distance(const slo_config* cfg, const double* sc1, const double* sc2, int* shift) {
    SCManager m(*cfg);
    std::vector<double> a(sc1, sc1 + cfg->sc_num_ring * cfg->sc_num_sector);
    std::vector<double> b(sc2, sc2 + cfg->sc_num_ring * cfg->sc_num_sector);
    auto r = m.distanceBtnScanContext(a, b);
    *shift = r.second;
    return r.first;
}
double oracle_sc_dist_direct(const slo_config* cfg, const double* sc1, const double* sc2) {
    SCManager m(*cfg);
    std::vector<double> a(sc1, sc1 + cfg->sc_num_ring * cfg->sc_num_sector);
    std::vector<double> b(sc2, sc2 + cfg->sc_num_ring * cfg->sc_num_sector);
    return m.distDirectSC(a, b, 0);
}
int oracle_sc_fast_align(const slo_config* cfg, const double* vk1, const double* vk2) {
    SCManager m(*cfg);
    std::vector<double> a(vk1, vk1 + cfg->sc_num_sector), b(vk2, vk2 + cfg->sc_num_sector);
    return m.fastAlignUsingVkey(a, b);
}
void oracle_sc_make(const slo_config* cfg, const float* pts, int n, double* desc, double* ring, double* sector) {
    SCManager m(*cfg);
    Cloud c(n);
    memcpy(c.data(), pts, (size_t)n * 16);
    auto d = m.makeScancontext(c);
    auto rk = m.makeRingkey(d);
    auto vk = m.makeSectorkey(d);
    memcpy(desc, d.data(), d.size() * 8);
    memcpy(ring, rk.data(), rk.size() * 8);
    memcpy(sector, vk.data(), vk.size() * 8);
}
int oracle_voxel_grid(const float* pts, int n, float leaf, int stable, float* out, int cap) {
    Cloud c(n), o;
    memcpy(c.data(), pts, (size_t)n * 16);
    voxel_grid(c, leaf, o, stable != 0);
    return copy_cloud(o, out, cap);
}

// ---- Scan Context session (SCManager alone): add = VoxelGrid(leaf_sc) of the
// finite points + makeAndSaveScancontextAndKeys; detect = detectLoopClosureID.
void* oracle_sc_session_create(const slo_config* cfg) { return new SCManager(*cfg); }
void oracle_sc_session_destroy(void* h) { delete (SCManager*)h; }
// returns the DS size; ring_key_f (NR floats) = the tree row just appended
int oracle_sc_session_add(void* h, const float* pts, int n, int stable, float* ring_key_f) {
    SCManager* m = (SCManager*)h;
    Cloud c, ds;
    for (int i = 0; i < n; ++i) {
        const float* p = pts + 4 * (size_t)i;
        if (std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2])) c.push_back({p[0], p[1], p[2], p[3]});
    }
    voxel_grid(c, m->cfg.leaf_sc, ds, stable != 0);
    m->makeAndSaveScancontextAndKeys(ds);
    if (ring_key_f) memcpy(ring_key_f, m->invkeys_mat_.back().data(), sizeof(float) * m->NR);
    return (int)ds.size();
}
// out_i: loop_id, nn_idx, n_cand, cand[K]; out_f: yaw, min_dist
void oracle_sc_session_detect(void* h, int* out_i, double* out_f) {
    auto r = ((SCManager*)h)->detectLoopClosureID();
    out_i[0] = r.loop_id; out_i[1] = r.nn_idx; out_i[2] = r.n_cand;
    for (int c = 0; c < r.n_cand; ++c) out_i[3 + c] = r.cand[c];
    out_f[0] = r.yaw; out_f[1] = r.min_dist;
}
// exact K-NN of the restatement over `n` rows of `data` (the ring-key tree
// snapshot) in nanoflann's float L2 order; unfilled slots stay 0 / FLT_MAX
void oracle_sc_knn(const slo_config* cfg, const float* data, int n, const float* q, int K, int* idx, float* dist) {
    SCManager m(*cfg);
    for (int t = 0; t < n; ++t)
        m.invkeys_to_search_.emplace_back(data + (size_t)t * m.NR, data + (size_t)(t + 1) * m.NR);
    std::vector<int> ci;
    std::vector<float> cd;
    m.knn_search(q, K, ci, cd);
    for (int c = 0; c < K; ++c) { idx[c] = ci[c]; dist[c] = cd[c]; }
}

// ---- cross-stream Scan Context store (slo_xsc.hip) restated: per-stream
// rings of `cap` descriptors taken from the all-gathered records; a query runs
// detectLoopClosureID's candidate search (SCc:247-338) against every other
// stream's entries: K nearest ring keys by (nanoflann float L2, entry code =
// stream * cap + slot), distanceBtnScanContext each, first minimum, loop when
// below SC_DIST_THRES
struct XscOracle {
    slo_config cfg;
    int N, cap, NR, NS;
    SCManager m;
    std::vector<std::vector<double>> desc, sect;
    std::vector<std::vector<float>> ring;
    std::vector<int> kfi, cnt;
    XscOracle(const slo_config& c, int n, int k)
        : cfg(c), N(n), cap(k), NR(c.sc_num_ring), NS(c.sc_num_sector), m(c), desc((size_t)n * k), sect((size_t)n * k),
          ring((size_t)n * k), kfi((size_t)n * k, -1), cnt(n, 0) {}
    std::vector<double> desc_of(const float* rec) const {
        std::vector<double> d(NR * NS);
        for (int i = 0; i < NR * NS; ++i) d[i] = (double)rec[SLO_REC_DESC + i];
        return d;
    }
    std::vector<float> ring_of(const std::vector<double>& d) const {
        auto rk = m.makeRingkey(d);
        std::vector<float> f(NR);
        for (int r = 0; r < NR; ++r) f[r] = (float)rk[r];
        return f;
    }
};
void* oracle_xsc_create(const slo_config* cfg, int n_streams, int cap) { return new XscOracle(*cfg, n_streams, cap); }
void oracle_xsc_destroy(void* h) { delete (XscOracle*)h; }
void oracle_xsc_ingest(void* h, const float* recs, int n) {
    XscOracle& x = *(XscOracle*)h;
    for (int r = 0; r < n && r < x.N; ++r) {
        const float* rec = recs + (size_t)r * SLO_RECORD_FLOATS;
        if (rec[SLO_REC_KF_SAVED] == 0.0f || rec[SLO_REC_KF_INDEX] < 0.0f) continue;
        const size_t slot = (size_t)r * x.cap + x.cnt[r] % x.cap;
        x.desc[slot] = x.desc_of(rec);
        x.sect[slot] = x.m.makeSectorkey(x.desc[slot]);
        x.ring[slot] = x.ring_of(x.desc[slot]);
        x.kfi[slot] = (int)rec[SLO_REC_KF_INDEX];
        x.cnt[r]++;
    }
}
// out_i [nq][5] = valid, n_cand, nn_stream, nn_keyframe, loop; out_f [nq][2] = yaw, min_dist
void oracle_xsc_query(void* h, const float* recs, int nq, int global0, int32_t* out_i, double* out_f) {
    XscOracle& x = *(XscOracle*)h;
    const int K = x.cfg.sc_num_candidates;
    for (int q = 0; q < nq; ++q) {
        const float* rec = recs + (size_t)q * SLO_RECORD_FLOATS;
        int32_t* oi = out_i + 5 * q;
        double* of = out_f + 2 * q;
        oi[0] = 0; oi[1] = 0; oi[2] = -1; oi[3] = -1; oi[4] = 0; of[0] = 0; of[1] = 0;
        if (rec[SLO_REC_KF_SAVED] == 0.0f || rec[SLO_REC_KF_INDEX] < 0.0f) continue;
        const int self = global0 + q;
        auto qd = x.desc_of(rec);
        auto qr = x.ring_of(qd);
        std::vector<std::pair<float, long long>> all;
        for (int t = 0; t < x.N; ++t) {
            if (t == self) continue;
            for (int j = 0; j < std::min(x.cnt[t], x.cap); ++j) {
                const long long e = (long long)t * x.cap + j;
                all.push_back({SCManager::l2_nf(qr.data(), x.ring[e].data(), x.NR), e});
            }
        }
        std::sort(all.begin(), all.end());
        const int nc = std::min<int>(K, (int)all.size());
        double md = 10000000;
        int am = 0, bc = -1;
        for (int c = 0; c < nc; ++c) {
            auto r = x.m.distanceBtnScanContext(qd, x.desc[all[c].second]);
            if (r.first < md) { md = r.first; am = r.second; bc = c; }
        }
        oi[0] = 1; oi[1] = nc;
        of[1] = md;
        if (bc >= 0) {
            const long long e = all[bc].second;
            oi[2] = (int)(e / x.cap); oi[3] = x.kfi[e]; oi[4] = md < x.cfg.sc_dist_thres ? 1 : 0;
            of[0] = (float)((float)(am * (360.0 / (double)x.NS)) * M_PI / 180.0);
        }
    }
}

// ---- the normal equations' GEMMs (oracle_common.h gemm_AtA / gemm_AtB) in
// either accumulation mode, on an n x m float matrix A and n-vector B
void oracle_gemm_at(const float* A, const float* B, int n, int m, int mode, float* AtA, float* AtB) {
    const int m0 = t_gemm_mode;
    t_gemm_mode = mode;
    std::vector<float> a(A, A + (size_t)n * m), b(B, B + n);
    gemm_AtA(a, n, m, AtA);
    gemm_AtB(a, b, n, m, AtB);
    t_gemm_mode = m0;
}

// tally on / off (both modes evaluated while on); [entries computed, entries
// where the two modes differ] since the last call (tallies reset)
void oracle_gemm_tally(int on) { g_gemm_tally = on != 0; }
void oracle_gemm_stats(long long* out) {
    out[0] = g_gemm_entries.exchange(0);
    out[1] = g_gemm_differ.exchange(0);
}

// ---- slo_ddsum.h under test: sum of the exact float products a[i]*b[i]
// mode 0 = sequential add (the oracle's loop), 1 = a pairwise merge tree of
// per-element sums (the device reductions), 2 = 64 strided lane sums merged
// in a butterfly (a wave's shuffle reduction); returns the rounded float
float oracle_ddsum(const float* a, const float* b, int n, int mode) {
    using namespace slo_dd;
    if (mode == 0) {
        DD s = zero();
        for (int i = 0; i < n; ++i) add(s, (double)a[i] * (double)b[i]);
        return to_float(s);
    }
    std::vector<DD> v;
    if (mode == 1) {
        for (int i = 0; i < n; ++i) { DD s = zero(); add(s, (double)a[i] * (double)b[i]); v.push_back(s); }
    } else {
        v.assign(64, zero());
        for (int i = 0; i < n; ++i) add(v[i % 64], (double)a[i] * (double)b[i]);
    }
    if (v.empty()) return 0.0f;
    while (v.size() > 1) {
        std::vector<DD> w;
        for (size_t i = 0; i + 1 < v.size(); i += 2) { DD s = v[i]; merge(s, v[i + 1]); w.push_back(s); }
        if (v.size() & 1) w.push_back(v.back());
        v.swap(w);
    }
    return to_float(v[0]);
}

// ---- generator passthrough (same header the product library uses)
int oracle_gen_scan(int preset, int config_id, int stream_id, int k, float* out) {
    slo_config cfg;
    if (slo_config_preset_impl(preset, &cfg)) return -1;
    slo_gen::Stream s = slo_gen::make_stream(cfg, config_id, stream_id);
    return slo_gen::stream_scan(s, k, out);
}

// ---- CPU baseline (bench.py cpu_baseline leg; SURVEY §8(d) "(B) all host
// cores"): n_threads independent streams, one per thread, each timed over
// scans [preroll, preroll + n_scans) after an untimed pre-roll of scans
// [0, preroll) that fills its local map and Scan Context history (the same
// window the GPU bench times).  The pre-roll runs on n_distinct streams in
// parallel; thread t then continues from a copy of stream t % n_distinct
// (the state a stream reaches is data, not timing), so a many-core host pays
// the pre-roll once per distinct stream.  `history` seeds the SC history with
// that many earlier scans (bench --history).  Returns the wall seconds of the
// timed window; stage_s[4] = per-stage seconds summed over threads (ip, fa,
// mo, sc); stage_one[4] = the same for a copy of stream 0 run over the same
// scans alone, before the parallel run (the reference's one-stream
// 3-process topology, SURVEY (A)).
static double bench_impl(const slo_config& cfg, int config_id, int n_threads, int n_scans, int preroll, int history,
                         int n_distinct, double* stage_s, double* stage_one);
double oracle_bench(int preset, int config_id, int n_threads, int n_scans, int preroll, int history, int n_distinct,
                    double* stage_s, double* stage_one) {
    slo_config cfg;
    if (slo_config_preset_impl(preset, &cfg)) return -1;
    return bench_impl(cfg, config_id, n_threads, n_scans, preroll, history, n_distinct, stage_s, stage_one);
}
// the same with the caller's configuration (a preset with edits: SC off, K = 50, ...)
double oracle_bench_cfg(const slo_config* cfg, int config_id, int n_threads, int n_scans, int preroll, int history,
                        int n_distinct, double* stage_s, double* stage_one) {
    return bench_impl(*cfg, config_id, n_threads, n_scans, preroll, history, n_distinct, stage_s, stage_one);
}
static double bench_impl(const slo_config& cfg, int config_id, int n_threads, int n_scans, int preroll, int history,
                         int n_distinct, double* stage_s, double* stage_one) {
    if (n_threads <= 0 || n_scans <= 0) return -1;
    if (n_distinct <= 0 || n_distinct > n_threads) n_distinct = n_threads;
    const int P = cfg.n_scan * cfg.horizon_scan;
    std::vector<OracleStream*> base(n_distinct, nullptr);
    std::vector<std::vector<float>> scans((size_t)n_distinct * n_scans);
    {
        std::vector<std::thread> g;
        for (int t = 0; t < n_distinct; ++t)
            g.emplace_back([&, t]() {
                slo_gen::Stream s = slo_gen::make_stream(cfg, config_id, t);
                base[t] = new OracleStream(cfg);
                std::vector<float> buf((size_t)P * 4);
                for (int h = 0; h < history; ++h) {   // SC history seed: VoxelGrid(leaf_sc) + make&save
                    slo_gen::stream_scan(s, h - history, buf.data());
                    Cloud c, ds;
                    for (int i = 0; i < P; ++i) {
                        const float* p = &buf[4 * (size_t)i];
                        if (std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2])) c.push_back({p[0], p[1], p[2], p[3]});
                    }
                    voxel_grid(c, cfg.leaf_sc, ds, false);
                    base[t]->mo.sc.makeAndSaveScancontextAndKeys(ds);
                }
                for (int k = 0; k < preroll; ++k) {
                    slo_gen::stream_scan(s, k, buf.data());
                    base[t]->step(buf.data(), P, 0.1 * k);
                }
                for (int k = 0; k < n_scans; ++k) {
                    auto& v = scans[(size_t)t * n_scans + k];
                    v.resize((size_t)P * 4);
                    slo_gen::stream_scan(s, preroll + k, v.data());
                }
            });
        for (auto& th : g) th.join();
    }
    // one scan of stream s through the three nodes (+ SC detect), per-stage seconds added to acc[4]
    auto run_scan = [&](OracleStream& s, const float* p, int k, double* acc) {
        const double tk = 0.1 * (preroll + k);
        auto a = std::chrono::steady_clock::now();
        s.det_valid = false;
        s.ip.cloudHandler(p, P);
        auto b = std::chrono::steady_clock::now();
        s.fa.run(s.ip.segmentedCloud, s.ip.segMsg, s.ip.outlierCloud, tk);
        auto c = std::chrono::steady_clock::now();
        bool kf = false;
        if (s.fa.published_to_mapping) {
            bool ran = s.mo.run(s.fa.laserCloudCornerLast, s.fa.laserCloudSurfLast, s.fa.outlierCloud,
                                s.fa.transformSum, p, P, tk);
            kf = ran && s.mo.saved_keyframe;
        }
        auto d = std::chrono::steady_clock::now();
        if (kf && cfg.loop_closure_enable) s.det = s.mo.sc.detectLoopClosureID();
        auto e = std::chrono::steady_clock::now();
        s.scan_index++;
        acc[0] += std::chrono::duration<double>(b - a).count();
        acc[1] += std::chrono::duration<double>(c - b).count();
        acc[2] += std::chrono::duration<double>(d - c).count();
        acc[3] += std::chrono::duration<double>(e - d).count();
    };
    // (A): stream 0 alone on an otherwise idle process, so its stage times are
    // not diluted by the other streams' threads
    if (stage_one) {
        OracleStream solo(*base[0]);
        for (int k = 0; k < 4; ++k) stage_one[k] = 0;
        for (int k = 0; k < n_scans; ++k) run_scan(solo, scans[(size_t)k].data(), k, stage_one);
    }
    std::vector<OracleStream*> streams(n_threads, nullptr);
    for (int t = 0; t < n_threads; ++t) streams[t] = t < n_distinct ? base[t] : new OracleStream(*base[t % n_distinct]);
    std::vector<double> st(4 * n_threads, 0.0);
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<double> tstart(n_threads), tend(n_threads);
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t)
        th.emplace_back([&, t]() {
            OracleStream& s = *streams[t];
            const int src = t % n_distinct;
            ready++;
            while (!go.load()) std::this_thread::yield();
            auto T0 = std::chrono::steady_clock::now();
            tstart[t] = std::chrono::duration<double>(T0.time_since_epoch()).count();
            for (int k = 0; k < n_scans; ++k) run_scan(s, scans[(size_t)src * n_scans + k].data(), k, &st[4 * t]);
            tend[t] = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        });
    while (ready.load() < n_threads) std::this_thread::yield();
    go = true;
    for (auto& x : th) x.join();
    for (auto* p : streams) delete p;
    double t0 = *std::min_element(tstart.begin(), tstart.end());
    double t1 = *std::max_element(tend.begin(), tend.end());
    for (int k = 0; k < 4; ++k) {
        if (stage_s) {
            stage_s[k] = 0;
            for (int t = 0; t < n_threads; ++t) stage_s[k] += st[4 * t + k];
        }
    }
    return t1 - t0;
}

// keyframes held by a stream after `preroll` scans (what the bench's window sees)
int oracle_stream_keyframes(void* h) { return (int)((OracleStream*)h)->mo.keyPoses.size(); }

}  // extern "C"
