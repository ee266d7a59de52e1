// slo_pgwire.hip — the pose-graph back end (slo_pg.hip) wired into the batched
// pipeline (cfg.pose_graph), in the reference's order (mapOptmization.cpp):
//
//   mapping step, after saveKeyFramesAndFactor's scan-to-map part:
//     a saved keyframe adds its odometry factor (MO:1547-1555) and takes the
//     graph's estimate as its key pose / transformAftMapped / transformLast /
//     transformTobeMapped (MO:1566-1611); then correctPoses (MO:1642-1664):
//     if a loop was closed since the last mapping step, every key pose is
//     rewritten from the estimate of the last keyframe save and the recent
//     keyframe deque is cleared, so the next local map is rebuilt from the
//     corrected poses; publishTF follows with the corrected transform.
//   after SC detect + loop verification (performLoopClosure, MO:964-1110):
//     each accepted candidate adds a Cauchy loop factor — RS (MO:1030-1046):
//     poseFrom = the ICP correction applied to the newest key pose in the
//     lidar axes, poseTo = the candidate's key pose; SC (MO:1078-1091):
//     poseFrom = the ICP correction itself, poseTo = identity — and the graph
//     is solved (isam->update); the loop is then "closed" for the next
//     mapping step.
//
// Without a closed loop the estimate of a new keyframe equals its initial
// value up to rounding, so nothing is written back and the device's own
// keyframe estimate (slo_pose::keyframe_estimate) stands.  Host code: one
// small graph per stream; the device state is read and patched between the
// batched launches (one synchronisation per mapping step, only with
// cfg.pose_graph).
#include "slo_internal.h"
#include "slo_pose.h"
#include "slo_libm.h"
#include "../../include/slo_abi.h"
#include <string.h>
#include <vector>

namespace slo {

// correctPoses / the new keyframe's estimate into stream s's device state:
// key poses [0, n) (x y z roll pitch yaw); with has_tf the transforms
// (transformAftMapped = transformLast = transformTobeMapped, MO:1601-1611)
// and the publishTF hand-off; the recent keyframe deque cleared when asked
__global__ void k_pg_writeback(DevView v, int s, const float* poses, int n, int has_tf, PgTf tf, int clear_deque) {
    StreamState& st = v.st[s];
    float* kp = v.kf_pose + (size_t)s * v.KFMAX * 6;
    for (int i = threadIdx.x; i < n * 6; i += blockDim.x) kp[i] = poses[i];
    if (threadIdx.x != 0) return;
    if (has_tf) {
        for (int k = 0; k < 6; ++k) {
            st.transformAftMapped[k] = tf.t[k]; st.transformLast[k] = tf.t[k]; st.transformTobeMapped[k] = tf.t[k];
        }
        slo_pose::odom_handoff(st.transformAftMapped, st.tf_aft);   // publishTF after correctPoses (MO:1701)
    }
    if (clear_deque) st.recent_n = 0;   // recent*CloudKeyFrames.clear() (MO:1644-1646)
}

// pcl::getTransformation(x, y, z, roll, pitch, yaw) (PCL common/eigen.hpp) as a row-major 4x4
static void pcl_transform(float x, float y, float z, float roll, float pitch, float yaw, float T[16]) {
    using namespace slo_libm;
    const float A = cosf_(yaw), B = sinf_(yaw), C = cosf_(pitch), D = sinf_(pitch), E = cosf_(roll), F = sinf_(roll);
    const float DE = D * E, DF = D * F;
    T[0] = A * C; T[1] = A * DF - B * E; T[2] = B * F + A * DE; T[3] = x;
    T[4] = B * C; T[5] = A * E + B * DF; T[6] = B * DE - A * F; T[7] = y;
    T[8] = -D;    T[9] = C * F;          T[10] = C * E;         T[11] = z;
    T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
}

// RS loop factor's poseFrom (MO:1027-1037): correctionLidarFrame * tWrong,
// read back with pcl::getTranslationAndEulerAngles, as the Pose3(RzRyRx(roll,
// pitch, yaw), Point3(x, y, z)) arguments.  Affine products in float, row by
// column left to right (Eigen's own order is unpinned: Eigen is absent here).
void rs_loop_from(const float corr_xyzrpy[6], const float latest[6], float out[6]) {
    float L[16], W[16], C[16];
    // correctionLidarFrame = getTransformation(z, x, y, yaw, roll, pitch) of the camera-frame correction
    pcl_transform(corr_xyzrpy[2], corr_xyzrpy[0], corr_xyzrpy[1], corr_xyzrpy[5], corr_xyzrpy[3], corr_xyzrpy[4], L);
    // tWrong = pclPointToAffine3fCameraToLidar(cloudKeyPoses6D[latest]) (MO:1118-1120)
    pcl_transform(latest[2], latest[0], latest[1], latest[5], latest[3], latest[4], W);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) C[4 * r + c] = (L[4 * r] * W[c] + L[4 * r + 1] * W[4 + c]) + L[4 * r + 2] * W[8 + c];
        C[4 * r + 3] = ((L[4 * r] * W[3] + L[4 * r + 1] * W[7]) + L[4 * r + 2] * W[11]) + L[4 * r + 3];
    }
    out[3] = C[3]; out[4] = C[7]; out[5] = C[11];
    out[0] = slo_libm::atan2f_(C[9], C[10]);
    out[1] = slo_libm::asinf_(-C[8]);
    out[2] = slo_libm::atan2f_(C[4], C[0]);
}

static int pg_upload(slo_ctx* ctx, const std::vector<float>& poses) {
    if (poses.size() > ctx->pg_cap) {
        if (ctx->d_pg_poses) hipFree(ctx->d_pg_poses);
        ctx->d_pg_poses = nullptr;
        ctx->pg_cap = 0;
        SLO_CHECK(hipMalloc(&ctx->d_pg_poses, sizeof(float) * poses.size()));
        ctx->pg_cap = poses.size();
    }
    if (!poses.empty())
        SLO_CHECK(hipMemcpyAsync(ctx->d_pg_poses, poses.data(), sizeof(float) * poses.size(), hipMemcpyHostToDevice,
                                 ctx->stream));
    return 0;
}

int pg_after_mapping(slo_ctx* ctx) {
    const int S = ctx->S;
    SLO_CHECK(hipMemcpyAsync(ctx->h_st, ctx->v.st, sizeof(StreamState) * S, hipMemcpyDeviceToHost, ctx->stream));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    for (int s = 0; s < S; ++s) {
        const StreamState& st = ctx->h_st[s];
        slo_pg* g = ctx->pg[s];
        if (st.kf_saved) {
            float out[6], key[6];
            if (slo_pg_add_keyframe(g, st.kf_pre, out, key) != SLO_OK) { ctx->err = slo_pg_last_error(g); return SLO_E_STATE; }
            if (!ctx->pg_pending[s]) continue;
            // saveKeyFramesAndFactor after a loop: the new pose and the
            // transforms from the estimate; correctPoses: every key pose
            const int n = slo_pg_size(g);
            std::vector<float> poses((size_t)n * 6);
            if (slo_pg_get_key_poses(g, poses.data(), n) != n) { ctx->err = slo_pg_last_error(g); return SLO_E_STATE; }
            if (int r = pg_upload(ctx, poses)) return r;
            PgTf tf;
            memcpy(tf.t, out, sizeof out);
            SLO_LAUNCH(ctx, "pg_writeback", k_pg_writeback, dim3(1), dim3(256), 0, ctx->v, s, ctx->d_pg_poses, n, 1,
                       tf, 1);
        } else if (ctx->pg_pending[s]) {
            // correctPoses without a new keyframe: isamCurrentEstimate is the
            // one of the last save, taken before the loop factor went in
            const std::vector<float>& snap = ctx->pg_snap[s];
            if (int r = pg_upload(ctx, snap)) return r;
            PgTf tf{};
            SLO_LAUNCH(ctx, "pg_writeback", k_pg_writeback, dim3(1), dim3(256), 0, ctx->v, s, ctx->d_pg_poses,
                       (int)(snap.size() / 6), 0, tf, 1);
        } else {
            continue;
        }
        ctx->pg_pending[s] = 0;   // aLoopIsClosed = false (MO:1662)
        SLO_CHECK(hipStreamSynchronize(ctx->stream));   // d_pg_poses is reused by the next stream
    }
    return 0;
}

int pg_after_loops(slo_ctx* ctx) {
    const int S = ctx->S;
    std::vector<slo_loop_result> res((size_t)S * 2);
    SLO_CHECK(hipMemcpyAsync(ctx->h_st, ctx->v.st, sizeof(StreamState) * S, hipMemcpyDeviceToHost, ctx->stream));
    SLO_CHECK(hipMemcpyAsync(res.data(), ctx->lc.res, sizeof(slo_loop_result) * 2 * S, hipMemcpyDeviceToHost,
                             ctx->stream));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    for (int s = 0; s < S; ++s) {
        const StreamState& st = ctx->h_st[s];
        if (!st.det_valid || !st.kf_saved) continue;
        const slo_loop_result& rs = res[2 * s];
        const slo_loop_result& sc = res[2 * s + 1];
        const bool use_rs = rs.ran && rs.accepted && rs.id >= 0, use_sc = sc.ran && sc.accepted && sc.id >= 0;
        // performLoopClosure got past detectLoopClosure: aLoopIsClosed is set
        // whether or not an ICP was accepted (MO:1107-1108), so correctPoses
        // runs at the next mapping step either way
        if (!rs.ran && !sc.ran) continue;
        slo_pg* g = ctx->pg[s];
        const int latest = st.n_keyframes - 1;   // latestFrameIDLoopCloure (MO:849)
        if (latest < 0 || latest >= slo_pg_size(g)) continue;
        // isamCurrentEstimate as of the last save, for a correctPoses without a new keyframe
        std::vector<float>& snap = ctx->pg_snap[s];
        snap.resize((size_t)slo_pg_size(g) * 6);
        slo_pg_get_key_poses(g, snap.data(), slo_pg_size(g));
        if (use_rs) {
            float latest6[6], to6[6], from[6], to[6];
            SLO_CHECK(hipMemcpy(latest6, ctx->v.kf_pose + ((size_t)s * ctx->v.KFMAX + latest) * 6, 24,
                                hipMemcpyDeviceToHost));
            SLO_CHECK(hipMemcpy(to6, ctx->v.kf_pose + ((size_t)s * ctx->v.KFMAX + rs.id) * 6, 24,
                                hipMemcpyDeviceToHost));
            rs_loop_from(rs.xyzrpy, latest6, from);
            // pclPointTogtsamPose3 (MO:1113-1115): RzRyRx(yaw, roll, pitch), Point3(z, x, y)
            to[0] = to6[5]; to[1] = to6[3]; to[2] = to6[4]; to[3] = to6[2]; to[4] = to6[0]; to[5] = to6[1];
            if (slo_pg_add_loop(g, latest, rs.id, from, to) != SLO_OK) { ctx->err = slo_pg_last_error(g); return SLO_E_STATE; }
        }
        if (use_sc) {
            const float from[6] = {sc.xyzrpy[3], sc.xyzrpy[4], sc.xyzrpy[5], sc.xyzrpy[0], sc.xyzrpy[1], sc.xyzrpy[2]};
            const float to[6] = {0, 0, 0, 0, 0, 0};
            if (slo_pg_add_loop(g, latest, sc.id, from, to) != SLO_OK) { ctx->err = slo_pg_last_error(g); return SLO_E_STATE; }
        }
        if ((use_rs || use_sc) && slo_pg_optimize(g, 0, nullptr, nullptr) < 0) {   // isam->update (MO:1045, 1090)
            ctx->err = slo_pg_last_error(g);
            return SLO_E_STATE;
        }
        ctx->pg_pending[s] = 1;   // aLoopIsClosed = true (MO:1107)
    }
    return 0;
}

int pg_alloc(slo_ctx* ctx) {
    ctx->pg.assign(ctx->S, nullptr);
    ctx->pg_pending.assign(ctx->S, 0);
    ctx->pg_snap.assign(ctx->S, {});
    for (int s = 0; s < ctx->S; ++s)
        if (slo_pg_create(&ctx->pg[s]) != SLO_OK) return SLO_E_CAPACITY;
    return 0;
}

void pg_free(slo_ctx* ctx) {
    for (slo_pg* g : ctx->pg) slo_pg_destroy(g);
    ctx->pg.clear();
    if (ctx->d_pg_poses) hipFree(ctx->d_pg_poses);
    ctx->d_pg_poses = nullptr;
    ctx->pg_cap = 0;
}

}  // namespace slo

extern "C" {

int slo_set_key_poses(slo_ctx* ctx, int stream, const float* poses6, int n, const float* transform6) {
    if (!ctx || stream < 0 || stream >= ctx->S || n < 0 || n > ctx->v.KFMAX || (n > 0 && !poses6)) return SLO_E_ARG;
    SLO_CHECK(hipSetDevice(ctx->dev));
    std::vector<float> p(poses6, poses6 + (size_t)n * 6);
    if (int r = slo::pg_upload(ctx, p)) return r;
    slo::PgTf tf{};
    if (transform6) memcpy(tf.t, transform6, sizeof tf.t);
    SLO_LAUNCH(ctx, "pg_writeback", slo::k_pg_writeback, dim3(1), dim3(256), 0, ctx->v, stream, ctx->d_pg_poses, n,
               transform6 ? 1 : 0, tf, 1);
    SLO_CHECK(hipStreamSynchronize(ctx->stream));
    return SLO_OK;
}

}  // extern "C"
