// slo_imu.hip — FeatureAssociation::imuHandler for a batch of streams
// (featureAssociation.cpp:459-486 with AccumulateIMUShiftAndRotation,
// FA:417-457) and the C ABI of the IMU input.  The handlers of one stream
// run in message order on one lane (each message integrates on the
// previous one); the streams run side by side.  The scan-side use of the
// ring is in slo_fa.hip (k_fa_imu_start, k_fa_points) and slo_odom.hip
// (updateInitialGuess, TransformToEnd, integrateTransformation).
#include "slo_internal.h"
#include "slo_imu.h"

namespace slo {

__global__ void k_imu_init(DevView v) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    v.imu[s].last = -1;        // imuPointerLast (FA:251)
    v.imu[s].last_iter = 0;    // imuPointerLastIteration (FA:252)
}

__global__ void k_imu_ingest(DevView v, const slo_imu_msg* msgs, int per, const int32_t* counts) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= v.S) return;
    ImuState& m = v.imu[s];
    const int n = min(counts[s], per);
    for (int k = 0; k < n; ++k) slo_imu::imu_handler(m, msgs[(size_t)s * per + k], v.cfg.scan_period);
}

int imu_init(slo_ctx* ctx) {
    SLO_LAUNCH(ctx, "imu_init", k_imu_init, dim3((ctx->S + 63) / 64), dim3(64), 0, ctx->v);
    SLO_CHECK(hipGetLastError());
    return 0;
}

// a context Mode S ran on takes no IMU messages (slo_ctx.hip modes_enter)
int imu_enter(slo_ctx* ctx) {
    if (ctx->modes_used) {
        ctx->err = "IMU messages on a context a Mode S entry point ran on (Mode S carries no IMU ring)";
        return SLO_E_STATE;
    }
    ctx->imu_fed = true;
    return 0;
}

}  // namespace slo

extern "C" {

int slo_batch_imu(slo_ctx* ctx, const slo_imu_msg* d_msgs, int msgs_per_stream, const int32_t* d_counts) {
    if (!ctx || msgs_per_stream < 0 || (msgs_per_stream > 0 && (!d_msgs || !d_counts))) return SLO_E_ARG;
    if (msgs_per_stream == 0) return SLO_OK;
    if (int r = slo::imu_enter(ctx)) return r;
    SLO_CHECK(hipSetDevice(ctx->dev));
    SLO_LAUNCH(ctx, "imu_ingest", slo::k_imu_ingest, dim3((ctx->S + 63) / 64), dim3(64), 0, ctx->v, d_msgs,
               msgs_per_stream, d_counts);
    SLO_CHECK(hipGetLastError());
    return SLO_OK;
}

int slo_imu_handler(slo_ctx* ctx, const slo_imu_msg* msg) {
    if (!ctx || !msg) return SLO_E_ARG;
    if (ctx->S != 1) { ctx->err = "slo_imu_handler needs a context with n_streams == 1"; return SLO_E_STATE; }
    if (int r = slo::imu_enter(ctx)) return r;
    SLO_CHECK(hipSetDevice(ctx->dev));
    slo_imu_msg* d = nullptr;
    SLO_CHECK(hipMallocAsync((void**)&d, sizeof(slo_imu_msg) + sizeof(int32_t), ctx->stream));
    const int32_t one = 1;
    SLO_CHECK(hipMemcpyAsync(d, msg, sizeof(slo_imu_msg), hipMemcpyHostToDevice, ctx->stream));
    SLO_CHECK(hipMemcpyAsync((char*)d + sizeof(slo_imu_msg), &one, sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    SLO_LAUNCH(ctx, "imu_ingest", slo::k_imu_ingest, dim3(1), dim3(64), 0, ctx->v, d, 1,
               (const int32_t*)((char*)d + sizeof(slo_imu_msg)));
    SLO_CHECK(hipFreeAsync(d, ctx->stream));
    SLO_CHECK(hipStreamSynchronize(ctx->stream));   // the host message and `one` are read by the copies
    return SLO_OK;
}

}  // extern "C"
