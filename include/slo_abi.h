/* slo_abi.h — C ABI of the MI355X-native SC-LeGO-LOAM hot path (libslo.so).
 *
 * Drop-in boundary for the four per-scan entry points of the reference
 * (SURVEY §8(b)); every function is extern "C", noexcept, returns 0 on
 * success or a negative SLO_E* code (text via slo_last_error()).
 *
 *   reference entry point                                  replaced by
 *   ImageProjection::cloudHandler   imageProjection.cpp:181   slo_image_projection / slo_batch_image_projection
 *   FeatureAssociation::runFeatureAssociation
 *                                featureAssociation.cpp:1817  slo_feature_association / slo_batch_feature_association
 *   mapOptimization::run            mapOptmization.cpp:1673   slo_map_optimization / slo_batch_map_optimization
 *   SCManager::makeAndSaveScancontextAndKeys Scancontext.h:72 (called inside the mapping step, MO:1630)
 *   SCManager::detectLoopClosureID  Scancontext.h:73 / MO:916 slo_sc_detect / slo_batch_sc_detect
 *
 * One context serves `n_streams` independent LiDAR streams (the batch
 * dimension): a batched call advances every stream by one scan.  The
 * single-scan calls act on stream 0 and take host memory, exactly like the
 * reference callbacks.  A context is single-caller; the caller serialises
 * (the reference's `mtx`, mapOptmization.cpp:197).  Every entry point sets
 * the context's HIP device first, so calls may come from any host thread.
 */
#ifndef SLO_ABI_H
#define SLO_ABI_H

#include <stddef.h>
#include <stdint.h>
#include "slo_config.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SLO_OK 0
#define SLO_E_ARG (-1)
#define SLO_E_HIP (-2)
#define SLO_E_CAPACITY (-3)
#define SLO_E_STATE (-4)
/* a positive status is a result with a caveat, not an error: slo_pg_optimize
 * stopped at max_iters before its convergence test held (the estimate is the
 * last accepted iterate) */
#define SLO_NOT_CONVERGED 1

typedef struct slo_ctx slo_ctx;

/* Fill *out with a named preset (SLO_PRESET_*), reference defaults. */
int slo_config_preset(int preset, slo_config* out);

/* Create a context on HIP device `hip_device` for `n_streams` streams. */
int slo_create(const slo_config* cfg, int hip_device, int n_streams, slo_ctx** out);
void slo_destroy(slo_ctx* ctx);
const char* slo_last_error(const slo_ctx* ctx);
/* The hipStream_t all work of this context is queued on. */
void* slo_stream(slo_ctx* ctx);
/* Block until all queued work of the context is done. */
int slo_synchronize(slo_ctx* ctx);
/* Allocate now every workspace a mapping step will use (the VoxelGrid and
 * PCL-order sort workspaces of mapOptimization, MO:1224-1263), sized from the
 * configured capacities; otherwise the first call that can map does it.  A
 * caller budgeting device memory calls it right after slo_create; a Mode S
 * front or odometry context never maps and never holds them. */
int slo_prepare_mapping(slo_ctx* ctx);

/* ---------------------------------------------------------------- batched
 * d_points: device array [n_streams][cfg.max_points] of (x,y,z,intensity)
 * float4 in firing order, NaN for no return; d_counts: device int32
 * [n_streams].  All batched calls are asynchronous on slo_stream(). */
int slo_batch_image_projection(slo_ctx* ctx, const void* d_points, const int32_t* d_counts);
/* cfg.use_cloud_ring: device uint16 [n_streams][cfg.max_points], the ring of
 * each input point (indexed like d_points); kept for the following calls */
int slo_batch_set_rings(slo_ctx* ctx, const uint16_t* d_rings);
/* features (FA:1833-1839) + scan-to-scan odometry (FA:1846-1859) */
int slo_batch_feature_association(slo_ctx* ctx);
/* mapping step for streams whose FA published this scan and whose
 * t_scan - t_last >= mappingProcessInterval (MO:1675-1706), incl. keyframe
 * save and Scan Context make (MO:1630); d_points as above (raw cloud, Q16) */
int slo_batch_map_optimization(slo_ctx* ctx, const void* d_points, const int32_t* d_counts, double t_scan);
/* SC loop detection for every stream that saved a keyframe this scan */
int slo_batch_sc_detect(slo_ctx* ctx);
/* whole pipeline for one scan per stream with the deterministic gating of
 * IP -> FA -> [mapping + SC make] -> [SC detect].  After the
 * first scan each step is one HIP graph launch (captured per step kind, with
 * and without the mapping stage) unless graphs are off, timing is on, or
 * cfg.loop_verify / cfg.pose_graph need host round trips. */
int slo_batch_process(slo_ctx* ctx, const void* d_points, const int32_t* d_counts, double t_scan);
/* on != 0 (the default): slo_batch_process replays captured graphs; 0:
 * every launch issued eagerly (the captured graphs are released) */
int slo_graph_mode(slo_ctx* ctx, int on);

/* ---------------------------------------------------------------- IMU (FeatureAssociation::imuHandler)
 * sensor_msgs/Imu as imuHandler reads it (featureAssociation.cpp:459-486):
 * header stamp, orientation quaternion, linear acceleration, angular
 * velocity, all float64.  Each message is pushed on the stream's 200-entry
 * IMU ring (imuQueLength) and integrated (AccumulateIMUShiftAndRotation,
 * FA:417-457); the next scans deskew against the ring (adjustDistortion,
 * FA:525-616), seed the odometry (updateInitialGuess, FA:1639-1664) and
 * plug the IMU rotation into the integration (FA:1697-1725).  Without any
 * message every IMU term is the reference's zero. */
typedef struct slo_imu_msg {
    double stamp;
    double qx, qy, qz, qw;
    double ax, ay, az;
    double wx, wy, wz;
} slo_imu_msg;
/* d_msgs: device [n_streams][msgs_per_stream]; d_counts: device int32
 * [n_streams]: the messages each stream's imuHandler receives, in order,
 * before its next scan (async on slo_stream()) */
int slo_batch_imu(slo_ctx* ctx, const slo_imu_msg* d_msgs, int msgs_per_stream, const int32_t* d_counts);
/* the stamp of the scan the next feature step deskews (cloudHeader.stamp,
 * FA:488-491; slo_batch_process and slo_feature_association set it) */
int slo_batch_scan_time(slo_ctx* ctx, double t_scan);
/* imuHandler of a one-stream context on a host message */
int slo_imu_handler(slo_ctx* ctx, const slo_imu_msg* msg);

/* ---------------------------------------------------------------- single scan (stream 0, host memory) */
typedef struct slo_seg_view {
    int32_t n_segmented;           /* |segmentedCloud| */
    const float* segmented;        /* n_segmented x (x,y,z,intensity) */
    const uint8_t* ground_flag;    /* cloud_info.segmentedCloudGroundFlag */
    const uint32_t* col_ind;       /* cloud_info.segmentedCloudColInd */
    const float* range;            /* cloud_info.segmentedCloudRange */
    const int32_t* start_ring_index;
    const int32_t* end_ring_index;
    float start_orientation, end_orientation, orientation_diff;
    int32_t n_outlier;
    const float* outlier;          /* n_outlier x 4 */
} slo_seg_view;

typedef struct slo_fa_view {
    int32_t n_sharp, n_less_sharp, n_flat, n_less_flat;
    const float* sharp;            /* each n x (x,y,z,intensity), camera frame */
    const float* less_sharp;
    const float* flat;
    const float* less_flat;
    float transform_sum[6];        /* /laser_odom_to_init (rx,ry,rz,tx,ty,tz) */
    int32_t published;             /* 1 if this scan went to mapping (FA:1790) */
} slo_fa_view;

typedef struct slo_map_view {
    int32_t ran;                   /* mapping ran for this scan */
    int32_t keyframe_saved;
    int32_t n_keyframes;
    float transform_aft_mapped[6]; /* /aft_mapped_to_init */
} slo_map_view;

/* pts: n points, stride_bytes apart, xyz at off_xyz (3 floats), intensity at off_i */
int slo_image_projection(slo_ctx* ctx, const void* pts, size_t n, size_t stride_bytes, size_t off_xyz,
                         size_t off_i, slo_seg_view* out);
/* useCloudRing (cfg.use_cloud_ring, IP:172-178, 225-226): rings[k] is the
 * "ring" of input point k in the message's order; the reference reads it at
 * the point's index AFTER NaN removal (laserCloudInRing->points[i]), which
 * is the same point only for the dense clouds it accepts (IP:174-177) */
int slo_image_projection_ring(slo_ctx* ctx, const void* pts, size_t n, size_t stride_bytes, size_t off_xyz,
                              size_t off_i, const uint16_t* rings, slo_seg_view* out);
int slo_feature_association(slo_ctx* ctx, double t_scan, slo_fa_view* out);
/* raw_pts: the raw cloud of the scan being mapped (same layout arguments) */
int slo_map_optimization(slo_ctx* ctx, const void* raw_pts, size_t n, size_t stride_bytes, size_t off_xyz,
                         size_t off_i, double t_scan, slo_map_view* out);
int slo_sc_detect(slo_ctx* ctx, int32_t* loop_id, float* yaw_rad, double* min_dist);
/* SCManager::makeAndSaveScancontextAndKeys (Scancontext.cpp:230) on stream 0:
 * pts is the already downsampled cloud, as in the reference call (MO:1630) */
int slo_sc_make_and_save(slo_ctx* ctx, const void* pts, size_t n, size_t stride_bytes, size_t off_xyz,
                         size_t off_i);
/* batched: VoxelGrid(0.5) + makeAndSaveScancontextAndKeys for every stream
 * (used to seed the Scan Context history, e.g. from a previous session) */
int slo_batch_sc_make(slo_ctx* ctx, const void* d_points, const int32_t* d_counts);

/* The public SCManager helpers (Scancontext.h:63-69), computed on the device
 * in the reference's evaluation order (Eigen 3.3 packet sums).  A descriptor
 * is NR x NS doubles, row-major (ring r, sector c at [r * NS + c]; Eigen's
 * MatrixXd is column-major, so bind it through a RowMajor Map); a ring key is
 * NR doubles, a sector key NS doubles (cfg.sc_num_ring / sc_num_sector).
 * Host pointers; synchronous. */
/* makeScancontext (SCc:151-195): n points of stride_bytes with x, y, z floats at off_xyz */
int slo_sc_make_scancontext(slo_ctx* ctx, const void* pts, size_t n, size_t stride_bytes, size_t off_xyz,
                            double* desc);
/* makeRingkeyFromScancontext (SCc:198-211): the row means */
int slo_sc_ring_key(slo_ctx* ctx, const double* desc, double* ring_key);
/* makeSectorkeyFromScancontext (SCc:214-227): the column means */
int slo_sc_sector_key(slo_ctx* ctx, const double* desc, double* sector_key);
/* fastAlignUsingVkey (SCc:93-113): the shift of least |vkey1 - circshift(vkey2, shift)| */
int slo_sc_fast_align(slo_ctx* ctx, const double* vkey1, const double* vkey2, int32_t* shift);
/* distDirectSC (SCc:69-90): 1 - mean cosine of the columns non-zero in both */
int slo_sc_dist_direct(slo_ctx* ctx, const double* sc1, const double* sc2, double* dist);
/* distanceBtnScanContext (SCc:116-148): (min distance over the aligned shift
 * window, its shift) */
int slo_sc_distance(slo_ctx* ctx, const double* sc1, const double* sc2, double* dist, int32_t* shift);
/* batched distanceBtnScanContext on device arrays: n pairs (d_sc1[i], d_sc2[i]),
 * each NR x NS; asynchronous on slo_stream(ctx) */
int slo_batch_sc_distance(slo_ctx* ctx, const double* d_sc1, const double* d_sc2, int n, double* d_dist,
                          int32_t* d_shift);

/* pcl::VoxelGrid<PointXYZI> setLeafSize(leaf) + filter (PCL 1.8 applyFilter,
 * the reference's downsize filters: featureAssociation.cpp:779-780,
 * mapOptmization.cpp:1224-1262) on every stream's device cloud at once:
 * stream s's d_n[s] float4 points (x, y, z, intensity; non-finite ones
 * skipped) at d_in + s * in_stride points; its centroids, in voxel-index
 * order, to d_out + s * out_stride, at most out_cap (more are clipped and
 * flagged in slo_get(.., "vg_stats")[1]), their count to d_nout[s].  The
 * order inside a voxel follows cfg.voxel_order (SLO_VOXEL_PCL: std::sort's,
 * as PCL).  vg_stats[0] counts the ranges the PCL-order sort finished on one
 * lane (a spent introsort depth budget: adversarial inputs), [2] / [3] / [4]
 * inconsistent wave-sort steps, tail cuts and tail partners (internal checks;
 * always 0).  A stream whose range tripped one of the checks [2]-[4] also
 * gets bit 16 (SORT) of slo_get(.., s, "err"); a stream of 2^24 or more
 * finite points is not sorted and gets bit 4 (CAPACITY).  Returns SLO_E_ARG
 * when out_cap > out_stride (the output rows would overlap) and
 * SLO_E_CAPACITY when n_streams * in_stride exceeds INT32_MAX items (the
 * sort's positions are 32-bit).  Asynchronous on slo_stream(ctx). */
int slo_batch_voxel_grid(slo_ctx* ctx, const void* d_in, size_t in_stride, const int32_t* d_n, float leaf,
                         void* d_out, size_t out_stride, int32_t* d_nout, int out_cap);

/* ---------------------------------------------------------------- Mode S: one stream over several contexts
 * One vehicle's stream split over contexts, on one GPU or several (SURVEY
 * §8(e) mode S; the reference deploys the same split as processes,
 * launch/run.launch:14-17).  Front contexts take turns at the scans' front
 * ends — imageProjection::cloudHandler and featureAssociation's feature
 * extraction (adjustDistortion .. extractFeatures, FA:1833-1841) — and one
 * owner context runs every scan's back end: the odometry (FA:1843-1858),
 * mapOptimization and Scan Context.  Two device buffers travel per scan:
 * - the carry, from a scan's front end to the next scan's: the state a front
 *   end inherits (featureAssociation's persistent arrays, read where a scan
 *   does not rewrite them; the cloud_info arrays past the scan's points; the
 *   orientations an empty scan keeps — SURVEY Appendix A Q5);
 * - the features, from a scan's front end to the owner.
 * Every context needs the same config and n_streams.  Not with IMU input (its
 * ring would have to travel too).  Asynchronous on slo_stream(ctx); the caller
 * moves the buffers (hipMemcpyPeer, RCCL send / recv: slo_amd/modes.py). */
size_t slo_modes_carry_bytes(slo_ctx* ctx);
size_t slo_modes_features_bytes(slo_ctx* ctx);
/* the front end of the scan in d_points / d_counts (as slo_batch_process);
 * d_carry_in: the previous scan's carry (NULL for a stream's first scan, or
 * when the previous scan's front end ran on this same context); writes this
 * scan's carry (NULL: not needed, the next front end runs here too) and its
 * features (device buffers of the sizes above) */
int slo_front_process(slo_ctx* ctx, const void* d_points, const int32_t* d_counts, double t_scan,
                      const void* d_carry_in, void* d_carry_out, void* d_features_out);
/* the back end of the scan whose front end wrote d_features; d_points /
 * d_counts: that scan again (mapping reads the raw cloud, MO:1236) */
int slo_back_process(slo_ctx* ctx, const void* d_features, const void* d_points, const int32_t* d_counts,
                     double t_scan);
/* The back end in two stages (the reference's featureAssociation |
 * mapOptimization process boundary, launch/run.launch:15-16): an odometry
 * context runs slo_odom_process — featureAssociation's odometry and publish
 * gate (FA:1843-1858, 1790-1814) — and hands a third buffer to a mapping
 * context, which runs slo_map_process — transformFusion's
 * laserOdometryHandler (TF:186-219), mapOptimization (MO:1685-1699) and Scan
 * Context, in scan order.  The mapping context then holds what the owner of
 * slo_back_process would: slo_get on it reads the same poses, keyframes,
 * descriptors and detect records.  The odometry buffer: the published corner /
 * surf clouds (after TransformToEnd), the outliers, their counts, the
 * stream's err bits and transformSum. */
size_t slo_modes_odom_bytes(slo_ctx* ctx);
int slo_odom_process(slo_ctx* ctx, const void* d_features, const void* d_points, const int32_t* d_counts,
                     double t_scan, void* d_odom_out);
int slo_map_process(slo_ctx* ctx, const void* d_odom, const void* d_points, const int32_t* d_counts, double t_scan);

/* The same three-stage split inside ONE context (the reference's three
 * processes, launch/run.launch:14-17, as three HIP streams): after
 * slo_pipeline(ctx, depth >= 2) on a fresh context, slo_batch_process(ctx, ..)
 * runs a scan's front end on an internal front context, its odometry on an
 * internal odometry context and transformFusion + mapOptimization + Scan
 * Context on ctx itself, each on its own HIP stream, the stages chained by
 * events through rings of `depth` feature / odometry buffers and input copies —
 * so scan k + 2's front end, scan k + 1's odometry and scan k's mapping step
 * run at once, and the host only enqueues.  Results are bit-identical to the
 * context without it (Mode S above).  slo_get reads each field from the stage
 * that computes it; slo_synchronize waits for all three; slo_stream(ctx) is
 * the mapping stage's stream, the last one a scan passes (its completion
 * covers every stage of every scan issued).  depth 0 turns it off again (only
 * before the first scan).  Not with IMU input, loop verification or the pose
 * graph (their host round trips need the one-context path): SLO_E_STATE. */
int slo_pipeline(slo_ctx* ctx, int depth);

/* ---------------------------------------------------------------- loop-closure verification
 * mapOptmization.cpp:841-1110 (detectLoopClosure + performLoopClosure, minus
 * the GTSAM factors).  Needs cfg.loop_verify = 1 and
 * cfg.loop_archive_points > 0 at slo_create (the keyframe archive).  One
 * record per candidate, [0] = radius search (RS), [1] = Scan Context (SC). */
typedef struct slo_loop_result {
    int32_t id;          /* candidate keyframe, -1 none */
    int32_t ran;         /* ICP ran (only when an SC candidate exists, MO:925-927) */
    int32_t converged;   /* icp.hasConverged() */
    int32_t accepted;    /* converged && fitness <= historyKeyframeFitnessScore (MO:1020 / 1071) */
    int32_t iters;       /* ICP iterations */
    int32_t n_src, n_tgt;  /* source cloud / downsampled submap sizes */
    int32_t pad;
    double fitness;      /* icp.getFitnessScore() */
    float T[16];         /* icp.getFinalTransformation(), row-major */
    float xyzrpy[6];     /* pcl::getTranslationAndEulerAngles(T): x, y, z, roll, pitch, yaw */
} slo_loop_result;

/* RS + SC verification for every stream whose SC detect ran this scan
 * (slo_batch_process calls it when cfg.loop_verify is set); results via
 * slo_get(.., "loop") */
int slo_batch_loop_closure(slo_ctx* ctx);
/* the same for stream 0 after slo_sc_detect; out[0] = RS, out[1] = SC */
int slo_loop_closure(slo_ctx* ctx, slo_loop_result* out);
/* pcl::IterativeClosestPoint::align + getFitnessScore (MO:1006-1016) on given
 * device clouds, one pair per stream: d_src [n_streams][src_stride] float4,
 * d_nsrc int32 [n_streams], d_tgt [n_streams][tgt_stride], d_ntgt; counts
 * must fit loop_archive_points.  Writes n_streams records to host h_out. */
int slo_icp_align_batch(slo_ctx* ctx, const void* d_src, size_t src_stride, const int32_t* d_nsrc, const void* d_tgt,
                        size_t tgt_stride, const int32_t* d_ntgt, slo_loop_result* h_out);

/* ---------------------------------------------------------------- multi-GPU records
 * Pack one fixed-size record per stream into device memory d_out
 * [n_streams][SLO_RECORD_FLOATS] floats for the RCCL all-gather (SURVEY
 * §8(e)): odometry pose (transformSum), mapped pose (transformAftMapped),
 * keyframe count, keyframe-saved flag, this step's loop result, the newest
 * ring key, and — when a keyframe was saved — its Scan Context descriptor
 * (20 x 60 cell maxima: floats or 0, so the f32 copy is exact; the ring and
 * sector keys are derived from it bit for bit, Scancontext.cpp:198-227). */
#define SLO_RECORD_FLOATS 1240
#define SLO_REC_POSE 0          /* [6] transformSum */
#define SLO_REC_MAPPED 6        /* [6] transformAftMapped */
#define SLO_REC_N_KEYFRAMES 12
#define SLO_REC_KF_SAVED 13     /* 1 when this step saved a keyframe */
#define SLO_REC_LOOP_ID 14      /* detect: loop id, -1 none, -2 no detect this step */
#define SLO_REC_MIN_DIST 15
#define SLO_REC_RING_KEY 16     /* [20] newest ring key (f32 tree row) */
#define SLO_REC_SC_COUNT 36
#define SLO_REC_ERR 37
#define SLO_REC_KF_INDEX 38     /* keyframe index of the descriptor, -1 none */
#define SLO_REC_YAW 39
#define SLO_REC_DESC 40         /* [NR*NS <= 1200] descriptor, row-major (ring, sector) */
int slo_pack_records(slo_ctx* ctx, void* d_out);
int slo_record_floats(void);

/* Cross-stream Scan Context store over the all-gathered records (multi-
 * session loop candidates, csrc/slo_xsc.hip).  One store per rank holds the
 * descriptor history of all n_streams global streams (a ring of `cap` per
 * stream).  slo_xsc_ingest appends the descriptors of the records that saved
 * a keyframe (d_records = the whole gathered table, n_records == n_streams);
 * slo_xsc_query runs detectLoopClosureID (SCc:247-338) for each of n_query
 * records (global stream ids global0 ..) against every OTHER stream's
 * history: K nearest ring keys (exact f32 L2), distanceBtnScanContext, first
 * minimum, loop when below sc_dist_thres.  Asynchronous on hip_stream. */
typedef struct slo_xsc slo_xsc;
typedef struct slo_xsc_match {
    int32_t valid;          /* the record carried a new keyframe */
    int32_t n_cand;         /* candidates compared (<= sc_num_candidates) */
    int32_t nn_stream;      /* global stream of the best candidate, -1 none */
    int32_t nn_keyframe;    /* its keyframe index */
    int32_t loop;           /* min_dist < sc_dist_thres */
    float yaw;              /* alignment shift in radians */
    double min_dist;
} slo_xsc_match;
int slo_xsc_create(const slo_config* cfg, int hip_device, int n_streams, int cap, slo_xsc** out);
void slo_xsc_destroy(slo_xsc* g);
int slo_xsc_ingest(slo_xsc* g, const void* d_records, int n_records, void* hip_stream);
int slo_xsc_query(slo_xsc* g, const void* d_records, int n_query, int global0, void* d_out, void* hip_stream);

/* ---------------------------------------------------------------- readback
 * Copy a named per-stream result to host memory (synchronises).  Returns the
 * element count (copies at most cap_bytes), or < 0.  Names: "range",
 * "label", "ground", "seg_pts", "seg_ground", "seg_col", "seg_range",
 * "ring_start", "ring_end", "orient", "outlier", "fa_seg_pts", "curvature",
 * "picked", "cloud_label", "smooth_ind", "sharp", "less_sharp", "flat",
 * "less_flat", "corner_last", "surf_last", "transform_sum", "transform_cur",
 * "fa_iters", "mapped", "n_keyframes", "keyposes", "sc_desc", "ring_key",
 * "sector_key", "detect", "detect_f", "flags", "loop" (2 x slo_loop_result), "key_times",
 * "integrated" (transformFusion's /integrated_to_init for this scan, 6 floats:
 * transformFusion.cpp:186-219 on this scan's odometry and the last
 * published mapping result). */
int slo_get(slo_ctx* ctx, int stream, const char* name, void* dst, size_t cap_bytes);

/* per-kernel timing (HIP events around every launch when enabled) */
int slo_timing_enable(slo_ctx* ctx, int enable);
/* fills up to cap entries of names (NUL-separated into buf) and total ms and
 * launch counts; returns number of kernels */
int slo_timing_read(slo_ctx* ctx, char* names_buf, size_t buf_bytes, double* total_ms, int64_t* launches, int cap);
int slo_timing_reset(slo_ctx* ctx);
/* time only the launches named `name` — one name or a comma-separated list
 * (NULL or "" = all, by HIP events, eager launches).  With a filter the
 * launches are timed by in-stream device timestamps (the constant-rate wall
 * clock) that are captured into the step graphs, so the bench times its
 * roofline kernels this way inside the timed region */
int slo_timing_filter(slo_ctx* ctx, const char* name);

/* ---------------------------------------------------------------- wire format
 * sensor_msgs/PointCloud2 -> pcl::PointCloud<PointXYZI>, the conversion of
 * ImageProjection::copyPointCloud (imageProjection.cpp:167,
 * pcl::fromROSMsg).  PCL's field mapping (pcl/conversions.h FieldMapper /
 * FieldMatches): each of x, y, z, intensity takes the FIRST message field of
 * the same name whose datatype is FLOAT32 (7) and whose count is 1 or 0; a
 * field with no match stays 0 (PointXYZI's constructor) — e.g. an intensity
 * sent as UINT16 reads as 0, exactly like the reference.  Point (r, c) is at
 * data + r * row_step + c * point_step; is_bigendian is not looked at (PCL
 * copies bytes as they are).  NaN removal (IP:170) is part of the projection. */
#define SLO_PF_INT8 1
#define SLO_PF_UINT8 2
#define SLO_PF_INT16 3
#define SLO_PF_UINT16 4
#define SLO_PF_INT32 5
#define SLO_PF_UINT32 6
#define SLO_PF_FLOAT32 7
#define SLO_PF_FLOAT64 8

typedef struct slo_pc2_field {   /* sensor_msgs/PointField */
    const char* name;
    uint32_t offset;
    uint8_t datatype;
    uint32_t count;
} slo_pc2_field;

typedef struct slo_pc2 {         /* sensor_msgs/PointCloud2 (header omitted: t_scan is passed separately) */
    uint32_t height, width;
    const slo_pc2_field* fields;
    int32_t n_fields;
    uint8_t is_bigendian;
    uint32_t point_step, row_step;
    const uint8_t* data;
    size_t data_bytes;
    uint8_t is_dense;
} slo_pc2;

/* byte offsets of x, y, z, intensity (FLOAT32) and ring (UINT16, the
 * reference's PointXYZIR, utility.h:158-169) inside a point, -1 = no match */
typedef struct slo_pc2_layout {
    uint32_t point_step;
    int32_t off_x, off_y, off_z, off_intensity;
    int32_t off_ring;
} slo_pc2_layout;

/* the field mapping alone; SLO_E_ARG if a matched field does not fit in point_step */
int slo_pc2_layout_of(const slo_pc2* msg, slo_pc2_layout* out);
/* fromROSMsg into host (x,y,z,intensity) float4s; *n_out = width * height.
 * SLO_E_CAPACITY (with *n_out set) when cap_points is too small, SLO_E_ARG
 * when data_bytes cannot hold the last point. */
int slo_pc2_to_xyzi(const slo_pc2* msg, float* out_xyzi, size_t cap_points, size_t* n_out);
/* ImageProjection::cloudHandler (IP:181) taking the message itself; with
 * cfg.use_cloud_ring the rows come from the uint16 "ring" field exactly as
 * IP:172-178 / 225-226 read them (SLO_E_ARG unless is_dense) */
int slo_image_projection_pc2(slo_ctx* ctx, const slo_pc2* msg, slo_seg_view* out);
/* batched, on the device: n_streams messages of one point layout, message s
 * at d_bytes + s * msg_stride with d_dims[3 s .. 3 s + 2] = (width, height,
 * row_step); writes the d_points / d_counts of slo_batch_image_projection.
 * A message of more than cfg.max_points points keeps its first max_points
 * (the context's capacity; bit 8 of slo_get(.., "err") is set); one whose
 * points would reach past msg_stride is not read (count 0, same bit).  d_rings
 * (optional, NULL = none) receives each point's ring for slo_batch_set_rings
 * (0 where the layout has no uint16 ring).  Asynchronous. */
int slo_batch_pc2_unpack(slo_ctx* ctx, const uint8_t* d_bytes, size_t msg_stride, const int32_t* d_dims,
                         const slo_pc2_layout* layout, void* d_points, int32_t* d_counts, uint16_t* d_rings);

/* synthetic stream generator (sc-lego-loam_amd/csrc/slo_gen.h), host side */
int slo_gen_scan(int preset, int config_id, int stream_id, int scan_index, float* out_xyzi);
/* n_streams x n_scans scans, layout [scan][stream][max_points][4], host threads */
int slo_gen_batch(int preset, int config_id, int stream0, int n_streams, int scan0, int n_scans, float* out,
                  int n_threads);

/* The same generator on the device (csrc/slo_gendev.hip; benchmark inputs):
 * scans of streams stream0 .. stream0+n_streams-1, bit-identical to
 * slo_gen_batch.  slo_gen_device_scans writes [n_scans][n_streams][max_points][4]
 * floats to device memory d_out on hip_stream (a hipStream_t, NULL = default)
 * and returns when they are written; n_scans * n_streams <= 65535 per call. */
typedef struct slo_gen_dev slo_gen_dev;
int slo_gen_device_create(int preset, int config_id, int stream0, int n_streams, int hip_device, slo_gen_dev** out);
int slo_gen_device_scans(slo_gen_dev* g, int scan0, int n_scans, void* d_out, void* hip_stream);
void slo_gen_device_destroy(slo_gen_dev* g);

/* Pose-graph back end (sc-lego-loam_amd/csrc/slo_pg.hip), host side.  Replaces
 * mapOptimization's GTSAM iSAM2 graph: prior + odometry between factors
 * (MO:365-368, 1541-1611), robust Cauchy loop factors (MO:985-997, 1038-1046,
 * 1083-1091, the isam->update after them) and correctPoses (MO:1642-1664). */
typedef struct slo_pg slo_pg;
int slo_pg_create(slo_pg** out);
void slo_pg_destroy(slo_pg* g);
const char* slo_pg_last_error(slo_pg* g);
int slo_pg_size(slo_pg* g);
/* saveKeyFramesAndFactor's graph step: transform = transformAftMapped (transformTobeMapped
 * for the first key frame), LeGO order rx ry rz tx ty tz; writes the updated
 * transformAftMapped and the new cloudKeyPoses6D entry (x y z roll pitch yaw); either may be NULL */
int slo_pg_add_keyframe(slo_pg* g, const float transform[6], float transform_out[6], float key_pose6d[6]);
/* BetweenFactor(from_id, to_id, poseFrom.between(poseTo)), each pose given as the
 * Pose3(Rot3::RzRyRx(v0, v1, v2), Point3(v3, v4, v5)) arguments the reference builds */
int slo_pg_add_loop(slo_pg* g, int from_id, int to_id, const float pose_from[6], const float pose_to[6]);
/* solve to convergence (max_iters <= 0: 100); iters_out / cost_out may be NULL.
 * SLO_OK when the relative cost decrease fell below 1e-12 or no damping lowered
 * the cost any more (converged to rounding); SLO_NOT_CONVERGED when max_iters
 * ran out first */
int slo_pg_optimize(slo_pg* g, int max_iters, int* iters_out, double* cost_out);
/* correctPoses: all key poses, 6 floats each; returns the count or a negative code */
int slo_pg_get_key_poses(slo_pg* g, float* out6, int cap);
int slo_pg_last_transform(slo_pg* g, float out[6]);
/* correctPoses into a stream's device state (synchronises): key poses
 * [0, n) (cloudKeyPoses6D order x y z roll pitch yaw); transform6 (may be
 * NULL) becomes transformAftMapped, transformLast and transformTobeMapped
 * (MO:1601-1611); the recent keyframe deque is cleared, so the next mapping
 * step rebuilds its local map from the corrected poses (MO:1642-1664).
 * cfg.pose_graph does this itself; a caller driving slo_pg by hand uses it. */
int slo_set_key_poses(slo_ctx* ctx, int stream, const float* poses6, int n, const float* transform6);

#ifdef __cplusplus
}
#endif
#endif
