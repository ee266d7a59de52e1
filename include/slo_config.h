/* slo_config.h — the runtime sensor / algorithm configuration of the C ABI
 * (include/slo_abi.h).  The reference compiles these as `extern const`
 * globals (utility.h:55-141, Scancontext.h:77-96, voxel leaves
 * mapOptmization.cpp:263-272 and featureAssociation.cpp:225); here they are
 * a plain struct so one library serves every sensor.  slo_config_preset()
 * fills it with the reference's values. */
#ifndef SLO_CONFIG_H
#define SLO_CONFIG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct slo_config {
    /* sensor geometry (utility.h:101-106) */
    int32_t n_scan;          /* rows R */
    int32_t horizon_scan;    /* columns C */
    float ang_res_x;         /* degrees per column */
    float ang_res_y;         /* degrees per row */
    float ang_bottom;        /* degrees below horizon of row 0 */
    int32_t ground_scan_ind; /* rows [0, gsi] are ground candidates */
    /* segmentation (utility.h:115-121) */
    float sensor_minimum_range;
    float sensor_mount_angle;
    float segment_theta;
    int32_t segment_valid_point_num;
    int32_t segment_valid_line_num;
    float segment_alpha_x;
    float segment_alpha_y;
    /* glibc sinf/cosf of the two alphas (imageProjection.cpp:421 evaluates
       sin(alpha)/cos(alpha) in float per edge; they are constants) */
    float sin_alpha_x, cos_alpha_x, sin_alpha_y, cos_alpha_y;
    /* features (utility.h:111, 124-129) */
    float scan_period;
    int32_t edge_feature_num;
    int32_t surf_feature_num;
    int32_t sections_total;
    float edge_threshold;
    float surf_threshold;
    float nearest_feature_search_sq_dist;
    /* mapping (utility.h:108-109, 134) */
    int32_t loop_closure_enable;
    double mapping_process_interval;
    int32_t surrounding_keyframe_search_num;
    /* voxel leaves (featureAssociation.cpp:225; mapOptmization.cpp:263-266) */
    float leaf_less_flat;    /* 0.2 */
    float leaf_corner;       /* 0.2 */
    float leaf_surf;         /* 0.3 */
    float leaf_outlier;      /* 0.4 */
    float leaf_sc;           /* 0.5 */
    /* Scan Context (Scancontext.h:77-96) */
    double sc_lidar_height;
    int32_t sc_num_ring;
    int32_t sc_num_sector;
    double sc_max_radius;
    int32_t sc_num_exclude_recent;
    int32_t sc_num_candidates;
    double sc_search_ratio;
    double sc_dist_thres;
    int32_t sc_tree_making_period;
    /* Scancontext.cpp:26 `atan(float)`: 1 = float overload (atanf, default),
       0 = double ::atan */
    int32_t sc_atan_float;
    /* FA frame skip (featureAssociation.cpp:284) */
    int32_t skip_frame_num;
    /* capacity: maximum points per input scan */
    int32_t max_points;
    /* capacity: points of one keyframe's surf / outlier cloud kept for the
       local map (mapOptmization.cpp:1580-1594); 0 = the worst case (R*C /
       R*ceil(C/5), never clipped).  A keyframe cloud larger than a non-zero
       cap is clipped and sets SLO_ERR_MAP_CAPACITY in the stream's error
       bits, so a run that stays exact reports no error.  Host-side only: the
       CPU restatement ignores it. */
    int32_t keyframe_cloud_cap;
    /* loop-closure verification (performLoopClosure, mapOptmization.cpp:
       964-1110, with detectLoopClosure 841-962): after every SC detect that
       reports a loop, the radius-search (RS) and Scan Context (SC) candidate
       submaps are assembled and each is aligned by ICP.  0 = off (the
       reference's loop thread, ICP and GTSAM factors are then not run). */
    int32_t loop_verify;
    /* capacity: points per stream of the keyframe archive (corner + surf DS
       clouds of every keyframe, body frame: cornerCloudKeyFrames /
       surfCloudKeyFrames, MO:1587-1594) the submaps are built from; required
       (> 0) when loop_verify is set */
    int32_t loop_archive_points;
    float history_keyframe_search_radius;   /* 20.0 m (utility.h:137) */
    int32_t history_keyframe_search_num;    /* 25 (utility.h:138): submap = keyframes id-25..id+25 */
    float history_keyframe_fitness_score;   /* 1.5 (utility.h:139) */
    float leaf_history;                     /* 0.3 (downSizeFilterHistoryKeyFrames, MO:268) */
    double loop_time_gap;                   /* 30.0 s (MO:866) */
    int32_t icp_max_iterations;             /* 100 (MO:1008 / 1059) */
    double icp_max_corr_dist;               /* 100 (MO:1007 / 1058) */
    double icp_transformation_epsilon;      /* 1e-6 (MO:1009 / 1060) */
    double icp_fitness_epsilon;             /* 1e-6 (MO:1010 / 1061) */
    /* useCloudRing (utility.h:64, false in the reference): the row of a point
       is its "ring" field instead of its elevation (IP:225-226); rings come
       from slo_batch_set_rings or the PointCloud2's uint16 "ring" field */
    int32_t use_cloud_ring;
    /* loopClosureEnableFlag == false branch of extractSurroundingKeyFrames
       (MO:1167-1222): key poses within surroundingKeyframeSearchRadius of
       the robot (kd-tree radius search), VoxelGrid'ed at 1 m, form the local
       map.  The reference then keeps every keyframe's clouds, so:
         map_keyframes   keyframes the local map may hold (0 = default:
                         surroundingKeyframeSearchNum with loop closure, 128
                         without); more sets SLO_ERR_MAP_CAPACITY
         keyframe_ring   keyframe cloud slots (0 = default:
                         surroundingKeyframeSearchNum + 2 with loop closure,
                         1024 without); a map that needs a keyframe whose
                         slot was reused sets SLO_ERR_MAP_CAPACITY */
    float surrounding_keyframe_search_radius;   /* 50.0 m (utility.h:133) */
    float leaf_surrounding_key_poses;           /* 1.0 (downSizeFilterSurroundingKeyPoses, MO:269) */
    int32_t map_keyframes;
    int32_t keyframe_ring;
    /* pose-graph back end in the batched pipeline (csrc/slo_pgwire.hip): the
       key poses come from an SE(3) factor graph per stream (GTSAM iSAM2's
       role, MO:1541-1611) that takes the loops loop_verify accepts, and a
       closed loop rewrites every key pose (correctPoses, MO:1642-1664).
       0 = off (the keyframe estimate is its initial value, as in the
       reference while no loop is closed) */
    int32_t pose_graph;
    /* the order of the points inside a voxel, which fixes every VoxelGrid
       centroid's float sum (PCL VoxelGrid, FA:779-780, MO:1224-1262):
         SLO_VOXEL_PCL (0, default)  std::sort's order, as the reference's PCL
                                     (slo_vgpcl.hip, slo_pclsort.h);
         SLO_VOXEL_STABLE (1)        input order (a stable radix sort; faster,
                                     centroids differ from PCL's by rounding) */
    int32_t voxel_order;
} slo_config;

enum { SLO_VOXEL_PCL = 0, SLO_VOXEL_STABLE = 1 };

/* preset ids */
enum {
    SLO_PRESET_VLP16 = 0,      /* utility.h:67-72 */
    SLO_PRESET_HDL32 = 1,      /* utility.h:75-80 */
    SLO_PRESET_VLS128 = 2,     /* utility.h:83-88 */
    SLO_PRESET_OS1_16 = 3,     /* utility.h:93-98 */
    SLO_PRESET_OS1_64 = 4,     /* utility.h:101-106 (the shipped one) */
    SLO_PRESET_OS64_1800 = 5,  /* build-defined: OS1-64 vertical, C=1800 (config C2) */
    SLO_PRESET_HDL64_1800 = 6, /* build-defined: KITTI HDL-64E shape (config C3) */
    SLO_PRESET_DENSE128 = 7    /* build-defined: VLS-128 vertical, C=2048 (config C5) */
};

#ifdef __cplusplus
}
#endif

#endif
