// slo_config.h — runtime sensor/algorithm configuration.
//
// The reference compiles these as `extern const` globals (utility.h:55-141,
// Scancontext.h:77-96, voxel leaves mapOptmization.cpp:263-272 and
// featureAssociation.cpp:225).  Here they are a plain struct so one library
// serves every sensor; slo_config_preset() fills it with the reference's
// values.  Derived float constants are computed exactly the way the
// reference's initialisers compute them (double expression, then narrowed to
// float), e.g. ang_res_y = 33.2/float(N_SCAN-1) (utility.h:104).
#pragma once

#include <stdint.h>
#include <math.h>
#include "../../include/slo_config.h"

#ifdef __cplusplus
#include "slo_libm.h"

/* Fill cfg with the preset; returns 0 or -1 for an unknown id. */
inline int slo_config_preset_impl(int preset, slo_config* c) {
    const double PI_ = 3.14159265358979323846;  /* M_PI */
    int R, C, gsi;
    float rx, ry, bot;
    switch (preset) {
        case SLO_PRESET_VLP16:
            R = 16; C = 1800; rx = (float)0.2; ry = (float)2.0; bot = (float)(15.0 + 0.1); gsi = 7; break;
        case SLO_PRESET_HDL32:
            R = 32; C = 1800; rx = (float)(360.0 / (float)C); ry = (float)(41.33 / (float)(R - 1));
            bot = (float)30.67; gsi = 20; break;
        case SLO_PRESET_VLS128:
            R = 128; C = 1800; rx = (float)0.2; ry = (float)0.3; bot = (float)25.0; gsi = 10; break;
        case SLO_PRESET_OS1_16:
            R = 16; C = 1024; rx = (float)(360.0 / (float)C); ry = (float)(33.2 / (float)(R - 1));
            bot = (float)(16.6 + 0.1); gsi = 7; break;
        case SLO_PRESET_OS1_64:
            R = 64; C = 1024; rx = (float)(360.0 / (float)C); ry = (float)(33.2 / (float)(R - 1));
            bot = (float)(16.6 + 0.1); gsi = 15; break;
        case SLO_PRESET_OS64_1800:
            R = 64; C = 1800; rx = (float)(360.0 / (float)C); ry = (float)(33.2 / (float)(R - 1));
            bot = (float)(16.6 + 0.1); gsi = 15; break;
        case SLO_PRESET_HDL64_1800:   /* gsi 50: the LeGO-LOAM KITTI parameter set in common use */
            R = 64; C = 1800; rx = (float)(360.0 / (float)C); ry = (float)(26.9 / (float)(R - 1));
            bot = (float)(24.9 + 0.1); gsi = 50; break;
        case SLO_PRESET_DENSE128:
            R = 128; C = 2048; rx = (float)(360.0 / (float)C); ry = (float)0.3; bot = (float)25.0; gsi = 10; break;
        default:
            return -1;
    }
    c->n_scan = R;
    c->horizon_scan = C;
    c->ang_res_x = rx;
    c->ang_res_y = ry;
    c->ang_bottom = bot;
    c->ground_scan_ind = gsi;
    c->sensor_minimum_range = (float)1.0;
    c->sensor_mount_angle = (float)0.0;
    c->segment_theta = (float)(60.0 / 180.0 * PI_);
    c->segment_valid_point_num = 5;
    c->segment_valid_line_num = 3;
    c->segment_alpha_x = (float)(rx / 180.0 * PI_);
    c->segment_alpha_y = (float)(ry / 180.0 * PI_);
    c->sin_alpha_x = slo_libm::sinf_(c->segment_alpha_x);
    c->cos_alpha_x = slo_libm::cosf_(c->segment_alpha_x);
    c->sin_alpha_y = slo_libm::sinf_(c->segment_alpha_y);
    c->cos_alpha_y = slo_libm::cosf_(c->segment_alpha_y);
    c->scan_period = (float)0.1;
    c->edge_feature_num = 2;
    c->surf_feature_num = 4;
    c->sections_total = 6;
    c->edge_threshold = (float)0.1;
    c->surf_threshold = (float)0.1;
    c->nearest_feature_search_sq_dist = (float)25;
    c->loop_closure_enable = 1;
    c->mapping_process_interval = 0.3;
    c->surrounding_keyframe_search_num = 50;
    c->leaf_less_flat = (float)0.2;
    c->leaf_corner = (float)0.2;
    c->leaf_surf = (float)0.3;
    c->leaf_outlier = (float)0.4;
    c->leaf_sc = (float)0.5;
    c->sc_lidar_height = 2.0;
    c->sc_num_ring = 20;
    c->sc_num_sector = 60;
    c->sc_max_radius = 80.0;
    c->sc_num_exclude_recent = 50;
    c->sc_num_candidates = 10;
    c->sc_search_ratio = 0.1;
    c->sc_dist_thres = 0.5;
    c->sc_tree_making_period = 10;
    c->sc_atan_float = 1;
    c->skip_frame_num = 1;
    c->max_points = R * C;
    c->keyframe_cloud_cap = 0;
    c->loop_verify = 0;
    c->loop_archive_points = 0;
    c->history_keyframe_search_radius = (float)20.0;
    c->history_keyframe_search_num = 25;
    c->history_keyframe_fitness_score = (float)1.5;
    c->leaf_history = (float)0.3;
    c->loop_time_gap = 30.0;
    c->icp_max_iterations = 100;
    c->icp_max_corr_dist = 100.0;
    c->icp_transformation_epsilon = 1e-6;
    c->icp_fitness_epsilon = 1e-6;
    c->use_cloud_ring = 0;
    c->surrounding_keyframe_search_radius = (float)50.0;
    c->leaf_surrounding_key_poses = (float)1.0;
    c->map_keyframes = 0;
    c->keyframe_ring = 0;
    c->pose_graph = 0;
    c->voxel_order = 0;   /* SLO_VOXEL_PCL */
    return 0;
}
#endif
