"""slo_config_preset against the reference's constants, transcribed by hand.

The reference compiles its parameters as `extern const` globals
(utility.h:66-141; Scancontext.h:77-96; voxel leaves MO:263-268 and FA:225).
The table below restates each literal initialiser as written there and
evaluates it the way C++ does (double expression, narrowed to float where the
global is a float), independently of csrc/slo_config.h.  The three presets
the reference does not ship (C2, C3, C5 shapes) are listed with
the rule that defines them."""
import ctypes

import numpy as np
import pytest

f32 = np.float32
PI = 3.14159265358979323846

# utility.h:66-106 — (N_SCAN, Horizon_SCAN, ang_res_x, ang_res_y, ang_bottom, groundScanInd)
SENSORS = {
    0: (16, 1800, f32(0.2), f32(2.0), f32(15.0 + 0.1), 7),                                   # VLP-16   UT:67-72
    1: (32, 1800, f32(360.0 / float(f32(1800))), f32(41.33 / float(f32(31))), f32(30.67), 20),  # HDL-32E UT:75-80
    2: (128, 1800, f32(0.2), f32(0.3), f32(25.0), 10),                                        # VLS-128  UT:83-88
    3: (16, 1024, f32(360.0 / 1024.0), f32(33.2 / 15.0), f32(16.6 + 0.1), 7),                 # OS1-16   UT:93-98
    4: (64, 1024, f32(360.0 / 1024.0), f32(33.2 / 63.0), f32(16.6 + 0.1), 15),                # OS1-64   UT:101-106
    # build-defined: OS1-64 vertical geometry with C = 1800 (C2)
    5: (64, 1800, f32(360.0 / 1800.0), f32(33.2 / 63.0), f32(16.6 + 0.1), 15),
    # build-defined KITTI HDL-64E shape (C3): 0.2 deg columns, +2 .. -24.9 deg
    # over 64 rows; groundScanInd = 50 is the value of the LeGO-LOAM KITTI
    # parameter set in common use (rows 0..50 = elevations below ~-3.6 deg;
    # see DESIGN.md §1 on why not SURVEY's "< -7 deg" rule, which would give 42)
    6: (64, 1800, f32(360.0 / 1800.0), f32(26.9 / 63.0), f32(24.9 + 0.1), 50),
    # build-defined VLS-128 vertical geometry with C = 2048 (C5)
    7: (128, 2048, f32(360.0 / 2048.0), f32(0.3), f32(25.0), 10),
}

# utility.h:108-141, Scancontext.h:77-96, MO:263-268, FA:225 (sensor independent)
COMMON = {
    "loop_closure_enable": 1,                        # UT:108
    "mapping_process_interval": 0.3,                 # UT:109
    "scan_period": f32(0.1),                         # UT:111
    "sensor_minimum_range": f32(1.0),                # UT:115
    "sensor_mount_angle": f32(0.0),                  # UT:116
    "segment_theta": f32(60.0 / 180.0 * PI),         # UT:117
    "segment_valid_point_num": 5,                    # UT:118
    "segment_valid_line_num": 3,                     # UT:119
    "edge_feature_num": 2,                           # UT:124
    "surf_feature_num": 4,                           # UT:125
    "sections_total": 6,                             # UT:126
    "edge_threshold": f32(0.1),                      # UT:127
    "surf_threshold": f32(0.1),                      # UT:128
    "nearest_feature_search_sq_dist": f32(25),       # UT:129
    "surrounding_keyframe_search_num": 50,           # UT:134
    "surrounding_keyframe_search_radius": f32(50.0), # UT:133
    "leaf_surrounding_key_poses": f32(1.0),          # MO:269
    "history_keyframe_search_radius": f32(20.0),     # UT:137
    "history_keyframe_search_num": 25,               # UT:138
    "history_keyframe_fitness_score": f32(1.5),      # UT:139
    "leaf_less_flat": f32(0.2),                      # FA:225
    "leaf_corner": f32(0.2),                         # MO:263
    "leaf_sc": f32(0.5),                             # MO:264
    "leaf_surf": f32(0.3),                           # MO:265
    "leaf_outlier": f32(0.4),                        # MO:266
    "leaf_history": f32(0.3),                        # MO:268
    "sc_lidar_height": 2.0,                          # SCh:77
    "sc_num_ring": 20,                               # SCh:79
    "sc_num_sector": 60,                             # SCh:80
    "sc_max_radius": 80.0,                           # SCh:81
    "sc_num_exclude_recent": 50,                     # SCh:86
    "sc_num_candidates": 10,                         # SCh:87
    "sc_search_ratio": 0.1,                          # SCh:90
    "sc_dist_thres": 0.5,                            # SCh:92
    "sc_tree_making_period": 10,                     # SCh:95
    "skip_frame_num": 1,                             # FA:284
    "icp_max_iterations": 100,                       # MO:1008
    "icp_max_corr_dist": 100.0,                      # MO:1007
    "icp_transformation_epsilon": 1e-6,              # MO:1009
    "icp_fitness_epsilon": 1e-6,                     # MO:1010
    "loop_time_gap": 30.0,                           # MO:866
}


@pytest.mark.parametrize("pid", sorted(SENSORS))
def test_preset_matches_the_reference_constants(pid):
    from slo_amd import _abi
    lib = _abi.lib()
    c = _abi.SloConfig()
    assert lib.slo_config_preset(pid, ctypes.byref(c)) == 0
    R, C, rx, ry, bot, gsi = SENSORS[pid]
    assert (c.n_scan, c.horizon_scan, c.ground_scan_ind) == (R, C, gsi)
    for name, want in (("ang_res_x", rx), ("ang_res_y", ry), ("ang_bottom", bot)):
        assert np.float32(getattr(c, name)).view(np.uint32) == np.float32(want).view(np.uint32), name
    # segmentAlphaX/Y = ang_res / 180.0 * M_PI, float promoted to double (UT:120-121)
    assert np.float32(c.segment_alpha_x) == f32(float(rx) / 180.0 * PI)
    assert np.float32(c.segment_alpha_y) == f32(float(ry) / 180.0 * PI)
    # their float sin / cos are glibc's sinf / cosf (IP:421): within an ulp of numpy's
    for got, want in ((c.sin_alpha_x, np.sin(np.float64(f32(c.segment_alpha_x)))),
                      (c.cos_alpha_y, np.cos(np.float64(f32(c.segment_alpha_y))))):
        assert abs(float(got) - want) <= float(np.spacing(f32(want)))
    for name, want in COMMON.items():
        got = getattr(c, name)
        if isinstance(want, np.float32):
            assert np.float32(got).view(np.uint32) == want.view(np.uint32), name
        else:
            assert got == want, name
    assert c.max_points == R * C


def test_the_shipped_sensor_is_os1_64():
    # utility.h:101-106 is the one preset not commented out
    from slo_amd import _abi
    c = _abi.SloConfig()
    assert _abi.lib().slo_config_preset(4, ctypes.byref(c)) == 0
    assert (c.n_scan, c.horizon_scan, c.ground_scan_ind) == (64, 1024, 15)
