"""ctypes binding of include/slo_abi.h (libslo.so, the gfx950 product library).

This is the same binding a maintainer would add to call the C ABI from any
host language.  There is no CPU fallback: if libslo.so is
missing or no HIP device is present the calls raise.
"""
import ctypes

import numpy as np
import os
import subprocess

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # sc-lego-loam_amd/
LIB_PATH = os.environ.get("SLO_LIB") or os.path.join(_PKG, "libslo.so")   # SLO_LIB: an experiment build
_LIB = None


class SloConfig(ctypes.Structure):
    """Mirror of struct slo_config (csrc/slo_config.h)."""
    _fields_ = [
        ("n_scan", ctypes.c_int32), ("horizon_scan", ctypes.c_int32),
        ("ang_res_x", ctypes.c_float), ("ang_res_y", ctypes.c_float), ("ang_bottom", ctypes.c_float),
        ("ground_scan_ind", ctypes.c_int32),
        ("sensor_minimum_range", ctypes.c_float), ("sensor_mount_angle", ctypes.c_float),
        ("segment_theta", ctypes.c_float), ("segment_valid_point_num", ctypes.c_int32),
        ("segment_valid_line_num", ctypes.c_int32), ("segment_alpha_x", ctypes.c_float),
        ("segment_alpha_y", ctypes.c_float),
        ("sin_alpha_x", ctypes.c_float), ("cos_alpha_x", ctypes.c_float),
        ("sin_alpha_y", ctypes.c_float), ("cos_alpha_y", ctypes.c_float),
        ("scan_period", ctypes.c_float), ("edge_feature_num", ctypes.c_int32),
        ("surf_feature_num", ctypes.c_int32), ("sections_total", ctypes.c_int32),
        ("edge_threshold", ctypes.c_float), ("surf_threshold", ctypes.c_float),
        ("nearest_feature_search_sq_dist", ctypes.c_float),
        ("loop_closure_enable", ctypes.c_int32), ("mapping_process_interval", ctypes.c_double),
        ("surrounding_keyframe_search_num", ctypes.c_int32),
        ("leaf_less_flat", ctypes.c_float), ("leaf_corner", ctypes.c_float), ("leaf_surf", ctypes.c_float),
        ("leaf_outlier", ctypes.c_float), ("leaf_sc", ctypes.c_float),
        ("sc_lidar_height", ctypes.c_double), ("sc_num_ring", ctypes.c_int32), ("sc_num_sector", ctypes.c_int32),
        ("sc_max_radius", ctypes.c_double), ("sc_num_exclude_recent", ctypes.c_int32),
        ("sc_num_candidates", ctypes.c_int32), ("sc_search_ratio", ctypes.c_double),
        ("sc_dist_thres", ctypes.c_double), ("sc_tree_making_period", ctypes.c_int32),
        ("sc_atan_float", ctypes.c_int32), ("skip_frame_num", ctypes.c_int32), ("max_points", ctypes.c_int32),
        ("keyframe_cloud_cap", ctypes.c_int32),
        ("loop_verify", ctypes.c_int32), ("loop_archive_points", ctypes.c_int32),
        ("history_keyframe_search_radius", ctypes.c_float), ("history_keyframe_search_num", ctypes.c_int32),
        ("history_keyframe_fitness_score", ctypes.c_float), ("leaf_history", ctypes.c_float),
        ("loop_time_gap", ctypes.c_double), ("icp_max_iterations", ctypes.c_int32),
        ("icp_max_corr_dist", ctypes.c_double), ("icp_transformation_epsilon", ctypes.c_double),
        ("icp_fitness_epsilon", ctypes.c_double),
        ("use_cloud_ring", ctypes.c_int32),
        ("surrounding_keyframe_search_radius", ctypes.c_float), ("leaf_surrounding_key_poses", ctypes.c_float),
        ("map_keyframes", ctypes.c_int32), ("keyframe_ring", ctypes.c_int32), ("pose_graph", ctypes.c_int32), ("voxel_order", ctypes.c_int32),
    ]


class SegView(ctypes.Structure):
    _fields_ = [("n_segmented", ctypes.c_int32), ("segmented", ctypes.c_void_p), ("ground_flag", ctypes.c_void_p),
                ("col_ind", ctypes.c_void_p), ("range", ctypes.c_void_p), ("start_ring_index", ctypes.c_void_p),
                ("end_ring_index", ctypes.c_void_p), ("start_orientation", ctypes.c_float),
                ("end_orientation", ctypes.c_float), ("orientation_diff", ctypes.c_float),
                ("n_outlier", ctypes.c_int32), ("outlier", ctypes.c_void_p)]


class Pc2Field(ctypes.Structure):
    """slo_pc2_field (include/slo_abi.h) = sensor_msgs/PointField"""
    _fields_ = [("name", ctypes.c_char_p), ("offset", ctypes.c_uint32), ("datatype", ctypes.c_uint8),
                ("count", ctypes.c_uint32)]


class Pc2(ctypes.Structure):
    """slo_pc2 (include/slo_abi.h) = sensor_msgs/PointCloud2 without the header"""
    _fields_ = [("height", ctypes.c_uint32), ("width", ctypes.c_uint32), ("fields", ctypes.POINTER(Pc2Field)),
                ("n_fields", ctypes.c_int32), ("is_bigendian", ctypes.c_uint8), ("point_step", ctypes.c_uint32),
                ("row_step", ctypes.c_uint32), ("data", ctypes.c_void_p), ("data_bytes", ctypes.c_size_t),
                ("is_dense", ctypes.c_uint8)]


class Pc2Layout(ctypes.Structure):
    _fields_ = [("point_step", ctypes.c_uint32), ("off_x", ctypes.c_int32), ("off_y", ctypes.c_int32),
                ("off_z", ctypes.c_int32), ("off_intensity", ctypes.c_int32), ("off_ring", ctypes.c_int32)]


class FaView(ctypes.Structure):
    _fields_ = [("n_sharp", ctypes.c_int32), ("n_less_sharp", ctypes.c_int32), ("n_flat", ctypes.c_int32),
                ("n_less_flat", ctypes.c_int32), ("sharp", ctypes.c_void_p), ("less_sharp", ctypes.c_void_p),
                ("flat", ctypes.c_void_p), ("less_flat", ctypes.c_void_p),
                ("transform_sum", ctypes.c_float * 6), ("published", ctypes.c_int32)]


class MapView(ctypes.Structure):
    _fields_ = [("ran", ctypes.c_int32), ("keyframe_saved", ctypes.c_int32), ("n_keyframes", ctypes.c_int32),
                ("transform_aft_mapped", ctypes.c_float * 6)]


class XscMatch(ctypes.Structure):
    """slo_xsc_match (include/slo_abi.h)"""
    _fields_ = [("valid", ctypes.c_int32), ("n_cand", ctypes.c_int32), ("nn_stream", ctypes.c_int32),
                ("nn_keyframe", ctypes.c_int32), ("loop", ctypes.c_int32), ("yaw", ctypes.c_float),
                ("min_dist", ctypes.c_double)]


# slo_imu_msg (include/slo_abi.h): sensor_msgs/Imu as imuHandler reads it
IMU_DTYPE = np.dtype([("stamp", "<f8"), ("qx", "<f8"), ("qy", "<f8"), ("qz", "<f8"), ("qw", "<f8"),
                      ("ax", "<f8"), ("ay", "<f8"), ("az", "<f8"), ("wx", "<f8"), ("wy", "<f8"), ("wz", "<f8")])

# record layout (include/slo_abi.h SLO_REC_*)
RECORD_FLOATS = 1240
REC = {"pose": 0, "mapped": 6, "n_keyframes": 12, "kf_saved": 13, "loop_id": 14, "min_dist": 15, "ring_key": 16,
       "sc_count": 36, "err": 37, "kf_index": 38, "yaw": 39, "desc": 40}


# symbols declared in include/slo_abi.h (tests check every one is exported)
EXPORTS = [
    "slo_config_preset", "slo_create", "slo_destroy", "slo_last_error", "slo_stream", "slo_synchronize",
    "slo_prepare_mapping",
    "slo_batch_image_projection", "slo_batch_feature_association", "slo_batch_map_optimization",
    "slo_batch_sc_detect", "slo_batch_process", "slo_graph_mode", "slo_batch_imu", "slo_batch_scan_time",
    "slo_imu_handler", "slo_image_projection", "slo_feature_association",
    "slo_map_optimization", "slo_sc_detect", "slo_sc_make_and_save", "slo_batch_sc_make", "slo_batch_voxel_grid", "slo_sc_make_scancontext", "slo_sc_ring_key",
    "slo_sc_sector_key", "slo_sc_fast_align", "slo_sc_dist_direct", "slo_sc_distance", "slo_batch_sc_distance", "slo_pack_records",
    "slo_record_floats", "slo_get", "slo_timing_enable", "slo_timing_read", "slo_timing_reset", "slo_gen_scan",
    "slo_gen_batch", "slo_batch_loop_closure", "slo_loop_closure", "slo_icp_align_batch",
    "slo_timing_filter", "slo_image_projection_ring", "slo_batch_set_rings", "slo_pc2_layout_of", "slo_pc2_to_xyzi", "slo_image_projection_pc2", "slo_batch_pc2_unpack",
    # cross-stream Scan Context store over the gathered records (csrc/slo_xsc.hip)
    "slo_xsc_create", "slo_xsc_destroy", "slo_xsc_ingest", "slo_xsc_query",
    # synthetic stream generator on the device (csrc/slo_gendev.hip)
    "slo_gen_device_create", "slo_gen_device_scans", "slo_gen_device_destroy",
    # Mode S: one stream's front ends and back end on different contexts
    "slo_modes_carry_bytes", "slo_modes_features_bytes", "slo_front_process", "slo_back_process",
    "slo_modes_odom_bytes", "slo_odom_process", "slo_map_process", "slo_pipeline",
    # pose-graph back end (csrc/slo_pg.hip, host side)
    "slo_pg_create", "slo_pg_destroy", "slo_pg_last_error", "slo_pg_size", "slo_pg_add_keyframe", "slo_pg_add_loop", "slo_pg_optimize", "slo_pg_get_key_poses", "slo_pg_last_transform", "slo_set_key_poses",
]


def build():
    subprocess.run(["make", "-s", "-C", _PKG], check=True)


def lib():
    """Load libslo.so (raises if it is not built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libslo.so not built (run __graft_entry__.build() or make -C sc-lego-loam_amd)")
    # One HIP runtime per process: PyTorch bundles its own libamdhip64.so.7
    # (same soname as /opt/rocm's).  Whichever is loaded first serves both, and
    # torch cannot initialise on the system one, so load torch's first when
    # torch is in use (bench, tests); libslo then binds to it.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    L.slo_config_preset.argtypes = [ctypes.c_int, ctypes.POINTER(SloConfig)]
    L.slo_create.argtypes = [ctypes.POINTER(SloConfig), ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
    L.slo_destroy.argtypes = [P]
    L.slo_last_error.argtypes = [P]
    L.slo_last_error.restype = ctypes.c_char_p
    L.slo_stream.argtypes = [P]
    L.slo_stream.restype = P
    L.slo_synchronize.argtypes = [P]
    L.slo_prepare_mapping.argtypes = [P]
    L.slo_pipeline.argtypes = [P, ctypes.c_int]
    L.slo_batch_image_projection.argtypes = [P, P, P]
    L.slo_batch_feature_association.argtypes = [P]
    L.slo_batch_map_optimization.argtypes = [P, P, P, ctypes.c_double]
    L.slo_batch_sc_detect.argtypes = [P]
    L.slo_batch_process.argtypes = [P, P, P, ctypes.c_double]
    L.slo_graph_mode.argtypes = [P, ctypes.c_int]
    L.slo_batch_imu.argtypes = [P, P, ctypes.c_int, P]
    L.slo_batch_scan_time.argtypes = [P, ctypes.c_double]
    L.slo_imu_handler.argtypes = [P, P]
    L.slo_image_projection.argtypes = [P, P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                       ctypes.POINTER(SegView)]
    L.slo_feature_association.argtypes = [P, ctypes.c_double, ctypes.POINTER(FaView)]
    L.slo_map_optimization.argtypes = [P, P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                       ctypes.c_double, ctypes.POINTER(MapView)]
    L.slo_sc_detect.argtypes = [P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float),
                                ctypes.POINTER(ctypes.c_double)]
    L.slo_get.argtypes = [P, ctypes.c_int, ctypes.c_char_p, P, ctypes.c_size_t]
    L.slo_timing_enable.argtypes = [P, ctypes.c_int]
    L.slo_timing_reset.argtypes = [P]
    L.slo_timing_filter.argtypes = [P, ctypes.c_char_p]
    L.slo_image_projection_ring.argtypes = [P, P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                            P, ctypes.POINTER(SegView)]
    L.slo_batch_set_rings.argtypes = [P, P]
    L.slo_timing_read.argtypes = [P, P, ctypes.c_size_t, P, P, ctypes.c_int]
    L.slo_gen_scan.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
    L.slo_gen_batch.argtypes = [ctypes.c_int] * 6 + [P, ctypes.c_int]
    L.slo_set_key_poses.argtypes = [P, ctypes.c_int, P, ctypes.c_int, P]
    L.slo_xsc_create.argtypes = [ctypes.POINTER(SloConfig), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
    L.slo_xsc_destroy.argtypes = [P]
    L.slo_xsc_ingest.argtypes = [P, P, ctypes.c_int, P]
    L.slo_xsc_query.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P, P]
    L.slo_gen_device_create.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(P)]
    L.slo_gen_device_scans.argtypes = [P, ctypes.c_int, ctypes.c_int, P, P]
    L.slo_gen_device_destroy.argtypes = [P]
    L.slo_batch_loop_closure.argtypes = [P]
    L.slo_loop_closure.argtypes = [P, P]
    L.slo_icp_align_batch.argtypes = [P, P, ctypes.c_size_t, P, P, ctypes.c_size_t, P, P]
    L.slo_sc_make_and_save.argtypes = [P, P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
    L.slo_batch_sc_make.argtypes = [P, P, P]
    L.slo_sc_make_scancontext.argtypes = [P, P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, P]
    L.slo_sc_ring_key.argtypes = [P, P, P]
    L.slo_sc_sector_key.argtypes = [P, P, P]
    L.slo_sc_fast_align.argtypes = [P, P, P, P]
    L.slo_sc_dist_direct.argtypes = [P, P, P, P]
    L.slo_sc_distance.argtypes = [P, P, P, P, P]
    L.slo_batch_sc_distance.argtypes = [P, P, P, ctypes.c_int, P, P]
    L.slo_batch_voxel_grid.argtypes = [P, P, ctypes.c_size_t, P, ctypes.c_float, P, ctypes.c_size_t, P, ctypes.c_int]
    L.slo_pack_records.argtypes = [P, P]
    L.slo_pc2_layout_of.argtypes = [ctypes.POINTER(Pc2), ctypes.POINTER(Pc2Layout)]
    L.slo_pc2_to_xyzi.argtypes = [ctypes.POINTER(Pc2), P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    L.slo_image_projection_pc2.argtypes = [P, ctypes.POINTER(Pc2), ctypes.POINTER(SegView)]
    L.slo_batch_pc2_unpack.argtypes = [P, P, ctypes.c_size_t, P, ctypes.POINTER(Pc2Layout), P, P, P]
    L.slo_record_floats.argtypes = []
    L.slo_modes_carry_bytes.argtypes = [P]
    L.slo_modes_carry_bytes.restype = ctypes.c_size_t
    L.slo_modes_features_bytes.argtypes = [P]
    L.slo_modes_features_bytes.restype = ctypes.c_size_t
    L.slo_front_process.argtypes = [P, P, P, ctypes.c_double, P, P, P]
    L.slo_back_process.argtypes = [P, P, P, P, ctypes.c_double]
    L.slo_modes_odom_bytes.argtypes = [P]
    L.slo_modes_odom_bytes.restype = ctypes.c_size_t
    L.slo_odom_process.argtypes = [P, P, P, P, ctypes.c_double, P]
    L.slo_map_process.argtypes = [P, P, P, P, ctypes.c_double]
    _LIB = L
    return L
