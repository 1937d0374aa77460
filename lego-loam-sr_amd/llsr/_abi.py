"""ctypes mirror of include/llsr.h (the C-ABI boundary). Plain data types only."""
from __future__ import annotations

import ctypes as C

import numpy as np

ABI_VERSION = 2  # LLSR_ABI_VERSION of include/llsr.h these bindings mirror (checked at load)
LLSR_OK = 0
LLSR_LIDAR_VLP16 = 0
LLSR_LIDAR_HDL64E = 2
LLSR_MODE_FAITHFUL = 0
LLSR_MODE_LM_APPLIED = 1
LLSR_VOXEL_ORDER_INPUT = 0
LLSR_VOXEL_ORDER_PCL = 1
NE_WORDS = 32  # LLSR_NE_WORDS: int64 words per problem exchanged by llsr_scan2map_shard_*


class Config(C.Structure):
    _fields_ = [
        ("num_vertical_scans", C.c_int32),
        ("num_horizontal_scans", C.c_int32),
        ("vertical_angle_bottom", C.c_float),
        ("vertical_angle_top", C.c_float),
        ("sensor_mount_angle", C.c_float),
        ("ground_scan_index", C.c_int32),
        ("use_kitti", C.c_int32),
        ("use_vlp32c", C.c_int32),
        ("segment_theta", C.c_float),
        ("segment_valid_point_num", C.c_int32),
        ("segment_valid_line_num", C.c_int32),
        ("scan_period", C.c_float),
        ("edge_threshold", C.c_float),
        ("surf_threshold", C.c_float),
        ("nearest_feature_search_distance", C.c_float),
        ("DBFr", C.c_float),
        ("RatioXY", C.c_float),
        ("RatioZ", C.c_float),
        ("mapping_frequency_divider", C.c_int32),
        ("iterCountThres", C.c_int32),
        ("step_size", C.c_float),
        ("stop_thres", C.c_float),
        ("mode", C.c_int32),
    ]


def config_for(lidar: str, horizontal: int | None = None) -> Config:
    """The loam_config.yaml block (VLP-16: lines 1-67, HDL-64E: 137-203) as a Config.

    Pure-Python copy of llsr_config_default so the oracle can be configured without the
    product library; tests check both agree.
    """
    c = Config()
    if lidar == "vlp16":
        c.num_vertical_scans, c.num_horizontal_scans = 16, 1800
        c.vertical_angle_bottom, c.vertical_angle_top = -15.0, 15.0
        c.ground_scan_index, c.use_kitti = 7, 0
        c.DBFr, c.RatioXY, c.RatioZ = 5.0, 0.5, 2.5
        c.edge_threshold, c.surf_threshold, c.nearest_feature_search_distance = 0.03, 0.03, 5.0
    elif lidar == "hdl64e":
        c.num_vertical_scans, c.num_horizontal_scans = 64, 1800
        c.vertical_angle_bottom, c.vertical_angle_top = -24.8, 2.0
        c.ground_scan_index, c.use_kitti = 50, 1
        c.DBFr, c.RatioXY, c.RatioZ = 7.5, 0.3, 5.0
        c.edge_threshold, c.surf_threshold, c.nearest_feature_search_distance = 0.005, 0.005, 25.0
    else:
        raise ValueError(lidar)
    if horizontal is not None:
        c.num_horizontal_scans = horizontal
    c.sensor_mount_angle = 0.0
    c.use_vlp32c = 0
    c.segment_theta, c.segment_valid_point_num, c.segment_valid_line_num = 60.0, 5, 3
    c.scan_period = 0.1
    c.mapping_frequency_divider = 1
    c.iterCountThres, c.step_size, c.stop_thres = 200, 1.0, 0.05
    c.mode = LLSR_MODE_FAITHFUL
    return c


_P = C.c_void_p


class VisOut(C.Structure):
    """llsr_vis_out (include/llsr.h): publishClouds' visualization clouds of one slot."""
    _fields_ = [("full_cloud", _P), ("full_info_cloud", _P), ("ground_cloud", _P), ("nonground_cloud", _P),
                ("unknownground_cloud", _P), ("segmented_cloud_pure", _P), ("n_ground", C.c_int32),
                ("n_nonground", C.c_int32), ("n_unknownground", C.c_int32), ("n_segmented_pure", C.c_int32)]


VIS_CLOUDS = [("full_cloud", None), ("full_info_cloud", None), ("ground_cloud", "n_ground"),
              ("nonground_cloud", "n_nonground"), ("unknownground_cloud", "n_unknownground"),
              ("segmented_cloud_pure", "n_segmented_pure")]


class ScanOut(C.Structure):
    _fields_ = [
        ("n_points", C.c_int32),
        ("orientation", C.c_float * 3),
        ("range_image", _P),
        ("cell_point", _P),
        ("ground_image", _P),
        ("label_image", _P),
        ("start_ring_index", _P),
        ("end_ring_index", _P),
        ("n_segmented", C.c_int32),
        ("seg_xyzi", _P),
        ("seg_ground_flag", _P),
        ("seg_col_ind", _P),
        ("seg_range", _P),
        ("seg_intensity", _P),
        ("n_outlier", C.c_int32),
        ("outlier_xyzi", _P),
        ("outlier_intensity", _P),
        ("n_near", C.c_int32),
        ("n_ransac_inliers", C.c_int32),
        ("ransac_iterations", C.c_int32),
        ("loam_xyzi", _P),
        ("curvature", _P),
        ("picked", _P),
        ("label", _P),
        ("n_less_sharp", C.c_int32),
        ("less_sharp_ind", _P),
        ("dbscan_cluster", _P),
        ("n_sharp", C.c_int32),
        ("sharp_ind", _P),
        ("n_flat", C.c_int32),
        ("flat_ind", _P),
        ("n_less_flat", C.c_int32),
        ("less_flat_xyzi", _P),
    ]


class LmReport(C.Structure):
    """llsr_lm_report (include/llsr.h): result of one scan-to-map optimisation."""
    _fields_ = [
        ("iterations", C.c_int32),
        ("converged", C.c_int32),
        ("degenerate", C.c_int32),
        ("min_lambda", C.c_float),
        ("cf_mean", C.c_float),
        ("n_corner_corr", C.c_int32),
        ("n_surf_corr", C.c_int32),
        ("matX0", C.c_float * 6),
        ("pose", C.c_float * 6),
        ("ms", C.c_float),
    ]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["matX0"] = np.array(self.matX0[:], dtype=np.float32)
        d["pose"] = np.array(self.pose[:], dtype=np.float32)
        return d


class S2SReport(C.Structure):
    """llsr_s2s_report (include/llsr.h): result of one scan-to-scan updateTransformation."""
    _fields_ = [
        ("surf_iterations", C.c_int32),
        ("corner_iterations", C.c_int32),
        ("n_surf_corr", C.c_int32),
        ("n_corner_corr", C.c_int32),
        ("degenerate", C.c_int32),
        ("skipped", C.c_int32),
        ("transform_cur", C.c_float * 6),
        ("ms", C.c_float),
    ]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["transform_cur"] = np.array(self.transform_cur[:], dtype=np.float32)
        return d


class OdomSlot(C.Structure):
    """llsr_odom_slot (include/llsr.h): one sequence's odometry state after the last scan."""
    _fields_ = [
        ("frames", C.c_int32),
        ("n_corner_last", C.c_int32),
        ("n_surf_last", C.c_int32),
        ("n_corner_scan", C.c_int32),
        ("n_surf_scan", C.c_int32),
        ("transform_cur", C.c_float * 6),
        ("transform_sum", C.c_float * 6),
        ("lm", S2SReport),
    ]


class S2SBatch(C.Structure):
    """llsr_s2s_batch (include/llsr.h): device pointers of one scan-to-scan batch."""
    _fields_ = [
        ("n_problems", C.c_int32),
        ("sharp", C.c_void_p), ("sharp_off", C.c_void_p),
        ("flat", C.c_void_p), ("flat_off", C.c_void_p),
        ("corner_last", C.c_void_p), ("corner_last_off", C.c_void_p),
        ("surf_last", C.c_void_p), ("surf_last_off", C.c_void_p),
        ("transform_cur", C.c_void_p),
        ("is_degenerate", C.c_void_p),
        ("report", C.c_void_p),
    ]


class S2MBatch(C.Structure):
    """llsr_s2m_batch (include/llsr.h): device pointers of one scan-to-map batch."""
    _fields_ = [
        ("n_problems", C.c_int32),
        ("corner_q", C.c_void_p), ("corner_q_off", C.c_void_p),
        ("surf_q", C.c_void_p), ("surf_q_off", C.c_void_p),
        ("corner_map", C.c_void_p), ("corner_map_off", C.c_void_p),
        ("surf_map", C.c_void_p), ("surf_map_off", C.c_void_p),
        ("pose", C.c_void_p),
        ("report", C.c_void_p),
    ]


class S2MStats(C.Structure):
    _fields_ = [("batches", C.c_int32), ("iteration_launches", C.c_int32), ("grid_ms", C.c_float),
                ("iterate_ms", C.c_float)]


class S2SStats(C.Structure):
    _fields_ = [("batches", C.c_int32), ("reserved", C.c_int32), ("grid_ms", C.c_float), ("lm_ms", C.c_float)]


class OdometryMsg(C.Structure):
    """llsr_odometry_msg: the nav_msgs/Odometry fields the nodes use."""
    _fields_ = [("orientation", C.c_double * 4), ("position", C.c_double * 3),
                ("twist_angular", C.c_double * 3), ("twist_linear", C.c_double * 3)]


class FusionState(C.Structure):
    """llsr_fusion_state: TransformFusion's members (transformFusion.h)."""
    _fields_ = [("transform_sum", C.c_float * 6), ("transform_incre", C.c_float * 6),
                ("transform_mapped", C.c_float * 6), ("transform_bef_mapped", C.c_float * 6),
                ("transform_aft_mapped", C.c_float * 6)]


class MapConfig(C.Structure):
    """llsr_map_config (include/llsr.h): MapOptimization's local-map parameters."""
    _fields_ = [("surrounding_radius", C.c_float), ("keypose_leaf", C.c_float), ("corner_leaf", C.c_float),
                ("surf_leaf", C.c_float), ("outlier_leaf", C.c_float), ("enable_loop_closure", C.c_int32),
                ("surrounding_keyframe_search_num", C.c_int32)]


class MapReport(C.Structure):
    """llsr_map_report (include/llsr.h): one extractSurroundingKeyFrames call."""
    _fields_ = [("n_in_radius", C.c_int32), ("n_poses_ds", C.c_int32), ("n_keyframes", C.c_int32),
                ("n_transformed", C.c_int32), ("n_corner_map", C.c_int64), ("n_surf_map", C.c_int64),
                ("n_corner_ds", C.c_int64), ("n_surf_ds", C.c_int64), ("ms", C.c_float)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class MappingSlot(C.Structure):
    """llsr_mapping_slot (include/llsr.h): one sequence's MapOptimization state after the last call."""
    _fields_ = [("frames", C.c_int32), ("mo_frames", C.c_int32), ("keyframes", C.c_int32), ("lm_ran", C.c_int32),
                ("transform_sum", C.c_float * 6), ("transform_tobe_mapped", C.c_float * 6),
                ("transform_bef_mapped", C.c_float * 6), ("transform_aft_mapped", C.c_float * 6),
                ("n_corner_q", C.c_int32), ("n_surf_q", C.c_int32), ("lm", LmReport), ("map", MapReport)]


PC2_FLOAT32 = 7
PC2_MAX_FIELDS = 16
KITTI_MAX_FLOATS = 1000000


class Pc2Field(C.Structure):
    """llsr_pc2_field: sensor_msgs/PointField."""
    _fields_ = [("name", C.c_char * 16), ("offset", C.c_int32), ("datatype", C.c_int32), ("count", C.c_int32)]


class Pc2Layout(C.Structure):
    """llsr_pc2_layout: the PointCloud2 fields + point_step."""
    _fields_ = [("point_step", C.c_int32), ("num_fields", C.c_int32), ("fields", Pc2Field * PC2_MAX_FIELDS)]


class Pc2Msg(C.Structure):
    """llsr_pc2_msg: one message of a decode batch."""
    _fields_ = [("data_offset", C.c_int64), ("width", C.c_int32), ("height", C.c_int32),
                ("row_step", C.c_int32), ("pad", C.c_int32)]


class Sizes(C.Structure):
    _fields_ = [("cells", C.c_int32), ("rings", C.c_int32), ("max_points", C.c_int32),
                ("shadow_points", C.c_int32)]


# (field, dtype, elements per cell/point) for the array outputs; "HW" arrays sized H*W, "H"
# arrays sized H, the rest sized to the H*W bound and trimmed by their count field.
ARRAYS = [
    ("range_image", np.float32, "HW", 1, None),
    ("cell_point", np.int32, "HW", 1, None),
    ("ground_image", np.int8, "HW", 1, None),
    ("label_image", np.int32, "HW", 1, None),
    ("start_ring_index", np.int32, "H", 1, None),
    ("end_ring_index", np.int32, "H", 1, None),
    ("seg_xyzi", np.float32, "HW", 4, "n_segmented"),
    ("seg_ground_flag", np.uint8, "HW", 1, "n_segmented"),
    ("seg_col_ind", np.uint32, "HW", 1, "n_segmented"),
    ("seg_range", np.float32, "HW", 1, "n_segmented"),
    ("seg_intensity", np.float32, "HW", 1, "n_segmented"),
    ("outlier_xyzi", np.float32, "HW", 4, "n_outlier"),
    ("outlier_intensity", np.float32, "HW", 1, "n_outlier"),
    ("loam_xyzi", np.float32, "HW", 4, "n_segmented"),
    ("curvature", np.float32, "HW", 1, "n_segmented"),
    ("picked", np.uint8, "HW", 1, "n_segmented"),
    ("label", np.int8, "HW", 1, "n_segmented"),
    ("less_sharp_ind", np.int32, "HW", 1, "n_less_sharp"),
    ("dbscan_cluster", np.int32, "HW", 1, "n_less_sharp"),
    ("sharp_ind", np.int32, "HW", 1, "n_sharp"),
    ("flat_ind", np.int32, "HW", 1, "n_flat"),
    ("less_flat_xyzi", np.float32, "HW", 4, "n_less_flat"),
]

COUNTS = ["n_points", "n_segmented", "n_outlier", "n_near", "n_ransac_inliers",
          "ransac_iterations", "n_less_sharp", "n_sharp", "n_flat", "n_less_flat"]


class OutBuffers:
    """Host numpy buffers bound to a ScanOut; `result()` returns trimmed copies."""

    def __init__(self, H: int, W: int):
        self.H, self.W = H, W
        self.struct = ScanOut()
        self.bufs = {}
        for name, dt, kind, per, _ in ARRAYS:
            n = (H * W if kind == "HW" else H) * per
            a = np.zeros(n, dtype=dt)
            self.bufs[name] = a
            setattr(self.struct, name, a.ctypes.data)

    def result(self) -> dict:
        s = self.struct
        r = {k: int(getattr(s, k)) for k in COUNTS}
        r["orientation"] = np.array(s.orientation[:], dtype=np.float32)
        for name, dt, kind, per, cnt in ARRAYS:
            a = self.bufs[name]
            if cnt is not None:
                a = a[: r[cnt] * per]
            if per == 4:
                a = a.reshape(-1, 4)
            r[name] = a.copy()
        return r
