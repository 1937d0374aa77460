"""Python host binding of the MI355X LeGO-LOAM-SR hot path (ctypes over include/llsr.h).

Mirrors the reference's node-level interface for this path:

* `ImageProjection.cloud_handler(points)` ~ ImageProjection::cloudHandler (imageProjection.cpp:189)
  -> a ProjectionOut-like dict (segmented / outlier clouds + CloudInfo fields).
* `FeatureAssociation.extract(...)` ~ the feature stage of runFeatureAssociation
  (featureAssociation.cpp:2766-2775).
* `MapOptimization.scan2map_optimization(...)` ~ MapOptimization::scan2MapOptimization
  (mapOptmization.cpp:1572-1610): kNN-5 correspondences + the 6x6 LM against a local map.
* `Pipeline.process_scan` runs both for one scan; `Pipeline.process_batch` runs B scans that are
  already resident in HBM (device pointers, e.g. from torch tensors).

There is no CPU fallback: if libllsr.so (the HIP build) is missing or no HIP device is present,
construction raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi
from ._abi import Config, config_for  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("LLSR_LIB") or os.path.join(_PKG, "libllsr.so")  # override: A/B builds
_LIB = None

EXPORTS = [
    "llsr_abi_version", "llsr_build_id", "llsr_config_default", "llsr_get_config", "llsr_create", "llsr_destroy", "llsr_last_error", "llsr_query_sizes",
    "llsr_reset_state", "llsr_process_scan", "llsr_process_batch", "llsr_fetch_scan", "llsr_fetch_vis_clouds",
    "llsr_batch_counts", "llsr_kernel_times_ms", "llsr_kernel_name", "llsr_set_profiling",
    "llsr_scan2map_reserve", "llsr_scan2map_batch", "llsr_scan2map", "llsr_scan2map_stats",
    "llsr_shadow_points", "llsr_scan2scan_reserve", "llsr_scan2scan_batch", "llsr_scan2scan_check",
    "llsr_scan2scan", "llsr_scan2map_shard_begin", "llsr_scan2map_shard_partial",
    "llsr_scan2map_shard_step", "llsr_scan2map_shard_end", "llsr_odometry_batch", "llsr_odometry_fetch",
    "llsr_odometry_reset", "llsr_map_config_default", "llsr_map_config_lidar", "llsr_map_create", "llsr_map_destroy",
    "llsr_map_last_error", "llsr_map_reset", "llsr_map_voxel_grid", "llsr_map_downsample_scan",
    "llsr_map_add_keyframe", "llsr_map_num_keyframes", "llsr_map_extract", "llsr_map_keyframe_ids",
    "llsr_decode_pointcloud2", "llsr_kitti_count", "llsr_kitti_read", "llsr_kitti_load",
    "llsr_mapping_init", "llsr_mapping_batch", "llsr_mapping_fetch", "llsr_mapping_keyposes", "llsr_mapping_reset",
    "llsr_mapping_associate", "llsr_set_voxel_order", "llsr_scan2scan_stats", "llsr_fusion_init",
    "llsr_pose_to_odometry", "llsr_odometry_to_transform", "llsr_fusion_laser_odometry", "llsr_fusion_aft_mapped",
    "llsr_integrate_transformation", "llsr_transform_to_end",
]


class LlsrError(RuntimeError):
    pass


def build_id() -> str:
    """The loaded library's llsr_build_id() (hash of the kernel sources it was built from)."""
    return lib().llsr_build_id().decode()


def lib():
    """Load libllsr.so (raises if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise LlsrError(f"{LIB_PATH} missing: build it with `make -C lego-loam-sr_amd` "
                            "(there is no CPU fallback for the HIP path)")
        L = C.CDLL(LIB_PATH)
        L.llsr_abi_version.restype = C.c_int32
        L.llsr_abi_version.argtypes = []
        if L.llsr_abi_version() != _abi.ABI_VERSION:
            raise LlsrError(f"{LIB_PATH} has ABI version {L.llsr_abi_version()}, the bindings expect "
                            f"{_abi.ABI_VERSION}: rebuild with `make -C lego-loam-sr_amd`")
        L.llsr_build_id.restype = C.c_char_p
        L.llsr_build_id.argtypes = []
        L.llsr_config_default.argtypes = [C.POINTER(Config), C.c_int32]
        L.llsr_create.argtypes = [C.POINTER(Config), C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
        L.llsr_destroy.argtypes = [C.c_void_p]
        L.llsr_last_error.restype = C.c_char_p
        L.llsr_last_error.argtypes = [C.c_void_p]
        L.llsr_query_sizes.argtypes = [C.c_void_p, C.POINTER(_abi.Sizes)]
        L.llsr_reset_state.argtypes = [C.c_void_p]
        L.llsr_process_scan.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(_abi.ScanOut)]
        L.llsr_process_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        L.llsr_fetch_scan.argtypes = [C.c_void_p, C.c_int32, C.POINTER(_abi.ScanOut)]
        L.llsr_fetch_vis_clouds.argtypes = [C.c_void_p, C.c_int32, C.POINTER(_abi.VisOut)]
        L.llsr_batch_counts.argtypes = [C.c_void_p, C.c_void_p]
        L.llsr_kernel_times_ms.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.llsr_kernel_name.restype = C.c_char_p
        L.llsr_kernel_name.argtypes = [C.c_int32]
        L.llsr_set_profiling.argtypes = [C.c_void_p, C.c_int32]
        L.llsr_scan2map_reserve.argtypes = [C.c_void_p] + [C.c_int32] * 5
        L.llsr_scan2map_batch.argtypes = [C.c_void_p, C.POINTER(_abi.S2MBatch), C.c_void_p]
        L.llsr_scan2map_stats.argtypes = [C.c_void_p, C.POINTER(_abi.S2MStats)]
        L.llsr_scan2scan_stats.argtypes = [C.c_void_p, C.POINTER(_abi.S2SStats)]
        L.llsr_fusion_init.argtypes = [C.POINTER(_abi.FusionState)]
        L.llsr_pose_to_odometry.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(_abi.OdometryMsg)]
        L.llsr_odometry_to_transform.argtypes = [C.POINTER(_abi.OdometryMsg), C.c_void_p]
        L.llsr_fusion_laser_odometry.argtypes = [C.POINTER(_abi.FusionState), C.POINTER(_abi.OdometryMsg),
                                                 C.POINTER(_abi.OdometryMsg)]
        L.llsr_fusion_aft_mapped.argtypes = [C.POINTER(_abi.FusionState), C.POINTER(_abi.OdometryMsg)]
        L.llsr_shadow_points.argtypes = [C.c_void_p]
        L.llsr_integrate_transformation.argtypes = [C.c_void_p, C.c_void_p]
        L.llsr_transform_to_end.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        L.llsr_scan2scan_reserve.argtypes = [C.c_void_p] + [C.c_int32] * 5
        L.llsr_scan2scan_batch.argtypes = [C.c_void_p, C.POINTER(_abi.S2SBatch), C.c_void_p]
        L.llsr_scan2scan_check.argtypes = [C.c_void_p]
        L.llsr_scan2scan.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p,
                                     C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                     C.POINTER(_abi.S2SReport)]
        L.llsr_scan2map.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p,
                                    C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(_abi.LmReport)]
        L.llsr_scan2map_shard_begin.argtypes = [C.c_void_p, C.POINTER(_abi.S2MBatch), C.c_void_p]
        L.llsr_scan2map_shard_partial.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.llsr_scan2map_shard_step.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.c_void_p]
        L.llsr_scan2map_shard_end.argtypes = [C.c_void_p, C.c_void_p]
        L.llsr_odometry_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        L.llsr_odometry_fetch.argtypes = [C.c_void_p, C.c_int32, C.POINTER(_abi.OdomSlot)] + [C.c_void_p] * 4
        L.llsr_odometry_reset.argtypes = [C.c_void_p]
        L.llsr_map_config_default.argtypes = [C.POINTER(_abi.MapConfig)]
        L.llsr_map_config_lidar.argtypes = [C.POINTER(_abi.MapConfig), C.c_int32]
        L.llsr_map_create.argtypes = [C.POINTER(_abi.MapConfig), C.c_int32]
        L.llsr_map_destroy.argtypes = [C.c_void_p]
        L.llsr_map_last_error.argtypes = [C.c_void_p]
        L.llsr_map_reset.argtypes = [C.c_void_p]
        L.llsr_map_voxel_grid.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_void_p]
        L.llsr_map_downsample_scan.argtypes = [C.c_void_p] + [C.c_void_p, C.c_int32] * 5 + [C.c_void_p] * 3
        L.llsr_map_add_keyframe.argtypes = [C.c_void_p, C.c_void_p] + [C.c_void_p, C.c_int32] * 3 + [C.c_void_p]
        L.llsr_map_num_keyframes.argtypes = [C.c_void_p]
        L.llsr_map_extract.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                                       C.POINTER(_abi.MapReport), C.c_void_p]
        L.llsr_map_keyframe_ids.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.llsr_mapping_init.argtypes = [C.c_void_p, C.c_int32, C.POINTER(_abi.MapConfig)]
        L.llsr_mapping_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        L.llsr_mapping_fetch.argtypes = [C.c_void_p, C.c_int32, C.POINTER(_abi.MappingSlot)]
        L.llsr_mapping_keyposes.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32]
        L.llsr_mapping_reset.argtypes = [C.c_void_p]
        L.llsr_mapping_associate.argtypes = [C.c_void_p] * 6
        L.llsr_set_voxel_order.argtypes = [C.c_void_p, C.c_int32]
        L.llsr_decode_pointcloud2.argtypes = [C.POINTER(_abi.Pc2Layout), C.c_void_p, C.c_void_p, C.c_int32,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.llsr_kitti_count.argtypes = [C.c_char_p]
        L.llsr_kitti_read.argtypes = [C.c_char_p, C.c_void_p, C.c_int32, C.POINTER(C.c_int32)]
        L.llsr_kitti_load.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p,
                                      C.c_void_p, C.c_void_p]
        for fn in EXPORTS:
            if fn not in ("llsr_last_error", "llsr_kernel_name", "llsr_destroy", "llsr_map_create",
                          "llsr_map_destroy", "llsr_map_last_error", "llsr_build_id"):
                getattr(L, fn).restype = C.c_int32
        L.llsr_destroy.restype = None
        L.llsr_map_create.restype = C.c_void_p
        L.llsr_map_destroy.restype = None
        L.llsr_map_last_error.restype = C.c_char_p
        _LIB = L
    return _LIB


def default_config(lidar: str, horizontal: int | None = None) -> Config:
    c = Config()
    code = {"vlp16": _abi.LLSR_LIDAR_VLP16, "hdl64e": _abi.LLSR_LIDAR_HDL64E}[lidar]
    rc = lib().llsr_config_default(C.byref(c), code)
    if rc != 0:
        raise LlsrError(f"llsr_config_default: {rc}")
    if horizontal is not None:
        c.num_horizontal_scans = horizontal
    return c


class Pipeline:
    """One llsr handle: ImageProjection + FeatureAssociation feature stage on a HIP device."""

    def __init__(self, cfg: Config, device: int = 0, max_batch: int = 1, max_points: int | None = None):
        self.cfg = cfg
        H, W = cfg.num_vertical_scans, cfg.num_horizontal_scans
        self.max_points = max_points or 2 * H * W
        self.max_batch = max_batch
        h = C.c_void_p()
        rc = lib().llsr_create(C.byref(cfg), device, max_batch, self.max_points, C.byref(h))
        if rc != 0:
            raise LlsrError(f"llsr_create failed ({rc}): no HIP device or invalid config")
        self._h = h
        self.out = _abi.OutBuffers(H, W)

    def close(self):
        if getattr(self, "_h", None):
            lib().llsr_destroy(self._h)
            self._h = None

    __del__ = close

    def _check(self, rc, what):
        if rc != 0:
            raise LlsrError(f"{what} failed ({rc}): {lib().llsr_last_error(self._h).decode()}")

    def reset(self):
        self._check(lib().llsr_reset_state(self._h), "llsr_reset_state")

    def set_voxel_order(self, order: int):
        """_abi.LLSR_VOXEL_ORDER_PCL (default: the reference's std::sort order) or LLSR_VOXEL_ORDER_INPUT
        (ring order inside each voxel) for the less-flat VoxelGrid."""
        self._check(lib().llsr_set_voxel_order(self._h, order), "llsr_set_voxel_order")

    def process_scan(self, xyzi: np.ndarray) -> dict:
        xyzi = np.ascontiguousarray(xyzi, dtype=np.float32).reshape(-1, 4)
        self._check(lib().llsr_process_scan(self._h, xyzi.ctypes.data, xyzi.shape[0], C.byref(self.out.struct)),
                    "llsr_process_scan")
        return self.out.result()

    def process_batch(self, d_xyzi: int, d_offsets: int, B: int, stream: int = 0):
        """Enqueue B device-resident scans (raw device pointers) on a hipStream_t (0 = own)."""
        self._check(lib().llsr_process_batch(self._h, C.c_void_p(d_xyzi), C.c_void_p(d_offsets), B,
                                             C.c_void_p(stream)), "llsr_process_batch")

    def fetch(self, b: int) -> dict:
        self._check(lib().llsr_fetch_scan(self._h, b, C.byref(self.out.struct)), "llsr_fetch_scan")
        return self.out.result()

    def fetch_vis_clouds(self, b: int) -> dict:
        """publishClouds' visualization clouds of slot b (llsr_fetch_vis_clouds): {name: float32 [n, 4]}."""
        HW = self.cfg.num_vertical_scans * self.cfg.num_horizontal_scans
        bufs = {name: np.zeros((HW, 4), np.float32) for name, _ in _abi.VIS_CLOUDS}
        v = _abi.VisOut(*(bufs[name].ctypes.data for name, _ in _abi.VIS_CLOUDS))
        self._check(lib().llsr_fetch_vis_clouds(self._h, b, C.byref(v)), "llsr_fetch_vis_clouds")
        return {name: bufs[name][: (HW if cnt is None else getattr(v, cnt))].copy() for name, cnt in _abi.VIS_CLOUDS}

    def batch_counts(self, B: int) -> np.ndarray:
        buf = np.zeros((B, 8), dtype=np.int32)
        self._check(lib().llsr_batch_counts(self._h, buf.ctypes.data), "llsr_batch_counts")
        return buf

    def set_profiling(self, on: bool):
        self._check(lib().llsr_set_profiling(self._h, 1 if on else 0), "llsr_set_profiling")

    def debug_phase_ms(self, kernel: int, phase: int, reps: int = 5) -> float:
        """Diagnostics: mean ms of kernel `kernel` re-launched with an early exit at `phase`."""
        f = lib().llsr_debug_phase_ms
        f.restype, f.argtypes = C.c_float, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]
        return float(f(self._h, kernel, phase, reps))

    def debug_s2s_prof(self, out: np.ndarray) -> int:
        """Diagnostics build (libllsr_prof.so): the last scan-to-scan launch's per-problem phase ticks
        into out (float32 [P, 8]); returns the number of problems copied."""
        f = lib().llsr_debug_s2s_prof
        f.restype, f.argtypes = C.c_int32, [C.c_void_p, C.c_void_p, C.c_int32]
        n = f(self._h, out.ctypes.data, out.shape[0])
        if n < 0:
            raise LlsrError(f"llsr_debug_s2s_prof: {n}")
        return n

    def kernel_times(self) -> dict:
        buf = np.zeros(32, dtype=np.float32)
        n = lib().llsr_kernel_times_ms(self._h, buf.ctypes.data, 32)
        if n < 0:
            self._check(n, "llsr_kernel_times_ms")
        return {lib().llsr_kernel_name(k).decode(): float(buf[k]) for k in range(n)}


    # ---- scan-to-map (MapOptimization) -------------------------------------------------------
    def scan2map_reserve(self, problems: int, corner_map: int, surf_map: int, corner_q: int, surf_q: int):
        self._check(lib().llsr_scan2map_reserve(self._h, problems, corner_map, surf_map, corner_q, surf_q),
                    "llsr_scan2map_reserve")

    def scan2map(self, corner_q, surf_q, corner_map, surf_map, pose) -> dict:
        """One problem from host arrays ((n, 4) float32 clouds, pose[6]); returns the report."""
        arrs = [np.ascontiguousarray(a, dtype=np.float32).reshape(-1, 4) for a in (corner_q, surf_q, corner_map, surf_map)]
        pose = np.ascontiguousarray(pose, dtype=np.float32).copy()
        rep = _abi.LmReport()
        args = []
        for a in arrs:
            args += [C.c_void_p(a.ctypes.data if len(a) else None), len(a)]
        self._check(lib().llsr_scan2map(self._h, *args, pose.ctypes.data, C.byref(rep)), "llsr_scan2map")
        d = rep.as_dict()
        d["pose"] = pose
        return d

    @staticmethod
    def _s2m_batch(ptrs: dict, P: int) -> _abi.S2MBatch:
        b = _abi.S2MBatch()
        b.n_problems = P
        for k, v in ptrs.items():
            setattr(b, k, v)
        return b

    def scan2map_batch(self, ptrs: dict, P: int, stream: int = 0):
        """Device-resident batch: ptrs maps the llsr_s2m_batch field names to device pointers."""
        b = self._s2m_batch(ptrs, P)
        self._check(lib().llsr_scan2map_batch(self._h, C.byref(b), C.c_void_p(stream)), "llsr_scan2map_batch")

    # split-correspondence mode (llsr_scan2map_shard_*): the LM loop is the caller's (llsr.dist)
    def scan2map_shard_begin(self, ptrs: dict, P: int, stream: int = 0):
        b = self._s2m_batch(ptrs, P)
        self._check(lib().llsr_scan2map_shard_begin(self._h, C.byref(b), C.c_void_p(stream)),
                    "llsr_scan2map_shard_begin")

    def scan2map_shard_partial(self, rank: int, world: int, d_ne: int, stream: int = 0):
        self._check(lib().llsr_scan2map_shard_partial(self._h, rank, world, C.c_void_p(d_ne), C.c_void_p(stream)),
                    "llsr_scan2map_shard_partial")

    def scan2map_shard_step(self, d_ne: int, poll: bool, stream: int = 0) -> int:
        """Solve from the summed words; with poll, sync and return the problems still active
        (else -1)."""
        n = C.c_int32(-1)
        self._check(lib().llsr_scan2map_shard_step(self._h, C.c_void_p(d_ne), C.byref(n) if poll else None,
                                                    C.c_void_p(stream)), "llsr_scan2map_shard_step")
        return int(n.value)

    def scan2map_shard_end(self, stream: int = 0):
        self._check(lib().llsr_scan2map_shard_end(self._h, C.c_void_p(stream)), "llsr_scan2map_shard_end")


    def scan2map_stats(self) -> dict:
        st = _abi.S2MStats()
        self._check(lib().llsr_scan2map_stats(self._h, C.byref(st)), "llsr_scan2map_stats")
        return {k: getattr(st, k) for k, _ in st._fields_}


    def scan2scan_stats(self) -> dict:
        st = _abi.S2SStats()
        self._check(lib().llsr_scan2scan_stats(self._h, C.byref(st)), "llsr_scan2scan_stats")
        return {k: getattr(st, k) for k, _ in st._fields_}

    # ---- scan-to-scan (FeatureAssociation::updateTransformation) ------------------------------
    def scan2scan_reserve(self, problems: int, sharp: int, flat: int, corner_last: int, surf_last: int):
        self._check(lib().llsr_scan2scan_reserve(self._h, problems, sharp, flat, corner_last, surf_last),
                    "llsr_scan2scan_reserve")

    def scan2scan(self, sharp, flat, corner_last, surf_last, transform_cur, is_degenerate: int = 0) -> dict:
        """One scan from host arrays; returns the report (+ transform_cur, is_degenerate)."""
        arrs = [np.ascontiguousarray(a, dtype=np.float32).reshape(-1, 4) for a in (sharp, flat, corner_last, surf_last)]
        t = np.ascontiguousarray(transform_cur, dtype=np.float32).copy()
        deg = C.c_int32(is_degenerate)
        rep = _abi.S2SReport()
        args = []
        for a in arrs:
            args += [C.c_void_p(a.ctypes.data if len(a) else None), len(a)]
        self._check(lib().llsr_scan2scan(self._h, *args, t.ctypes.data, C.byref(deg), C.byref(rep)), "llsr_scan2scan")
        d = rep.as_dict()
        d["transform_cur"] = t
        d["is_degenerate"] = deg.value
        return d

    def scan2scan_batch(self, ptrs: dict, P: int, stream: int = 0):
        b = _abi.S2SBatch()
        b.n_problems = P
        for k, v in ptrs.items():
            setattr(b, k, v)
        self._check(lib().llsr_scan2scan_batch(self._h, C.byref(b), C.c_void_p(stream)), "llsr_scan2scan_batch")

    def scan2scan_check(self):
        self._check(lib().llsr_scan2scan_check(self._h), "llsr_scan2scan_check")


    # ---- end-to-end odometry (runFeatureAssociation) -------------------------------------------
    def odometry_batch(self, d_xyzi: int, d_offsets: int, B: int, stream: int = 0):
        """One device-resident scan per slot through features + scan-to-scan LM + last clouds."""
        self._check(lib().llsr_odometry_batch(self._h, C.c_void_p(d_xyzi), C.c_void_p(d_offsets), B,
                                              C.c_void_p(stream)), "llsr_odometry_batch")

    def odometry_fetch(self, b: int, clouds: bool = False) -> dict:
        st = _abi.OdomSlot()
        cap = self.cfg.num_vertical_scans * self.cfg.num_horizontal_scans + 160
        bufs = [np.zeros((cap, 4), np.float32) for _ in range(4)] if clouds else [None] * 4
        ptrs = [C.c_void_p(a.ctypes.data) if a is not None else None for a in bufs]
        self._check(lib().llsr_odometry_fetch(self._h, b, C.byref(st), *ptrs), "llsr_odometry_fetch")
        d = {k: getattr(st, k) for k in ("frames", "n_corner_last", "n_surf_last", "n_corner_scan", "n_surf_scan")}
        d["transform_cur"] = np.array(st.transform_cur[:], np.float32)
        d["transform_sum"] = np.array(st.transform_sum[:], np.float32)
        d["lm"] = st.lm.as_dict()
        if clouds:
            for name, a, n in zip(("corner_last", "surf_last", "corner_scan", "surf_scan"), bufs,
                                  (st.n_corner_last, st.n_surf_last, st.n_corner_scan, st.n_surf_scan)):
                d[name] = a[:n].copy()
        return d

    def odometry_reset(self):
        self._check(lib().llsr_odometry_reset(self._h), "llsr_odometry_reset")

    # ---- mapping chain (FeatureAssociation -> MapOptimization::run) ----------------------------
    def mapping_init(self, mo_mode: int = _abi.LLSR_MODE_LM_APPLIED, map_cfg: _abi.MapConfig | None = None):
        """Per-slot MapOptimization state; mo_mode is MapOptimization's LM mode."""
        self._check(lib().llsr_mapping_init(self._h, mo_mode, C.byref(map_cfg) if map_cfg is not None else None),
                    "llsr_mapping_init")

    def mapping_batch(self, d_xyzi: int, d_offsets: int, B: int, stream: int = 0):
        """One device-resident scan per slot through IP + FA + odometry + MapOptimization."""
        self._check(lib().llsr_mapping_batch(self._h, C.c_void_p(d_xyzi), C.c_void_p(d_offsets), B,
                                             C.c_void_p(stream)), "llsr_mapping_batch")

    def mapping_fetch(self, b: int) -> dict:
        st = _abi.MappingSlot()
        self._check(lib().llsr_mapping_fetch(self._h, b, C.byref(st)), "llsr_mapping_fetch")
        d = {k: getattr(st, k) for k in ("frames", "mo_frames", "keyframes", "lm_ran", "n_corner_q", "n_surf_q")}
        for k in ("transform_sum", "transform_tobe_mapped", "transform_bef_mapped", "transform_aft_mapped"):
            d[k] = np.array(getattr(st, k)[:], np.float32)
        d["lm"] = st.lm.as_dict()
        d["map"] = st.map.as_dict()
        return d

    def mapping_keyposes(self, b: int) -> np.ndarray:
        n = lib().llsr_mapping_keyposes(self._h, b, None, 0)
        if n < 0:
            self._check(n, "llsr_mapping_keyposes")
        out = np.zeros((max(n, 1), 6), np.float32)
        lib().llsr_mapping_keyposes(self._h, b, out.ctypes.data, n)
        return out[:n].copy()

    def mapping_reset(self):
        self._check(lib().llsr_mapping_reset(self._h), "llsr_mapping_reset")


def mapping_associate(transform_sum_fa, bef, aft):
    """Host-only pose glue of the mapping chain (llsr_mapping_associate): OdometryToTransform then
    transformAssociateToMap; returns (transform_sum, transform_tobe_mapped, transform_incre)."""
    a = [np.ascontiguousarray(x, np.float32) for x in (transform_sum_fa, bef, aft)]
    out = [np.zeros(6, np.float32) for _ in range(3)]
    rc = lib().llsr_mapping_associate(*(x.ctypes.data for x in a), *(x.ctypes.data for x in out))
    if rc != 0:
        raise LlsrError(f"llsr_mapping_associate: {rc}")
    return tuple(out)


def _msg_to_array(m: "_abi.OdometryMsg") -> np.ndarray:
    return np.array(list(m.orientation) + list(m.position) + list(m.twist_angular) + list(m.twist_linear),
                    np.float64)


def _array_to_msg(a) -> "_abi.OdometryMsg":
    a = np.asarray(a, np.float64)
    m = _abi.OdometryMsg()
    m.orientation[:] = a[0:4].tolist()
    m.position[:] = a[4:7].tolist()
    m.twist_angular[:] = a[7:10].tolist()
    m.twist_linear[:] = a[10:13].tolist()
    return m


def pose_to_odometry(pose, twist=None) -> np.ndarray:
    """The publishers' pose -> nav_msgs/Odometry encoding (llsr_pose_to_odometry: FA:2612-2625,
    MO:704-723, TF:193-206), as 13 doubles: orientation xyzw, position, twist angular, twist linear."""
    p = np.ascontiguousarray(pose, np.float32)
    t = None if twist is None else np.ascontiguousarray(twist, np.float32)
    m = _abi.OdometryMsg()
    rc = lib().llsr_pose_to_odometry(p.ctypes.data, None if t is None else t.ctypes.data, C.byref(m))
    if rc != 0:
        raise LlsrError(f"llsr_pose_to_odometry: {rc}")
    return _msg_to_array(m)


def odometry_to_transform(msg) -> np.ndarray:
    """OdometryToTransform (UT:99-113) of a 13-double odometry message."""
    out = np.zeros(6, np.float32)
    m = _array_to_msg(msg)
    rc = lib().llsr_odometry_to_transform(C.byref(m), out.ctypes.data)
    if rc != 0:
        raise LlsrError(f"llsr_odometry_to_transform: {rc}")
    return out


class TransformFusion:
    """The TransformFusion node's arithmetic (transformFusion.cpp) over the C-ABI's host entry points:
    `laser_odometry_handler(msg)` takes /laser_odom_to_init and returns /integrated_to_init (TF:188-280),
    `odom_aft_mapped_handler(msg)` takes /aft_mapped_to_init (TF:282-304). Messages are 13 doubles."""

    def __init__(self):
        self.state = _abi.FusionState()
        rc = lib().llsr_fusion_init(C.byref(self.state))
        if rc != 0:
            raise LlsrError(f"llsr_fusion_init: {rc}")

    def laser_odometry_handler(self, msg) -> np.ndarray:
        m, out = _array_to_msg(msg), _abi.OdometryMsg()
        rc = lib().llsr_fusion_laser_odometry(C.byref(self.state), C.byref(m), C.byref(out))
        if rc != 0:
            raise LlsrError(f"llsr_fusion_laser_odometry: {rc}")
        return _msg_to_array(out)

    def odom_aft_mapped_handler(self, msg):
        m = _array_to_msg(msg)
        rc = lib().llsr_fusion_aft_mapped(C.byref(self.state), C.byref(m))
        if rc != 0:
            raise LlsrError(f"llsr_fusion_aft_mapped: {rc}")

    def state_array(self) -> np.ndarray:
        """transformSum, transformIncre, transformMapped, transformBefMapped, transformAftMapped."""
        st = self.state
        return np.concatenate([np.array(getattr(st, f), np.float32) for f, _ in st._fields_])


def shadow_points() -> np.ndarray:
    """GenerateShadowPoint (FA:412-439): the 160 virtual points appended to the flat / surf-last clouds."""
    out = np.zeros((160, 4), np.float32)
    rc = lib().llsr_shadow_points(out.ctypes.data)
    if rc != 0:
        raise LlsrError(f"llsr_shadow_points: {rc}")
    return out


def integrate_transformation(transform_sum, transform_cur) -> np.ndarray:
    """integrateTransformation (FA:2537-2568) on the host side of the library: the new transformSum."""
    ts = np.array(transform_sum, np.float32).reshape(6).copy()
    tc = np.ascontiguousarray(transform_cur, np.float32).reshape(6)
    rc = lib().llsr_integrate_transformation(ts.ctypes.data, tc.ctypes.data)
    if rc != 0:
        raise LlsrError(f"llsr_integrate_transformation: {rc}")
    return ts


def transform_to_end(transform_cur, xyzi) -> np.ndarray:
    """TransformToEnd (FA:1414-1490) of float4 rows on the host side of the library."""
    tc = np.ascontiguousarray(transform_cur, np.float32).reshape(6)
    a = np.ascontiguousarray(xyzi, np.float32).reshape(-1, 4)
    out = np.empty_like(a)
    rc = lib().llsr_transform_to_end(tc.ctypes.data, a.ctypes.data, len(a), out.ctypes.data)
    if rc != 0:
        raise LlsrError(f"llsr_transform_to_end: {rc}")
    return out


class FeatureAssociation:
    """Drop-in for FeatureAssociation::updateTransformation's arithmetic (FA:2505-2535)."""

    def __init__(self, pipeline: Pipeline):
        self.p = pipeline
        self.transform_cur = np.zeros(6, np.float32)
        self.is_degenerate = 0

    def update_transformation(self, corner_points_sharp, surf_points_flat, laser_cloud_corner_last,
                              laser_cloud_surf_last) -> dict:
        r = self.p.scan2scan(corner_points_sharp, surf_points_flat, laser_cloud_corner_last,
                             laser_cloud_surf_last, self.transform_cur, self.is_degenerate)
        self.transform_cur = r["transform_cur"]
        self.is_degenerate = r["is_degenerate"]
        return r


class MapOptimization:
    """Drop-in for MapOptimization::scan2MapOptimization's arithmetic (MO:1572-1610)."""

    def __init__(self, pipeline: Pipeline):
        self.p = pipeline

    def scan2map_optimization(self, laser_cloud_corner_scan_ds, laser_cloud_surf_total_last_ds,
                              laser_cloud_corner_from_map_ds, laser_cloud_surf_from_map_ds,
                              transform_tobe_mapped) -> dict:
        return self.p.scan2map(laser_cloud_corner_scan_ds, laser_cloud_surf_total_last_ds,
                               laser_cloud_corner_from_map_ds, laser_cloud_surf_from_map_ds,
                               transform_tobe_mapped)


class ImageProjection:
    """Drop-in for ImageProjection::cloudHandler's arithmetic (IP:189-222)."""

    def __init__(self, pipeline: Pipeline):
        self.p = pipeline

    def cloud_handler(self, xyzi: np.ndarray) -> dict:
        r = self.p.process_scan(xyzi)
        return {
            "segmented_cloud": r["seg_xyzi"], "outlier_cloud": r["outlier_xyzi"],
            "seg_msg": {
                "start_ring_index": r["start_ring_index"], "end_ring_index": r["end_ring_index"],
                "start_orientation": float(r["orientation"][0]), "end_orientation": float(r["orientation"][1]),
                "orientation_diff": float(r["orientation"][2]),
                "segmented_cloud_ground_flag": r["seg_ground_flag"].astype(bool),
                "segmented_cloud_col_ind": r["seg_col_ind"], "segmented_cloud_range": r["seg_range"],
            },
            "outlierCloud_Intensity": r["outlier_intensity"].astype(np.float64),
            "segmentedCloud_Intensity": r["seg_intensity"].astype(np.float64),
            "_full": r,
        }


def map_config(lidar: str | None = None, **kw) -> _abi.MapConfig:
    """llsr_map_config_default (lidar None) or the loam_config.yaml block of `lidar`
    (llsr_map_config_lidar: "hdl64e" enables the loop-closure local map), then the overrides."""
    c = _abi.MapConfig()
    if lidar is None:
        lib().llsr_map_config_default(C.byref(c))
    else:
        code = {"vlp16": _abi.LLSR_LIDAR_VLP16, "hdl64e": _abi.LLSR_LIDAR_HDL64E}[lidar]
        if lib().llsr_map_config_lidar(C.byref(c), code) != 0:
            raise LlsrError("llsr_map_config_lidar failed")
    for k, v in kw.items():
        setattr(c, k, v)
    return c


class LocalMap:
    """MapOptimization's keyframe store + local map on a HIP device (llsr_map, include/llsr.h):
    saveKeyFramesAndFactor's clouds (MO:1686-1752), extractSurroundingKeyFrames (MO:1096-1232),
    downsampleCurrentScan (MO:1234-1267) and the VoxelGrid filters they use.

    Clouds are torch CUDA float32 tensors of shape (n, 4) (x, y, z, intensity); torch is only the
    device allocator here. Calls run on a private stream ordered after the caller's current stream
    and return once their results are ready (as the reference's calls do)."""

    def __init__(self, device: int = 0, cfg: _abi.MapConfig | None = None):
        import torch
        self._torch = torch
        self.cfg = cfg or map_config()
        self.device = torch.device("cuda", device)
        self._m = lib().llsr_map_create(C.byref(self.cfg), device)
        if not self._m:
            raise LlsrError("llsr_map_create failed: no HIP device")
        self._s = torch.cuda.Stream(device=self.device)
        self._n_corner = 0
        self._n_surf = 0

    def close(self):
        if getattr(self, "_m", None):
            lib().llsr_map_destroy(self._m)
            self._m = None

    def __del__(self):
        self.close()

    def _check(self, rc, what):
        if rc < 0:
            raise LlsrError(f"{what} failed ({rc}): {lib().llsr_map_last_error(self._m).decode()}")
        return rc

    def _enter(self):
        self._s.wait_stream(self._torch.cuda.current_stream(self.device))
        return C.c_void_p(self._s.cuda_stream)

    def _leave(self):
        self._torch.cuda.current_stream(self.device).wait_stream(self._s)

    def _cloud(self, a):
        t = self._torch.as_tensor(a, dtype=self._torch.float32, device=self.device).reshape(-1, 4).contiguous()
        return t

    def reset(self):
        self._check(lib().llsr_map_reset(self._m), "llsr_map_reset")
        self._n_corner = self._n_surf = 0

    def voxel_grid(self, clouds, leaves):
        """pcl::VoxelGrid::filter of every cloud (list) with its leaf size; returns the filtered clouds."""
        torch = self._torch
        cl = [self._cloud(c) for c in clouds]
        off = np.zeros(len(cl) + 1, np.int64)
        off[1:] = np.cumsum([c.shape[0] for c in cl])
        packed = torch.cat(cl) if off[-1] else torch.zeros((0, 4), dtype=torch.float32, device=self.device)
        out = torch.empty((max(int(off[-1]), 1), 4), dtype=torch.float32, device=self.device)
        out_off = np.zeros(len(cl) + 1, np.int64)
        leaf = np.asarray(leaves, np.float32)
        s = self._enter()
        self._check(lib().llsr_map_voxel_grid(self._m, C.c_void_p(packed.data_ptr()), off.ctypes.data, len(cl),
                                              leaf.ctypes.data, C.c_void_p(out.data_ptr()), out_off.ctypes.data, s),
                    "llsr_map_voxel_grid")
        self._leave()
        return [out[out_off[k]:out_off[k + 1]] for k in range(len(cl))]

    def downsample_scan(self, corner_last, surf_last, outlier_last, corner_scan, surf_scan) -> dict:
        """downsampleCurrentScan (MO:1234-1267): the six ...DS clouds."""
        torch = self._torch
        cl = [self._cloud(c) for c in (corner_last, surf_last, outlier_last, corner_scan, surf_scan)]
        n = [c.shape[0] for c in cl]
        out = torch.empty((max(sum(n) + n[1] + n[2], 1), 4), dtype=torch.float32, device=self.device)
        out_off = np.zeros(7, np.int64)
        args = []
        for c, k in zip(cl, n):
            args += [C.c_void_p(c.data_ptr() if k else 0), k]
        s = self._enter()
        self._check(lib().llsr_map_downsample_scan(self._m, *args, C.c_void_p(out.data_ptr()), out_off.ctypes.data,
                                                   s), "llsr_map_downsample_scan")
        self._leave()
        names = ("corner_last_ds", "surf_last_ds", "outlier_last_ds", "corner_scan_ds", "surf_scan_ds",
                 "surf_total_last_ds")
        return {nm: out[out_off[k]:out_off[k + 1]] for k, nm in enumerate(names)}

    def add_keyframe(self, pose6, corner, surf, outlier) -> int:
        """Store a keyframe: PointTypePose x, y, z, roll, pitch, yaw + its three clouds."""
        pose = np.ascontiguousarray(pose6, np.float32)
        cl = [self._cloud(c) for c in (corner, surf, outlier)]
        args = []
        for c in cl:
            args += [C.c_void_p(c.data_ptr() if c.shape[0] else 0), c.shape[0]]
        s = self._enter()
        k = self._check(lib().llsr_map_add_keyframe(self._m, pose.ctypes.data, *args, s), "llsr_map_add_keyframe")
        self._s.synchronize()  # the copies read the caller's tensors
        self._n_corner += cl[0].shape[0]
        self._n_surf += cl[1].shape[0] + cl[2].shape[0]
        return k

    @property
    def num_keyframes(self) -> int:
        return lib().llsr_map_num_keyframes(self._m)

    def extract(self, robot_pos):
        """extractSurroundingKeyFrames: (laserCloudCornerFromMapDS, laserCloudSurfFromMapDS, report)."""
        torch = self._torch
        pos = np.ascontiguousarray(robot_pos, np.float32)
        cc, cs = max(self._n_corner, 1), max(self._n_surf, 1)
        oc = torch.empty((cc, 4), dtype=torch.float32, device=self.device)
        os_ = torch.empty((cs, 4), dtype=torch.float32, device=self.device)
        rep = _abi.MapReport()
        s = self._enter()
        self._check(lib().llsr_map_extract(self._m, pos.ctypes.data, C.c_void_p(oc.data_ptr()), cc,
                                           C.c_void_p(os_.data_ptr()), cs, C.byref(rep), s), "llsr_map_extract")
        self._leave()
        return oc[:rep.n_corner_ds], os_[:rep.n_surf_ds], rep.as_dict()

    def keyframe_ids(self) -> np.ndarray:
        n = lib().llsr_map_keyframe_ids(self._m, None, 0)
        out = np.zeros(max(n, 1), np.int32)
        lib().llsr_map_keyframe_ids(self._m, out.ctypes.data, n)
        return out[:n]


# ---- input wire formats (llsr_input.hip) ----

def pc2_layout(fields, point_step: int) -> _abi.Pc2Layout:
    """fields: iterable of (name, offset, datatype, count) as in sensor_msgs/PointField."""
    lay = _abi.Pc2Layout()
    fields = list(fields)
    if len(fields) > _abi.PC2_MAX_FIELDS:
        raise ValueError("too many PointCloud2 fields")
    lay.point_step = point_step
    lay.num_fields = len(fields)
    for k, (name, off, dt, cnt) in enumerate(fields):
        lay.fields[k].name = name.encode()
        lay.fields[k].offset, lay.fields[k].datatype, lay.fields[k].count = off, dt, cnt
    return lay


def decode_pointcloud2(layout: _abi.Pc2Layout, messages, device: int = 0, stream: int = 0):
    """pcl::fromROSMsg<PointXYZI> of a batch of PointCloud2 messages. messages: list of
    (data bytes, width, height, row_step). The bytes are uploaded, decoded on the device, and the
    float4 points returned as a torch tensor (n, 4) with host and device point offsets [B+1]."""
    import torch
    dev = torch.device("cuda", device)
    B = len(messages)
    msgs = (_abi.Pc2Msg * B)()
    blobs, pos = [], 0
    for b, (data, width, height, row_step) in enumerate(messages):
        raw = np.frombuffer(bytes(data), np.uint8)
        pad = (-pos) % 16                     # keep every message 16-byte aligned in the pack
        if pad:
            blobs.append(np.zeros(pad, np.uint8))
            pos += pad
        msgs[b].data_offset, msgs[b].width, msgs[b].height, msgs[b].row_step = pos, width, height, row_step
        blobs.append(raw)
        pos += len(raw)
    data = torch.from_numpy(np.concatenate(blobs) if blobs else np.zeros(1, np.uint8)).to(dev)
    n = sum(w * h for _, w, h, _ in messages)
    out = torch.empty((max(n, 1), 4), dtype=torch.float32, device=dev)
    off = np.zeros(B + 1, np.int64)
    d_off = torch.empty(B + 1, dtype=torch.int64, device=dev)
    torch.cuda.current_stream(dev).synchronize()
    rc = lib().llsr_decode_pointcloud2(C.byref(layout), C.c_void_p(data.data_ptr()), msgs, B,
                                       C.c_void_p(out.data_ptr()), off.ctypes.data, C.c_void_p(d_off.data_ptr()),
                                       C.c_void_p(stream))
    if rc != 0:
        raise LlsrError(f"llsr_decode_pointcloud2 failed ({rc})")
    return out[:n], off, d_off


def kitti_count(velodyne_dir: str) -> int:
    return lib().llsr_kitti_count(velodyne_dir.encode())


def kitti_read(path: str) -> np.ndarray:
    """One KITTI .bin frame as (n, 4) float32, read the way the reference's loader reads it."""
    out = np.zeros((_abi.KITTI_MAX_FLOATS // 4, 4), np.float32)
    n = C.c_int32()
    rc = lib().llsr_kitti_read(path.encode(), out.ctypes.data, len(out), C.byref(n))
    if rc != 0:
        raise LlsrError(f"llsr_kitti_read({path}) failed ({rc})")
    return out[:n.value].copy()


def kitti_load(velodyne_dir: str, first: int, B: int, cap_points: int, device: int = 0, stream: int = 0):
    """Frames first .. first+B-1 into HBM: (points tensor (n, 4), host offsets, device offsets)."""
    import torch
    dev = torch.device("cuda", device)
    out = torch.empty((max(cap_points, 1), 4), dtype=torch.float32, device=dev)
    off = np.zeros(B + 1, np.int64)
    d_off = torch.empty(B + 1, dtype=torch.int64, device=dev)
    torch.cuda.current_stream(dev).synchronize()
    rc = lib().llsr_kitti_load(velodyne_dir.encode(), first, B, C.c_void_p(out.data_ptr()), cap_points,
                               off.ctypes.data, C.c_void_p(d_off.data_ptr()), C.c_void_p(stream))
    if rc != 0:
        raise LlsrError(f"llsr_kitti_load failed ({rc})")
    return out[:off[-1]], off, d_off
