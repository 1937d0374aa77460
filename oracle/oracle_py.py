"""TEST INFRASTRUCTURE ONLY — ctypes loader for the CPU restatement (oracle/_build/liboracle.so).

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the
product package. Builds the library with `make` if it is missing (gcc is on both boxes).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
sys.path.insert(0, os.path.join(_REPO, "lego-loam-sr_amd"))
from llsr import _abi  # noqa: E402

_LIB = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "_build", "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "liboracle.so")
        srcs = [os.path.join(_HERE, f) for f in ("oracle_ipfa.cpp", "oracle_mo.cpp", "oracle_fa_lm.cpp",
                                                        "oracle_map.cpp", "oracle_mapping.cpp", "oracle_voxel.h")]
        if not os.path.exists(path) or os.path.getmtime(path) < max(map(os.path.getmtime, srcs)):
            build()
        L = C.CDLL(path)
        L.oracle_create.restype = C.c_void_p
        L.oracle_create.argtypes = [C.POINTER(_abi.Config)]
        L.oracle_destroy.argtypes = [C.c_void_p]
        L.oracle_reset.argtypes = [C.c_void_p]
        L.oracle_process_scan.restype = C.c_int32
        L.oracle_process_scan.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(_abi.ScanOut)]
        L.oracle_stage_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.oracle_ransac_inliers.restype = C.c_int32
        L.oracle_ransac_inliers.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int32]
        L.oracle_std_sort_by_value.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
        L.oracle_set_voxel_order.argtypes = [C.c_void_p, C.c_int32]
        L.oracle_phantom_index.restype = C.c_int32
        L.oracle_phantom_index.argtypes = [C.c_void_p]
        for f in ("oracle_eig3", "oracle_eig6"):
            getattr(L, f).restype = C.c_int32
            getattr(L, f).argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        for f in ("oracle_qr_solve_5x3", "oracle_qr_solve_6x6"):
            getattr(L, f).argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        _bind_mo(L, "oracle_")
        L.oracle_transform_to_end.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.oracle_shadow_points.argtypes = [C.c_void_p]
        L.oracle_integrate_transformation.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_s2m_shard_create.restype = C.c_void_p
        L.oracle_s2m_shard_create.argtypes = [C.POINTER(_abi.Config)] + [C.c_void_p, C.c_int32] * 4 + [C.c_void_p]
        L.oracle_s2m_shard_destroy.argtypes = [C.c_void_p]
        L.oracle_s2m_shard_partial.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
        L.oracle_s2m_shard_step.restype = C.c_int32
        L.oracle_s2m_shard_step.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_s2m_shard_result.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(_abi.LmReport)]
        L.oracle_voxel_grid.restype = C.c_int64
        L.oracle_voxel_grid.argtypes = [C.c_void_p, C.c_int64, C.c_float, C.c_int32, C.c_void_p]
        L.oracle_keypose_radius.restype = C.c_int32
        L.oracle_keypose_radius.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_float, C.c_void_p]
        L.oracle_map_create.restype = C.c_void_p
        L.oracle_map_create.argtypes = [C.c_float] * 4 + [C.c_int32] * 2
        L.oracle_map_destroy.argtypes = [C.c_void_p]
        L.oracle_transform_cloud.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
        L.oracle_map_add_keyframe.restype = C.c_int32
        L.oracle_map_add_keyframe.argtypes = [C.c_void_p, C.c_void_p] + [C.c_void_p, C.c_int32] * 3
        L.oracle_map_extract.restype = C.c_int32
        L.oracle_map_extract.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p,
                                         C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p,
                                         C.c_void_p]
        L.oracle_scan2map_carry.restype = C.c_int32
        L.oracle_scan2map_carry.argtypes = [C.POINTER(_abi.Config)] + [C.c_void_p, C.c_int32] * 4 + \
            [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(_abi.LmReport)]
        L.oracle_odometry_to_transform.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_associate_to_map.argtypes = [C.c_void_p] * 5
        L.oracle_pose_to_odometry.argtypes = [C.c_void_p] * 3
        L.oracle_fusion_laser_odometry.argtypes = [C.c_void_p] * 3
        L.oracle_fusion_aft_mapped.argtypes = [C.c_void_p] * 2
        _LIB = L
    return _LIB


def _bind_mo(L, prefix):
    f = getattr(L, prefix + "scan2scan")
    f.restype = C.c_int32
    f.argtypes = [C.POINTER(_abi.Config), C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32,
                  C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.POINTER(_abi.S2SReport)]
    f = getattr(L, prefix + "scan2map")
    f.restype = C.c_int32
    f.argtypes = [C.POINTER(_abi.Config), C.c_void_p, C.c_int32, C.c_void_p, C.c_int32,
                  C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(_abi.LmReport)]
    f = getattr(L, prefix + "knn5_batch")
    f.restype = C.c_int32
    f.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]


_REF = None
REF_PATH = os.path.join(_HERE, "_ref", "libref_mo.so")
REF_SRC = "/root/reference/LeGO-LOAM/include/lego_loam/nanoflann.hpp"


def ref_lib():
    """oracle/_ref/libref_mo.so: the MO restatement over the reference's own nanoflann kd-tree.
    Built from /root/reference when that exists (build container); elsewhere only the prebuilt
    copy can be used. Returns None when neither is available."""
    global _REF
    if _REF is None:
        if os.path.exists(REF_SRC):
            subprocess.run(["make", "-s", "-C", _HERE, "ref"], check=True)
        if not os.path.exists(REF_PATH):
            return None
        L = C.CDLL(REF_PATH)
        _bind_mo(L, "ref_")
        _REF = L
    return _REF


class Oracle:
    """One reference pipeline (IP + FA feature stage) with its own carry-over state."""

    def __init__(self, cfg: _abi.Config, pcl_voxel_order: bool = True):
        self.cfg = cfg
        self._h = lib().oracle_create(C.byref(cfg))
        if not self._h:
            raise ValueError("oracle_create rejected the config")
        lib().oracle_set_voxel_order(self._h, 1 if pcl_voxel_order else 0)
        self.out = _abi.OutBuffers(cfg.num_vertical_scans, cfg.num_horizontal_scans)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_destroy(self._h)
            self._h = None

    def reset(self):
        lib().oracle_reset(self._h)

    def process(self, xyzi: np.ndarray) -> dict:
        xyzi = np.ascontiguousarray(xyzi, dtype=np.float32).reshape(-1, 4)
        rc = lib().oracle_process_scan(self._h, xyzi.ctypes.data, xyzi.shape[0], C.byref(self.out.struct))
        if rc != 0:
            raise RuntimeError(f"oracle_process_scan: {rc}")
        return self.out.result()

    def stage_ms(self):
        a, b = C.c_double(), C.c_double()
        lib().oracle_stage_ms(self._h, C.byref(a), C.byref(b))
        return a.value, b.value

    def phantom_index(self) -> int:
        """cloudSmoothness[4].ind after the last scan (the next ring-0 sort's phantom entry)."""
        return int(lib().oracle_phantom_index(self._h))

    def ransac_inliers(self, seed: int) -> np.ndarray:
        cap = self.cfg.num_vertical_scans * self.cfg.num_horizontal_scans
        buf = np.zeros(cap, dtype=np.int32)
        n = lib().oracle_ransac_inliers(self._h, seed, buf.ctypes.data, cap)
        return buf[:n].copy()


def std_sort_by_value(vals) -> np.ndarray:
    """Positions of `vals` in libstdc++ std::sort order under the value-only comparator (FA:1172)."""
    v = np.ascontiguousarray(vals, dtype=np.float32)
    out = np.zeros(len(v), dtype=np.int32)
    lib().oracle_std_sort_by_value(v.ctypes.data, len(v), out.ctypes.data)
    return out


def _f4(a) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] != 4:
        raise ValueError("expected (n, 4) float32 x,y,z,intensity")
    return a


def _mo_fn(name, knn):
    if knn == "grid":
        return getattr(lib(), "oracle_" + name)
    if knn == "kdtree":
        L = ref_lib()
        if L is None:
            raise FileNotFoundError(f"{REF_PATH} not built (needs {REF_SRC})")
        return getattr(L, "ref_" + name)
    raise ValueError(knn)


def scan2map(cfg: _abi.Config, corner_q, surf_q, corner_map, surf_map, pose0, knn: str = "grid") -> dict:
    """MapOptimization::scan2MapOptimization (MO:1572-1610) on explicit clouds; returns the
    report dict (pose = final transformTobeMapped). knn: "grid" (self-contained restatement)
    or "kdtree" (the reference's nanoflann, oracle/_ref)."""
    cq, sq, cm, sm = (_f4(a) for a in (corner_q, surf_q, corner_map, surf_map))
    pose = np.ascontiguousarray(pose0, dtype=np.float32).copy()
    rep = _abi.LmReport()
    rc = _mo_fn("scan2map", knn)(C.byref(cfg), cq.ctypes.data, len(cq), sq.ctypes.data, len(sq),
                                 cm.ctypes.data, len(cm), sm.ctypes.data, len(sm), pose.ctypes.data,
                                 C.byref(rep))
    if rc != 0:
        raise RuntimeError(f"oracle_scan2map: {rc}")
    d = rep.as_dict()
    d["pose"] = pose
    return d


def knn5(map_pts, queries, knn: str = "grid"):
    """kNN-5 with the MO acceptance (5th d^2 < 1.0): (idx [Q,5] with -1 rows = rejected, d2)."""
    m, q = _f4(map_pts), _f4(queries)
    idx = np.zeros((len(q), 5), np.int32)
    d2 = np.zeros((len(q), 5), np.float32)
    _mo_fn("knn5_batch", knn)(m.ctypes.data, len(m), q.ctypes.data, len(q), idx.ctypes.data, d2.ctypes.data)
    return idx, d2


def eig(A: np.ndarray):
    """Eigen SelfAdjointEigenSolver restatement (3x3 or 6x6): ascending evals, evec columns."""
    n = A.shape[0]
    a = np.asfortranarray(A, dtype=np.float32).ravel(order="F")
    ev = np.zeros(n, np.float32)
    V = np.zeros(n * n, np.float32)
    f = lib().oracle_eig3 if n == 3 else lib().oracle_eig6
    rc = f(a.ctypes.data, ev.ctypes.data, V.ctypes.data)
    if rc != 0:
        raise RuntimeError("eig did not converge")
    return ev, V.reshape(n, n, order="F")


def qr_solve(A: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Eigen ColPivHouseholderQR::solve restatement for 5x3 and 6x6 systems."""
    a = np.asfortranarray(A, dtype=np.float32).ravel(order="F")
    b = np.ascontiguousarray(b, dtype=np.float32)
    x = np.zeros(A.shape[1], np.float32)
    f = lib().oracle_qr_solve_5x3 if A.shape == (5, 3) else lib().oracle_qr_solve_6x6
    f(a.ctypes.data, b.ctypes.data, x.ctypes.data)
    return x


def scan2scan(cfg: _abi.Config, sharp, flat, corner_last, surf_last, transform_cur, is_degenerate: int = 0,
              knn: str = "grid") -> dict:
    """FeatureAssociation::updateTransformation (FA:2505-2535) on explicit clouds. knn: "grid"
    (brute-force restatement) or "kdtree" (the reference's nanoflann, oracle/_ref)."""
    a, b, c, d = (_f4(x) for x in (sharp, flat, corner_last, surf_last))
    t = np.ascontiguousarray(transform_cur, dtype=np.float32).copy()
    deg = C.c_int32(is_degenerate)
    rep = _abi.S2SReport()
    rc = _mo_fn("scan2scan", knn)(C.byref(cfg), a.ctypes.data, len(a), b.ctypes.data, len(b), c.ctypes.data, len(c),
                                  d.ctypes.data, len(d), t.ctypes.data, C.byref(deg), C.byref(rep))
    if rc != 0:
        raise RuntimeError(f"oracle_scan2scan: {rc}")
    out = rep.as_dict()
    out["transform_cur"] = t
    out["is_degenerate"] = deg.value
    return out


def transform_to_end(transform_cur, xyzi) -> np.ndarray:
    p = _f4(xyzi).copy()
    t = np.ascontiguousarray(transform_cur, dtype=np.float32)
    lib().oracle_transform_to_end(t.ctypes.data, p.ctypes.data, len(p))
    return p


def shadow_points() -> np.ndarray:
    out = np.zeros((160, 4), np.float32)
    lib().oracle_shadow_points(out.ctypes.data)
    return out


def fa_lm_inputs(prev: dict, cur: dict, transform_prev=None):
    """(sharp, flat, corner_last, surf_last) for the scan-to-scan LM from two consecutive
    feature-stage outputs (oracle/product result dicts), as runFeatureAssociation builds them:
    flat += shadow points (FA:1310-1314); last clouds = TransformToEnd(prev less-sharp / less-flat)
    + shadow points on the surf side (FA:2666-2707)."""
    sh = shadow_points()
    tp = np.zeros(6, np.float32) if transform_prev is None else transform_prev
    sharp = cur["loam_xyzi"][cur["sharp_ind"]]
    flat = np.concatenate([cur["loam_xyzi"][cur["flat_ind"]], sh])
    corner_last = transform_to_end(tp, prev["loam_xyzi"][prev["less_sharp_ind"]])
    surf_last = np.concatenate([transform_to_end(tp, prev["less_flat_xyzi"]), sh])
    return sharp, flat, corner_last, surf_last


class OracleShardEngine:
    """CPU statement of llsr_scan2map_shard_* for a batch of problems (llsr.dist engine protocol):
    the gloo tests' per-rank engine and the bit-exact reference of the device's split mode.
    problems: list of (corner_q, surf_q, corner_map, surf_map, pose0)."""

    def __init__(self, cfg: _abi.Config, problems):
        self.cfg = cfg
        self._keep = []
        self.h = []
        for cq, sq, cm, sm, pose in problems:
            arrs = [_f4(a) for a in (cq, sq, cm, sm)]
            p = np.ascontiguousarray(pose, dtype=np.float32)
            self._keep.append((arrs, p))
            args = []
            for a in arrs:
                args += [a.ctypes.data, len(a)]
            h = lib().oracle_s2m_shard_create(C.byref(cfg), *args, p.ctypes.data)
            if not h:
                raise ValueError("oracle_s2m_shard_create rejected the problem")
            self.h.append(h)
        self.P = len(self.h)

    def __del__(self):
        for h in getattr(self, "h", []):
            lib().oracle_s2m_shard_destroy(h)
        self.h = []

    def new_ne(self, device=None):
        import torch
        return torch.zeros((self.P, _abi.NE_WORDS), dtype=torch.int64)

    def begin(self):
        pass

    def partial(self, rank: int, world: int, ne):
        a = ne.numpy() if hasattr(ne, "numpy") else ne
        for p, h in enumerate(self.h):
            lib().oracle_s2m_shard_partial(h, rank, world, a[p].ctypes.data)

    def step(self, ne, poll: bool) -> int:
        a = ne.numpy() if hasattr(ne, "numpy") else ne
        active = sum(lib().oracle_s2m_shard_step(h, a[p].ctypes.data) for p, h in enumerate(self.h))
        return active if poll else -1

    def end(self):
        pass

    def results(self):
        out = []
        for h in self.h:
            pose = np.zeros(6, np.float32)
            rep = _abi.LmReport()
            lib().oracle_s2m_shard_result(h, pose.ctypes.data, C.byref(rep))
            d = rep.as_dict()
            d["pose"] = pose
            out.append(d)
        return out


def shard_run_local(cfg: _abi.Config, problems, world: int) -> list:
    """The split scan-to-map with `world` ranks simulated in one process: each iteration sums
    the ranks' words, exactly what an all-reduce delivers. Returns the per-problem reports."""
    engines = [OracleShardEngine(cfg, problems) for _ in range(world)]
    P = len(problems)
    for it in range(cfg.iterCountThres):
        tot = np.zeros((P, _abi.NE_WORDS), np.int64)
        part = np.zeros_like(tot)
        for r, e in enumerate(engines):
            e.partial(r, world, part)
            tot += part
        active = [e.step(tot, True) for e in engines]
        assert len(set(active)) == 1
        if active[0] == 0:
            break
    res = [e.results() for e in engines]
    for r in res[1:]:
        for a, b in zip(res[0], r):
            assert np.array_equal(a["pose"], b["pose"])
    return res[0]


def integrate_transformation(transform_sum, transform_cur) -> np.ndarray:
    ts = np.ascontiguousarray(transform_sum, dtype=np.float32).copy()
    tc = np.ascontiguousarray(transform_cur, dtype=np.float32)
    lib().oracle_integrate_transformation(ts.ctypes.data, tc.ctypes.data)
    return ts


class OracleOdometry:
    """runFeatureAssociation (FA:2742-2853) in the lm_applied mode for one sequence: the IP +
    feature stage, then updateTransformation against the last clouds, integrateTransformation and
    publishCloudsLast's TransformToEnd (first scan: checkSystemInitialization)."""

    def __init__(self, cfg: _abi.Config, pcl_voxel_order: bool = True):
        self.cfg = cfg
        self.ora = Oracle(cfg, pcl_voxel_order)
        self.shadow = shadow_points()
        self.tcur = np.zeros(6, np.float32)
        self.tsum = np.zeros(6, np.float32)
        self.deg = 0
        self.corner_last = None
        self.surf_last = None
        self.frames = 0

    def process(self, xyzi: np.ndarray) -> dict:
        r = self.ora.process(xyzi)
        loam = r["loam_xyzi"]
        sharp = loam[r["sharp_ind"]]
        flat = np.concatenate([loam[r["flat_ind"]], self.shadow])
        less_sharp, less_flat = loam[r["less_sharp_ind"]], r["less_flat_xyzi"]
        out = {"features": r}
        if self.corner_last is None:  # checkSystemInitialization (FA:2291-2315)
            self.corner_last = less_sharp.copy()
            self.surf_last = np.concatenate([less_flat, self.shadow])
            out["lm"] = None
            out["corner_scan"] = out["surf_scan"] = None
        else:
            lm = scan2scan(self.cfg, sharp, flat, self.corner_last, self.surf_last, self.tcur, self.deg)
            self.tcur, self.deg = lm["transform_cur"], lm["is_degenerate"]
            self.tsum = integrate_transformation(self.tsum, self.tcur)
            self.corner_last = transform_to_end(self.tcur, less_sharp)
            self.surf_last = np.concatenate([transform_to_end(self.tcur, less_flat), self.shadow])
            out["lm"] = lm
            out["corner_scan"] = transform_to_end(self.tcur, sharp)
            out["surf_scan"] = transform_to_end(self.tcur, flat)
        self.frames += 1
        out.update(frames=self.frames, transform_cur=self.tcur.copy(), transform_sum=self.tsum.copy(),
                   corner_last=self.corner_last, surf_last=self.surf_last)
        return out


def voxel_grid(xyzi, leaf: float, stable: bool = False) -> np.ndarray:
    """pcl::VoxelGrid::filter (oracle_voxel.h); stable=True sums each voxel in input order."""
    a = _f4(xyzi)
    out = np.zeros((max(len(a), 1), 4), np.float32)
    n = lib().oracle_voxel_grid(a.ctypes.data, len(a), leaf, int(stable), out.ctypes.data)
    if n < 0:
        raise ValueError("oracle_voxel_grid: bad arguments")
    return out[:n].copy()


def keypose_radius(poses4, pos, radius: float, knn: str = "brute") -> np.ndarray:
    """Indices (ascending) of key poses with d^2 < float(radius^2); knn="kdtree" runs the reference's
    nanoflann radiusSearch (oracle/_ref)."""
    p = _f4(poses4)
    q = np.ascontiguousarray(pos, np.float32)
    out = np.zeros(max(len(p), 1), np.int32)
    if knn == "kdtree":
        L = ref_lib()
        f = L.ref_keypose_radius
        f.restype = C.c_int32
        f.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_float, C.c_void_p]
    else:
        f = lib().oracle_keypose_radius
    n = f(p.ctypes.data, len(p), q.ctypes.data, radius, out.ctypes.data)
    return out[:n].copy()


def transform_keyframe(pose6, xyzi) -> np.ndarray:
    """transformPointCloud (MO:671-701) of a keyframe cloud by its key pose (x, y, z, roll, pitch, yaw)."""
    p = np.ascontiguousarray(pose6, np.float32)
    a = _f4(xyzi)
    out = np.zeros_like(a)
    if len(a):
        lib().oracle_transform_cloud(p.ctypes.data, a.ctypes.data, len(a), out.ctypes.data)
    return out


class OracleMap:
    """MapOptimization keyframe store + extractSurroundingKeyFrames (oracle_map.cpp)."""

    def __init__(self, radius=50.0, keypose_leaf=1.0, corner_leaf=0.2, surf_leaf=0.4, stable=False,
                 loop_closure: bool = False, search_num: int = 50):
        self._m = lib().oracle_map_create(radius, keypose_leaf, corner_leaf, surf_leaf, int(loop_closure), search_num)
        self.stable = stable
        self._nc = self._ns = 0

    def __del__(self):
        if getattr(self, "_m", None):
            lib().oracle_map_destroy(self._m)
            self._m = None

    def add_keyframe(self, pose6, corner, surf, outlier) -> int:
        pose = np.ascontiguousarray(pose6, np.float32)
        cl = [_f4(c) for c in (corner, surf, outlier)]
        args = []
        for c in cl:
            args += [c.ctypes.data, len(c)]
        self._nc += len(cl[0])
        self._ns += len(cl[1]) + len(cl[2])
        return lib().oracle_map_add_keyframe(self._m, pose.ctypes.data, *args)

    def extract(self, robot_pos):
        pos = np.ascontiguousarray(robot_pos, np.float32)
        oc = np.zeros((max(self._nc, 1), 4), np.float32)
        os_ = np.zeros((max(self._ns, 1), 4), np.float32)
        ids = np.zeros(4096, np.int32)
        nc, ns, nid = C.c_int64(), C.c_int64(), C.c_int32()
        raw = np.zeros(4, np.int64)
        rc = lib().oracle_map_extract(self._m, pos.ctypes.data, int(self.stable), oc.ctypes.data, len(oc),
                                      C.byref(nc), os_.ctypes.data, len(os_), C.byref(ns), ids.ctypes.data,
                                      len(ids), C.byref(nid), raw.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"oracle_map_extract: {rc}")
        rep = {"n_corner_map": int(raw[0]), "n_surf_map": int(raw[1]), "n_in_radius": int(raw[2]),
               "n_poses_ds": int(raw[3]), "n_keyframes": nid.value}
        return oc[:nc.value].copy(), os_[:ns.value].copy(), ids[:nid.value].copy(), rep


def decode_pointcloud2(fields, point_step: int, data: bytes, width: int, height: int, row_step: int) -> np.ndarray:
    """pcl::fromROSMsg<PointXYZI> (PCL 1.10 createMapping + copy, IP:196) restated with numpy:
    x / y / z / intensity are copied from the field of that name when its datatype is FLOAT32 (7)
    and count 1, else left at PointXYZI's default 0; points in row-major order, row r starting at
    byte r * row_step. NaN points are kept (removeNaNFromPointCloud is a separate step)."""
    raw = np.frombuffer(bytes(data), np.uint8)
    n = width * height
    out = np.zeros((n, 4), np.float32)
    idx = np.arange(n)
    base = (idx // max(width, 1)) * row_step + (idx % max(width, 1)) * point_step
    for a, name in enumerate(("x", "y", "z", "intensity")):
        for fname, off, dt, cnt in fields:
            if fname == name and dt == 7 and cnt == 1:
                b = base[:, None] + off + np.arange(4)[None, :]
                out[:, a] = raw[b].copy().view(np.float32).reshape(n) if n else out[:, a]
                break
    return out


def kitti_read(path: str) -> np.ndarray:
    """KittiLoader::get_cloud / offlineKittiService (imageProjection.h:159-170, IP:234-241): at most
    1,000,000 floats are read and floor(floats_read / 4) points kept."""
    buf = np.fromfile(path, dtype=np.float32, count=1000000)
    n = len(buf) // 4
    return buf[:4 * n].reshape(n, 4).copy()


def odometry_to_transform(transform_sum_fa) -> np.ndarray:
    """publishOdometry -> OdometryToTransform (FA:2612-2625, utility.h:99-113): the tf2 round trip."""
    t = np.ascontiguousarray(transform_sum_fa, np.float32)
    out = np.zeros(6, np.float32)
    lib().oracle_odometry_to_transform(t.ctypes.data, out.ctypes.data)
    return out


def pose_to_odometry(pose, twist=None) -> np.ndarray:
    """The publishers' pose -> nav_msgs/Odometry encoding (FA:2612-2625, MO:704-723, TF:193-206):
    13 doubles (orientation xyzw, position, twist angular, twist linear)."""
    p = np.ascontiguousarray(pose, np.float32)
    t = None if twist is None else np.ascontiguousarray(twist, np.float32)
    out = np.zeros(13, np.float64)
    lib().oracle_pose_to_odometry(p.ctypes.data, None if t is None else t.ctypes.data, out.ctypes.data)
    return out


class OracleTransformFusion:
    """TransformFusion (transformFusion.cpp): state = 5 x 6 floats (sum, incre, mapped, bef, aft)."""

    def __init__(self):
        self.state = np.zeros(30, np.float32)

    def laser_odometry(self, msg: np.ndarray) -> np.ndarray:
        m = np.ascontiguousarray(msg, np.float64)
        out = np.zeros(13, np.float64)
        lib().oracle_fusion_laser_odometry(self.state.ctypes.data, m.ctypes.data, out.ctypes.data)
        return out

    def aft_mapped(self, msg: np.ndarray):
        m = np.ascontiguousarray(msg, np.float64)
        lib().oracle_fusion_aft_mapped(self.state.ctypes.data, m.ctypes.data)


class OracleMapping:
    """MapOptimization::run (MO:1854-1896) fed by OracleOdometry, one sequence: the CPU statement of
    llsr_mapping_batch. Every VoxelGrid follows PCL (std::sort's order of equal voxel ids), as the
    device does; `stable` = True would sum each voxel in input order instead (diagnostics)."""

    def __init__(self, cfg: _abi.Config, mo_mode: int, radius=50.0, keypose_leaf=1.0, corner_leaf=0.2,
                 surf_leaf=0.4, outlier_leaf=0.4, stable: bool = False, pcl_voxel_order: bool = True,
                 loop_closure: bool | None = None, search_num: int = 50):
        """loop_closure None: the config block of the lidar (enable_loop_closure true for the
        HDL-64E block, CFG:159; false for VLP-16, CFG:23)."""
        import copy
        self.odo = OracleOdometry(cfg, pcl_voxel_order)
        self.cfg_mo = copy.copy(cfg)
        self.cfg_mo.mode = mo_mode
        if loop_closure is None:
            loop_closure = cfg.num_vertical_scans == 64
        self.map = OracleMap(radius, keypose_leaf, corner_leaf, surf_leaf, stable=stable,
                             loop_closure=loop_closure, search_num=search_num)
        self.divider = cfg.mapping_frequency_divider
        self.cycle = 0  # FeatureAssociation::_cycle_count (FA:92, 2818-2821)
        self.leaf = (corner_leaf, surf_leaf, outlier_leaf)
        self.stable = stable
        z = lambda: np.zeros(6, np.float32)  # noqa: E731
        self.transform_sum, self.bef, self.aft, self.tobe, self.incre, self.last = z(), z(), z(), z(), z(), z()
        self.robot = np.zeros(3, np.float32)
        self.deg = C.c_int32(0)
        self.matP = np.zeros(36, np.float32)
        self.keyposes = []
        self.mo_frames = 0

    def _vg(self, a, leaf):
        return voxel_grid(a, leaf, self.stable) if len(a) else np.zeros((0, 4), np.float32)

    def process(self, xyzi: np.ndarray) -> dict:
        o = self.odo.process(xyzi)
        out = {"odo": o, "step": False, "frames": o["frames"]}
        if o["lm"] is None:  # checkSystemInitialization: no AssociationOut (FA:2781-2784)
            return out
        self.cycle += 1  # FA:2818-2821: an AssociationOut on every divider-th frame
        if self.cycle != self.divider:
            return out
        self.cycle = 0
        lc, ls, lo = self.leaf
        # OdometryToTransform + transformAssociateToMap (MO:1878-1880)
        self.transform_sum = odometry_to_transform(o["transform_sum"])
        lib().oracle_associate_to_map(self.transform_sum.ctypes.data, self.bef.ctypes.data, self.aft.ctypes.data,
                                      self.tobe.ctypes.data, self.incre.ctypes.data)
        # extractSurroundingKeyFrames (MO:1096-1232)
        cmap = smap = np.zeros((0, 4), np.float32)
        mrep = None
        if self.keyposes:
            cmap, smap, _, mrep = self.map.extract(self.robot)
        # downsampleCurrentScan (MO:1234-1267); outliers after adjustOutlierCloud (FA:2600-2610)
        outlier = np.ascontiguousarray(o["features"]["outlier_xyzi"][:, [1, 2, 0, 3]])
        cl_ds = self._vg(o["corner_last"], lc)
        sl_ds = self._vg(o["surf_last"], ls)
        cs_ds = self._vg(o["corner_scan"], lc)
        ss_ds = self._vg(o["surf_scan"], ls)
        ol_ds = self._vg(outlier, lo)
        tot_ds = self._vg(np.concatenate([sl_ds, ol_ds]), ls)
        # scan2MapOptimization (MO:1572-1610) with the members carried across frames
        rep = _abi.LmReport()
        pose = self.tobe.copy()
        cq, sq, cm, sm = (_f4(a) for a in (cs_ds, tot_ds, cmap, smap))
        rc = lib().oracle_scan2map_carry(C.byref(self.cfg_mo), cq.ctypes.data, len(cq), sq.ctypes.data, len(sq),
                                         cm.ctypes.data, len(cm), sm.ctypes.data, len(sm), pose.ctypes.data,
                                         C.byref(self.deg), self.matP.ctypes.data, C.byref(rep))
        if rc != 0:
            raise RuntimeError(f"oracle_scan2map_carry: {rc}")
        lm_ran = len(cm) > 10 and len(sm) > 100
        if lm_ran:  # transformUpdate (MO:583-589)
            self.tobe = pose.copy()
            self.bef = self.transform_sum.copy()
            self.aft = self.tobe.copy()
        # saveKeyFramesAndFactor (MO:1612-1755): iSAM2 returns its initial values
        self.robot = self.aft[3:6].copy()
        first = not self.keyposes
        est = (self.tobe if first else self.aft).copy()
        self.last = est.copy()
        if not first:
            self.tobe = self.aft.copy()
        kp = np.array([est[3], est[4], est[5], est[0], est[1], est[2]], np.float32)
        self.map.add_keyframe(kp, o["corner_scan"], sl_ds, ol_ds)
        self.keyposes.append(kp)
        self.mo_frames += 1
        out.update(step=True, lm=rep.as_dict(), lm_ran=lm_ran, map=mrep, n_corner_q=len(cq), n_surf_q=len(sq),
                   n_corner_map=len(cm), n_surf_map=len(sm), transform_sum=self.transform_sum.copy(),
                   transform_tobe_mapped=self.tobe.copy(), transform_bef_mapped=self.bef.copy(),
                   transform_aft_mapped=self.aft.copy(), keyframes=len(self.keyposes))
        return out
