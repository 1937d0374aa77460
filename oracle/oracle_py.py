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
        src = os.path.join(_HERE, "oracle_ipfa.cpp")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
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
        _LIB = L
    return _LIB


class Oracle:
    """One reference pipeline (IP + FA feature stage) with its own carry-over state."""

    def __init__(self, cfg: _abi.Config):
        self.cfg = cfg
        self._h = lib().oracle_create(C.byref(cfg))
        if not self._h:
            raise ValueError("oracle_create rejected the config")
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

    def ransac_inliers(self, seed: int) -> np.ndarray:
        cap = self.cfg.num_vertical_scans * self.cfg.num_horizontal_scans
        buf = np.zeros(cap, dtype=np.int32)
        n = lib().oracle_ransac_inliers(self._h, seed, buf.ctypes.data, cap)
        return buf[:n].copy()
