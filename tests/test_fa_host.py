"""CPU tests of the FA end-of-scan host entry points the FA node's thread calls
(llsr_integrate_transformation, llsr_transform_to_end; include/llsr.h): integrateTransformation
(FA:2537-2568) and TransformToEnd (FA:1414-1490) against the oracle's statement of the same lines
(oracle/oracle_fa_lm.cpp). Host-side code of libllsr.so, so no GPU is needed; the device copies of
the same functions (k_odo_finish) are compared with the oracle in tests/test_gpu_odometry.py.

Bar: bit-exact (the library uses the glibc-exact sin / cos / asin / atan2 ports of llsr_libm.h,
the oracle the host glibc)."""
import numpy as np

import oracle_py
import llsr


def _poses(rng, n, rot=0.3, trans=3.0):
    t = np.empty((n, 6), np.float32)
    t[:, :3] = rng.uniform(-rot, rot, (n, 3))
    t[:, 3:] = rng.uniform(-trans, trans, (n, 3))
    return t


def test_integrate_transformation_bit_exact():
    rng = np.random.default_rng(11)
    sums, curs = _poses(rng, 3000, rot=3.0, trans=50.0), _poses(rng, 3000, rot=0.05, trans=1.0)
    curs[:5] = 0  # a still sensor
    for ts, tc in zip(sums, curs):
        a = llsr.integrate_transformation(ts, tc)
        b = oracle_py.integrate_transformation(ts, tc)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (ts, tc, a, b)


def test_transform_to_end_bit_exact():
    rng = np.random.default_rng(12)
    n = 20000
    pts = np.empty((n, 4), np.float32)
    pts[:, :3] = rng.uniform(-80, 80, (n, 3))
    ring = rng.integers(0, 64, n).astype(np.float32)
    pts[:, 3] = ring + rng.uniform(0, 0.0999, n).astype(np.float32)  # ring + relTime / 10 (FA:565-598)
    pts[:7, 3] = ring[:7]  # relTime 0
    for tc in _poses(rng, 8, rot=0.05, trans=1.0):
        a = llsr.transform_to_end(tc, pts)
        b = oracle_py.transform_to_end(tc, pts)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_transform_to_end_empty_and_bad_args():
    import ctypes as C
    tc = np.zeros(6, np.float32)
    assert llsr.transform_to_end(tc, np.zeros((0, 4), np.float32)).shape == (0, 4)
    L = llsr.lib()
    assert L.llsr_transform_to_end(None, None, 0, None) != 0
    assert L.llsr_transform_to_end(tc.ctypes.data, None, 3, None) != 0
    assert L.llsr_integrate_transformation(None, tc.ctypes.data) != 0
    del C
