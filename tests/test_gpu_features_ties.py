"""GPU parity where the reference's unspecified orders decide the result.

* Ties in the per-ring curvature sort (FA:1172, std::sort by value only): 4-fold symmetric scans
  repeat every curvature exactly, so libstdc++'s order of equal values decides the order of the
  edge / flat lists; the device takes its exact introsort path (llsr_fa.hip exact_introsort) and
  must match the oracle's real std::sort bit for bit, over a sequence (carry-over state).
* The phantom entry cloudSmoothness[4]: an exact zero curvature in ring 0 can take position 4 and
  its index is visited first by the next frame's flat loop (tests/test_introsort.py shows the
  effect); device == oracle on such a pair of frames.
* PCL RANSAC with a decisive RNG (IP:716-721): a ground that turns into a ramp, whose near-ground
  inlier set depends on boost::mt19937(12345)'s sample sequence; device == oracle.
* The exact sort itself against std::sort on tie-heavy arrays (llsr_debug_exact_sort).
"""
import ctypes as C

import numpy as np
import pytest

import _scenes
import oracle_py
from _compare import compare
from llsr import Pipeline, default_config, lib, synth

pytestmark = pytest.mark.gpu
PHANTOM_CENTERS = (605, 400, 1455, 1310, 615, 730, 955)


def _sequence(scans):
    cfg = default_config("vlp16")
    pipe = Pipeline(cfg, max_points=40000)
    ora = oracle_py.Oracle(cfg)
    fails = []
    for k, pts in enumerate(scans):
        errs = compare(pipe.process_scan(pts), ora.process(pts))
        if errs:
            fails.append(f"frame {k}:\n  " + "\n  ".join(errs))
    pipe.close()
    return fails


def test_device_exact_sort_matches_std_sort(require_gpu):
    f = lib().llsr_debug_exact_sort
    f.restype, f.argtypes = C.c_int32, [C.c_void_p, C.c_int32, C.c_void_p]
    rng = np.random.default_rng(11)
    cases = []
    for n in (0, 1, 2, 16, 17, 33, 100, 129, 200, 300, 420, 511, 700, 1024, 1800, 2048):
        for levels in (1, 3, 20, 1000):
            cases.append((rng.integers(0, levels, n) * 0.25).astype(np.float32))
    k = 1024  # a median-of-3 killer: exhausts the depth limit -> libstdc++'s heap-sort fallback
    killer = np.empty(2 * k, np.float32)
    for i in range(k):
        killer[i] = (i + 1) if i % 2 == 0 else (k + i + 1)
        killer[k + i] = 2 * (i + 1)
    cases += [killer, np.floor(killer / 3)]
    bad = []
    for j, v in enumerate(cases):
        out = np.zeros(len(v), np.int32)
        assert f(v.ctypes.data, len(v), out.ctypes.data) == 0
        if not np.array_equal(out, oracle_py.std_sort_by_value(v)):
            bad.append(j)
    assert not bad, f"cases {bad} differ from std::sort"


def test_symmetric_scans_bit_exact(require_gpu):
    fails = _sequence([synth.make_symmetric_scan(s) for s in (1, 2, 3)] + [synth.make_symmetric_scan(4, quadrants=2)])
    assert not fails, "\n".join(fails)


def test_phantom_carry_bit_exact(require_gpu):
    fails = _sequence([_scenes.zero_curvature_scan(1, PHANTOM_CENTERS), synth.make_scan(5),
                       _scenes.zero_curvature_scan(2, PHANTOM_CENTERS), synth.make_symmetric_scan(2)])
    assert not fails, "\n".join(fails)


def test_ransac_rng_decisive_bit_exact(require_gpu):
    fails = _sequence([synth.make_scan(7, ground_ramp=(2.0, 0.15)), synth.make_scan(8, ground_ramp=(3.0, 0.2))])
    assert not fails, "\n".join(fails)


def _voxel_rank_cases(rng):
    """Rank sequences like a ring's voxel ranks (runs of equal ranks along a piecewise-monotone
    sweep) plus tie-heavy random ones, at the sizes around the one-wave / block thresholds, and the
    median-of-3 killer (heap-sort fallback)."""
    cases = []
    for n in (0, 1, 2, 16, 17, 64, 65, 100, 200, 420, 511, 512, 513, 700, 1024, 1500, 2048):
        for levels in (1, 3, 50, 1000):
            cases.append(rng.integers(0, levels, n).astype(np.uint32))
        if n > 2:  # a sweep: ranks rise, fall and rise again in runs of 1-6 equal values
            runs = rng.integers(1, 7, n)
            seq = np.repeat(np.arange(len(runs)), runs)[:n]
            turn = n // 3
            seq = np.concatenate([seq[:turn], seq[turn:2 * turn][::-1], seq[2 * turn:]])
            cases.append(seq.astype(np.uint32))
    k = 1024
    killer = np.empty(2 * k, np.uint32)
    for i in range(k):
        killer[i] = (i + 1) if i % 2 == 0 else (k + i + 1)
        killer[k + i] = 2 * (i + 1)
    cases += [killer, killer // 3, killer[:512], killer[:512] // 5]
    return cases


def test_device_exact_sort32_matches_std_sort(require_gpu):
    """The PCL-order VoxelGrid's 32-bit-key sort (VoxLess32: rank << 11 | position) as k_vox_pcl runs
    it (block_introsort) against libstdc++'s std::sort, including the heap-sort fallback and chains
    of lopsided partitions."""
    f = lib().llsr_debug_exact_sort32
    f.restype, f.argtypes = C.c_int32, [C.c_void_p, C.c_int32, C.c_void_p]
    bad = []
    for j, v in enumerate(_voxel_rank_cases(np.random.default_rng(12))):
        out = np.zeros(len(v), np.int32)
        assert f(v.ctypes.data, len(v), out.ctypes.data) == 0
        if not np.array_equal(out, oracle_py.std_sort_by_value(v.astype(np.float32))):
            bad.append((j, len(v)))
    assert not bad, f"cases {bad} differ from std::sort"
