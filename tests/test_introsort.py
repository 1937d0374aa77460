"""CPU: the wave-parallel statement of libstdc++'s std::sort that the device uses for the per-ring
curvature sort's tie path (FA:1172; llsr_fa.hip exact_introsort) equals std::sort on 30k
tie-heavy arrays, including median-of-3 killers that exhaust the depth limit (heap-sort fallback)
— tests/native/introsort_check.cpp. The scenes that make ties decide the feature lists are checked
here against the oracle; the device is compared with them in tests/test_gpu_features_ties.py."""
import os
import subprocess

import numpy as np

import _scenes
import oracle_py
from _compare import compare
from llsr import default_config, synth

HERE = os.path.dirname(os.path.abspath(__file__))
PHANTOM_CENTERS = (605, 400, 1455, 1310, 615, 730, 955)


def test_parallel_partition_formulation_equals_std_sort(tmp_path):
    exe = str(tmp_path / "introsort_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(HERE, "native", "introsort_check.cpp")],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    cases, bad, heap = (int(v) for v in r.stdout.split())
    assert r.returncode == 0 and bad == 0 and cases > 30000 and heap > 0, r.stdout


def test_std_sort_hook_orders_ties_like_libstdcxx():
    v = np.array([1, 0, 1, 0, 2, 0, 1] * 5, np.float32)
    order = oracle_py.std_sort_by_value(v)
    assert np.all(np.diff(v[order]) >= 0)
    assert sorted(order.tolist()) == list(range(len(v)))


def test_symmetric_scans_tie_everywhere():
    cfg = default_config("vlp16")
    r = oracle_py.Oracle(cfg).process(synth.make_symmetric_scan(1))
    c, st, en = r["curvature"], r["start_ring_index"], r["end_ring_index"]
    tied = 0
    for i in range(16):
        if st[i] < en[i] - 1:
            _, cnt = np.unique(c[max(st[i], 5):en[i] - 1], return_counts=True)
            tied += int((cnt > 1).sum())
    assert tied > 1000


def test_phantom_index_carries_into_next_frame():
    """An exact zero curvature in ring 0 can take position 4 (cloudSmoothness[4]) in the ring-0
    sort; the next frame's flat loop then visits that stale index first (FA:1211-1216)."""
    cfg = default_config("vlp16")
    ora = oracle_py.Oracle(cfg)
    ora.process(_scenes.zero_curvature_scan(1, PHANTOM_CENTERS))
    assert ora.phantom_index() != 0
    nxt = synth.make_scan(5)
    carried = ora.process(nxt)
    fresh = oracle_py.Oracle(cfg).process(nxt)
    assert carried["flat_ind"][0] == 72 and fresh["flat_ind"][0] == 0
    assert compare(carried, fresh)  # the carried state changes the outputs


def test_ramp_scene_ransac_depends_on_the_rng():
    """A ground that turns into a 15 % ramp 2 m ahead: two planes in the near-ground cloud, so
    PCL's RANSAC (IP:716-721) returns a different inlier set for almost every seed — the device has
    to reproduce boost::mt19937(12345)'s sample sequence, not just the geometry."""
    cfg = default_config("vlp16")
    ora = oracle_py.Oracle(cfg)
    ora.process(synth.make_scan(7, ground_ramp=(2.0, 0.15)))
    ref = ora.ransac_inliers(12345)
    assert sum(not np.array_equal(ora.ransac_inliers(s), ref) for s in range(1, 9)) >= 6
