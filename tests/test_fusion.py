"""CPU tests of TransformFusion (transformFusion.cpp) through the C-ABI's host
entry points (llsr_fusion_*, llsr_pose_to_odometry, llsr_odometry_to_transform): no device needed.

* The product against the oracle's independent statement of the node (oracle_mapping.cpp:
  oracle_fusion_*), bit for bit: the publishers' pose -> nav_msgs/Odometry encoding (FA:2612-2625,
  MO:704-723), OdometryToTransform (UT:99-113), and an interleaved stream of /laser_odom_to_init and
  /aft_mapped_to_init messages through laserOdometryHandler (TF:188-280) and odomAftMappedHandler
  (TF:282-304): every /integrated_to_init message and the node state after every message.
* What the fusion means: while the mapped pose agrees with the odometry (aft = bef = sum), the fused
  pose is the odometry pose; after a map correction it carries the correction forward.
"""
import numpy as np

import llsr
import oracle_py


def _poses(rng, n, rot=np.pi, trans=200.0):
    p = np.zeros((n, 6), np.float32)
    p[:, :3] = rng.uniform(-rot, rot, (n, 3)).astype(np.float32)
    p[:, 3:] = rng.uniform(-trans, trans, (n, 3)).astype(np.float32)
    return p


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


def test_encoding_and_odometry_to_transform_bitwise():
    rng = np.random.default_rng(5)
    P, T = _poses(rng, 2000), _poses(rng, 2000)
    P[:20, 0] = np.float32(np.pi / 2)  # tf2's gimbal branch of getRPY
    P[20:40, 0] = -np.float32(np.pi / 2)
    bad = 0
    for k in range(len(P)):
        tw = T[k] if k % 2 else None
        m = llsr.pose_to_odometry(P[k], tw)
        mo = oracle_py.pose_to_odometry(P[k], tw)
        t = llsr.odometry_to_transform(m)
        to = oracle_py.odometry_to_transform(P[k])  # publishOdometry -> OdometryToTransform
        bad += not (_same(m, mo) and _same(t, to))
    assert bad == 0, f"{bad} of {len(P)} differ"


def test_fusion_stream_bitwise():
    rng = np.random.default_rng(9)
    fu, fo = llsr.TransformFusion(), oracle_py.OracleTransformFusion()
    n = 1500
    odo = np.cumsum(_poses(rng, n, 0.02, 0.5), axis=0).astype(np.float32)  # a drifting drive
    bad = []
    for k in range(n):
        if k % 3 == 2:  # MapOptimization's /aft_mapped_to_init at a lower rate
            aft = (odo[k] + rng.normal(0, 0.01, 6)).astype(np.float32)
            msg = llsr.pose_to_odometry(aft, odo[k])
            assert _same(msg, oracle_py.pose_to_odometry(aft, odo[k]))
            fu.odom_aft_mapped_handler(msg)
            fo.aft_mapped(msg)
        else:
            msg = llsr.pose_to_odometry(odo[k])
            a, b = fu.laser_odometry_handler(msg), fo.laser_odometry(msg)
            if not _same(a, b):
                bad.append(k)
        if not _same(fu.state_array(), fo.state):
            bad.append(k)
    assert not bad, f"messages {bad[:10]} differ"


def test_fusion_follows_odometry_and_carries_corrections():
    fu = llsr.TransformFusion()
    pose = np.array([0.01, 0.3, -0.02, 1.0, 0.1, 5.0], np.float32)
    # mapped == odometry: the fused pose is the odometry pose
    fu.odom_aft_mapped_handler(llsr.pose_to_odometry(pose, pose))
    out = llsr.odometry_to_transform(fu.laser_odometry_handler(llsr.pose_to_odometry(pose)))
    assert np.allclose(out, pose, atol=2e-6)
    # the map corrected the pose by +0.5 m in z (LOAM frame): later odometry is shifted by it
    aft = pose.copy()
    aft[5] += 0.5
    fu.odom_aft_mapped_handler(llsr.pose_to_odometry(aft, pose))
    nxt = pose.copy()
    nxt[5] += 1.0
    out = llsr.odometry_to_transform(fu.laser_odometry_handler(llsr.pose_to_odometry(nxt)))
    exp = nxt.copy()
    exp[5] += 0.5
    assert np.allclose(out, exp, atol=1e-5)
