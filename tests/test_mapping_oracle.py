"""CPU tests of the mapping chain's host logic (MapOptimization::run, MO:1854-1896).

* The product's pose glue (llsr_mapping_associate: OdometryToTransform's tf2 round trip,
  FA:2612-2625 / utility.h:99-113, then transformAssociateToMap MO:458-581) against the oracle's
  independent restatement (oracle_mapping.cpp), bit for bit, on random and edge-case poses.
  Host-only entry: no device needed.
* The oracle's chain (oracle_py.OracleMapping) on a short VLP-16 drive: the first scan sends no
  AssociationOut, every later frame adds a keyframe, scan-to-map runs from the second MO frame on
  and, in the lm_applied mode, the mapped pose follows the sensor (0.5 m per scan along the lidar x
  axis = the LOAM z axis).
"""
import numpy as np
import pytest

import llsr
import oracle_py
from llsr import _abi, default_config, synth


def _poses(rng, n):
    p = np.zeros((n, 6), np.float32)
    p[:, :3] = rng.uniform(-np.pi, np.pi, (n, 3)).astype(np.float32)
    p[:, 3:] = rng.uniform(-200, 200, (n, 3)).astype(np.float32)
    return p


def test_pose_glue_matches_oracle_bitwise():
    rng = np.random.default_rng(11)
    n = 3000
    S, Bf, Af = _poses(rng, n), _poses(rng, n), _poses(rng, n)
    # small-motion cases (the common one) and pitch at / near +-pi/2 (tf2's gimbal branch)
    S[:500, :3] *= 1e-3
    Bf[:500] = S[:500] + rng.normal(0, 1e-3, (500, 6)).astype(np.float32)
    S[500:520, 0] = np.float32(np.pi / 2)
    S[520:540, 0] = -np.float32(np.pi / 2)
    S[540:560, 0] = np.nextafter(np.float32(np.pi / 2), np.float32(0))
    S[560:570] = 0
    Bf[560:570] = 0
    Af[560:570] = 0
    bad = 0
    for k in range(n):
        ts, tobe, inc = llsr.mapping_associate(S[k], Bf[k], Af[k])
        ts_o = oracle_py.odometry_to_transform(S[k])
        tobe_o = np.zeros(6, np.float32)
        inc_o = np.zeros(6, np.float32)
        oracle_py.lib().oracle_associate_to_map(ts_o.ctypes.data, Bf[k].ctypes.data, Af[k].ctypes.data,
                                                tobe_o.ctypes.data, inc_o.ctypes.data)
        same = lambda a, b: np.array_equal(a.view(np.uint32), b.view(np.uint32))  # noqa: E731
        if not (same(ts, ts_o) and same(tobe, tobe_o) and same(inc, inc_o)):
            bad += 1
    assert bad == 0, f"{bad} of {n} poses differ"


def test_odometry_roundtrip_is_near_identity():
    # OdometryToTransform(publishOdometry(t)) returns t up to the tf2 double round trip (|pitch| < pi/2)
    rng = np.random.default_rng(3)
    t = _poses(rng, 200)
    t[:, 0] = np.clip(t[:, 0], -1.4, 1.4)
    for k in range(len(t)):
        r = oracle_py.odometry_to_transform(t[k])
        d = np.abs(np.angle(np.exp(1j * (r[:3].astype(np.float64) - t[k, :3]))))
        assert d.max() < 1e-5 and np.array_equal(r[3:], t[k, 3:])


@pytest.mark.parametrize("mode", [_abi.LLSR_MODE_LM_APPLIED, _abi.LLSR_MODE_FAITHFUL])
def test_oracle_mapping_drive(mode):
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    if mode == _abi.LLSR_MODE_FAITHFUL:
        cfg.iterCountThres = 20  # the faithful LM never converges by itself; keep the CPU run short
    om = oracle_py.OracleMapping(cfg, mode)
    outs = [om.process(synth.make_scan(1 + k, "vlp16")) for k in range(5)]
    assert [o["step"] for o in outs] == [False, True, True, True, True]
    assert [o["keyframes"] for o in outs[1:]] == [1, 2, 3, 4]
    assert not outs[1]["lm_ran"] and all(o["lm_ran"] for o in outs[2:])
    for o in outs[2:]:
        assert o["n_corner_map"] > 10 and o["n_surf_map"] > 100
        assert o["lm"]["iterations"] >= 1
    if mode == _abi.LLSR_MODE_LM_APPLIED:
        z = [o["transform_aft_mapped"][5] for o in outs[2:]]
        assert np.allclose(np.diff(z), 0.5, atol=0.05), z
    kp = np.array(om.keyposes)
    assert kp.shape == (4, 6) and np.isfinite(kp).all()
