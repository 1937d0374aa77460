"""GPU parity of the end-to-end odometry (llsr_odometry_*, runFeatureAssociation FA:2742-2853).

B independent sequences advance one scan per call through IP + features + scan-to-scan LM +
integrateTransformation + publishCloudsLast on the device; each slot is compared after every
scan with the oracle's sequence restatement (oracle_py.OracleOdometry).

Bar: bit-exact — frame counts, LM skip flag, transformCur / transformSum and the last / scan
clouds equal the oracle's (the features are bit-exact, tests/_compare.py, and the scan-to-scan LM
sums its normal equations in Eigen's order, llsr_fa_lm.hip).
"""
import numpy as np
import pytest

import oracle_py
from llsr import Pipeline, _abi, default_config, synth

pytestmark = pytest.mark.gpu


def _sequence(lidar, horizontal, slots, frames):
    import torch
    cfg = default_config(lidar, horizontal)
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    H, W = cfg.num_vertical_scans, cfg.num_horizontal_scans
    pipe = Pipeline(cfg, max_batch=len(slots), max_points=H * W)
    oras = [oracle_py.OracleOdometry(cfg) for _ in slots]
    errs, surf_its = [], []
    for k in range(frames):
        scans = [synth.make_scan(s0 + k, lidar, motion=True) for s0 in slots]
        off = np.zeros(len(scans) + 1, np.int64)
        off[1:] = np.cumsum([len(s) for s in scans])
        d_pts = torch.from_numpy(np.concatenate(scans)).cuda()
        d_off = torch.from_numpy(off).cuda()
        torch.cuda.synchronize()
        pipe.odometry_batch(d_pts.data_ptr(), d_off.data_ptr(), len(scans))
        for b, ora in enumerate(oras):
            g = pipe.odometry_fetch(b, clouds=True)
            o = ora.process(scans[b])
            tag = f"{lidar} slot {b} frame {k}"
            if g["frames"] != o["frames"]:
                errs.append(f"{tag}: frames {g['frames']} vs {o['frames']}")
            if (g["lm"]["skipped"] == 1) != (o["lm"] is None):
                errs.append(f"{tag}: skipped {g['lm']['skipped']} vs oracle lm {o['lm'] is not None}")
            elif o["lm"] is not None:
                surf_its.append(o["lm"]["surf_iterations"])
                for key in ("surf_iterations", "corner_iterations", "n_surf_corr", "n_corner_corr", "degenerate"):
                    if g["lm"][key] != o["lm"][key]:
                        errs.append(f"{tag}: lm {key} {g['lm'][key]} vs {o['lm'][key]}")
            for key in ("transform_cur", "transform_sum"):
                if not np.array_equal(g[key], o[key]):
                    errs.append(f"{tag}: {key} {g[key]} vs {o[key]} (max |d| {np.abs(g[key] - o[key]).max():.3g})")
            for key in ("corner_last", "surf_last", "corner_scan", "surf_scan"):
                ref = o[key] if o[key] is not None else np.zeros((0, 4), np.float32)
                if g[key].shape != ref.shape:
                    errs.append(f"{tag}: {key} shape {g[key].shape} vs {ref.shape}")
                elif not np.array_equal(g[key], ref):
                    errs.append(f"{tag}: {key} max |d| {np.abs(g[key] - ref).max():.3g}")
    pipe.close()
    assert max(surf_its) >= 6, f"the drive never iterates the surf step: {surf_its}"
    return errs


def test_odometry_vlp16_sequences(require_gpu):
    """Three moving drives (synth.sensor_attitude), five frames each."""
    errs = _sequence("vlp16", None, [1, 65, 130], 5)
    assert not errs, "\n".join(errs)


def test_odometry_hdl64e_sequence(require_gpu):
    errs = _sequence("hdl64e", 2048, [5, 70], 3)
    assert not errs, "\n".join(errs)


def test_odometry_needs_lm_applied(require_gpu):
    import torch
    from llsr import LlsrError
    cfg = default_config("vlp16")
    pipe = Pipeline(cfg, max_batch=1, max_points=28800)
    pts = synth.make_scan(1, "vlp16")
    d_pts = torch.from_numpy(pts).cuda()
    d_off = torch.tensor([0, len(pts)], dtype=torch.int64).cuda()
    torch.cuda.synchronize()
    with pytest.raises(LlsrError):
        pipe.odometry_batch(d_pts.data_ptr(), d_off.data_ptr(), 1)
    pipe.close()
