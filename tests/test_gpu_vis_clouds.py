"""GPU: ImageProjection's visualization topics (llsr_fetch_vis_clouds; publishClouds,
imageProjection.cpp:933-967) against a numpy statement of the reference's loops applied to the
oracle's own images (range, cell -> point, ground, label; tests/_compare.py already holds those
bit-exact against the device):
  _full_cloud / _full_info_cloud (IP:337-347, resetParameters' nanPoint IP:170-179),
  ground / nonground / unknownground (IP:760-769), _segmented_cloud_pure (IP:833-842).
Bar: bit-exact (NaN payloads compared as bits)."""
import numpy as np
import pytest

import oracle_py
from llsr import Pipeline, default_config, synth

pytestmark = pytest.mark.gpu


def _expected(raw, o, H, W):
    """The reference's loops over the oracle's images (row-major cells)."""
    HW = H * W
    cp = o["cell_point"]
    rows, cols = np.divmod(np.arange(HW), W)
    nan = np.float32(np.nan)
    full = np.tile(np.array([nan, nan, nan, 0.0], np.float32), (HW, 1))
    info = full.copy()
    hit = cp >= 0
    pts = raw[cp[hit]]
    inten = (rows[hit].astype(np.float32).astype(np.float64) +
             cols[hit].astype(np.float32).astype(np.float64) / 10000.0).astype(np.float32)
    full[hit, :3] = pts[:, :3]
    full[hit, 3] = inten                                   # (float)row + (float)col / 10000.0
    info[hit, :3] = pts[:, :3]
    info[hit, 3] = o["range_image"][hit]                   # intensity = range
    g, lab = o["ground_image"], o["label_image"]
    pure = full[(lab > 0) & (lab != 999999)].copy()
    pure[:, 3] = lab[(lab > 0) & (lab != 999999)].astype(np.float32)
    return {"full_cloud": full, "full_info_cloud": info, "ground_cloud": full[g == 1],
            "nonground_cloud": full[g == 0], "unknownground_cloud": full[g == 2], "segmented_cloud_pure": pure}


@pytest.mark.parametrize("lidar,seeds", [("vlp16", [1, 2, 70]), ("hdl64e", [5])])
def test_vis_clouds_bit_exact(require_gpu, lidar, seeds):
    cfg = default_config(lidar, 2048 if lidar == "hdl64e" else None)
    H, W = cfg.num_vertical_scans, cfg.num_horizontal_scans
    pipe = Pipeline(cfg, max_points=H * W)
    ora = oracle_py.Oracle(cfg)
    counts = {}
    for s in seeds:
        raw = synth.make_scan(s, lidar, motion=True)
        pipe.process_scan(raw)
        got = pipe.fetch_vis_clouds(0)
        exp = _expected(raw, ora.process(raw), H, W)
        for k, e in exp.items():
            a = got[k]
            assert a.shape == e.shape, (s, k, a.shape, e.shape)
            assert np.array_equal(a.view(np.uint32), e.view(np.uint32)), (s, k)
            counts[k] = counts.get(k, 0) + len(e)
    pipe.close()
    assert counts["ground_cloud"] > 0 and counts["nonground_cloud"] > 0 and counts["segmented_cloud_pure"] > 0
