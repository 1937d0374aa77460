"""GPU parity of the mapping chain (llsr_mapping_*: IP -> FA -> odometry -> MapOptimization::run,
MO:1854-1896) against the oracle's sequence restatement (oracle_py.OracleMapping).

B independent moving drives (synth.sensor_attitude) advance one scan per call; after every call each slot's MapOptimization
state is compared with the oracle's: frame / keyframe counts, whether scan-to-map ran (MO:1573),
the query and local-map sizes, the LM report, transformSum / TobeMapped / BefMapped / AftMapped,
and at the end the key poses (cloudKeyPoses6D).

Bar: bit-exact end to end — counts, LM reports, every pose and the key poses equal the oracle's.
MapOptimization's VoxelGrids on both sides sum a voxel in the order libstdc++'s std::sort leaves
PCL's index_vector, the feature stage's less-flat VoxelGrid in the handle's order (PCL's by default,
the opt-in LLSR_VOXEL_ORDER_INPUT in one test), and both LMs sum their normal equations in Eigen's order.
"""
import numpy as np
import pytest

import oracle_py
from llsr import Pipeline, _abi, default_config, map_config, synth

pytestmark = pytest.mark.gpu
POSES = ("transform_sum", "transform_tobe_mapped", "transform_bef_mapped", "transform_aft_mapped")


def _drive(mode, seeds, frames, iters=None, pcl=True, lidar="vlp16", search_num=None, divider=1,
           spare_slots=0):
    """search_num None: the lidar's config block through map_cfg NULL (HDL-64E: loop closure,
    search num 50); else the block with that surrounding_keyframe_search_num. spare_slots: the
    handle has that many more slots than the batch carries (max_batch > B)."""
    import torch
    cfg = default_config(lidar, 2048 if lidar == "hdl64e" else None)
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    cfg.mapping_frequency_divider = divider
    if iters is not None:
        cfg.iterCountThres = iters
    H, W = cfg.num_vertical_scans, cfg.num_horizontal_scans
    pipe = Pipeline(cfg, max_batch=len(seeds) + spare_slots, max_points=H * W)
    lc = lidar == "hdl64e"
    if search_num is None:
        pipe.mapping_init(mode)
        search_num = 50
    else:
        pipe.mapping_init(mode, map_config(lidar, surrounding_keyframe_search_num=search_num))
    if not pcl:
        pipe.set_voxel_order(_abi.LLSR_VOXEL_ORDER_INPUT)
    oras = [oracle_py.OracleMapping(cfg, mode, pcl_voxel_order=pcl, loop_closure=lc, search_num=search_num)
            for _ in seeds]
    errs, surf_its = [], []
    queue_full = False
    for k in range(frames):
        scans = [synth.make_scan(s0 + k, lidar, motion=True) for s0 in seeds]
        off = np.zeros(len(scans) + 1, np.int64)
        off[1:] = np.cumsum([len(s) for s in scans])
        d_pts = torch.from_numpy(np.concatenate(scans)).cuda()
        d_off = torch.from_numpy(off).cuda()
        torch.cuda.synchronize()
        pipe.mapping_batch(d_pts.data_ptr(), d_off.data_ptr(), len(scans))
        for b, ora in enumerate(oras):
            o = ora.process(scans[b])
            g = pipe.mapping_fetch(b)
            tag = f"mode {mode} slot {b} frame {k}"
            if g["frames"] != o["frames"]:
                errs.append(f"{tag}: frames {g['frames']} vs {o['frames']}")
            if o["odo"]["lm"] is not None:
                surf_its.append(o["odo"]["lm"]["surf_iterations"])
            if g["mo_frames"] != ora.mo_frames or g["keyframes"] != len(ora.keyposes):
                errs.append(f"{tag}: MapOptimization frames / keyframes {g['mo_frames']} / {g['keyframes']} vs "
                            f"{ora.mo_frames} / {len(ora.keyposes)}")
            if not o["step"]:
                continue
            for key in ("keyframes", "n_corner_q", "n_surf_q"):
                if g[key] != o[key]:
                    errs.append(f"{tag}: {key} {g[key]} vs {o[key]}")
            if bool(g["lm_ran"]) != bool(o["lm_ran"]):
                errs.append(f"{tag}: lm_ran {g['lm_ran']} vs {o['lm_ran']}")
            if o["map"] is not None:
                for key, ok in (("n_corner_ds", "n_corner_map"), ("n_surf_ds", "n_surf_map")):
                    if g["map"][key] != o[ok]:
                        errs.append(f"{tag}: map {key} {g['map'][key]} vs {o[ok]}")
                for key in ("n_keyframes", "n_corner_map", "n_surf_map", "n_in_radius", "n_poses_ds"):
                    if g["map"][key] != o["map"][key]:
                        errs.append(f"{tag}: map {key} {g['map'][key]} vs {o['map'][key]}")
                queue_full |= lc and o["map"]["n_keyframes"] == search_num and g["keyframes"] > search_num
            if o["lm_ran"]:
                for key in ("iterations", "converged", "degenerate", "n_corner_corr", "n_surf_corr"):
                    if g["lm"][key] != o["lm"][key]:
                        errs.append(f"{tag}: lm {key} {g['lm'][key]} vs {o['lm'][key]}")
            for key in POSES:
                if not np.array_equal(g[key], o[key]):
                    errs.append(f"{tag}: {key} {g[key]} vs {o[key]} (max |d| {np.abs(g[key] - o[key]).max():.3g})")
    for b, ora in enumerate(oras):
        kg = pipe.mapping_keyposes(b)
        ko = np.array(ora.keyposes, np.float32).reshape(-1, 6)
        if kg.shape != ko.shape:
            errs.append(f"slot {b}: keyposes {kg.shape} vs {ko.shape}")
        elif not np.array_equal(kg, ko):
            errs.append(f"slot {b}: keyposes max |d| {np.abs(kg - ko).max():.3g}")
    pipe.close()
    assert max(surf_its) >= 6, f"the drives never iterate the FA surf step: {surf_its}"
    return errs, queue_full


def test_mapping_chain_lm_applied(require_gpu):
    errs, _ = _drive(_abi.LLSR_MODE_LM_APPLIED, [1, 65, 130], 6)
    assert not errs, "\n".join(errs)


def test_mapping_chain_input_voxel_order(require_gpu):
    errs, _ = _drive(_abi.LLSR_MODE_LM_APPLIED, [2, 140], 5, pcl=False)
    assert not errs, "\n".join(errs)


def test_mapping_chain_faithful(require_gpu):
    errs, _ = _drive(_abi.LLSR_MODE_FAITHFUL, [3, 200], 5, iters=50)
    assert not errs, "\n".join(errs)


def test_mapping_chain_hdl64e_loop_closure_queue(require_gpu):
    """HDL-64E 64 x 2048 with the block's enable_loop_closure (CFG:159): the local map is the
    recent-keyframe queue of MO:1099-1151. search_num 4 so that the queue fills (MapOptimization
    frame 5) and then pops the oldest / pushes the newest keyframe on every later frame."""
    errs, full = _drive(_abi.LLSR_MODE_LM_APPLIED, [5], 9, lidar="hdl64e", search_num=4)
    assert not errs, "\n".join(errs)
    assert full, "the queue never reached its pop / push regime"


def test_mapping_chain_hdl64e_default_block(require_gpu):
    """map_cfg NULL on an HDL-64E handle: the block's loop-closure queue at search num 50 (the
    refill regime), two drives in a handle with a spare slot (max_batch > B)."""
    errs, _ = _drive(_abi.LLSR_MODE_LM_APPLIED, [6, 71], 4, lidar="hdl64e", spare_slots=1)
    assert not errs, "\n".join(errs)


def test_mapping_chain_frequency_divider(require_gpu):
    """mapping_frequency_divider 2 (FA:2818-2821): MapOptimization runs on frames 3, 5, 7 only,
    with a spare slot in the handle."""
    errs, _ = _drive(_abi.LLSR_MODE_LM_APPLIED, [12], 7, divider=2, spare_slots=2)
    assert not errs, "\n".join(errs)


def test_mapping_reset_repeats(require_gpu):
    """llsr_mapping_reset starts every slot over: a second pass over the same scans repeats the first."""
    import torch
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    pipe = Pipeline(cfg, max_batch=1, max_points=28800)
    pipe.mapping_init(_abi.LLSR_MODE_LM_APPLIED)
    runs = []
    for _ in range(2):
        pipe.mapping_reset()
        for k in range(4):
            pts = synth.make_scan(9 + k, "vlp16", motion=True)
            d_pts = torch.from_numpy(pts).cuda()
            d_off = torch.tensor([0, len(pts)], dtype=torch.int64).cuda()
            torch.cuda.synchronize()
            pipe.mapping_batch(d_pts.data_ptr(), d_off.data_ptr(), 1)
        runs.append((pipe.mapping_fetch(0), pipe.mapping_keyposes(0)))
    (a, ka), (b, kb) = runs
    assert a["keyframes"] == b["keyframes"] == 3
    assert np.array_equal(ka, kb)
    for key in POSES:
        assert np.array_equal(a[key], b[key]), key
    pipe.close()
