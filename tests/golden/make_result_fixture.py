"""Convert the reference's own recorded mapping run (Result/0318_test/, written by
MapOptimization::saveMapService, mapOptmization.cpp:344-440) into tests/golden/result_0318.npz.

These are the only reference-held data on this path; the fixture holds them as
plain arrays, no reference text:

* corner_map  [84644, 4] — cornerMap.pcd: every keyframe's corner cloud moved into the map (LOAM)
  frame by its key pose and concatenated, not downsampled (MO:380-395);
* surf_map    [6014, 4]  — surfaceMap.pcd: the surf + outlier keyframe clouds in the map frame,
  VoxelGrid 0.4 (downSizeFilterSurf, MO:384-394);
* key_poses   [723, 6]   — cloudKeyPoses6D as PointTypePose (x, y, z, roll, pitch, yaw): x, y, z
  from trajectory.pcd (cloudKeyPoses3D, 8 significant digits) and the angles from pose.txt, whose
  columns are z, x, y, yaw, roll, pitch, time (MO:405-411: Pose6DOF << yaw, roll, pitch, z, x, y);
* key_times   [723]      — pose.txt's time column;
* pose_txt_xyz [723, 3]  — pose.txt's (x, y, z) (6 decimals), to check the column mapping above;
* map_iter_times [722]   — MapIterTimes.txt: scan2MapOptimization iterations per frame;
* map_ms [723]           — mapt.txt: MapOptimization wall time per frame (ms).

Run in the build container (the reference is not on the GPU box):

    python tests/golden/make_result_fixture.py [/root/reference/Result/0318_test]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def read_pcd_ascii(path: str) -> np.ndarray:
    """An ASCII PCD v0.7 (FIELDS x y z intensity, all F 4) as float32 [N, 4]."""
    with open(path) as f:
        fields, n = None, None
        for line in f:
            tok = line.split()
            if not tok or tok[0].startswith("#"):
                continue
            if tok[0] == "FIELDS":
                fields = tok[1:]
            elif tok[0] == "POINTS":
                n = int(tok[1])
            elif tok[0] == "DATA":
                if tok[1] != "ascii":
                    raise ValueError(f"{path}: DATA {tok[1]}")
                break
        assert fields == ["x", "y", "z", "intensity"], fields
        a = np.loadtxt(f, dtype=np.float64, ndmin=2)
    assert a.shape == (n, 4), (a.shape, n)
    return a.astype(np.float32)


def main(src: str = "/root/reference/Result/0318_test", out: str = os.path.join(HERE, "result_0318.npz")):
    corner = read_pcd_ascii(os.path.join(src, "cornerMap.pcd"))
    surf = read_pcd_ascii(os.path.join(src, "surfaceMap.pcd"))
    traj = read_pcd_ascii(os.path.join(src, "trajectory.pcd"))
    pose = np.loadtxt(os.path.join(src, "pose.txt"), delimiter=",", dtype=np.float64, ndmin=2)
    iters = np.loadtxt(os.path.join(src, "MapIterTimes.txt"), dtype=np.float64, ndmin=1)
    map_ms = np.loadtxt(os.path.join(src, "mapt.txt"), dtype=np.float64, ndmin=1)
    assert len(traj) == len(pose)
    key = np.zeros((len(pose), 6), np.float32)
    key[:, 0:3] = traj[:, 0:3]                         # x, y, z (cloudKeyPoses3D)
    key[:, 3] = pose[:, 4].astype(np.float32)          # roll
    key[:, 4] = pose[:, 5].astype(np.float32)          # pitch
    key[:, 5] = pose[:, 3].astype(np.float32)          # yaw
    np.savez_compressed(out, corner_map=corner, surf_map=surf, key_poses=key, key_times=pose[:, 6],
                        pose_txt_xyz=pose[:, [1, 2, 0]], map_iter_times=iters, map_ms=map_ms,
                        traj_index=traj[:, 3], source=np.array("Result/0318_test"))
    print(f"{out}: corner {len(corner)}, surf {len(surf)}, key poses {len(key)}, "
          f"MapIterTimes {len(iters)} (values {sorted(set(iters.tolist()))})")


if __name__ == "__main__":
    main(*sys.argv[1:])
