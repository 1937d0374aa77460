"""The device libm restatement (csrc/llsr_libm.h) against host glibc, strided over all 2^32
inputs (the exhaustive stride-1 sweep is committed under profiles/libm_check_r01.log)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_libm_ports_bit_exact_strided():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    exe = os.path.join(REPO, "oracle", "_build", "libm_check")
    r = subprocess.run([exe, "257", str(min(8, os.cpu_count() or 1))], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "0 function(s) with mismatches" in r.stdout


def test_exhaustive_log_committed_clean():
    log = open(os.path.join(REPO, "profiles", "libm_check_r01.log")).read()
    assert "stride 1: 0 mismatches" in log and "0 function(s) with mismatches" in log


# Coefficients of the certified projection fast path (csrc/llsr_ip.hip project_cell_fast): atan on
# [0, 1] as t * P(t^2), degree-15 odd minimax.
_ATAN_P = [float.fromhex(h) for h in (
    "0x1.ffffeap-1", "-0x1.554c3ap-2", "0x1.988174p-3", "-0x1.1cd946p-3", "0x1.8af1c2p-4",
    "-0x1.ca08a0p-5", "0x1.6633d8p-6", "-0x1.09b84ap-8")]


def _fast_atan2_f32(a, b):
    """Host statement of project_cell_fast's atan2(a, b) in float32 ops (fmaf via the exact
    double product rounded once; the device's 1-ulp v_rcp_f32 is modelled by the correctly
    rounded quotient, its extra <= 2^-23 relative error in t is budgeted in the test)."""
    import numpy as np
    f = np.float32
    ax, bx = np.abs(a), np.abs(b)
    mx, mn = np.maximum(ax, bx), np.minimum(ax, bx)
    t = (mn * (f(1) / mx)).astype(f)
    u = t * t
    pa = np.full_like(t, f(_ATAN_P[7]))
    for c in _ATAN_P[6::-1]:
        pa = (u.astype(np.float64) * pa.astype(np.float64) + c).astype(f)
    ha = pa * t
    ha = np.where(ax > bx, f(1.57079637) - ha, ha)
    ha = np.where(b < 0, f(3.14159274) - ha, ha)
    return np.where(a < 0, -ha, ha).astype(f)


def test_projection_fast_atan2_error_bound():
    """project_cell_fast certifies a column when the quotient is 4e-6 rad / res_X (plus the
    quotient's own rounding) away from a half-integer; that is sound if its atan2 is within 1e-6
    rad of glibc's atan2f. Measured here against the true angle (glibc is within 1 ulp of it):
    < 5e-7 over random directions at every octant, plus the rcp and glibc terms < 1e-6."""
    import numpy as np
    rng = np.random.default_rng(11)
    n = 2_000_000
    ang = rng.uniform(-np.pi, np.pi, n)
    r = np.exp(rng.uniform(np.log(0.05), np.log(200.0), n))
    a = (r * np.sin(ang)).astype(np.float32)
    b = (r * np.cos(ang)).astype(np.float32)
    # octant boundaries and near-axis directions
    k = rng.integers(0, 8, 200_000) * (np.pi / 4) + rng.choice([0.0, 1e-7, -1e-7, 1e-4, -1e-4], 200_000)
    a = np.concatenate([a, np.sin(k).astype(np.float32) * 10]); b = np.concatenate([b, np.cos(k).astype(np.float32) * 10])
    keep = (np.minimum(np.abs(a), np.abs(b)) > 0)
    a, b = a[keep], b[keep]
    err = np.abs(_fast_atan2_f32(a, b).astype(np.float64) - np.arctan2(a.astype(np.float64), b.astype(np.float64)))
    err = np.minimum(err, 2 * np.pi - err)
    bound = err.max() + 2.0 ** -23 + 2.0 ** -22  # + rcp's extra ulp in t (atan' <= 1) + glibc's 1 ulp at pi
    assert err.max() < 5e-7, err.max()
    assert bound < 1e-6, bound


def test_dbscan_fast_eps_margin_sound():
    """k_dbscan_adj's db_near_fast decides eps <= DBFr from reciprocal-based squared distances and
    defers to the exact expression (FA:1353-1354) within 2e-5 of DBFr^2. Statement in float32 with
    the hardware reciprocal's 1-ulp error applied in both directions: every decided pair agrees with
    the reference's float evaluation, including pairs placed on the boundary."""
    import numpy as np
    f = np.float32
    rng = np.random.default_rng(7)
    n = 400_000
    DBFr = f(1.5)
    kxy = rng.uniform(0.01, 0.5, n).astype(f)
    kz = rng.uniform(0.01, 0.5, n).astype(f)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    # scaled radius: uniform around DBFr plus a dense band within 1e-5 of it
    rad = np.where(rng.random(n) < 0.5, rng.uniform(0, 3, n), 1.5 * (1 + rng.uniform(-3e-5, 3e-5, n)))
    d = (u * rad[:, None] * np.stack([kxy, kxy, kz], 1)).astype(f)
    p0 = rng.uniform(-30, 30, (n, 3)).astype(f)
    pj = (p0 - d).astype(f)
    dx, dy, dz = (p0[:, 0] - pj[:, 0]), (p0[:, 1] - pj[:, 1]), (p0[:, 2] - pj[:, 2])
    k2, z2 = kxy * kxy, kz * kz
    exact = np.sqrt(dx * dx / k2 + dy * dy / k2 + dz * dz / z2) <= DBFr
    r2 = DBFr * DBFr
    lo, hi = r2 * f(1 - 2e-5), r2 * f(1 + 2e-5)
    for sgn in (-1, 1):  # v_rcp_f32 within 1 ulp of 1/x
        rk = (f(1) / k2) * f(1 + sgn * 2.0 ** -23)
        rz = (f(1) / z2) * f(1 + sgn * 2.0 ** -23)
        s = (dx * dx + dy * dy) * rk + dz * dz * rz
        decided = (s < lo) | (s > hi)
        fast = s < lo
        assert np.array_equal(fast[decided], exact[decided])
        assert decided.mean() > 0.4  # the band is narrow: most pairs never reach the exact path
