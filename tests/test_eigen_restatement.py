"""The two Eigen 3.3.7 restatements — the device's (lego-loam-sr_amd/csrc/llsr_eigen.h, compiled
here for the host) and the oracle's independent one (oracle/oracle_eigen.h) — agree bit for bit.

Eigen is absent from this image, so neither can be checked against Eigen itself
("parity unpinned" against the library); what is pinned here: (1) the device code equals a second,
separately written statement of the same algorithms (oracle_eigen.h follows Eigen's source layout:
Householder / GEMV / selfadjoint-GEMV / redux kernels, the device one is register-resident with
compile-time loops), on 160k matrices including rank-deficient and badly scaled ones and the
degeneracy projection matP = matV.inverse() * matV2 (FA:1983, MO:1530); (2) the oracle's results
are the right numbers (numpy: eigenvalues, inverses, least squares), test_mo_oracle.py and below.
"""
import os
import subprocess

import numpy as np
import pytest

import oracle_py

HERE = os.path.dirname(os.path.abspath(__file__))


def test_device_and_oracle_restatements_bit_identical(tmp_path):
    exe = str(tmp_path / "eigen_cross")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-Wno-unknown-pragmas",
                    "-o", exe, os.path.join(HERE, "native", "eigen_cross.cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    rows = [ln.split() for ln in r.stdout.splitlines() if ln and not ln.startswith(" ")]
    assert {row[0] for row in rows} == {"fa_3x3", "mo_6x6", "mo_5x3", "mo_cov3", "gemm_kc"}
    for name, cases, bad in rows:
        assert int(cases) > 0 and int(bad) == 0, f"{name}: {bad} of {cases} differ\n{r.stdout}"
    assert r.returncode == 0


def _inv(A):
    import ctypes as C
    A = np.asfortranarray(A, np.float32)
    out = np.zeros_like(A)
    f = oracle_py.lib().oracle_inverse3 if A.shape == (3, 3) else oracle_py.lib().oracle_inverse6
    f.argtypes = [C.c_void_p, C.c_void_p]
    f(A.ctypes.data, out.ctypes.data)
    return out


@pytest.mark.parametrize("n", [3, 6])
def test_inverse_of_eigenvectors_matches_numpy(n):
    """matV.inverse() of an eigenvector matrix (orthonormal up to rounding): the cofactor (3x3) and
    PartialPivLU (6x6) inverses are within float rounding of numpy's and NOT bitwise V^T."""
    rng = np.random.default_rng(7 + n)
    differs = 0
    for _ in range(300):
        Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
        A = ((Q * np.geomspace(0.01, 1e4, n)) @ Q.T).astype(np.float32)
        _, V = oracle_py.eig((A + A.T) / 2)
        Vi = _inv(V)
        ref = np.linalg.inv(V.astype(np.float64))
        np.testing.assert_allclose(Vi, ref, atol=2e-6 * n)
        differs += int(not np.array_equal(Vi, V.T))
    assert differs > 0, "the exact inverse should differ from V^T in the last bits somewhere"


def test_inverse6_pivoting_and_singular():
    # a permutation-heavy matrix exercises the row swaps; a zero column gives a zero pivot
    P = np.eye(6, dtype=np.float32)[[3, 0, 5, 1, 4, 2]] * np.float32(2.0)
    np.testing.assert_allclose(_inv(P), np.linalg.inv(P), atol=1e-7)
    S = np.eye(6, dtype=np.float32)
    S[:, 2] = 0
    assert not np.all(np.isfinite(_inv(S)))  # Eigen divides by the zero pivot: inf / nan
