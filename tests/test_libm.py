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
