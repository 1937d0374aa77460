"""CPU tests of the C-ABI boundary: the HIP library builds for gfx950, loads, exports every entry
point include/llsr.h declares, and its host-only helpers agree with the Python mirror. No compute
call is made here (no GPU in this container): creating a handle must fail loudly with ENODEV."""
import ctypes as C
import os
import re
import subprocess

import pytest

import llsr
from llsr import _abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "llsr.h")


def _declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(llsr_\w+)\s*\(", text)))


def test_header_declares_expected_surface():
    assert set(llsr.EXPORTS) == set(_declared())


def test_integration_maps_every_entry_point():
    """INTEGRATION.md §1 names every entry point of the header next to the reference function it
    replaces (or marks it as a diagnostic)."""
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    missing = [f for f in _declared() if f not in text]
    assert not missing, missing


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", llsr.LIB_PATH], check=True,
                         capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (llsr_\w+)", out))
    missing = set(_declared()) - exported
    assert not missing, missing


def test_library_has_gfx950_code_object():
    blob = open(llsr.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


@pytest.mark.parametrize("lidar,horizontal", [("vlp16", None), ("hdl64e", None)])
def test_config_default_matches_yaml_mirror(lidar, horizontal):
    a = llsr.default_config(lidar, horizontal)
    b = _abi.config_for(lidar, horizontal)
    for name, _ in _abi.Config._fields_:
        assert getattr(a, name) == getattr(b, name), name


def test_struct_sizes_match_header():
    # llsr_config: 23 4-byte fields; llsr_scan_out: pointer/int layout as declared
    assert C.sizeof(_abi.Config) == 23 * 4
    assert C.sizeof(_abi.Sizes) == 16


def test_create_without_device_fails_loudly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a HIP device is visible")
    except Exception:
        pass
    h = C.c_void_p()
    cfg = llsr.default_config("vlp16")
    rc = llsr.lib().llsr_create(C.byref(cfg), 0, 1, 1000, C.byref(h))
    assert rc == -19 and not h.value  # LLSR_ENODEV: no silent CPU fallback
    with pytest.raises(llsr.LlsrError):
        llsr.Pipeline(cfg)


def test_map_create_fails_loudly_without_device():
    """llsr_map_create returns NULL when no HIP device is visible (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is visible")
    assert not llsr.lib().llsr_map_create(None, 0)
    with pytest.raises(llsr.LlsrError):
        llsr.LocalMap(0)


@pytest.mark.parametrize("lang,std", [("c", "c99"), ("c++", "c++11")])
def test_header_is_plain_c_and_cxx(lang, std):
    """include/llsr.h is the FFI surface (cgo / ctypes / a C++ node): it must parse as strict C99
    and C++11 with no warnings."""
    cc = "gcc" if lang == "c" else "g++"
    subprocess.run([cc, f"-std={std}", "-Wall", "-Wextra", "-pedantic", "-Werror", "-fsyntax-only", "-x", lang,
                    HEADER], check=True)


def test_c99_consumer_compiles_and_links(tmp_path):
    """A strict-C99 caller links against libllsr.so (tests/native/consumer_c.c; build only)."""
    exe = str(tmp_path / "consumer_c")
    libdir = os.path.dirname(llsr.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", os.path.join(REPO, "include"),
                    "-o", exe, os.path.join(REPO, "tests", "native", "consumer_c.c"), "-L", libdir, "-lllsr",
                    f"-Wl,-rpath,{libdir}"], check=True)
    assert os.path.exists(exe)


def test_cxx_consumer_is_built_in_tree():
    """The C++ consumer that tests/test_gpu_consumer.py runs on the GPU box is built by build()
    (lego-loam-sr_amd/Makefile) against the header and resolves libllsr.so."""
    exe = os.path.join(REPO, "tests", "native", "llsr_consumer")
    assert os.path.exists(exe)
    out = subprocess.run(["ldd", exe], check=True, capture_output=True, text=True).stdout
    assert "libllsr.so" in out and "not found" not in out
