"""Per-kernel resources of the SHIPPED library (the -fgpu-rdc-linked code objects inside libllsr.so),
read from the code objects' AMDGPU metadata notes: VGPRs, AGPRs, SGPRs, scratch (private segment)
bytes per lane, static LDS, max workgroup size and the waves per SIMD the registers allow. These are
the figures of the code the bench runs (a standalone compile of one source can differ: the device
link inlines across files and re-allocates registers).

    python scripts/kres_linked.py [lego-loam-sr_amd/libllsr.so] [> profiles/<tag>_kernel_resources.json]
"""
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "lego-loam-sr_amd",
                                                          "libllsr.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def waves_per_simd(vgpr, agpr):
    # gfx950 unified register file: 512 per lane per SIMD, allocated in blocks of 8 (MI355X_MICROARCH.md)
    tot = ((vgpr + 7) // 8) * 8 + ((agpr + 7) // 8) * 8 if agpr else ((vgpr + 7) // 8) * 8
    return min(8, 512 // max(tot, 8))


with tempfile.TemporaryDirectory() as td:
    fb = os.path.join(td, "fatbin.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
    blob = open(fb, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)] + [len(blob)]
    kernels = {}
    for k, (s, e) in enumerate(zip(starts[:-1], starts[1:])):
        part = os.path.join(td, f"b{k}.bin")
        open(part, "wb").write(blob[s:e])
        co = os.path.join(td, f"co{k}.o")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode != 0 or not os.path.getsize(co):
            continue
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
        # one YAML block per kernel, fields in alphabetical order: split at each '- .agpr_count'
        for blk in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
            blk = ".agpr_count:" + blk
            f = dict(re.findall(r"\.(\w+):\s+([^\n]+)", blk))
            name = f.get("name", "").strip()
            if not name.startswith("_Z") or name.startswith("_ZN7rocprim"):
                continue  # (rocPRIM's own kernels, linked in by llsr_map.hip, are left out)
            short = re.sub(r"^_ZN4llsr\d+", "", name)
            short = re.sub(r"ENS_.*|EEEvNS_.*|Ev$", "", short)
            vg, ag = int(f.get("vgpr_count", 0)), int(f.get("agpr_count", 0))
            kernels[name] = {"kernel": short, "code_object": k, "vgpr": vg, "agpr": ag,
                             "sgpr": int(f.get("sgpr_count", 0)),
                             "scratch_bytes_per_lane": int(f.get("private_segment_fixed_size", 0)),
                             "lds_bytes": int(f.get("group_segment_fixed_size", 0)),
                             "max_workgroup": int(f.get("max_flat_workgroup_size", 0)),
                             "waves_per_simd_by_registers": waves_per_simd(vg, ag),
                             "sgpr_spill": int(f.get("sgpr_spill_count", 0)),
                             "vgpr_spill": int(f.get("vgpr_spill_count", 0))}
bid = subprocess.run(["python3", "-c", "import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); "
                      "L.llsr_build_id.restype=ctypes.c_char_p; print(L.llsr_build_id().decode())", lib],
                     capture_output=True, text=True).stdout.strip()
print(json.dumps({"library": os.path.basename(lib), "build_id": bid,
                  "kernels": dict(sorted(((v["kernel"], v) for v in kernels.values()), key=lambda kv: kv[0]))},
                 indent=1))
