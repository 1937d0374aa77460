"""Per-kernel resource usage of one HIP source (VGPRs, spills, scratch, occupancy, LDS) from the
compiler's kernel-resource-usage remarks: python scripts/kres.py lego-loam-sr_amd/csrc/llsr_fa.hip"""
import re
import subprocess
import sys

src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                      "-fPIC", "-c", src, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    name = re.sub(r"^_ZN4llsr\d+", "", k)[:40]
    print(f"{name:40s} vgpr {v.get('VGPRs', '?'):>4} spill {v.get('VGPRs Spill', '?'):>3} "
          f"scratch {v.get('ScratchSize [bytes/lane]', '?'):>4} occ {v.get('Occupancy [waves/SIMD]', '?'):>2} "
          f"lds {v.get('LDS Size [bytes/block]', '?')}")
