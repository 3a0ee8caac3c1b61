"""Per-kernel register / spill / LDS summary of one HIP source (compile-time
resource remarks).  usage: python tools/kres.py csrc/pe_batch.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-mllvm", "-amdgpu-atomic-optimizer-strategy=DPP",
       "-fPIC", "-std=c++17", "-I../include", "-Icsrc", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{k[:70]:70s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} vspill={v.get('VGPRs Spill')} "
              f"sspill={v.get('SGPRs Spill')} occ={v.get('Occupancy [waves/SIMD]')} scratch={v.get('ScratchSize [bytes/lane]')}")
