"""Per-kernel VGPR / spill / scratch summary of one HIP source (gfx950),
from clang's kernel-resource-usage remarks: tools/kres_diff.py <src.hip> <incdir>... [filter]"""
import re, subprocess, sys
src, rest = sys.argv[1], sys.argv[2:]
flt = rest.pop() if rest and not rest[-1].startswith("/") and not rest[-1].startswith(".") else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-mllvm", "-amdgpu-atomic-optimizer-strategy=DPP",
       "-std=c++17", "--cuda-device-only", "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
cmd += ["-I" + d for d in rest]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark: +([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+)", line)
    if m and cur: rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{k[:70]:70s} VGPR {v.get('VGPRs','?'):>4} AGPR {v.get('AGPRs','?'):>4} spillV {v.get('VGPRs Spill','?'):>4} scratch {v.get('ScratchSize','?'):>5}")
