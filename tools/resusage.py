"""Per-kernel register / scratch / occupancy summary of one translation unit
(hipcc -Rpass-analysis=kernel-resource-usage), demangled, one line per kernel.

    python tools/resusage.py csrc/engine.hip [name-filter ...]
"""
import re
import subprocess
import sys

SRC = sys.argv[1]
FILT = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-c", SRC, "-o", "/tmp/_ru.o",
       "-Rpass-analysis=kernel-resource-usage"]
if SRC.endswith("tnw.hip"):
    cmd[-3:-3] = ["-mllvm", "-amdgpu-mfma-vgpr-form=true"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs Spill|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).replace(" [bytes/lane]", "").replace(" [waves/SIMD]", "").replace(" [bytes/block]", "")] = int(m.group(2))
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    if FILT and not any(f in n for f in FILT):
        continue
    print(f"{n[:80]:80s} vgpr {r.get('VGPRs')} agpr {r.get('AGPRs')} spill {r.get('VGPRs Spill')} "
          f"scratch {r.get('ScratchSize')} occ {r.get('Occupancy')} lds {r.get('LDS Size')}")
