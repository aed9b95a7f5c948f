#!/usr/bin/env python3
"""Print VGPR / SGPR / scratch / occupancy per kernel of a .hip file (gfx950)."""
import re, subprocess, sys
src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I../../include",
                      "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for ln in out.splitlines():
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", ln)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    d = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    d = re.sub(r"x264hip::|typename |PT<\d+>::", "", d)[:90]
    print(f"{d:90s} vgpr={v.get('VGPRs')} sgpr={v.get('TotalSGPRs')} scratch={v.get('ScratchSize')} occ={v.get('Occupancy')} lds={v.get('LDS')}")
for ln in out.splitlines():
    if "error" in ln or "warning: loop not unrolled" in ln:
        print(ln)
