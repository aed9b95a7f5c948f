#!/usr/bin/env python3
"""Instruction histogram of one kernel: isa_hist.py <file.hip> <substring of mangled name> [n]"""
import subprocess, sys, collections, os, re
src, pat = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I../../include", "-c", src,
                "-o", f"/tmp/asm/{os.path.splitext(os.path.basename(src))[0]}.o", "-save-temps=obj"], check=True, capture_output=True)
base = os.path.splitext(os.path.basename(src))[0]
s = open(f"/tmp/asm/{base}-hip-amdgcn-amd-amdhsa-gfx950.s").read()
names = re.findall(r"^(_Z\S+):", s, re.M)
for name in names:
    if pat not in name:
        continue
    i = s.index(name + ":"); j = s.index(".Lfunc_end", i)
    lines = [l.strip() for l in s[i:j].split("\n") if l.strip() and not l.strip().startswith((";", ".", "_Z"))]
    c = collections.Counter(l.split()[0] for l in lines)
    print(name, "total", sum(c.values()))
    print("  " + "  ".join(f"{k}:{v}" for k, v in c.most_common(n)))
