#!/usr/bin/env python3
"""Interleaved A/B of library builds on one leg: lib_ab.py LEG STEPS ROUNDS KEY LIB [LIB ...]
runs tools/leg_time.py LEG STEPS once per library per round (X264HIP_LIBRARY = LIB; "default"
= the in-tree build) and prints KEY of every run plus the per-library median."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    leg, steps, rounds, key = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    libs = sys.argv[5:]
    got = {l: [] for l in libs}
    for r in range(rounds):
        for l in libs:
            env = dict(os.environ)
            if l != "default":
                env["X264HIP_LIBRARY"] = os.path.join(ROOT, l)
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "leg_time.py"), leg, steps],
                                 env=env, capture_output=True, text=True, timeout=300)
            if out.returncode:
                print(out.stdout[-2000:], out.stderr[-2000:])
                sys.exit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            got[l].append(d[key])
            print(r, l, {k: v for k, v in d.items() if k.endswith("_ms")}, flush=True)
    for l in libs:
        print("median", l, key, statistics.median(got[l]), got[l])


if __name__ == "__main__":
    main()
