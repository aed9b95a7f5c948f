#!/usr/bin/env python3
"""Interleaved A/B of an environment switch on one leg: env_ab.py LEG STEPS ROUNDS VAR V1 [V2 ...]
runs tools/leg_time.py LEG STEPS once per value per round (VAR=value) and prints every run's
*_ms keys plus the per-value medians."""
import ast  # noqa: F401
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    leg, steps, rounds, var = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    vals = sys.argv[5:]
    got = {}
    for r in range(rounds):
        for v in vals:
            env = dict(os.environ, **{var: v})
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "leg_time.py"), leg, steps],
                                 env=env, capture_output=True, text=True, timeout=300)
            if out.returncode:
                print(out.stdout[-2000:], out.stderr[-2000:])
                sys.exit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            ms = {k: x for k, x in d.items() if k.endswith("_ms")}
            for k, x in ms.items():
                got.setdefault((v, k), []).append(x)
            print(r, v, ms, flush=True)
    for (v, k), xs in sorted(got.items()):
        print("median", var, v, k, round(statistics.median(xs), 4))


if __name__ == "__main__":
    main()
