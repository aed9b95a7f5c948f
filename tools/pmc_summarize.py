#!/usr/bin/env python3
"""Summarise a gpu_profile.sh run into profiles/: per-kernel rocprofv3 stats and
the corrected HBM traffic of the full-search kernel.

gfx950 correction (/opt/skills/guides/MI355X_MICROARCH.md §HBM, cdna_hip_programming.md
§7): FETCH_SIZE (KiB) reads 1/2 of the bytes of a wide coalesced read stream, so
bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KiB) is exact for wide stores.
usage: pmc_summarize.py <round tag> [gpurun_out dir]"""
import csv, collections, json, os, shutil, sys
tag = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
dst = "profiles"
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "prof_trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
vals = collections.defaultdict(list)
for kind in ("fetch", "write"):
    path = os.path.join(src, f"prof_{kind}", "run_counter_collection.csv")
    shutil.copy(path, os.path.join(dst, f"{tag}_pmc_{kind}.csv"))
    for r in csv.DictReader(open(path)):
        vals[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
bench = open(os.path.join(src, "bench.log")).read()
b = json.loads(bench[bench.index("{"):])
cfg = b["config"]
out = {"tag": tag, "frames": cfg["frames_per_step_per_gpu"], "range": int(round(((cfg["candidates_per_mb"]) ** 0.5 - 1) / 2)),
       "width": 1920, "kernels": {}}
for (k, c), v in vals.items():
    out["kernels"].setdefault(k, {})[c] = sum(v) / len(v)
for k, d in out["kernels"].items():
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        d["hbm_bytes_corrected"] = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
    if "me_full_sad16" in k and "hbm_bytes_corrected" in d:
        out["hbm_bytes_per_launch"] = d["hbm_bytes_corrected"]
# per-dispatch durations of the headline kernel from the kernel trace: all
# dispatches, and the last `steps` ones (the bench's timed region follows its
# warmup launches of the same kernel; the GPU clock ramps during the first ~100)
KNAME = b["roofline"]["kernel"].split("<")[0]      # the headline kernel the bench names
durs = []
for r in csv.DictReader(open(os.path.join(src, "prof_trace", "run_kernel_trace.csv"))):
    if KNAME in r["Kernel_Name"]:
        durs.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3))
durs.sort()
# the headline leg runs first: its warmup then timed launches are the first warmup + steps
# dispatches of the kernel (the 2160p extra leg launches the same kernel later, per frame)
steps, warm = b["steps"], b["warmup"]
head = durs[:warm + steps]
timed = head[warm:]
trace = {"kernel": KNAME, "dispatches": len(durs), "headline_dispatches": len(head),
         "avg_us_headline_all": sum(d for _, d in head) / max(1, len(head)),
         "avg_us_timed_region": sum(d for _, d in timed) / max(1, len(timed)),
         "bench_event_launch_us": b["roofline"]["launch_ms"] * 1e3}
out["trace"] = trace
json.dump(trace, open(os.path.join(dst, f"{tag}_me_trace_summary.json"), "w"), indent=1)
json.dump(out, open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "bench.log"), os.path.join(dst, f"{tag}_bench.log"))
print(json.dumps(out, indent=1))
