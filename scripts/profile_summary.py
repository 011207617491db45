"""Summarise a gpu_check.sh session into profiles/<tag>_*.{csv,json} (committed).

  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the bench headline
                           (`python3 bench.py --no-cpu --no-plan --no-side`: one launch shape)
  <tag>_kernel_stats_full.csv  the same over the whole bench (`--no-cpu`: plan + side legs)
  <tag>_traffic.json       HBM bytes per k_states launch from the FETCH_SIZE / WRITE_SIZE passes,
                           corrected as MI355X_MICROARCH.md prescribes: FETCH_SIZE counts half the
                           bytes of a wide (16 B/lane) streaming read on gfx950 -> x2; both in KB.
"""
import csv
import glob
import json
import os
import shutil
import sys

out_dir, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")
os.makedirs(prof, exist_ok=True)

for sub, suffix in (("prof", "kernel_stats"), ("prof_full", "kernel_stats_full"), ("prof_plan", "kernel_stats_planner")):
    stats = glob.glob(os.path.join(out_dir, sub, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_{suffix}.csv"))
        rows = list(csv.DictReader(open(stats[0])))
        print(f"-- {suffix}")
        for r in rows[:12]:
            print(r.get("Name", "")[:70], r.get("Calls"), r.get("AverageNs"))


def per_kernel(counter):
    files = glob.glob(os.path.join(out_dir, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            vals.setdefault(r["Kernel_Name"], []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"]),
                                                         int(r["Grid_Size"])))
    return vals


fetch, write = per_kernel("FETCH_SIZE"), per_kernel("WRITE_SIZE")
summary = {}
for name, v in fetch.items():
    if "k_states" not in name:
        continue
    w = write.get(name, [])
    # bench.py's timed launches are all the same 1,048,576-state shape: average them
    f_kb = sum(x[1] for x in v) / len(v)
    w_kb = sum(x[1] for x in w) / len(w) if w else 0.0
    summary[name] = {"launches": len(v), "fetch_size_kb": f_kb, "write_size_kb": w_kb,
                     "hbm_bytes_per_launch": 2 * f_kb * 1024 + w_kb * 1024,
                     "correction": "FETCH_SIZE x2 (gfx950 wide-load rule), WRITE_SIZE as read"}
json.dump(summary, open(os.path.join(prof, f"{tag}_traffic.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))

# The planner probe's steady state: its first pre_compute_traj call is the cold plan (a fresh
# generator: workspaces, the fallback areas' one-time whole-table warm-up searches, first
# launches).  <tag>_kernel_stats_planner_steady.csv drops every kernel before the second
# call's first k_pb_sample.
traces = glob.glob(os.path.join(out_dir, "prof_plan", "**", "*kernel_trace.csv"), recursive=True)
if traces:
    rows = sorted(csv.DictReader(open(traces[0])), key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in rows if "k_pb_sample" in r["Kernel_Name"]]
    if len(starts) > 1:
        cut = starts[1]  # (one batch per pre_compute_traj call: its 9 segments together)
        steady = [r for r in rows if int(r["Start_Timestamp"]) >= cut]
        agg = {}
        for r in steady:
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            a = agg.setdefault(r["Kernel_Name"], [0, 0, 1 << 62, 0])
            a[0] += 1
            a[1] += d
            a[2] = min(a[2], d)
            a[3] = max(a[3], d)
        tot = sum(a[1] for a in agg.values()) or 1
        path = os.path.join(prof, f"{tag}_kernel_stats_planner_steady.csv")
        with open(path, "w", newline="") as f:
            wr = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            wr.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for name, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
                wr.writerow([name, a[0], a[1], a[1] / a[0], 100.0 * a[1] / tot, a[2], a[3]])
        print(f"-- kernel_stats_planner_steady (from the second call: {len(steady)} of {len(rows)} dispatches)")
        for name, a in sorted(agg.items(), key=lambda kv: -kv[1][1])[:12]:
            print(name[:70], a[0], a[1] / a[0])
