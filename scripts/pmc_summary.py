"""Per-kernel mean of rocprofv3 --pmc counters (diagnostics): argv[1] = a rocprofv3 output
directory (counter_collection.csv inside, any depth), argv[2] = kernel-name regex filter."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

files = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in files:
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if pat and not pat.search(name):
            continue
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for name, cs in acc.items():
    n = max(1, len(disp[name]))
    print(f"{name[:90]}  (dispatches {n})")
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {v / n:16.1f}")
