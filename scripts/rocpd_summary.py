"""Per-kernel time summary of a rocprofv3 SQLite (rocpd) output: name, calls, average /
max µs, share; plus memory copies.  Usage: rocpd_summary.py <results.db> [name filter]"""
import re
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
agg = defaultdict(list)
for n, s, e in rows:
    if flt in n:
        agg[n].append((e - s) / 1e3)
tot = sum(sum(v) for v in agg.values())
for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    short = re.sub(r"^void ", "", n).replace("epp::(anonymous namespace)::", "")
    short = short[:short.index("(", short.index(">") if "<" in short.split("(")[0] else 0)] if "(" in short else short
    print(f"{short[:60]:60s} {len(v):6d} {sum(v)/len(v):9.1f} {max(v):9.1f} {100*sum(v)/tot:6.1f}%")
try:
    mc = c.execute("select start, end, size from memory_copies").fetchall()
    if mc:
        d = [(e - s) / 1e3 for s, e, _ in mc]
        print(f"memory copies: {len(mc)}, avg {sum(d)/len(d):.1f} us, max {max(d):.1f} us, bytes avg {sum(x[2] for x in mc)/len(mc):.0f}")
except sqlite3.Error as e:
    print("memory copies:", e)
