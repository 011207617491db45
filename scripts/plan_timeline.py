"""Timeline of the planner's device pipeline (diagnostics): reads a rocprofv3 kernel +
memory-copy trace of `scripts/plan_probe.py` (one planner thread) and prints, for the
last `samples`-state segment plans, every kernel and copy with its start relative to the
segment's first event, its duration and the idle gap before it; then the per-segment
totals (busy vs idle) as medians over the segments.

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_plan \
      -o run -- python3 scripts/plan_probe.py --child
  python3 scripts/plan_timeline.py gpurun_out/prof_plan
"""
import csv
import glob
import os
import sys

import numpy as np


def short(name):
    n = name.replace("epp::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:44]


def main():
    d = sys.argv[1]
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Thread_Id"])))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kind = r.get("Direction") or r.get("Operation") or "copy"
            size = r.get("Size") or r.get("Bytes") or ""
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"COPY {kind} {size}", int(r.get("Thread_Id", 0) or 0)))
    ev.sort()
    # segments start at k_sample_uniform
    starts = [i for i, e in enumerate(ev) if e[2].startswith("k_sample_uniform")]
    segs = []
    for a, b in zip(starts, starts[1:] + [len(ev)]):
        segs.append(ev[a:b])
    if not segs:
        print("no k_sample_uniform found")
        return
    # the last segment in full
    show = segs[-2] if len(segs) > 1 else segs[-1]
    t0 = show[0][0]
    prev_end = t0
    print(f"{'event':46s} {'start_us':>9s} {'dur_us':>8s} {'gap_us':>8s}")
    for s, e, n, _ in show:
        print(f"{n:46s} {(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} {(s - prev_end) / 1e3:8.2f}")
        prev_end = max(prev_end, e)
    busy, span, gaps = [], [], {}
    for sg in segs[:-1]:
        t0 = sg[0][0]
        end = max(e for _, e, _, _ in sg)
        b, pe = 0, t0
        for s, e, n, _ in sg:
            b += max(0, e - max(s, pe))
            g = s - pe
            if g > 0:
                gaps.setdefault(n, []).append(g)
            pe = max(pe, e)
        busy.append(b)
        span.append(end - t0)
    print(f"segments {len(segs) - 1}: span p50 {np.median(span) / 1e3:.1f} us, busy p50 {np.median(busy) / 1e3:.1f} us")
    for n, g in sorted(gaps.items(), key=lambda kv: -np.median(kv[1]))[:10]:
        print(f"  gap before {n:44s} p50 {np.median(g) / 1e3:7.2f} us (n={len(g)})")


if __name__ == "__main__":
    main()
