"""Per-call timeline of the batched planner from a rocprofv3 SQLite output: for each
k_pb_sample (the start of a batch), the kernels on that stream until k_pb_emit, their
durations and the idle gaps between them (µs).  Usage: rocpd_timeline.py <db> [calls]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 3


def short(n):
    n = n.replace("void ", "").replace("epp::(anonymous namespace)::", "")
    return n.split("(")[0][:28]


shown, i, gaps_all, spans = 0, 0, [], []
while i < len(rows):
    if "k_pb_sample" not in rows[i][0]:
        i += 1
        continue
    st = rows[i][3]
    seq = [rows[i]]
    j = i + 1
    while j < len(rows) and "k_pb_emit" not in seq[-1][0]:
        if rows[j][3] == st:
            seq.append(rows[j])
        j += 1
    t0 = seq[0][1]
    gaps = sum(max(0, seq[k][1] - seq[k - 1][2]) for k in range(1, len(seq))) / 1e3
    gaps_all.append(gaps)
    spans.append((seq[-1][2] - t0) / 1e3)
    if shown < ncalls:
        print(f"batch at {t0 / 1e3:.1f} us: span {(seq[-1][2] - t0) / 1e3:.1f} us, idle gaps {gaps:.1f} us")
        prev = t0
        for n, s, e, _ in seq:
            print(f"   {short(n):28s} start +{(s - t0) / 1e3:7.1f}  dur {(e - s) / 1e3:6.1f}  gap {(s - prev) / 1e3:5.1f}")
            prev = e
        shown += 1
    i = j
if spans:
    spans.sort(), gaps_all.sort()
    print(f"{len(spans)} batches: span p50 {spans[len(spans) // 2]:.1f} us, idle gaps p50 {gaps_all[len(gaps_all) // 2]:.1f} us")
