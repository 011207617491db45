"""VALU roofline of the C3 motion kernels (round 6): reads the rocprofv3 --pmc passes of
scripts/gpu_pmc_motions.sh (gpurun_out/mpmc1..3) and the kernel trace of the same program
(gpurun_out/mkt), and writes per kernel: the SQ counters per launch, the average launch
duration, and

  valu_issue_frac = VALU issue cycles / (duration x 2.4 GHz x 1024 SIMDs), with 2 cycles per
                    32-bit VALU instruction and 4 per FP64 one (16 lanes per cycle: 78.6 TF
                    FP64 vector = half the 157.3 TF FP32 rate, MI355X_MICROARCH.md);
  fp64_frac       = FP64 flops (64 lanes x (add + mul + 2 fma + trans)) / duration / 78.6 TF;
  hbm_frac        = 49 B per edge x 1,048,576 / duration / 8 TB/s.

    python scripts/motions_valu.py OUT.json   (bench.py reads the newest profiles/r*_motions_valu.json)
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
CLOCK_HZ, SIMDS = 2.4e9, 1024
FP64_PEAK, HBM_PEAK = 78.6e12, 8.0e12
EDGES, BYTES_PER_EDGE = 1 << 20, 49


def counters():
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for d in ("mpmc1", "mpmc2", "mpmc3"):
        for f in glob.glob(os.path.join(OUT, d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                if "k_motions_v5" not in name:
                    continue
                c = r["Counter_Name"]
                acc[name][c] += float(r["Counter_Value"])
                # (dispatch ids restart in every pass's run: a counter in two passes is
                # averaged over both runs' dispatches)
                disp[name][c].add((d, r.get("Dispatch_Id", r.get("Correlation_Id", ""))))
    return {n: {c: v / max(1, len(disp[n][c])) for c, v in cs.items()} for n, cs in acc.items()}


def durations():
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(OUT, "mkt", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if "k_motions_v5" in name:
                acc[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {n: sum(v) / len(v) for n, v in acc.items()}


def short(name):
    m = re.search(r"k_motions_v5<([^>]*)>", name)
    return f"k_motions_v5<{m.group(1)}>" if m else name


def main():
    cs, ds = counters(), durations()
    out = {}
    for name, c in cs.items():
        key = short(name)
        dur = next((v for n, v in ds.items() if short(n) == key), None)
        fp64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                           "SQ_INSTS_VALU_TRANS_F64"))
        flops = 64 * (c.get("SQ_INSTS_VALU_ADD_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0) +
                      2 * c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_TRANS_F64", 0))
        valu = c.get("SQ_INSTS_VALU", 0.0)
        e = {"mode": "analytic" if ", 0," in key else "discrete32", "counters_per_launch": c,
             "valu_insts_per_launch": valu, "fp64_insts_per_launch": fp64, "fp64_flops_per_launch": flops,
             "valu_issue_cycles_per_launch": 2 * (valu - fp64) + 4 * fp64}
        if dur:
            s = dur * 1e-9
            e.update(kernel_ns=dur, valu_issue_frac=e["valu_issue_cycles_per_launch"] / (s * CLOCK_HZ * SIMDS),
                     fp64_frac=flops / s / FP64_PEAK, hbm_frac=BYTES_PER_EDGE * EDGES / s / HBM_PEAK)
        out[key] = e
    dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(OUT, "motions_valu.json")
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    for k, e in sorted(out.items()):
        print(k, {x: e.get(x) for x in ("kernel_ns", "valu_insts_per_launch", "valu_issue_frac", "fp64_frac",
                                         "hbm_frac")})


if __name__ == "__main__":
    main()
