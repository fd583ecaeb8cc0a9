"""Print a rocprofv3 output directory's per-kernel summary (run on the GPU box or here).

    python tools/pmc_summary.py <rocprofv3 -d dir>

Kernel trace: the top kernels of run_kernel_stats.csv.  Counter collection: the mean
of every counter per kernel name (first 60 characters), plus derived SQ ratios
(active / wait_inst / wait_any per wave-cycle, VALU instructions per wave).
"""
import collections
import csv
import glob
import os
import sys

base = sys.argv[1]
for path in glob.glob(os.path.join(base, "**", "*kernel_stats.csv"), recursive=True):
    rows = list(csv.DictReader(open(path)))
    for r in rows[:6]:
        print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:9.2f} us "
              f"{float(r['Percentage']):6.2f} %")
for path in glob.glob(os.path.join(base, "**", "*counter_collection.csv"), recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        if "SQ_WAVES" in a and a["SQ_WAVES"] < 1000:
            continue  # tiny helper kernels
        print(f"  {k}")
        print("    " + "  ".join(f"{c}={v:.6g}" for c, v in sorted(a.items())))
        w = a.get("SQ_WAVE_CYCLES")
        if w:
            print(f"    active {a.get('SQ_ACTIVE_INST_ANY', 0) / w:.3f} wait_inst {a.get('SQ_WAIT_INST_ANY', 0) / w:.3f} "
                  f"wait_any {a.get('SQ_WAIT_ANY', 0) / w:.3f} valu_active {a.get('SQ_ACTIVE_INST_VALU', 0) / w:.3f} "
                  f"valu/wave {a.get('SQ_INSTS_VALU', 0) / max(a.get('SQ_WAVES', 1), 1):.1f}")
