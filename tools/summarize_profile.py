"""Summarise a tools/profile.sh run into profiles/<tag>_summary.md (+ json).

Reads gpurun_out/prof_<tag>/{trace,pmc_fetch,pmc_write,pmc_sq}/ and reports, for the
dominant sweep kernel: rocprofv3 average duration, FETCH_SIZE / WRITE_SIZE per
launch (KB, as reported) and HBM bytes with the gfx950 correction of
MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of 16-B-per-lane reads:
x2 on the fetch side; WRITE_SIZE exact), and the SQ stall breakdown.
    python tools/summarize_profile.py <tag> [bytes_per_location] [rows]
"""
import collections
import csv
import json
import os
import sys

tag = sys.argv[1]
bpl = float(sys.argv[2]) if len(sys.argv) > 2 else 572.0
rows = float(sys.argv[3]) if len(sys.argv) > 3 else 1e6
base = os.path.join("gpurun_out", f"prof_{tag}")
stats = list(csv.DictReader(open(os.path.join(base, "trace", "run_kernel_stats.csv"))))
hot = max((r for r in stats if "bf_" in r["Name"] and "finalize" not in r["Name"]),
          key=lambda r: float(r["TotalDurationNs"]))
hot_key = hot["Name"].split("(")[0]


def pmc(sub):
    path = os.path.join(base, sub, "run_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].split("(")[0] == hot_key:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


fetch = pmc("pmc_fetch").get("FETCH_SIZE")
write = pmc("pmc_write").get("WRITE_SIZE")
sq = pmc("pmc_sq")
avg_ns = float(hot["AverageNs"])
out = {"tag": tag, "kernel": hot_key, "calls": int(hot["Calls"]), "avg_ns": avg_ns,
       "algorithmic_bytes": bpl * rows, "algorithmic_GBps": bpl * rows / avg_ns}
if fetch is not None and write is not None:
    hbm = 2 * fetch * 1024 + write * 1024
    out.update({"FETCH_SIZE_KB": fetch, "WRITE_SIZE_KB": write, "hbm_bytes_corrected": hbm,
                "hbm_GBps": hbm / avg_ns})
if sq:
    w = sq["SQ_WAVE_CYCLES"]
    out.update({"sq_active": sq["SQ_ACTIVE_INST_ANY"] / w, "sq_wait_inst": sq["SQ_WAIT_INST_ANY"] / w,
                "sq_wait_any": sq["SQ_WAIT_ANY"] / w, "valu_per_wave": sq["SQ_INSTS_VALU"] / sq["SQ_WAVES"]})
os.makedirs(os.path.join("profiles", tag), exist_ok=True)
json.dump(out, open(os.path.join("profiles", tag, "summary.json"), "w"), indent=1)
lines = [f"# rocprofv3 summary `{tag}`", "",
         f"command: `python3 bench.py {open(os.path.join(base, 'args.txt')).read().strip() if os.path.exists(os.path.join(base, 'args.txt')) else ''}`", "",
         "## kernel stats (`rocprofv3 --kernel-trace --stats`)", "",
         "| kernel | calls | avg ns | total ns | % |", "|---|---|---|---|---|"]
for r in stats[:10]:
    lines.append(f"| `{r['Name'][:100]}` | {r['Calls']} | {float(r['AverageNs']):.0f} | {r['TotalDurationNs']} | "
                 f"{float(r['Percentage']):.2f} |")
lines += ["", "## dominant kernel", ""] + [f"- {k}: {v}" for k, v in out.items()]
open(os.path.join("profiles", tag, "summary.md"), "w").write("\n".join(lines) + "\n")
print(json.dumps(out))
