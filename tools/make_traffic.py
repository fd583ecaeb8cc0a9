"""Turn a tools/gpu_provenance.sh run into committed roofline provenance for every bench preset.

    python tools/make_traffic.py <tag>

Reads gpurun_out/prov_<tag>/c<preset>/{trace,fetch,write,valuclass,valubusy} (rocprofv3 CSV output)
and writes
  * profiles/<tag>/c<preset>_kernel_stats.csv (the --kernel-trace --stats summary) and
    profiles/<tag>/summary.md + summary.json (per preset: the dominant kernels' average duration,
    HBM bytes per launch, VALU instructions per wave, the VALU class mix, VALU-active cycles per
    instruction and SIMD VALU busy);
  * profiles/traffic.json: one entry per preset kernel, which bench.py copies into the bench line's
    roofline.traffic and roofline_valu.
Presets the tag did not measure keep their entries in profiles/traffic.json.
HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024): on gfx950 FETCH_SIZE counts half the
bytes of 16-B-per-lane streaming reads, WRITE_SIZE counts 16-B stores exactly
(/opt/skills/guides/MI355X_MICROARCH.md, HBM / rocprofv3).  busy = sum over waves of VALU-active
cycles / (1,024 SIMDs x GRBM_GUI_ACTIVE / 8) (tools/valu_busy.py).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# preset -> (bench key fields, kernels: (role, name prefix))
PRESETS = {
    3: ({"n_per_gpu": 1_000_000, "m": 15, "kind": "exponential", "layout": "storage", "write_BF": True},
        [("sweep", "void nngp::bf_pairb<15, 0, 2, false>")]),
    2: ({"n_per_gpu": 100_000, "m": 15, "kind": "matern32", "layout": "storage", "write_BF": True},
        [("sweep", "void nngp::bf_pairb<15, 1, 2, false>")]),
    4: ({"n_per_gpu": 10_000_000, "m": 20, "kind": "exponential", "layout": "storage", "write_BF": True},
        [("sweep", "void nngp::bf_pairb<20, 0, 2, false>")]),
    5: ({"preset": 5, "n_per_gpu": 1_000_000, "m": 15, "kind": "exponential"},
        [("sweep", "void nngp::bf_pairb<15, 0, 2, false>"), ("colour", "void nngp::gibbs_w_color<false>")]),
}
BYTES_PER_LOC = {3: 36 * 15 + 32, 2: 36 * 15 + 32, 4: 36 * 20 + 32, 5: 36 * 15 + 32 + 8}
ROWS = {3: 1e6, 2: 1e5, 4: 1e7, 5: 1e6}


def counters(d, prefix):
    agg = collections.defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Kernel_Name"].startswith(prefix):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def stats(d):
    paths = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    return (paths[0], list(csv.DictReader(open(paths[0])))) if paths else (None, [])


def main():
    tag = sys.argv[1]
    base = os.path.join(ROOT, "gpurun_out", f"prov_{tag}")
    out_dir = os.path.join(ROOT, "profiles", tag)
    os.makedirs(out_dir, exist_ok=True)
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    doc = json.load(open(tpath)) if os.path.exists(tpath) else {"entries": []}
    doc["_doc"] = __doc__.split("\n\n")[0].strip() + " -- see tools/make_traffic.py for the definitions."

    def preset_of(e):
        for q, (key, _) in PRESETS.items():
            if all(e.get(k) == v for k, v in key.items()):
                return q
        return None

    ran = [p for p in PRESETS if os.path.isdir(os.path.join(base, f"c{p}"))]
    # the presets this tag measured are regenerated; the others keep their committed entries
    keep = [e for e in doc.get("entries", []) if preset_of(e) not in ran]
    summary, lines = {}, [f"# Roofline provenance `{tag}` (tools/gpu_provenance.sh + tools/make_traffic.py)", ""]
    for p, (key, kernels) in PRESETS.items():
        d = os.path.join(base, f"c{p}")
        if not os.path.isdir(d):
            continue
        spath, st = stats(os.path.join(d, "trace"))
        if spath:
            shutil.copy(spath, os.path.join(out_dir, f"c{p}_kernel_stats.csv"))
        args = open(os.path.join(d, "args.txt")).read().strip() if os.path.exists(os.path.join(d, "args.txt")) else ""
        lines += [f"## preset {p}: `{args}`", "", "| kernel | calls | avg us | share of kernel time |", "|---|---|---|---|"]
        for r in st[:6]:
            lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                         f"{float(r['Percentage']):.1f} % |")
        lines.append("")
        for role, prefix in kernels:
            row = next((r for r in st if r["Name"].startswith(prefix)), None)
            if row is None:
                continue
            fetch, nf = counters(os.path.join(d, "fetch"), prefix)
            write, nw = counters(os.path.join(d, "write"), prefix)
            cls, _ = counters(os.path.join(d, "valuclass"), prefix)
            busy, _ = counters(os.path.join(d, "valubusy"), prefix)
            e = dict(key)
            e.update({"kernel": prefix, "role": role, "avg_ns": float(row["AverageNs"]), "calls": int(row["Calls"]),
                      "source": f"profiles/{tag}", "source_tag": tag})
            if "FETCH_SIZE" in fetch and "WRITE_SIZE" in write:
                e["FETCH_SIZE_KB"], e["WRITE_SIZE_KB"] = fetch["FETCH_SIZE"], write["WRITE_SIZE"]
                e["bytes_per_launch"] = 2 * fetch["FETCH_SIZE"] * 1024 + write["WRITE_SIZE"] * 1024
                e["pmc_launches"] = [nf.get("FETCH_SIZE", 0), nw.get("WRITE_SIZE", 0)]
            if "SQ_INSTS_VALU" in cls and "SQ_WAVES" in cls:
                waves = cls["SQ_WAVES"]
                e["valu_per_wave"] = cls["SQ_INSTS_VALU"] / waves
                e["waves_per_launch"] = waves
                e["valu_mix_per_wave"] = {k[len("SQ_INSTS_VALU_"):]: v / waves for k, v in cls.items()
                                          if k.startswith("SQ_INSTS_VALU_")}
                if role == "sweep":
                    e["locations_per_wave"] = 32  # bf_pairb: two lanes per location
            if "SQ_ACTIVE_INST_VALU" in busy and "GRBM_GUI_ACTIVE" in busy and "valu_per_wave" in e:
                act = busy["SQ_ACTIVE_INST_VALU"] * 4 / busy["SQ_WAVES"]
                e["valu_active_cycles_per_instr"] = act / e["valu_per_wave"]
                e["simd_valu_busy"] = busy["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * busy["GRBM_GUI_ACTIVE"] / 8)
                e["wave_lifetime_cycles"] = busy["SQ_WAVE_CYCLES"] * 4 / busy["SQ_WAVES"]
                e["valu_source"] = (f"profiles/{tag} (rocprofv3 --pmc SQ_INSTS_VALU* class pass + SQ_ACTIVE_INST_VALU / "
                                    "GRBM_GUI_ACTIVE pass)")
            if role == "sweep":
                e["algorithmic_bytes_per_launch"] = BYTES_PER_LOC[p] * ROWS[p]
                e["algorithmic_hbm_frac"] = BYTES_PER_LOC[p] * ROWS[p] / (e["avg_ns"] * 1e-9) / 8e12
            keep.append(e)
            summary[f"c{p}_{role}"] = e
            lines += [f"- **{role}** `{prefix}`: {e['avg_ns'] / 1e3:.2f} us average over {e['calls']} launches"
                      + (f"; HBM {e['bytes_per_launch'] / 1e6:.1f} MB per launch (FETCH {e['FETCH_SIZE_KB']:.0f} KB x2 + "
                         f"WRITE {e['WRITE_SIZE_KB']:.0f} KB)" if "bytes_per_launch" in e else "")
                      + (f"; algorithmic {e['algorithmic_bytes_per_launch'] / 1e6:.0f} MB = "
                         f"{e['algorithmic_hbm_frac']:.3f} of 8 TB/s" if "algorithmic_hbm_frac" in e else "")
                      + (f"; {e['valu_per_wave']:.0f} VALU per wave" if "valu_per_wave" in e else "")
                      + (f", {e['valu_active_cycles_per_instr']:.2f} VALU-active cycles per instruction, SIMD VALU busy "
                         f"{e['simd_valu_busy']:.3f}" if "simd_valu_busy" in e else "")]
        lines.append("")
    doc["entries"] = keep
    json.dump(doc, open(tpath, "w"), indent=1)
    json.dump(summary, open(os.path.join(out_dir, "summary.json"), "w"), indent=1)
    open(os.path.join(out_dir, "summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
