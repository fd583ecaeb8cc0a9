#!/bin/bash
# Round 5: the batched chains' colour kernel -- chain tests, then its VALU busy / per-wave counters at C = 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05u
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_gibbs_chains.py tests/test_gpu_bench.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1; rc=$?
grep -E "^(FAILED|ERROR)" $o/pytest.txt | head; tail -1 $o/pytest.txt
case $rc in 0) ;; *) exit $rc;; esac
A="--config 5 --chains-per-gpu 4 --chain-mode batched --cpu-seconds 0 --steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python3 bench.py $A > $o/trace.json 2> $o/trace.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d $o/valubusy -o run -- python3 bench.py $A > $o/valubusy.json 2> $o/valubusy.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- python3 bench.py $A > $o/fetch.json 2> $o/fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/write -o run -- python3 bench.py $A > $o/write.json 2> $o/write.err || exit 1
python3 - <<'PY'
import csv, glob, collections
o = "gpurun_out/r05u"
st = [r for r in csv.DictReader(open(glob.glob(o + "/trace/**/*kernel_stats.csv", recursive=True)[0]))]
for r in st:
    if "gibbs_w_color_chains_il" in r["Name"]:
        print("avg_us", float(r["AverageNs"]) / 1e3, "calls", r["Calls"])
agg = collections.defaultdict(list)
for d in ("valubusy", "fetch", "write"):
    for f in glob.glob(f"{o}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gibbs_w_color_chains_il" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
a = {k: sum(v) / len(v) for k, v in agg.items()}
w = a["SQ_WAVES"]
busy = a["SQ_ACTIVE_INST_VALU"] / (1024 * a["GRBM_GUI_ACTIVE"] / 8)
print({"valu_per_wave": a["SQ_INSTS_VALU"] / w, "wave_cycles": a["SQ_WAVE_CYCLES"] / w, "simd_valu_busy": busy,
       "hbm_MB": (2 * a["FETCH_SIZE"] + a["WRITE_SIZE"]) * 1024 / 1e6, "waves": w})
PY
