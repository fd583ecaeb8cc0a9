#!/bin/bash
# Round 6: wave pair plans -- plan parity tests, same-box A/B (duration, VALU, clock) of the planned and
# unplanned kernels at configs 3 and 2, then per-wave LDS / wait counters and FETCH / WRITE of both at config 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/${TAG:-r06a}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1 || { tail -30 $o/pytest.txt; exit 1; }
tail -1 $o/pytest.txt
bash tools/ab_clock.sh ${TAG:-r06a} "c3_off||--plan off" "c3_on||--plan on" || exit 1
for p in off on; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES \
    --output-format csv -d $o/lds_$p -o run -- python3 bench.py --plan $p --steps 30 --warmup 30 --cpu-seconds 0 > $o/lds_$p.json 2> $o/lds_$p.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
    --output-format csv -d $o/wait_$p -o run -- python3 bench.py --plan $p --steps 30 --warmup 30 --cpu-seconds 0 > $o/wait_$p.json 2> $o/wait_$p.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch_$p -o run -- \
    python3 bench.py --plan $p --steps 30 --warmup 30 --cpu-seconds 0 > $o/fetch_$p.json 2> $o/fetch_$p.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/write_$p -o run -- \
    python3 bench.py --plan $p --steps 30 --warmup 30 --cpu-seconds 0 > $o/write_$p.json 2> $o/write_$p.err || exit 1
done
python3 - "$o" <<'PY'
import csv, glob, collections, sys
o = sys.argv[1]
for p in ("off", "on"):
    agg = collections.defaultdict(list)
    for d in (f"{o}/lds_{p}", f"{o}/wait_{p}", f"{o}/fetch_{p}", f"{o}/write_{p}"):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "bf_pairb" in r["Kernel_Name"] and (p == "off" or "true>" in r["Kernel_Name"]):
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    a = {k: sum(v) / len(v) for k, v in agg.items()}
    w = a.get("SQ_WAVES", 1)
    per_wave = {k: round(v / w, 1) for k, v in sorted(a.items())
                if k not in ("SQ_WAVES", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES", "FETCH_SIZE", "WRITE_SIZE")}
    print(p, "per wave", per_wave)
    print(p, "FETCH_SIZE kB/launch (x2 gfx950 streaming correction not applied)", a.get("FETCH_SIZE"),
          "WRITE_SIZE kB/launch", a.get("WRITE_SIZE"))
PY
