# Same-box A/B with clock accounting (run via gpurun): for each variant, a kernel-trace run
# (average duration) and a GRBM/SQ counter run (busy cycles, wave cycles) of bench.py;
# effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md, DVFS).
#   bash tools/ab_clock.sh <tag> "<name>|<env>|<bench args>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for spec in "$@"; do
  IFS='|' read -r name envs args <<< "$spec"
  echo "== $name ($envs) $args"
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${name}_trace -o run -- \
    python3 bench.py --cpu-seconds 0 --steps 100 --warmup 100 $args > $out/${name}_trace.json 2> $out/${name}_trace.err || exit 1
  env $envs timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
    --output-format csv -d $out/${name}_pmc -o run -- python3 bench.py --cpu-seconds 0 --steps 100 --warmup 100 $args \
    > $out/${name}_pmc.json 2> $out/${name}_pmc.err || exit 1
done
python3 - "$out" "$@" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for spec in sys.argv[2:]:
    name = spec.split('|')[0]
    st = [r for r in csv.DictReader(open(glob.glob(f'{out}/{name}_trace/**/*kernel_stats.csv', recursive=True)[0]))
          if 'bf_' in r['Name'] and 'finalize' not in r['Name']]
    dur = float(st[0]['AverageNs'])
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(glob.glob(f'{out}/{name}_pmc/**/*counter_collection.csv', recursive=True)[0])):
        if 'bf_' in r['Kernel_Name'] and 'finalize' not in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    a = {k: sum(v) / len(v) for k, v in agg.items()}
    cyc = a['GRBM_GUI_ACTIVE'] / 8
    print(f"{name:14s} dur {dur/1e3:8.2f} us  cycles {cyc:9.0f}  clock {cyc/dur:5.3f} GHz  "
          f"VALU {a['SQ_INSTS_VALU']:.4g}  wave-cycles {a['SQ_WAVE_CYCLES']:.4g}  "
          f"slot-occupancy {a['SQ_WAVE_CYCLES']*4/cyc/2048:.3f}  waves {a['SQ_WAVES']:.0f}")
PY
