# SQ stall breakdown for the bf kernels (one rocprofv3 --pmc pass per algo)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
for algo in ${ALGOS:-lane pair}; do
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/sq/$algo -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --algo $algo ${BENCH_ARGS:-} > gpurun_out/sq/$algo.json 2>>gpurun_out/sq/err.log || exit $?
python3 - "$algo" <<'PY'
import csv, collections, sys
algo = sys.argv[1]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f'gpurun_out/sq/{algo}/run_counter_collection.csv')):
    if 'bf_' in r['Kernel_Name'] and 'finalize' not in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
a = {k: sum(v) / len(v) for k, v in agg.items()}
w = a['SQ_WAVE_CYCLES']
print(algo, 'waves', a['SQ_WAVES'], 'VALU/wave', round(a['SQ_INSTS_VALU'] / a['SQ_WAVES']),
      'active %.2f inst-wait %.2f mem-wait %.2f' % (a['SQ_ACTIVE_INST_ANY'] / w, a['SQ_WAIT_INST_ANY'] / w, a['SQ_WAIT_ANY'] / w),
      'busy', a['SQ_BUSY_CYCLES'])
PY
done
