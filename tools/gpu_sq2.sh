# SQ / LDS counter passes for the bench's sweep kernel (run on the GPU box via gpurun).
#   bash tools/gpu_sq2.sh [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/sq2
mkdir -p $out
args="--steps 5 --warmup 1 --cpu-seconds 0 $*"
[ -f $out/counters.txt ] || timeout -s KILL 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
i=0
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $out/p$i -o run -- python3 bench.py $args > $out/p$i.json 2> $out/p$i.err || exit $?
done
python3 - <<'PY'
import csv, collections, glob
agg = collections.defaultdict(list)
for f in glob.glob('gpurun_out/sq2/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if 'bf_' in k and 'finalize' not in k:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
a = {k: sum(v) / len(v) for k, v in agg.items()}
for k in sorted(a): print(f'{k:28s} {a[k]:.6g}')
w = a.get('SQ_WAVE_CYCLES', 1)
print('per-wave VALU', a['SQ_INSTS_VALU'] / a['SQ_WAVES'], 'active', a['SQ_ACTIVE_INST_ANY'] / w,
      'wait_inst', a['SQ_WAIT_INST_ANY'] / w, 'wait_any', a['SQ_WAIT_ANY'] / w)
PY
