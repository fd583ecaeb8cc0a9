# A/B timing of library builds on the Gibbs iteration (tools/bench_gibbs.py), one GPU box.
#   VARIANTS="label:libpath ..." REPS=3 bash tools/gpu_ab_gibbs.sh [bench_gibbs args...]
# Interleaved repetitions; prints ms per iteration per run and the median per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/abg; mkdir -p gpurun_out/abg
for rep in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    label=${v%%:*}; lib=${v#*:}
    NNGP_LIB=$lib timeout -k 10 120 python tools/bench_gibbs.py "$@" \
      > gpurun_out/abg/$label.$rep.json 2>> gpurun_out/abg/err.log || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/abg/$label.$rep.json')); print('$label', $rep, round(d['ms_per_iter'],4), 'ms/iter')"
  done
done
python3 - <<'PY'
import glob, json, collections, statistics
t = collections.defaultdict(list)
for f in glob.glob('gpurun_out/abg/*.json'):
    t[f.split('/')[-1].rsplit('.', 2)[0]].append(json.load(open(f))['ms_per_iter'])
for k, v in sorted(t.items()):
    print('median', k, round(statistics.median(v), 4), 'ms over', len(v))
PY
