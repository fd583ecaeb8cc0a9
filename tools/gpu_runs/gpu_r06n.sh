#!/bin/bash
# Round 6: the general-nu Matern kind left-looking at one wave per SIMD (tools/variants/matern_left.patch)
# against the current right-looking kernel, m = 18..24 at N = 10^6 (nu = 1.3), same box, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06n
mkdir -p $o
for m in 18 19 20 21 22 23 24; do
  for r in 1 2; do for v in cur:pynngp_amd/_build/libnngp_hip.so left:ab/matern_left/libnngp_hip.so; do
    label=${v%%:*}; lib=$(pwd)/${v#*:}
    NNGP_LIB=$lib timeout -k 10 120 python bench.py --steps 30 --warmup 30 --cpu-seconds 0 --kind matern --nu 1.3 --m $m --n 1000000 \
      > $o/${label}_m$m.$r.json 2>> $o/err.log || exit 1
  done; done
done
python3 - $o <<'PY'
import glob, json, collections, statistics, sys
o = sys.argv[1]
t = collections.defaultdict(list)
for f in glob.glob(f'{o}/*.json'):
    d = json.load(open(f))
    t[f.split('/')[-1].rsplit('.', 2)[0]].append((d['roofline']['kernel_ms'], d['loglik']))
for k, v in sorted(t.items()):
    print(k, 'kernel ms', round(statistics.median([a for a, _ in v]), 4), 'loglik', v[0][1])
PY
