#!/bin/bash
# Round 6: tiled sweep -- the current build (unconditional staging loads) vs a timing-only probe without
# global loads (tools/variants/tile_noload.patch): per-launch kernel times by tiles per launch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06j
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gibbs_tiles.py \
  > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for v in cur:pynngp_amd/_build/libnngp_hip.so noload:ab/tile_noload/libnngp_hip.so; do
  label=${v%%:*}; lib=$(pwd)/${v#*:}
  for tn in 4096 2048 1024; do
    NNGP_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $o/${label}_${tn} -o run -- \
      python3 tools/bench_gibbs.py --iters 30 --warmup 10 --sweep tiled --tile-nodes $tn > $o/${label}_${tn}.json 2> $o/${label}_${tn}.err || exit 1
  done
done
python3 - $o <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for d in sorted(glob.glob(f'{o}/*_*/')):
    t = collections.defaultdict(list)
    col = []
    f = glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True)[0]
    for r in csv.DictReader(open(f)):
        dt = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        if 'gibbs_tile_phase' in r['Kernel_Name']:
            t[int(r['Grid_Size_X']) // 1024].append(dt)
        elif 'gibbs_w_color' in r['Kernel_Name']:
            col.append(dt)
    tot = sum(sum(v) for v in t.values()) / 140
    print(d, 'tile us per sweep', round(tot, 1), 'coarse colour launches per sweep', round(len(col) / 140, 1),
          'us', round(sum(col) / 140, 1), ' '.join(f'{k}:{round(sum(v)/len(v),1)}' for k, v in sorted(t.items(), reverse=True)))
PY
