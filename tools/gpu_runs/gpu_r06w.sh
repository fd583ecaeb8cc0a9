#!/bin/bash
# Round 6: the whole GPU suite, smoke and the bench at the driver's flags (headline and config 5) on the
# current tree (pruned pair kernel, tiled Gibbs sweep)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/${TAG:-r06w}
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --durations=15 --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -3 $o/tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { tail -20 $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench_driver.json 2> $o/bench_driver.err || exit 1
python3 -c "import json; d=json.load(open('$o/bench_driver.json')); r=d['roofline']; print('driver', round(d['value']/1e9,3), 'Gloc/s', round(d['ms_per_step'],4), 'ms', 'kernel_ms', round(r['kernel_ms'],4), r['kernel_ms_samples'], 'loop', round(r['kernel_ms_loop'],4), 'frac', round(r['frac'],3))"
timeout -k 10 300 python bench.py --config 5 --steps 300 --warmup 100 --cpu-seconds 0 > $o/bench_config5.json 2> $o/bench_config5.err || exit 1
timeout -k 10 300 python bench.py --config 5 --steps 300 --warmup 100 --cpu-seconds 0 --gibbs-sweep tiled > $o/bench_config5_tiled.json 2> $o/bench_config5_tiled.err || exit 1
for f in bench_config5 bench_config5_tiled; do python3 -c "import json; d=json.load(open('$o/$f.json')); b=d['breakdown']; print('$f', round(d['value'],1), 'it/s', round(d['ms_per_step'],4), 'ms', 'w_sweep', round(b['w_sweep_ms'],4), b.get('w_sweep'))"; done
