#!/bin/bash
# Round 6: the whole GPU suite, smoke and the bench at the driver's flags on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/${TAG:-r06d}
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --durations=15 --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -3 $o/tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { tail -20 $o/smoke.txt; exit 1; }
tail -2 $o/smoke.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench_driver.json 2> $o/bench_driver.err || exit 1
python3 -c "import json; d=json.load(open('$o/bench_driver.json')); r=d['roofline']; print('driver', round(d['value']/1e9,3), 'Gloc/s', round(d['ms_per_step'],4), 'ms', 'kernel_ms', round(r['kernel_ms'],4), r['kernel_ms_samples'], 'loop', round(r['kernel_ms_loop'],4), 'frac', round(r['frac'],3))"
