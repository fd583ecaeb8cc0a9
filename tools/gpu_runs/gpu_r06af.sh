#!/bin/bash
# round 6: member-row bound checks in the colour sweep wrappers (tests; config 5 unchanged)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
o=gpurun_out/r06af
mkdir -p $o
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gibbs.py tests/test_gpu_gibbs_chains.py tests/test_gpu_gibbs_sharded.py tests/test_gpu_gibbs_tiles.py tests/test_gpu_gibbs_ref.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
timeout -k 10 300 python bench.py --config 5 --steps 300 --warmup 100 --cpu-seconds 0 > $o/bench_config5.json 2> $o/bench_config5.err || exit 1
python3 -c "import json; d=json.load(open('$o/bench_config5.json')); print('config5', round(d['value'],1), 'it/s', round(d['ms_per_step'],4), 'ms')"
