#!/bin/bash
# Round 4: member records for the one-GPU Gibbs chain -- GPU tests, same-box A/B, colour-kernel profile.
set -euo pipefail
mkdir -p gpurun_out/r04i
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gibbs_members.py \
  tests/test_gpu_gibbs.py tests/test_gpu_gibbs_ref.py tests/test_gpu_gibbs_sharded.py > gpurun_out/r04i/pytest.txt 2>&1
for k in 1 2; do
  timeout -k 10 300 python tools/bench_gibbs.py --iters 200 --warmup 100 > gpurun_out/r04i/ab_members_$k.json
  timeout -k 10 300 python tools/bench_gibbs.py --iters 200 --warmup 100 --node-order > gpurun_out/r04i/ab_node_$k.json
done
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 > gpurun_out/r04i/bench_config5.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04i/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/bench_gibbs.py" --iters 30 --warmup 10 > "$GRAFT_REPO_ROOT/gpurun_out/r04i/prof_bench.json"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04i/fetch" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/bench_gibbs.py" --iters 5 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/r04i/fetch_bench.json"
