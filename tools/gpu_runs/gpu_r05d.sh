#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 PYTHONPATH=.
mkdir -p gpurun_out/r05d
timeout -k 10 300 python -u tools/diag_plan_dump.py --m 13 --out gpurun_out/r05d/plan13.npz
