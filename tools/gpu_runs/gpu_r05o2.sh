#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 PYTHONPATH=.
timeout -k 10 300 python -u tools/diag_pairs.py
