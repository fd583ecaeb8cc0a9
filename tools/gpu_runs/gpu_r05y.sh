#!/bin/bash
# Round 5: the final in-tree library -- smoke and the Gibbs / chain tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_gibbs_chains.py tests/test_gpu_gibbs.py -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
