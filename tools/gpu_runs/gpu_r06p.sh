#!/bin/bash
# Round 6: the covariance-blocks kind left-looking (tools/variants/blocks_left.patch) against the current
# right-looking kernel, m = 18..24 at N = 10^6, same box, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06p
mkdir -p $o
for r in 1 2; do for v in cur:pynngp_amd/_build/libnngp_hip.so left:ab/blocks_left/libnngp_hip.so; do
  label=${v%%:*}; lib=$(pwd)/${v#*:}
  NNGP_LIB=$lib timeout -k 10 300 python tools/bench_blocks_m.py 18 19 20 21 22 23 24 > $o/$label.$r.json 2>> $o/err.log || exit 1
  cat $o/$label.$r.json
done; done
