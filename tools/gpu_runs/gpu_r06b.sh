#!/bin/bash
# Round 6: where the planned kernel's time goes -- timing probes (wrong values, same instruction stream):
# conflict-free point reads (1), conflict-free fill reads (2), every wave on tile 0's cache-resident plan (4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06b
mkdir -p $o
for rep in 1 2; do
  for v in off:pynngp_amd/_build/libnngp_hip.so on:pynngp_amd/_build/libnngp_hip.so p1:ab/probe1/libnngp_hip.so \
           p2:ab/probe2/libnngp_hip.so p4:ab/probe4/libnngp_hip.so p7:ab/probe7/libnngp_hip.so; do
    label=${v%%:*}; lib=${v#*:}; plan=on; [ $label = off ] && plan=off
    NNGP_LIB=$(pwd)/$lib timeout -k 10 120 python bench.py --steps 200 --warmup 200 --cpu-seconds 0 --plan $plan \
      > $o/$label.$rep.json 2>> $o/err.log || exit 1
    python3 -c "import json; d=json.load(open('$o/$label.$rep.json')); print('$label', $rep, round(d['roofline']['kernel_ms'],4), 'ms', round(d['value']/1e9,3), 'Gloc/s', d['lib'])"
  done
done
