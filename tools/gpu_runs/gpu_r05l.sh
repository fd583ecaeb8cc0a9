#!/bin/bash
# Round 5: config 5 chain modes on one box -- batches of chains on their own streams / host threads
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05l2
mkdir -p $o
b() {  # name, args
  timeout -k 10 400 python bench.py --config 5 --cpu-seconds 0 --steps 300 --warmup 50 $2 > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$o/$1.json')); print('$1', round(d['value'], 1), round(d['ms_per_step'], 4), d['config'].get('chain_mode'), d['config'].get('chain_groups'))"
}
b c5_1 ""
b c5_4_g2 "--chains-per-gpu 4 --chain-mode batched-streams --chain-groups 2"
b c5_4_g4 "--chains-per-gpu 4 --chain-mode batched-streams --chain-groups 4"
b c5_6_g3 "--chains-per-gpu 6 --chain-mode batched-streams --chain-groups 3"
b c5_6_g2 "--chains-per-gpu 6 --chain-mode batched-streams --chain-groups 2"
b c5_8_g2 "--chains-per-gpu 8 --chain-mode batched-streams --chain-groups 2"
b c5_8_g4 "--chains-per-gpu 8 --chain-mode batched-streams --chain-groups 4"
b c5_3_g3 "--chains-per-gpu 3 --chain-mode batched-streams --chain-groups 3"
