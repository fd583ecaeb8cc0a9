#!/bin/bash
# Round 4: LDS counters of the m = 15 sweep (the exp-table reads): bank conflicts, LDS instructions, waits.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r04t
mkdir -p $o
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES \
  --output-format csv -d "$GRAFT_REPO_ROOT/$o/lds" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 30 --cpu-seconds 0 \
  > "$GRAFT_REPO_ROOT/$o/lds.json" 2> "$GRAFT_REPO_ROOT/$o/lds.err" || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$GRAFT_REPO_ROOT/$o/wait" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 30 --cpu-seconds 0 \
  > "$GRAFT_REPO_ROOT/$o/wait.json" 2> "$GRAFT_REPO_ROOT/$o/wait.err" || exit 1
