#!/bin/bash
# One rocprofv3 --pmc pass of the SQ stall counters (where a latency-bound kernel's wave cycles
# go: parked on s_waitcnt / barrier, issue-stalled, issuing; LDS instruction and bank-conflict
# cycles) for one bench command.  Usage (repo root, on the box):
#   bash scripts/pmc_stall.sh <outdir> [bench args...]      -> <outdir>/stall.csv
set -e -o pipefail
D=$(cd "$(dirname "$1")" && pwd)/$(basename "$1"); shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc $SQ --output-format csv -d $D/s -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-upload --steps 5 "$@" > /dev/null 2> $D/s.err
cp $(find $D/s -name "*counter_collection.csv") $D/stall.csv
rm -rf $D/s
