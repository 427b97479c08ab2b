#!/bin/bash
# Batch size x camera streams sweep of the headline command (C2 unless $1 names a config):
# one bench line per setting, timed region only (no CPU baseline, upload pass or roofline pass).
# Usage: bash scripts/sweep_batches.sh [C2] > gpurun_out/sweep.jsonl
set -e -o pipefail
CFG=${1:-C2}
for BS in "256 3" "512 3" "384 3" "256 4" "512 2" "128 6" "768 2"; do
  set -- $BS
  timeout -k 10 120 python -u bench.py --config $CFG --batch $1 --streams $2 --steps 20 \
    --no-cpu-baseline --no-upload --no-profile |
    python -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(json.dumps({'batch': $1, 'streams': $2, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))"
done
