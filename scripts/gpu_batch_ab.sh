#!/bin/bash
# Batch size A/B for the stereo and C5 configs (256 vs 512 frames per batch), alternated twice.
set -o pipefail
T=${1:-bab}
mkdir -p gpurun_out/$T
for rep in 1 2; do for C in C3 C4 C5; do for B in 512 256; do
  timeout -k 10 200 python bench.py --config $C --batch $B --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/$T/x.jsonl 2>/dev/null || exit 2
  python -c "import json; d=json.loads(open('gpurun_out/$T/x.jsonl').read().strip().splitlines()[-1]); print('$C B=$B', d['value'])"
done; done; done
