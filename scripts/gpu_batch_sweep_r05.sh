#!/bin/bash
# Camera streams x frames per stream for every config at the round-5 kernels (DESIGN.md, round 5
# not kept).  Usage on the GPU box: bash scripts/gpu_batch_sweep_r05.sh <out tag>
set -o pipefail
T=$1
mkdir -p gpurun_out/$T
run() { # cfg streams batch tag
  timeout -k 10 300 python bench.py --config $1 --streams $2 --batch $3 --steps 12 --warmup 3 --no-cpu-baseline --no-upload --no-profile > gpurun_out/$T/$1_s$2_b$3_$4.jsonl 2> gpurun_out/$T/$1_s$2_b$3_$4.err || { tail -5 gpurun_out/$T/$1_s$2_b$3_$4.err; exit 2; }
  python -c "import json; d=json.loads(open('gpurun_out/$T/$1_s$2_b$3_$4.jsonl').read().strip().splitlines()[-1]); print('$1 streams $2 batch $3', d['value'])"
}
for r in 1 2; do
  for sb in "3 512" "3 1024" "2 1024" "3 768" "2 1536" "3 1536" "3 2048" "4 384" "6 256"; do run C2 $sb $r || exit 2; done
  for c in AR C3 C4 C5; do for sb in "3 512" "3 1024" "2 1024"; do run $c $sb $r || exit 2; done; done
done
