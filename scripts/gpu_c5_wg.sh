#!/bin/bash
# C5 / C4 bench lines with the workgroup-per-node matcher kernels forced on for batches (A/B).
set -o pipefail
T=${1:-c5wg}
mkdir -p gpurun_out/$T
for C in C5 C4; do
  for v in default bow tri both; do
    case $v in
      default) E="";;
      bow) E="ORBX_BOW_WG_PROBS=100000";;
      tri) E="ORBX_TRI_WG_PROBS=100000";;
      both) E="ORBX_BOW_WG_PROBS=100000 ORBX_TRI_WG_PROBS=100000";;
    esac
    env $E timeout -k 10 200 python bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/$T/$C-$v.jsonl 2>/dev/null || exit 2
    python -c "import json; d=json.loads(open('gpurun_out/$T/$C-$v.jsonl').read().strip().splitlines()[-1]); st=d['roofline']['stages_ms_per_step']; print('$C $v', d['value'], st['k_bow'], st['k_tri'])"
  done
done
