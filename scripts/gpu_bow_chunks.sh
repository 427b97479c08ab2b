#!/bin/bash
# k_bow_nodes register chunks (ORBX_BOW_CHUNKS variants built by build_variants.sh) on C5 / C2.
set -o pipefail
T=${1:-bowch}
mkdir -p gpurun_out/$T
for C in C5 C2; do
  for v in default ch4 ch8; do
    if [ $v = default ]; then E=""; else E="ORBX_ALLOW_CUSTOM_BUILD=1 ORBX_LIB_DIR=ar_orbslam2_amd/_lib_exp/$v"; fi
    env $E timeout -k 10 200 python bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/$T/$C-$v.jsonl 2>/dev/null || exit 2
    python -c "import json; d=json.loads(open('gpurun_out/$T/$C-$v.jsonl').read().strip().splitlines()[-1]); st=d['roofline']['stages_ms_per_step']; print('$C $v', d['value'], st['k_bow'], st['k_tri'])"
  done
done
