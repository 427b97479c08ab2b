#!/bin/bash
# C2 headline and stage times of experiment builds (build_variants.sh) against the default
# library, alternated twice.  Usage: bash scripts/gpu_variant_ab.sh TAG variant1 variant2 ...
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
for rep in 1 2; do for v in default "$@"; do
  if [ $v = default ]; then E=""; else E="ORBX_ALLOW_CUSTOM_BUILD=1 ORBX_LIB_DIR=ar_orbslam2_amd/_lib_exp/$v"; fi
  env $E timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-upload > gpurun_out/$T/c2.jsonl 2>/dev/null || exit 2
  python -c "import json; d=json.loads(open('gpurun_out/$T/c2.jsonl').read().strip().splitlines()[-1]); st=d['roofline']['stages_ms_per_step']; print('$v', d['value'], st['k_pyramid'], st['k_blur'])"
done; done
