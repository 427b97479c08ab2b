#!/bin/bash
# Drop-in A/B: the parity tests of the extraction paths with the defaults, then the one-thread
# drop-in line under each setting of two environment switches, alternated.
# Usage: bash scripts/gpu_dropin_ab.sh TAG VAR1 VAR2 [tests...]
set -o pipefail
T=$1; A=$2; B=$3; shift 3
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest ${@:-tests} -m gpu -q -x --timeout 240 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for rep in 1 2; do
  for a in 1 0; do for b in 1 0; do
    env $A=$a $B=$b timeout -k 10 200 python bench.py --dropin --threads 1 --dropin-frames 400 > gpurun_out/$T/d$a$b.json 2> gpurun_out/$T/d$a$b.err || exit 4
    python -c "import json; d=json.load(open('gpurun_out/$T/d$a$b.json')); print('$A=$a $B=$b', d['value'], d['dropin']['median_ms'], d['dropin']['per_call_median_ms']['orbx_extract'])"
  done; done
done
