#!/bin/bash
# Drop-in A/B of one environment switch at 1 / 4 / 8 host threads (twice, alternated), after the
# threaded parity tests with the switch on.  Usage: bash scripts/gpu_dropin_threads_ab.sh TAG VAR=1
set -o pipefail
T=$1; V=$2
mkdir -p gpurun_out/$T
env $V timeout -k 10 400 python -u -m pytest tests/test_threads_gpu.py tests/test_extract_gpu.py -m gpu -q -x --timeout 240 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for rep in 1 2; do for th in 1 4 8; do for x in "$V" ""; do
  env $x timeout -k 10 200 python bench.py --dropin --threads $th --dropin-frames 300 > gpurun_out/$T/d.json 2>/dev/null || exit 4
  python -c "import json; d=json.load(open('gpurun_out/$T/d.json')); print('t$th [$x]', d['value'], d['dropin']['median_ms'])"
done; done; done
