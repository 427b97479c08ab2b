#!/bin/bash
# C2 headline A/B of an environment switch, alternated three times (after the extraction tests).
set -o pipefail
T=$1; V=$2
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_extract_gpu.py tests/test_pipeline_gpu.py -m gpu -q -x --timeout 240 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for rep in 1 2 3; do for x in "$V" ""; do
  env $x timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-upload > gpurun_out/$T/c2.jsonl 2>/dev/null || exit 2
  python -c "import json; d=json.loads(open('gpurun_out/$T/c2.jsonl').read().strip().splitlines()[-1]); print('[$x]', d['value'])"
done; done
