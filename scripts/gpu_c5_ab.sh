#!/bin/bash
# C5 headline A/B of an environment switch, alternated three times (after the pipeline tests).
set -o pipefail
T=$1; V=$2
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_pipeline_gpu.py tests/test_match_gpu.py -m gpu -q -x --timeout 240 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for rep in 1 2 3; do for x in "$V" ""; do
  env $x timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/$T/c5.jsonl 2>/dev/null || exit 2
  python -c "import json; d=json.loads(open('gpurun_out/$T/c5.jsonl').read().strip().splitlines()[-1]); st=d['roofline']['stages_ms_per_step']; print('[$x]', d['value'], st['k_bow'], st['k_tri'])"
done; done
