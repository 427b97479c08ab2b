#!/bin/bash
# Selected -m gpu test files, then the C5 and C2 bench lines (stage times of the matchers).
set -o pipefail
T=${1:-c5q}; shift
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest ${@:-tests} -m gpu -q -x --timeout 240 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for C in C5 C2; do
  timeout -k 10 200 python bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/$T/$C.jsonl 2>/dev/null || exit 2
  python -c "import json; d=json.loads(open('gpurun_out/$T/$C.jsonl').read().strip().splitlines()[-1]); st=d['roofline']['stages_ms_per_step']; print('$C', d['value'], st['k_bow'], st['k_tri'])"
done
