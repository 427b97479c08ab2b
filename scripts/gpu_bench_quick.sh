#!/bin/bash
# Bench lines only (no tests): C2 and optionally more configs; prints stage times.
# Usage: bash scripts/gpu_bench_quick.sh TAG "C2 C5"
set -o pipefail
T=${1:-bq}
mkdir -p gpurun_out/$T
for C in ${2:-C2}; do
  timeout -k 10 300 python bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-upload \
    > gpurun_out/$T/$C.jsonl 2> gpurun_out/$T/$C.err || exit 2
done
python - <<PY
import json
for c in "${2:-C2}".split():
    d = json.loads(open("gpurun_out/$T/%s.jsonl" % c).read())
    st = d["roofline"]["stages_ms_per_step"]
    print(c, d["value"], {k: v for k, v in st.items() if v})
PY
