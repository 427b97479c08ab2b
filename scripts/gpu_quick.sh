#!/bin/bash
# Quick iteration: selected -m gpu test files, then the C2 bench line and the one-thread drop-in
# line.  Usage: bash scripts/gpu_quick.sh TAG "tests/test_a.py tests/test_b.py"
set -o pipefail
T=${1:-quick}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest ${2:-tests} -m gpu -q -x --timeout 240 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-upload > gpurun_out/$T/c2.jsonl 2> gpurun_out/$T/c2.err || exit 2
timeout -k 10 200 python bench.py --dropin --threads 1 --dropin-frames 400 > gpurun_out/$T/d1.json 2> gpurun_out/$T/d1.err || exit 4
python - <<PY
import json
d = json.loads(open("gpurun_out/$T/c2.jsonl").read())
st = d["roofline"]["stages_ms_per_step"]
print("c2", d["value"], {k: v for k, v in st.items() if v})
d = json.loads(open("gpurun_out/$T/d1.json").read())
print("dropin d1", d["value"], {k: v for k, v in d["dropin"].items() if "median" in k})
PY
