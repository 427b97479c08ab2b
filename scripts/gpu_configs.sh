#!/bin/bash
# Iteration check: the whole -m gpu suite (or the test files given as $2), then the bench line of
# every configuration (C2 C3 C4 C5 AR) and the one-thread drop-in line, with each line's stage
# times.  Usage: bash scripts/gpu_configs.sh TAG ["tests/test_a.py ..."]
set -o pipefail
T=${1:-cfg}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest ${2:-tests} -m gpu -q -x --timeout 300 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for C in C2 C3 C4 C5 AR; do
  timeout -k 10 200 python bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-upload \
    > gpurun_out/$T/$C.jsonl 2> gpurun_out/$T/$C.err || { tail -5 gpurun_out/$T/$C.err; exit 2; }
  python - gpurun_out/$T/$C.jsonl $C <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
st = d["roofline"]["stages_ms_per_step"]
print(sys.argv[2], round(d["value"]), {k: v for k, v in st.items() if v > 0.02})
PY
done
timeout -k 10 200 python bench.py --dropin --threads 1 --dropin-frames 400 > gpurun_out/$T/d1.json 2> gpurun_out/$T/d1.err || exit 4
python - gpurun_out/$T/d1.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("dropin d1", d["value"], {k: v for k, v in d["dropin"].items() if "median" in k})
PY
