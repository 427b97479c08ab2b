#!/bin/bash
# Full iteration: the whole -m gpu suite, then the C2 / C5 bench lines and the one-thread
# drop-in line.  Usage: bash scripts/gpu_all_iter.sh TAG
set -o pipefail
T=${1:-iter}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-upload > gpurun_out/$T/c2.jsonl 2> gpurun_out/$T/c2.err || exit 2
timeout -k 10 200 python bench.py --dropin --threads 1 --dropin-frames 400 > gpurun_out/$T/d1.json 2> gpurun_out/$T/d1.err || exit 4
timeout -k 10 200 python bench.py --dropin --threads 8 --dropin-frames 300 > gpurun_out/$T/d8.json 2> gpurun_out/$T/d8.err || exit 5
python - <<PY
import json
d = json.loads(open("gpurun_out/$T/c2.jsonl").read())
st = d["roofline"]["stages_ms_per_step"]
print("c2", d["value"], {k: v for k, v in st.items() if v})
for t in ("d1", "d8"):
    d = json.loads(open("gpurun_out/$T/%s.json" % t).read())
    print("dropin", t, d["value"], {k: v for k, v in d["dropin"].items() if "median" in k})
PY
