#!/bin/bash
# Quick iteration on the FAST kernel: extraction parity tests, then the C2 and C5 bench lines
# and the one-thread drop-in line (no CPU baseline, no PCIe leg).  Usage: bash scripts/gpu_fast_iter.sh TAG
set -o pipefail
T=${1:-iter}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_pipeline_gpu.py tests/test_cvorb_gpu.py -m gpu -q -x \
  --timeout 300 --timeout-method thread -k "not topology" > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-upload > gpurun_out/$T/c2.jsonl 2> gpurun_out/$T/c2.err || exit 2
timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/$T/c5.jsonl 2> gpurun_out/$T/c5.err || exit 3
timeout -k 10 200 python bench.py --dropin --threads 1 --dropin-frames 400 > gpurun_out/$T/d1.json 2> gpurun_out/$T/d1.err || exit 4
python - <<PY
import json
for c in ("c2", "c5"):
    d = json.loads(open("gpurun_out/$T/%s.jsonl" % c).read())
    st = d["roofline"]["stages_ms_per_step"]
    print(c, d["value"], {k: v for k, v in st.items() if v})
d = json.loads(open("gpurun_out/$T/d1.json").read())
print("dropin t1", d["value"], {k: v for k, v in d["dropin"].items() if "median" in k or "mean" in k})
PY
