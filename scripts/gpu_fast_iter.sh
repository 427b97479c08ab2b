#!/bin/bash
# Quick iteration on the FAST kernels: extraction parity tests (single-image and batch plans),
# the batch pipeline tests, then the C2 / C4 / C5 bench lines and the one-thread drop-in line
# (no CPU baseline, no PCIe leg).  Usage: bash scripts/gpu_fast_iter.sh TAG
set -o pipefail
T=${1:-iter}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_extract_gpu.py tests/test_pipeline_gpu.py -m gpu -v -x \
  --timeout 300 --timeout-method thread -k "not topology" > gpurun_out/$T/tests.txt 2>&1 || { tail -40 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for C in C2 C4 C5; do
  timeout -k 10 200 python bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/$T/$C.jsonl 2> gpurun_out/$T/$C.err || exit 2
done
timeout -k 10 200 python bench.py --dropin --threads 1 --dropin-frames 400 > gpurun_out/$T/d1.json 2> gpurun_out/$T/d1.err || exit 4
python - <<PY
import json
for c in ("C2", "C4", "C5"):
    d = json.loads(open("gpurun_out/$T/%s.jsonl" % c).read())
    st = d["roofline"]["stages_ms_per_step"]
    print(c, d["value"], {k: v for k, v in st.items() if v})
d = json.loads(open("gpurun_out/$T/d1.json").read())
print("dropin t1", d["value"], {k: v for k, v in d["dropin"].items() if "median" in k})
PY
