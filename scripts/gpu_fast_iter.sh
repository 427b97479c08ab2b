#!/bin/bash
# FAST iteration: the extraction and pipeline parity tests (every batch plan runs k_fast_pairs),
# then the C2 / C5 bench lines (stage times).  Usage: bash scripts/gpu_fast_iter.sh TAG
set -o pipefail
T=${1:-fast}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_extract_gpu.py tests/test_pipeline_gpu.py -m gpu -q -x \
  --timeout 240 --timeout-method thread > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-upload > gpurun_out/$T/c2.jsonl 2> gpurun_out/$T/c2.err || exit 2
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/$T/c5.jsonl 2> gpurun_out/$T/c5.err || exit 3
python - <<PY
import json
for c in ("c2", "c5"):
    d = json.loads(open("gpurun_out/$T/%s.jsonl" % c).read())
    st = d["roofline"]["stages_ms_per_step"]
    print(c, d["value"], {k: v for k, v in st.items() if v})
PY
