#!/bin/bash
# Full -m gpu suite, then the drop-in lines (C ABI and shim-shaped, one thread).
# Usage: bash scripts/gpu_full.sh TAG
set -o pipefail
T=${1:-full}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -40 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
timeout -k 10 200 python bench.py --dropin --threads 1 --dropin-frames 400 > gpurun_out/$T/d1.json 2> gpurun_out/$T/d1.err || exit 4
timeout -k 10 200 python bench.py --dropin --dropin-mode shim --threads 1 --dropin-frames 400 > gpurun_out/$T/d1s.json 2> gpurun_out/$T/d1s.err || exit 5
python - <<PY
import json
for f in ("d1", "d1s"):
    d = json.loads(open("gpurun_out/$T/%s.json" % f).read())
    print(f, d["value"], d["dropin"]["median_ms"], {k: v for k, v in d["dropin"]["per_call_median_ms"].items()})
PY
