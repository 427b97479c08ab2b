#!/bin/bash
# One-thread drop-in lines of the default build and of experiment builds in
# ar_orbslam2_amd/_lib_exp/, alternating, after the drop-in tests.
# Usage: bash scripts/gpu_dropin_ab.sh TAG "variant ..."
set -o pipefail
T=${1:-dab}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_dropin_gpu.py tests/test_extract_gpu.py -m gpu -q -x --timeout 240 \
  --timeout-method thread > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for round in 1 2 3; do
  for v in default $2; do
    if [ $v = default ]; then env=""; else env="ORBX_LIB_DIR=ar_orbslam2_amd/_lib_exp/$v ORBX_ALLOW_CUSTOM_BUILD=1"; fi
    env $env timeout -k 10 200 python bench.py --dropin --threads 1 --dropin-frames 400 > gpurun_out/$T/${v}.$round.json 2> gpurun_out/$T/${v}.$round.err || { tail -5 gpurun_out/$T/${v}.$round.err; exit 2; }
    python - gpurun_out/$T/${v}.$round.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["dropin"]["median_ms"], d["dropin"]["per_call_median_ms"])
PY
  done
done
