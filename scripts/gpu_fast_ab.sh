#!/bin/bash
# FAST A/B: the extraction + pipeline parity tests on the default build, then the C2 / C5 bench
# lines (stage times) of the default build and of experiment builds in ar_orbslam2_amd/_lib_exp/
# (make OUT=../_lib_exp/<name>), alternating, two rounds.
# Usage: bash scripts/gpu_fast_ab.sh TAG "variant ..." ["C2 C5"] [tests]
set -o pipefail
T=${1:-fab}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest ${4:-tests/test_extract_gpu.py tests/test_pipeline_gpu.py} -m gpu -q -x \
  --timeout 240 --timeout-method thread > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for round in 1 2; do
  for v in default $2; do
    for C in ${3:-C2 C5}; do
      if [ $v = default ]; then env=""; else env="ORBX_LIB_DIR=ar_orbslam2_amd/_lib_exp/$v ORBX_ALLOW_CUSTOM_BUILD=1"; fi
      env $env timeout -k 10 300 python bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-upload \
        > gpurun_out/$T/${v}_$C.$round.jsonl 2> gpurun_out/$T/${v}_$C.$round.err || { tail -5 gpurun_out/$T/${v}_$C.$round.err; exit 2; }
      python - gpurun_out/$T/${v}_$C.$round.jsonl $v $C <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
st = d["roofline"]["stages_ms_per_step"]
print(sys.argv[2], sys.argv[3], round(d["value"]), {k: v for k, v in st.items() if k in ("k_pyramid", "k_blur", "k_fast_cells", "k_describe", "k_octree")})
PY
    done
  done
done
