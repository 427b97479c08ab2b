#!/bin/bash
# Bench lines only (no parity tests: timing experiments) of the default build and experiment
# builds in ar_orbslam2_amd/_lib_exp/<name>, stage times printed.
# Usage: bash scripts/gpu_bench_variants.sh TAG "variant ..." ["C2 C5"] [rounds]
set -o pipefail
T=${1:-bv}
mkdir -p gpurun_out/$T
for round in $(seq 1 ${4:-1}); do
  for v in default $2; do
    for C in ${3:-C2 C5}; do
      if [ $v = default ]; then env=""; else env="ORBX_LIB_DIR=ar_orbslam2_amd/_lib_exp/$v ORBX_ALLOW_CUSTOM_BUILD=1"; fi
      env $env timeout -k 10 300 python bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --no-upload \
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
