#!/bin/bash
# Octree A/B: extraction + pipeline parity on the default build, then C2 / C5 bench lines and the
# one-thread drop-in line of the default build and of experiment builds (ar_orbslam2_amd/_lib_exp).
# Usage: bash scripts/gpu_oct_ab.sh TAG "variant ..."
set -o pipefail
T=${1:-oab}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_extract_gpu.py tests/test_pipeline_gpu.py -m gpu -q -x \
  --timeout 240 --timeout-method thread > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
for round in 1 2; do
  for v in default $2; do
    if [ $v = default ]; then env=""; else env="ORBX_LIB_DIR=ar_orbslam2_amd/_lib_exp/$v ORBX_ALLOW_CUSTOM_BUILD=1"; fi
    for C in C2 C5; do
      env $env timeout -k 10 300 python bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --no-upload \
        > gpurun_out/$T/${v}_$C.$round.jsonl 2> gpurun_out/$T/${v}_$C.$round.err || { tail -5 gpurun_out/$T/${v}_$C.$round.err; exit 2; }
    done
    env $env timeout -k 10 200 python bench.py --dropin --threads 1 --dropin-frames 400 > gpurun_out/$T/${v}_d1.$round.json 2> gpurun_out/$T/${v}_d1.$round.err || exit 4
    python - gpurun_out/$T $v $round <<'PY'
import json, sys
o, v, r = sys.argv[1:]
for C in ("C2", "C5"):
    d = json.loads(open("%s/%s_%s.%s.jsonl" % (o, v, C, r)).read())
    st = d["roofline"]["stages_ms_per_step"]
    print(v, C, round(d["value"]), {k: x for k, x in st.items() if k in ("k_octree", "k_fast_cells", "k_pyramid")})
d = json.loads(open("%s/%s_d1.%s.json" % (o, v, r)).read())
print(v, "dropin", d["dropin"]["median_ms"], d["dropin"]["per_call_median_ms"]["orbx_extract"])
PY
  done
done
