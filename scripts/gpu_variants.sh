#!/bin/bash
# Bench lines (C2, and C5 when $2 = c5) for each experiment build in ar_orbslam2_amd/_lib_exp/
# and the default build, with optional per-variant environment: arguments are
# "name[:ENV=V,...]" items (name "default" = the tree's build).  Parity of a variant must be
# checked before adopting it.  Usage: bash scripts/gpu_variants.sh TAG "c2|c5" item...
set -o pipefail
T=$1; CFG=$2; shift 2
O=gpurun_out/$T; mkdir -p $O
for item in "$@"; do
  name=${item%%:*}; envs=""; [ "$item" != "$name" ] && envs=${item#*:}
  ( export ORBX_ALLOW_CUSTOM_BUILD=1
    [ "$name" != default ] && export ORBX_LIB_DIR=$PWD/ar_orbslam2_amd/_lib_exp/$name
    for kv in ${envs//,/ }; do export "$kv"; done
    args="--steps 20 --warmup 3"; [ "$CFG" = c5 ] && args="--config C5 --steps 10 --warmup 2"
    timeout -k 10 200 python bench.py $args --no-cpu-baseline --no-upload > $O/$item.jsonl 2> $O/$item.err
  ) || { echo "$item failed"; tail -5 "$O/$item.err"; exit 1; }
  python - "$O/$item.jsonl" "$item" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
st = d["roofline"]["stages_ms_per_step"]
print(sys.argv[2], d["value"], {k: v for k, v in st.items() if k.startswith("k_fast")})
PY
done
